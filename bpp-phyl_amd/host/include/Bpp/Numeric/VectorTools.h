// bpp-core VectorTools subset: element-wise vector arithmetic operators and vectorUnion.
#ifndef BPP_AMD_VECTORTOOLS_H
#define BPP_AMD_VECTORTOOLS_H

#include <algorithm>
#include <vector>

namespace bpp {

template <class T, class U>
std::vector<T>& operator/=(std::vector<T>& v, const U& c) {
  for (auto& x : v) x /= c;
  return v;
}
template <class T, class U>
std::vector<T>& operator*=(std::vector<T>& v, const U& c) {
  for (auto& x : v) x *= c;
  return v;
}
template <class T>
std::vector<T>& operator+=(std::vector<T>& v, const std::vector<T>& w) {
  for (size_t i = 0; i < v.size() && i < w.size(); i++) v[i] += w[i];
  return v;
}

struct VectorTools {
  // elements of v1 then those of v2 not in v1, each once, in order of appearance
  template <class T>
  static std::vector<T> vectorUnion(const std::vector<T>& v1, const std::vector<T>& v2) {
    std::vector<T> out;
    for (const T& x : v1)
      if (std::find(out.begin(), out.end(), x) == out.end()) out.push_back(x);
    for (const T& x : v2)
      if (std::find(out.begin(), out.end(), x) == out.end()) out.push_back(x);
    return out;
  }
  template <class T>
  static T sum(const std::vector<T>& v) {
    T s = T();
    for (const T& x : v) s += x;
    return s;
  }
};

}  // namespace bpp

#endif
