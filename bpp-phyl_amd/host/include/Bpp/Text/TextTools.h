#ifndef BPP_AMD_TEXTTOOLS_H
#define BPP_AMD_TEXTTOOLS_H
#include <sstream>
#include <string>
namespace bpp {
struct TextTools {
  template <class T>
  static std::string toString(T t) {
    std::ostringstream o;
    o << t;
    return o.str();
  }
  template <class T>
  static std::string toString(T t, int precision) {
    std::ostringstream o;
    o.precision(precision);
    o << t;
    return o.str();
  }
  template <class T>
  static T to(const std::string& s) {
    std::istringstream i(s);
    T t;
    i >> t;
    return t;
  }
  static double toDouble(const std::string& s) { return to<double>(s); }
  static int toInt(const std::string& s) { return to<int>(s); }
  static bool isEmpty(const std::string& s) { return s.find_first_not_of(" \t\n\r") == std::string::npos; }
  static std::string removeSurroundingWhiteSpaces(const std::string& s) {
    size_t a = s.find_first_not_of(" \t\n\r");
    if (a == std::string::npos) return "";
    size_t b = s.find_last_not_of(" \t\n\r");
    return s.substr(a, b - a + 1);
  }
};
}  // namespace bpp
#endif
