// Dense row-major matrices (bpp-core RowMatrix subset) and the symmetric
// eigen-solver used by the reversible models.
#ifndef BPP_AMD_MATRIX_H
#define BPP_AMD_MATRIX_H

#include <vector>

namespace bpp {

typedef std::vector<double> Vdouble;
typedef std::vector<Vdouble> VVdouble;
typedef std::vector<VVdouble> VVVdouble;
typedef std::vector<int> Vint;

template <class T>
class RowMatrix {
  size_t nRows_ = 0, nCols_ = 0;
  std::vector<T> data_;

 public:
  RowMatrix() {}
  RowMatrix(size_t r, size_t c) : nRows_(r), nCols_(c), data_(r * c, T()) {}
  void resize(size_t r, size_t c) {
    nRows_ = r;
    nCols_ = c;
    data_.assign(r * c, T());
  }
  size_t getNumberOfRows() const { return nRows_; }
  size_t getNumberOfColumns() const { return nCols_; }
  T& operator()(size_t i, size_t j) { return data_[i * nCols_ + j]; }
  const T& operator()(size_t i, size_t j) const { return data_[i * nCols_ + j]; }
  const T* data() const { return data_.data(); }
  T* data() { return data_.data(); }
  std::vector<T> row(size_t i) const { return std::vector<T>(data_.begin() + i * nCols_, data_.begin() + (i + 1) * nCols_); }
};

// Symmetric eigen-decomposition of the n x n row-major matrix A (Householder
// reduction to tridiagonal form followed by implicit-shift QL).  On return
// d[k] are the eigenvalues and column k of U (row-major) the eigenvectors.
void symmetricEigen(size_t n, const std::vector<double>& A, std::vector<double>& d, std::vector<double>& U);

}  // namespace bpp

#endif
