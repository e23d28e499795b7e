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

// Real eigen-decomposition of a general (nonsymmetric) n x n row-major matrix A, in the
// layout of the reference's EigenValue (getV / getRealEigenValues / getImagEigenValues,
// used by Model/AbstractSubstitutionModel.cpp:276-281): a complex pair a +- ib occupies
// positions k, k+1 with wi[k] = b > 0, wi[k+1] = -b, and columns k, k+1 of V (row-major)
// hold Re v, Im v of the eigenvector of a + ib, so that A V = V D with D block-diagonal,
// D(k,k) = D(k+1,k+1) = a, D(k,k+1) = b, D(k+1,k) = -b.  Eigenvalues: complex shifted QR
// on the Hessenberg form; eigenvectors: inverse iteration (vectors of a repeated
// eigenvalue deflated against each other).  Returns false if the iteration does not
// converge.
bool generalEigen(size_t n, const std::vector<double>& A, std::vector<double>& wr, std::vector<double>& wi,
                  std::vector<double>& V);

// Inverse of the n x n row-major matrix A (LU with partial pivoting); false if singular.
bool invertMatrix(size_t n, const std::vector<double>& A, std::vector<double>& Ainv);

}  // namespace bpp

#endif
