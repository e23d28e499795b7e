// bpp-core MatrixTools subset (print) over the mirror's RowMatrix.
#ifndef BPP_AMD_MATRIXTOOLS_H
#define BPP_AMD_MATRIXTOOLS_H

#include <iostream>

#include "Matrix.h"

namespace bpp {

struct MatrixTools {
  template <class T>
  static void print(const RowMatrix<T>& m, std::ostream& out = std::cout) {
    out << m.getNumberOfRows() << "x" << m.getNumberOfColumns() << std::endl << "[" << std::endl;
    for (size_t i = 0; i < m.getNumberOfRows(); i++) {
      out << "[";
      for (size_t j = 0; j < m.getNumberOfColumns(); j++) out << (j ? ", " : "") << m(i, j);
      out << "]" << std::endl;
    }
    out << "]" << std::endl;
  }
};

}  // namespace bpp

#endif
