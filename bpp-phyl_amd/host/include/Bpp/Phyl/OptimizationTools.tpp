// Brent's method (golden section + successive parabolic interpolation) on [a, b].
#include <cmath>

namespace bpp {

template <class F>
double OptimizationTools::brent(F f, double a, double b, double x0, double tol, unsigned int maxEval, double* fmin,
                                unsigned int* nEval) {
  const double cgold = 0.3819660112501051;
  double x = std::min(std::max(x0, a), b), w = x, v = x;
  double fx = f(x), fw = fx, fv = fx;
  unsigned int n = 1;
  double d = 0., e = 0.;
  while (n < maxEval) {
    const double xm = 0.5 * (a + b);
    const double tol1 = tol * std::fabs(x) + 1e-10, tol2 = 2. * tol1;
    if (std::fabs(x - xm) <= tol2 - 0.5 * (b - a)) break;
    bool golden = true;
    if (std::fabs(e) > tol1) {
      double r = (x - w) * (fx - fv);
      double q = (x - v) * (fx - fw);
      double p = (x - v) * q - (x - w) * r;
      q = 2. * (q - r);
      if (q > 0.) p = -p;
      q = std::fabs(q);
      const double etemp = e;
      e = d;
      if (!(std::fabs(p) >= std::fabs(0.5 * q * etemp) || p <= q * (a - x) || p >= q * (b - x))) {
        d = p / q;
        const double u = x + d;
        if (u - a < tol2 || b - u < tol2) d = (xm - x >= 0.) ? tol1 : -tol1;
        golden = false;
      }
    }
    if (golden) {
      e = (x >= xm) ? a - x : b - x;
      d = cgold * e;
    }
    const double u = (std::fabs(d) >= tol1) ? x + d : x + ((d >= 0.) ? tol1 : -tol1);
    const double fu = f(u);
    n++;
    if (fu <= fx) {
      if (u >= x) a = x; else b = x;
      v = w; fv = fw;
      w = x; fw = fx;
      x = u; fx = fu;
    } else {
      if (u < x) a = u; else b = u;
      if (fu <= fw || w == x) {
        v = w; fv = fw;
        w = u; fw = fu;
      } else if (fu <= fv || v == x || v == w) {
        v = u; fv = fu;
      }
    }
  }
  if (fmin) *fmin = fx;
  if (nEval) *nEval += n;
  return x;
}

}  // namespace bpp
