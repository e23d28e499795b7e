// Host mirror: optimisers over the GPU likelihood (see OptimizationTools.h).
#include "Bpp/Phyl/OptimizationTools.h"

#include <cmath>
#include <limits>

namespace bpp {

const std::string OptimizationTools::OPTIMIZATION_NEWTON = "newton";
const std::string OptimizationTools::OPTIMIZATION_GRADIENT = "gradient";
const std::string OptimizationTools::OPTIMIZATION_BRENT = "Brent";
const std::string OptimizationTools::OPTIMIZATION_BFGS = "BFGS";

namespace {

double setAndEval(TreeLikelihood* tl, ParameterList& pl, size_t i, double value) {
  pl[i].setValue(value);
  ParameterList one;
  one.addParameter(pl[i]);
  tl->setParameters(one);
  return tl->getValue();
}

// Search interval for one parameter: positive unbounded parameters are searched on a
// log scale around the current value, bounded ones over their (open) interval.
void searchInterval(const Parameter& p, double* lo, double* hi, bool* logScale) {
  double a = -1e300, b = 1e300;
  bool sa = false, sb = false;
  if (p.hasConstraint()) {
    a = p.getConstraint()->getLowerBound();
    b = p.getConstraint()->getUpperBound();
    sa = p.getConstraint()->strictLowerBound();
    sb = p.getConstraint()->strictUpperBound();
  }
  const double x = p.getValue();
  if (a >= 0. && !std::isfinite(b)) {
    *logScale = true;
    const double la = std::log(std::max(a, 1e-12) * (sa ? 1.0001 : 1.)), lx = std::log(std::max(x, 1e-12));
    *lo = std::max(la, lx - 4.);
    *hi = lx + 4.;
  } else {
    *logScale = false;
    const double eps = 1e-7 * std::max(1., std::fabs(b - a));
    *lo = std::isfinite(a) ? a + (sa ? eps : 0.) : x - 10. * std::max(1., std::fabs(x));
    *hi = std::isfinite(b) ? b - (sb ? eps : 0.) : x + 10. * std::max(1., std::fabs(x));
    if (std::isfinite(b) && std::isfinite(a) && b - a > 1e3) {
      *lo = std::max(*lo, x - 10. * std::max(1., std::fabs(x)));
      *hi = std::min(*hi, x + 10. * std::max(1., std::fabs(x)));
    }
  }
}

}  // namespace

unsigned int OptimizationTools::optimizeTreeScale(TreeLikelihood* tl, double tolerance, unsigned int tlEvalMax,
                                                  OutputStream*, OutputStream*, unsigned int) {
  ParameterList bl = tl->getBranchLengthsParameters();
  std::vector<double> b0(bl.size());
  for (size_t i = 0; i < bl.size(); i++) b0[i] = bl[i].getValue();
  unsigned int nEval = 0;
  auto f = [&](double logScale) {
    const double s = std::exp(logScale);
    ParameterList pl = bl;
    for (size_t i = 0; i < pl.size(); i++) pl[i].setValue(std::min(std::max(b0[i] * s, 0.000001), 10000.));
    tl->setParameters(pl);
    return tl->getValue();
  };
  double fmin = 0.;
  const double best = brent(f, std::log(0.01), std::log(100.), 0., tolerance, tlEvalMax, &fmin, &nEval);
  f(best);
  return nEval;
}

unsigned int OptimizationTools::optimizeNumericalParameters2(TreeLikelihood* tl, const ParameterList& parameters,
                                                             OptimizationListener*, double tolerance,
                                                             unsigned int tlEvalMax, OutputStream*, OutputStream*,
                                                             bool, bool, unsigned int, const std::string&) {
  ParameterList pl = tl->getParameters().getCommonParametersWith(parameters);
  unsigned int nEval = 0;
  double fcur = tl->getValue();
  for (int round = 0; round < 200 && nEval < tlEvalMax; round++) {
    const double fstart = fcur;
    for (size_t i = 0; i < pl.size(); i++) {
      double lo, hi;
      bool logScale;
      searchInterval(pl[i], &lo, &hi, &logScale);
      const double x0 = logScale ? std::log(std::max(pl[i].getValue(), 1e-12)) : pl[i].getValue();
      auto f = [&](double u) {
        double v = logScale ? std::exp(u) : u;
        if (pl[i].hasConstraint() && !pl[i].getConstraint()->isCorrect(v)) v = pl[i].getConstraint()->getAcceptedLimit(v);
        return setAndEval(tl, pl, i, v);
      };
      double fmin = 0.;
      const double u = brent(f, lo, hi, x0, 1e-8, 200, &fmin, &nEval);
      double fu = f(u);
      if (fu > fcur) fu = f(x0);  // never accept a worse point
      fcur = fu;
    }
    if (fstart - fcur < tolerance) break;
  }
  return nEval;
}

}  // namespace bpp
