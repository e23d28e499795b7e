// Host mirror: optimisers over the GPU likelihood (see OptimizationTools.h).
#include "Bpp/Phyl/OptimizationTools.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <vector>

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

// One parameter of a PseudoNewton problem: its constraint (CONSTRAINTS_AUTO maps an
// out-of-range value to the accepted limit, bpp-core AutoParameter) and whether the
// likelihood supplies analytic derivatives for it.
struct PNParam {
  std::string name;
  std::shared_ptr<Constraint> constraint;
  bool analytic = false;
  double accept(double v) const {
    return (constraint && !constraint->isCorrect(v)) ? constraint->getAcceptedLimit(v) : v;
  }
  bool correct(double v) const { return !constraint || constraint->isCorrect(v); }
};

// PseudoNewtonOptimizer (Likelihood/PseudoNewtonOptimizer.cpp:96-190) as
// optimizeNumericalParameters2 sets it up for OPTIMIZATION_NEWTON (OptimizationTools.cpp:
// 266-353): the function is -lnL; branch lengths take the likelihood's analytic d1 / d2
// (getFirstOrderDerivative / getSecondOrderDerivative, the device path derivatives), the
// non-derivable parameters a ThreePointsNumericalDerivative of interval 1e-4 (:311-314,
// 330-331).  Each step moves every parameter by d1 / |d2| at once (0 if d2 == 0 or the move
// is NaN), clamped into its constraint; while f grows by more than the tolerance (or is NaN)
// the Felsenstein-Churchill correction halves all moves, at most 10 times, the fourth
// correction being a conjugate-gradient search from the current point (useCG_, :151-170);
// a step that cannot improve keeps the point.  Stop: |f_new - f_old| < tolerance
// (FunctionStopCondition) or the evaluation budget.  f(x) sets every parameter and returns
// -lnL; evaluations are counted in *nEval.
// First derivatives at x (the likelihood sits at x on entry and on return): analytic for the
// derivable parameters, ThreePointsNumericalDerivative (interval 1e-4, one-sided at a
// constraint) for the others; d2 alike when asked for.  With points == 2 the numerical
// derivatives are bpp-core's TwoPointsNumericalDerivative instead: the forward difference
// (f(x + h) - f(x)) / h, backward where x + h leaves the constraint, no d2.
struct Derivatives {
  const std::vector<PNParam>& par;
  const std::function<double(const std::vector<double>&)>& eval;
  const std::function<void(size_t, double*, double*)>& analytic;
  int points = 3;
  double interval = 0.0001;
  void operator()(const std::vector<double>& x, double fx, std::vector<double>& d1, std::vector<double>* d2) const {
    const size_t n = par.size();
    const double kInterval = interval;
    std::vector<double> y(n);
    bool moved_away = false;
    for (size_t i = 0; i < n; i++) {
      double a1 = 0., a2 = 0.;
      if (par[i].analytic) {
        if (moved_away) {
          eval(x);
          moved_away = false;
        }
        analytic(i, &a1, &a2);
      } else {
        const double v = x[i], h = (1. + std::fabs(v)) * kInterval;
        y = x;
        double fm, fp, f2;
        if (points == 2) {
          y[i] = par[i].correct(v + h) ? v + h : v - h;
          a1 = (eval(y) - fx) / (y[i] - v);
        } else if (par[i].correct(v - h) && par[i].correct(v + h)) {
          y[i] = v - h;
          fm = eval(y);
          y[i] = v + h;
          fp = eval(y);
          a1 = (fp - fm) / (2. * h);
          a2 = (fp - 2. * fx + fm) / (h * h);
        } else if (par[i].correct(v + 2. * h)) {  // left limit: forward
          y[i] = v + h;
          fp = eval(y);
          y[i] = v + 2. * h;
          f2 = eval(y);
          a1 = (fp - fx) / h;
          a2 = (f2 - 2. * fp + fx) / (h * h);
        } else {  // right limit: backward
          y[i] = v - h;
          fm = eval(y);
          y[i] = v - 2. * h;
          f2 = eval(y);
          a1 = (fx - fm) / h;
          a2 = (fx - 2. * fm + f2) / (h * h);
        }
        moved_away = true;
      }
      d1[i] = a1;
      if (d2) (*d2)[i] = a2;
    }
    if (moved_away) eval(x);
  }
};

// bpp-core ConjugateGradientMultiDimensions as PseudoNewtonOptimizer uses it (Polak-Ribiere
// directions, a Brent line minimisation along each, FunctionStopCondition |f - f_old| < tol),
// from x / fx; the constraints bound every line search.  Returns the value at the new x.
// *nEval is the caller's evaluation counter (eval counts).
double conjugateGradient(const std::vector<PNParam>& par, std::vector<double>& x, double fx,
                         const std::function<double(const std::vector<double>&)>& eval, const Derivatives& der,
                         double tol, unsigned int maxEval, unsigned int* nEval) {
  const size_t n = par.size();
  std::vector<double> g(n), h(n), xi(n), y(n);
  der(x, fx, xi, nullptr);
  for (size_t j = 0; j < n; j++) g[j] = h[j] = xi[j] = -xi[j];
  for (int it = 0; it < 200 && *nEval < maxEval; it++) {
    // the largest step along xi that stays inside every constraint
    double amax = std::numeric_limits<double>::infinity(), xn = 1., dn = 0.;
    for (size_t j = 0; j < n; j++) {
      xn = std::max(xn, std::fabs(x[j]));
      dn = std::max(dn, std::fabs(xi[j]));
      if (xi[j] == 0. || !par[j].constraint) continue;
      const double lo = par[j].constraint->getLowerBound(), hi = par[j].constraint->getUpperBound();
      const double lim = xi[j] > 0. ? (hi - x[j]) / xi[j] : (lo - x[j]) / xi[j];
      if (std::isfinite(lim)) amax = std::min(amax, lim * (1. - 1e-9));
    }
    if (dn == 0.) break;
    if (!std::isfinite(amax)) amax = 10. * xn / dn;
    auto fl = [&](double a) {
      for (size_t j = 0; j < n; j++) y[j] = par[j].accept(x[j] + a * xi[j]);
      return eval(y);
    };
    double fmin = fx;
    unsigned int ne = 0;
    const double a = OptimizationTools::brent(fl, 0., std::max(amax, 0.), std::min(amax, 0.1 * xn / dn), 1e-6, 100,
                                              &fmin, &ne);
    const double fold = fx;
    if (fmin < fx) {
      for (size_t j = 0; j < n; j++) x[j] = par[j].accept(x[j] + a * xi[j]);
      fx = eval(x);
    } else {
      eval(x);
    }
    if (std::fabs(fx - fold) < tol) break;
    std::vector<double> gn(n);
    der(x, fx, gn, nullptr);
    double gg = 0., dgg = 0.;
    for (size_t j = 0; j < n; j++) {
      gg += g[j] * g[j];
      dgg += (gn[j] + g[j]) * gn[j];  // Polak-Ribiere
    }
    if (gg == 0.) break;
    const double gam = dgg / gg;
    for (size_t j = 0; j < n; j++) {
      g[j] = -gn[j];
      h[j] = g[j] + gam * h[j];
      xi[j] = h[j];
    }
  }
  return fx;
}

unsigned int pseudoNewton(const std::vector<PNParam>& par, std::vector<double>& x,
                          const std::function<double(const std::vector<double>&)>& f,
                          const std::function<void(size_t, double*, double*)>& analytic, double tolerance,
                          unsigned int maxEval, unsigned int* steps_out,
                          const std::function<void(unsigned int, const std::vector<double>&, double)>& onStep) {
  const size_t n = par.size();
  unsigned int nEval = 0, steps = 0;
  std::function<double(const std::vector<double>&)> eval = [&](const std::vector<double>& y) {
    nEval++;
    return f(y);
  };
  const Derivatives der{par, eval, analytic};
  double fcur = eval(x), fprev = 0.;  // previousValue_ starts at 0 (PseudoNewtonOptimizer.cpp:72)
  std::vector<double> d1(n), d2(n), mv(n), y(n);
  while (nEval < maxEval) {
    steps++;
    der(x, fcur, d1, &d2);  // derivatives at x (the likelihood sits at x)
    // Newton moves (PseudoNewtonOptimizer.cpp:108-135)
    for (size_t i = 0; i < n; i++) {
      double m = d2[i] == 0. ? 0. : (d2[i] < 0. ? -d1[i] / d2[i] : d1[i] / d2[i]);
      if (std::isnan(m)) m = 0.;
      y[i] = par[i].accept(x[i] - m);
      mv[i] = x[i] - y[i];
    }
    double fnew = eval(y);
    // Felsenstein-Churchill correction, the fourth try a conjugate-gradient search (:140-175)
    for (unsigned int count = 0; count < 10 && (fnew > fcur + tolerance || std::isnan(fnew)); count++) {
      if (count == 3) {
        const double tol = std::max(std::fabs(fcur - fprev) / 2., tolerance);
        eval(x);
        y = x;
        fnew = conjugateGradient(par, y, fcur, eval, der, tol, maxEval, &nEval);
        continue;
      }
      for (size_t i = 0; i < n; i++) {
        mv[i] /= 2.;
        y[i] = par[i].accept(x[i] - mv[i]);
      }
      fnew = eval(y);
    }
    if (fnew > fcur + tolerance || std::isnan(fnew)) {
      eval(x);  // could not be ameliorated: stay at x
      fnew = fcur;
    } else {
      x = y;
    }
    const bool done = std::fabs(fnew - fcur) < tolerance;
    fprev = fcur;
    fcur = fnew;
    if (onStep) onStep(steps, x, fcur);
    if (done) break;
  }
  if (steps_out) *steps_out = steps;
  return nEval;
}

}  // namespace

unsigned int OptimizationTools::optimizeTreeScale(TreeLikelihood* tl, double tolerance, unsigned int tlEvalMax,
                                                  OutputStream*, OutputStream*, unsigned int) {
  // ScaleFunction (OptimizationTools.cpp:77-115): every branch length but RootPosition
  ParameterList bl = tl->getBranchLengthsParameters();
  if (bl.hasParameter("RootPosition")) bl.deleteParameter("RootPosition");
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

namespace {

// Global molecular clock (OptimizationTools.cpp:266-353 with useClock = true, i.e.
// GlobalClockTreeLikelihoodFunctionWrapper): branch lengths of a rooted tree are
// derived from node heights, h(leaf) = 0, h(root) = TotalHeight and, for every
// other internal node v, h(v) = HeightP_v * h(father(v)) with HeightP_v in (0, 1).
struct ClockMap {
  std::vector<const Node*> nodes;       // postorder, root last: BrLen<i> = nodes[i]
  std::map<const Node*, size_t> index;
  std::vector<int> internalNonRoot;     // indices into nodes
  double totalHeight = 0.;
  std::vector<double> heightP;          // per internalNonRoot

  explicit ClockMap(const TreeTemplate<Node>& tree) {
    nodes = tree.getNodes();
    for (size_t i = 0; i < nodes.size(); i++) index[nodes[i]] = i;
    if (nodes.back()->getNumberOfSons() != 2)
      throw Exception("optimizeNumericalParameters2(useClock = true): the tree must be rooted");
    std::vector<double> h(nodes.size(), 0.);
    for (size_t i = 0; i < nodes.size(); i++) {
      const Node* n = nodes[i];
      double m = 0.;
      for (size_t k = 0; k < n->getNumberOfSons(); k++) {
        const Node* c = n->getSon(k);
        m = std::max(m, h[index[c]] + c->getDistanceToFather());
      }
      h[i] = n->isLeaf() ? 0. : m;
    }
    totalHeight = h.back();
    for (size_t i = 0; i + 1 < nodes.size(); i++)
      if (!nodes[i]->isLeaf()) {
        internalNonRoot.push_back((int)i);
        heightP.push_back(std::min(std::max(h[i] / h[index[nodes[i]->getFather()]], 1e-6), 1. - 1e-6));
      }
  }
  std::vector<double> branchLengths() const {
    std::vector<double> h(nodes.size(), 0.);
    h.back() = totalHeight;
    // heights top-down (reverse postorder)
    std::map<int, double> p;
    for (size_t k = 0; k < internalNonRoot.size(); k++) p[internalNonRoot[k]] = heightP[k];
    for (size_t i = nodes.size() - 1; i-- > 0;) {
      const Node* n = nodes[i];
      h[i] = n->isLeaf() ? 0. : p[(int)i] * h[index.at(n->getFather())];
    }
    std::vector<double> bl(nodes.size() - 1);
    for (size_t i = 0; i + 1 < nodes.size(); i++)
      bl[i] = std::min(std::max(h[index.at(nodes[i]->getFather())] - h[i], 0.000001), 10000.);
    return bl;
  }
};

}  // namespace

// optimizeNumericalParameters2 with OPTIMIZATION_NEWTON (the default): PseudoNewton over
// the requested parameters, or with useClock over the non-branch parameters plus the clock
// heights of GlobalClockTreeLikelihoodFunctionWrapper (TotalHeight, HeightP_v), whose
// derivatives are numerical (OptimizationTools.cpp:277-288, 329-331).
unsigned int OptimizationTools::pseudoNewtonParameters(TreeLikelihood* tl, const ParameterList& pl, double tolerance,
                                                       unsigned int tlEvalMax, bool useClock, OutputStream* messenger,
                                                       OutputStream* profiler) {
  std::vector<PNParam> par;
  std::vector<double> x;
  std::vector<size_t> plIndex;  // parameter -> index in pl (non-clock parameters)
  std::unique_ptr<ClockMap> clock;
  ParameterList brl;
  const bool deriv = tl->derivativesEnabled();
  // analytic derivatives for the likelihood's derivable parameters (the branch lengths,
  // BrLenRoot and RootPosition included), ThreePointsNumericalDerivative for the others
  // (OptimizationTools.cpp:330-331 getNonDerivableParameters)
  const ParameterList derivable = tl->getDerivableParameters();
  for (size_t i = 0; i < pl.size(); i++) {
    const bool br = derivable.hasParameter(pl[i].getName());
    if (useClock && br) continue;
    PNParam p;
    p.name = pl[i].getName();
    if (pl[i].hasConstraint()) p.constraint.reset(pl[i].getConstraint()->clone());
    p.analytic = br && deriv;
    par.push_back(p);
    x.push_back(pl[i].getValue());
    plIndex.push_back(i);
  }
  const size_t nPlain = par.size();
  if (useClock) {
    const TreeTemplate<Node>* tree = dynamic_cast<const TreeTemplate<Node>*>(&tl->getTree());
    clock.reset(new ClockMap(*tree));
    brl = tl->getBranchLengthsParameters();
    PNParam th;
    th.name = "TotalHeight";
    th.constraint.reset(new IntervalConstraint(0., 1e300, false, true));
    par.push_back(th);
    x.push_back(clock->totalHeight);
    for (size_t k = 0; k < clock->heightP.size(); k++) {
      PNParam hp;
      hp.name = "HeightP" + std::to_string(k);
      hp.constraint.reset(new IntervalConstraint(1e-6, 1. - 1e-6, true, true));
      par.push_back(hp);
      x.push_back(clock->heightP[k]);
    }
  }
  ParameterList cur = pl;
  auto f = [&](const std::vector<double>& y) {
    ParameterList set;
    for (size_t i = 0; i < nPlain; i++) {
      Parameter q = cur[plIndex[i]];
      q.setValue(y[i]);
      set.addParameter(q);
    }
    if (clock) {
      clock->totalHeight = y[nPlain];
      for (size_t k = 0; k < clock->heightP.size(); k++) clock->heightP[k] = y[nPlain + 1 + k];
      const std::vector<double> bl = clock->branchLengths();
      for (size_t i = 0; i < brl.size(); i++) {
        Parameter q = brl[i];
        q.setValue(bl[i]);
        set.addParameter(q);
      }
    }
    tl->setParameters(set);
    return tl->getValue();
  };
  auto an = [&](size_t i, double* d1, double* d2) {
    *d1 = tl->getFirstOrderDerivative(par[i].name);
    *d2 = tl->getSecondOrderDerivative(par[i].name);
  };
  // profiler: one line per step with every parameter and the function value (the
  // optimisers' profile format: a header of names, then tab-separated values)
  if (profiler) {
    *profiler << "Step";
    for (auto& p : par) *profiler << "\t" << p.name;
    *profiler << "\tFunction";
    profiler->endLine();
  }
  auto onStep = [&](unsigned int step, const std::vector<double>& y, double fy) {
    if (profiler) {
      *profiler << (long)step;
      for (double v : y) *profiler << "\t" << v;
      *profiler << "\t" << fy;
      profiler->endLine();
    }
    if (messenger) {
      *messenger << "PseudoNewton step " << (long)step << ": f = " << fy;
      messenger->endLine();
    }
  };
  unsigned int steps = 0;
  const unsigned int nEval = pseudoNewton(par, x, f, an, tolerance, tlEvalMax, &steps, onStep);
  f(x);  // leave the likelihood at the accepted point
  lastSteps_ = steps;
  if (std::getenv("BPP_AMD_OPT_LOG"))
    std::fprintf(stderr, "PseudoNewton: %u steps, %u function evaluations, -lnL = %.12f\n", steps, nEval,
                 tl->getValue());
  return nEval;
}

unsigned int OptimizationTools::lastSteps_ = 0;

unsigned int OptimizationTools::optimizeNumericalParametersWithGlobalClock2(
    DiscreteRatesAcrossSitesClockTreeLikelihood* cl, const ParameterList& parameters, OptimizationListener*,
    double tolerance, unsigned int tlEvalMax, OutputStream* messenger, OutputStream* profiler, unsigned int,
    const std::string& optMethodDeriv) {
  if (optMethodDeriv != OPTIMIZATION_GRADIENT && optMethodDeriv != OPTIMIZATION_NEWTON)
    throw Exception("OptimizationTools::optimizeBranchLengthsParameters. Unknown optimization method: " +
                    optMethodDeriv);
  TreeLikelihood* tl = cl;
  const ParameterList pl = tl->getParameters().getCommonParametersWith(parameters);
  std::vector<PNParam> par(pl.size());
  std::vector<double> x(pl.size());
  for (size_t i = 0; i < pl.size(); i++) {
    par[i].name = pl[i].getName();
    if (pl[i].hasConstraint()) par[i].constraint.reset(pl[i].getConstraint()->clone());
    x[i] = pl[i].getValue();
  }
  ParameterList cur = pl;
  std::function<double(const std::vector<double>&)> f = [&](const std::vector<double>& y) {
    for (size_t i = 0; i < y.size(); i++) cur[i].setValue(y[i]);
    tl->setParameters(cur);
    return tl->getValue();
  };
  const std::function<void(size_t, double*, double*)> none = [](size_t, double*, double*) {
    throw Exception("optimizeNumericalParametersWithGlobalClock2: no analytic derivative");
  };
  if (profiler) {
    *profiler << "Step";
    for (auto& p : par) *profiler << "\t" << p.name;
    *profiler << "\tFunction";
    profiler->endLine();
  }
  auto onStep = [&](unsigned int step, const std::vector<double>& y, double fy) {
    if (profiler) {
      *profiler << (long)step;
      for (double v : y) *profiler << "\t" << v;
      *profiler << "\t" << fy;
      profiler->endLine();
    }
    if (messenger) {
      *messenger << "step " << (long)step << ": f = " << fy;
      messenger->endLine();
    }
  };
  unsigned int nEval = 0, steps = 0;
  if (optMethodDeriv == OPTIMIZATION_NEWTON) {
    nEval = pseudoNewton(par, x, f, none, tolerance, tlEvalMax, &steps, onStep);
  } else {
    // ConjugateGradientMultiDimensions over TwoPointsNumericalDerivative (interval 1e-7,
    // OptimizationTools.cpp:499-504), FunctionStopCondition |f - f_old| < tolerance
    std::function<double(const std::vector<double>&)> eval = [&](const std::vector<double>& y) {
      nEval++;
      return f(y);
    };
    const Derivatives der{par, eval, none, 2, 0.0000001};
    const double f0 = eval(x);
    const double f1 = conjugateGradient(par, x, f0, eval, der, tolerance, tlEvalMax, &nEval);
    onStep(++steps, x, f1);
  }
  f(x);  // leave the likelihood at the accepted point
  lastSteps_ = steps;
  if (std::getenv("BPP_AMD_OPT_LOG"))
    std::fprintf(stderr, "GlobalClock2 (%s): %u function evaluations, -lnL = %.12f\n", optMethodDeriv.c_str(), nEval,
                 tl->getValue());
  return nEval;
}

unsigned int OptimizationTools::optimizeNumericalParameters2(TreeLikelihood* tl, const ParameterList& parameters,
                                                             OptimizationListener*, double tolerance,
                                                             unsigned int tlEvalMax, OutputStream* messenger,
                                                             OutputStream* profiler, bool, bool useClock, unsigned int,
                                                             const std::string& optMethodDeriv) {
  ParameterList pl = tl->getParameters().getCommonParametersWith(parameters);
  if (optMethodDeriv == OPTIMIZATION_NEWTON && !std::getenv("BPP_AMD_OPT_BRENT"))
    return pseudoNewtonParameters(tl, pl, tolerance, tlEvalMax, useClock, messenger, profiler);
  unsigned int nEval = 0;
  std::unique_ptr<ClockMap> clock;
  ParameterList brl;
  if (useClock) {
    const TreeTemplate<Node>* tree = dynamic_cast<const TreeTemplate<Node>*>(&tl->getTree());
    clock.reset(new ClockMap(*tree));
    brl = tl->getBranchLengthsParameters();
    // branch lengths are replaced by the clock parameters
    ParameterList rest;
    for (size_t i = 0; i < pl.size(); i++)
      if (pl[i].getName().compare(0, 5, "BrLen") != 0) rest.addParameter(pl[i]);
    pl = rest;
    for (size_t i = 0; i < brl.size(); i++) brl[i].setValue(clock->branchLengths()[i]);
    tl->setParameters(brl);
  }
  auto applyClock = [&]() {
    std::vector<double> bl = clock->branchLengths();
    for (size_t i = 0; i < brl.size(); i++) brl[i].setValue(bl[i]);
    tl->setParameters(brl);
    return tl->getValue();
  };
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
    if (clock) {
      // TotalHeight on a log scale, then every HeightP in (0, 1)
      {
        const double x0 = std::log(clock->totalHeight);
        auto f = [&](double u) {
          clock->totalHeight = std::exp(u);
          return applyClock();
        };
        double fmin = 0.;
        const double u = brent(f, x0 - 4., x0 + 4., x0, 1e-8, 200, &fmin, &nEval);
        double fu = f(u);
        if (fu > fcur) fu = f(x0);
        fcur = fu;
      }
      for (size_t k = 0; k < clock->heightP.size(); k++) {
        const double x0 = clock->heightP[k];
        auto f = [&](double v) {
          clock->heightP[k] = v;
          return applyClock();
        };
        double fmin = 0.;
        const double u = brent(f, 1e-6, 1. - 1e-6, x0, 1e-8, 200, &fmin, &nEval);
        double fu = f(u);
        if (fu > fcur) fu = f(x0);
        fcur = fu;
      }
    }
    if (fstart - fcur < tolerance) break;
  }
  return nEval;
}

}  // namespace bpp
