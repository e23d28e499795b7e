// Host mirror: optimisers over the GPU likelihood (see OptimizationTools.h).
#include "Bpp/Phyl/OptimizationTools.h"

#include <cmath>
#include <limits>
#include <map>
#include <memory>

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

unsigned int OptimizationTools::optimizeNumericalParameters2(TreeLikelihood* tl, const ParameterList& parameters,
                                                             OptimizationListener*, double tolerance,
                                                             unsigned int tlEvalMax, OutputStream*, OutputStream*,
                                                             bool, bool useClock, unsigned int, const std::string&) {
  ParameterList pl = tl->getParameters().getCommonParametersWith(parameters);
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
