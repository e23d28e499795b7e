// Host-side optimisers driving repeated likelihood evaluations (the callers of the
// hot path): optimizeTreeScale (OptimizationTools.cpp:119-143) and
// optimizeNumericalParameters2 (:266-353).  Every function evaluation is one GPU
// evaluation through fireParameterChanged.  optimizeNumericalParameters2 with
// OPTIMIZATION_NEWTON (the default) restates PseudoNewtonOptimizer::doStep
// (Likelihood/PseudoNewtonOptimizer.cpp:96-190) with the device's analytic branch-length
// derivatives; other methods (and BPP_AMD_OPT_BRENT=1) use a bounded Brent line search per
// parameter, cycled to convergence.  optimizeTreeScale is Brent on the log scale factor as in
// the reference (:119-143).
#ifndef BPP_AMD_OPTIMIZATIONTOOLS_H
#define BPP_AMD_OPTIMIZATIONTOOLS_H

#include <string>

#include "../App/ApplicationTools.h"
#include "../Io/OutputStream.h"
#include "Likelihood/ClockTreeLikelihood.h"
#include "Likelihood/TreeLikelihood.h"

namespace bpp {

class OptimizationListener {
 public:
  virtual ~OptimizationListener() {}
};

struct OptimizationTools {
  static const std::string OPTIMIZATION_NEWTON;
  static const std::string OPTIMIZATION_GRADIENT;
  static const std::string OPTIMIZATION_BRENT;
  static const std::string OPTIMIZATION_BFGS;

  static unsigned int optimizeTreeScale(TreeLikelihood* tl, double tolerance = 0.000001,
                                        unsigned int tlEvalMax = 1000000, OutputStream* messageHandler = nullptr,
                                        OutputStream* profiler = nullptr, unsigned int verbose = 1);

  static unsigned int optimizeNumericalParameters2(TreeLikelihood* tl, const ParameterList& parameters,
                                                   OptimizationListener* listener = nullptr,
                                                   double tolerance = 0.000001, unsigned int tlEvalMax = 1000000,
                                                   OutputStream* messageHandler = nullptr,
                                                   OutputStream* profiler = nullptr, bool reparametrization = false,
                                                   bool useClock = false, unsigned int verbose = 1,
                                                   const std::string& optMethodDeriv = OPTIMIZATION_NEWTON);

  // OptimizationTools.cpp:484-539: every given parameter of a global-clock likelihood
  // (TotalHeight, HeightP<id>, the model and rate parameters) optimised together,
  // with numerical derivatives: OPTIMIZATION_GRADIENT (the default) is a conjugate-gradient
  // descent over TwoPointsNumericalDerivative (interval 1e-7), OPTIMIZATION_NEWTON the
  // PseudoNewton optimiser over ThreePointsNumericalDerivative (interval 1e-4).
  static unsigned int optimizeNumericalParametersWithGlobalClock2(
      DiscreteRatesAcrossSitesClockTreeLikelihood* cl, const ParameterList& parameters,
      OptimizationListener* listener = nullptr, double tolerance = 0.000001, unsigned int tlEvalMax = 1000000,
      OutputStream* messageHandler = nullptr, OutputStream* profiler = nullptr, unsigned int verbose = 1,
      const std::string& optMethodDeriv = OPTIMIZATION_GRADIENT);

  // PseudoNewton steps of the last OPTIMIZATION_NEWTON run (diagnostics)
  static unsigned int lastSteps_;
  static unsigned int pseudoNewtonParameters(TreeLikelihood* tl, const ParameterList& pl, double tolerance,
                                             unsigned int tlEvalMax, bool useClock, OutputStream* messenger = nullptr,
                                             OutputStream* profiler = nullptr);

  // Bounded 1-D Brent minimisation of f on [a, b]; returns the argmin, *fmin the value.
  template <class F>
  static double brent(F f, double a, double b, double x0, double tol, unsigned int maxEval, double* fmin,
                      unsigned int* nEval);
};

}  // namespace bpp

#include "OptimizationTools.tpp"

#endif
