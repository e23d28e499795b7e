// Likelihood/ClockTreeLikelihood.h:58-81 and DiscreteRatesAcrossSitesTreeLikelihood.h:
// interfaces of the likelihoods whose branch lengths follow a global molecular clock
// (parameters TotalHeight and HeightP<id> instead of BrLen<i>).  The optimisers take
// these interfaces (OptimizationTools::optimizeNumericalParametersWithGlobalClock2).
#ifndef BPP_AMD_CLOCKTREELIKELIHOOD_H
#define BPP_AMD_CLOCKTREELIKELIHOOD_H

#include "TreeLikelihood.h"

namespace bpp {

class DiscreteRatesAcrossSitesTreeLikelihood : public virtual TreeLikelihood {
 public:
  ~DiscreteRatesAcrossSitesTreeLikelihood() override {}
};

class ClockTreeLikelihood : public virtual TreeLikelihood {
 public:
  ~ClockTreeLikelihood() override {}
};

class DiscreteRatesAcrossSitesClockTreeLikelihood : public virtual ClockTreeLikelihood,
                                                    public virtual DiscreteRatesAcrossSitesTreeLikelihood {
 public:
  ~DiscreteRatesAcrossSitesClockTreeLikelihood() override {}
};

}  // namespace bpp

#endif
