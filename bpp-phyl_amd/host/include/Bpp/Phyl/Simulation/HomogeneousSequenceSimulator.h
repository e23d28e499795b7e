// Simulation/HomogeneousSequenceSimulator.h:53-72: the non-homogeneous simulator with one
// model on every branch and its equilibrium frequencies at the root.  Host-side input
// generation (not the hot path).
#ifndef BPP_AMD_HOMOGENEOUSSEQUENCESIMULATOR_H
#define BPP_AMD_HOMOGENEOUSSEQUENCESIMULATOR_H

#include "NonHomogeneousSequenceSimulator.h"

namespace bpp {

class HomogeneousSequenceSimulator : public NonHomogeneousSequenceSimulator {
 public:
  HomogeneousSequenceSimulator(const SubstitutionModel* model, const DiscreteDistribution* rate, const Tree* tree)
      : NonHomogeneousSequenceSimulator(model, rate, tree) {}
  const SubstitutionModel* getModel() const { return getSubstitutionModelSet()->getModel(0); }
};

}  // namespace bpp

#endif
