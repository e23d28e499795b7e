// Likelihood/RHomogeneousClockTreeLikelihood.h / .cpp: the homogeneous likelihood of a rooted
// bifurcating tree under a global molecular clock.  The branch lengths are not parameters;
// they follow from the node heights: TotalHeight (the root's height) and, for every internal
// non-root node v, HeightP<id(v)> = h(v) / h(father(v)) in [0, 1] (:118-145), with leaves at
// height 0 (:150-168).  Every evaluation is the same plk_evaluate call as the unconstrained
// likelihood: the branches whose derived length moved get a new P(t) on the device, the
// traversal and root reduction follow.  No analytic derivatives (:172-199): the optimisers
// differentiate numerically.
#ifndef BPP_AMD_RHOMOGENEOUSCLOCKTREELIKELIHOOD_H
#define BPP_AMD_RHOMOGENEOUSCLOCKTREELIKELIHOOD_H

#include <map>
#include <string>
#include <vector>

#include "ClockTreeLikelihood.h"
#include "TreeLikelihood.h"

namespace bpp {

class RHomogeneousClockTreeLikelihood : public RHomogeneousTreeLikelihood,
                                        public DiscreteRatesAcrossSitesClockTreeLikelihood {
  std::map<const Node*, std::string> heightNames_;  // "HeightP<id>" of every internal non-root node

  // RHomogeneousClockTreeLikelihood.cpp:87-93: rooted and bifurcating, branch lengths >= 0
  void init_();
  // lengths of the sons' branches below `node` of height `height` (:150-168); appends the
  // nodes whose length changed
  void branchLengthsFromHeights(Node* node, double height, std::vector<const Node*>& changed);

 protected:
  void initBranchLengthsParameters() override;
  std::vector<const Node*> applyBranchLengths() override;

 public:
  RHomogeneousClockTreeLikelihood(const Tree& tree, SubstitutionModel* model, DiscreteDistribution* rDist,
                                  bool checkRooted = true, bool verbose = true);
  RHomogeneousClockTreeLikelihood(const Tree& tree, const SiteContainer& data, SubstitutionModel* model,
                                  DiscreteDistribution* rDist, bool checkRooted = true, bool verbose = true);

  ParameterList getDerivableParameters() const override;
  ParameterList getNonDerivableParameters() const override;
  double getFirstOrderDerivative(const std::string& variable) const override;
  double getSecondOrderDerivative(const std::string& variable) const override;
  double getSecondOrderDerivative(const std::string&, const std::string&) const { return 0.; }
};

}  // namespace bpp

#endif
