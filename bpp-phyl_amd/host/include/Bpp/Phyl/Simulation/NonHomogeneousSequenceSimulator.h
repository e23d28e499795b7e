// Site simulation along a tree under a (non-)homogeneous model set, the generator the
// reference's test_likelihood_nh.cpp fits models to
// (Simulation/NonHomogeneousSequenceSimulator.cpp:110-160 init, 306-353 simulate, 433-483
// evolve / multipleEvolve): root states from the root frequencies, one rate class per site
// uniformly, then every branch in preorder draws the child state from the cumulative row of
// P(t . r_c) of its own model.  Host-side input generation (not the hot path); the random
// numbers come from RandomTools.
#ifndef BPP_AMD_NONHOMOGENEOUSSEQUENCESIMULATOR_H
#define BPP_AMD_NONHOMOGENEOUSSEQUENCESIMULATOR_H

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../Numeric/Prob/DiscreteDistribution.h"
#include "../../Numeric/Random/RandomTools.h"
#include "../../Seq/Container/SiteContainer.h"
#include "../Model/SubstitutionModelSet.h"
#include "../TreeTemplate.h"

namespace bpp {

class NonHomogeneousSequenceSimulator {
  const SubstitutionModelSet* modelSet_;
  std::unique_ptr<SubstitutionModelSet> ownModelSet_;
  const Alphabet* alphabet_;
  const DiscreteDistribution* rate_;
  std::unique_ptr<TreeTemplate<Node> > tree_;
  std::vector<const Node*> leaves_;
  std::vector<std::string> seqNames_;
  size_t nbClasses_, nbStates_;
  bool outputInternalSequences_ = false;
  // per non-root node id: cumulative transition rows [class][x][y]
  std::map<int, VVVdouble> cumpxy_;

  void init();
  void multipleEvolve(const Node* node, const std::vector<size_t>& rateClasses,
                      std::map<int, std::vector<size_t> >& states) const;

 public:
  NonHomogeneousSequenceSimulator(const SubstitutionModelSet* modelSet, const DiscreteDistribution* rate,
                                  const Tree* tree);
  // homogeneous case: the model on every branch, its equilibrium frequencies at the root
  NonHomogeneousSequenceSimulator(const SubstitutionModel* model, const DiscreteDistribution* rate,
                                  const Tree* tree);
  virtual ~NonHomogeneousSequenceSimulator() {}
  NonHomogeneousSequenceSimulator(const NonHomogeneousSequenceSimulator&) = delete;
  NonHomogeneousSequenceSimulator& operator=(const NonHomogeneousSequenceSimulator&) = delete;

  SiteContainer* simulate(size_t numberOfSites) const;
  // the same with given root states and rate classes (one per site)
  SiteContainer* multipleEvolve(const std::vector<size_t>& initialStateIndices,
                                const std::vector<size_t>& rateClasses) const;
  std::vector<std::string> getSequencesNames() const { return seqNames_; }
  const Alphabet* getAlphabet() const { return alphabet_; }
  const SubstitutionModelSet* getSubstitutionModelSet() const { return modelSet_; }
  void outputInternalSequences(bool yn);
};

}  // namespace bpp

#endif
