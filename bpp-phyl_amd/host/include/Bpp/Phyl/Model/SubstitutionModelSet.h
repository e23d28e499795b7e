// Non-homogeneous model sets: one model per branch, shared ("aliased") parameters, root
// frequencies.  After Model/SubstitutionModelSet.h (getModelForNode :329-341,
// getNodesWithParameter .cpp:110-130, getNodeParameters :457-466, getRootFrequencies
// :429-435) and SubstitutionModelSetTools::createNonHomogeneousModelSet
// (Model/SubstitutionModelSetTools.cpp:81-175).  Parameter names follow the reference: the
// root frequencies' parameters first ("GC.theta"), then every model parameter with the
// suffix "_<k>" (k = 1-based model index, "T92.kappa_1", "T92.theta_1", ...).  A global
// parameter is the first model's copy with every other model's copy aliased to it
// (aliasParameters, bpp-core AbstractParameterAliasable): the aliases follow their source
// and are left out of getIndependentParameters().
#ifndef BPP_AMD_SUBSTITUTIONMODELSET_H
#define BPP_AMD_SUBSTITUTIONMODELSET_H

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../TreeTemplate.h"
#include "Models.h"

namespace bpp {

class SubstitutionModelSet : public AbstractParametrizable {
  const Alphabet* alphabet_;
  std::vector<std::shared_ptr<SubstitutionModel> > models_;
  std::vector<std::vector<int> > nodesOfModel_;
  std::map<int, size_t> modelOfNode_;
  std::shared_ptr<FrequencySet> rootFreqs_;
  std::map<std::string, std::string> aliasOf_;  // alias name -> source name
  // bookkeeping of the last fireParameterChanged (which models / root frequencies changed)
  std::vector<size_t> lastChangedModels_;
  bool lastRootFreqsChanged_ = false;

  // the model index (0-based) a suffixed parameter name belongs to, or -1
  long modelIndexOfParameter(const std::string& name) const;

 public:
  explicit SubstitutionModelSet(const Alphabet* alpha) : AbstractParametrizable(""), alphabet_(alpha) {}
  SubstitutionModelSet(const SubstitutionModelSet& s);
  SubstitutionModelSet& operator=(const SubstitutionModelSet&) = delete;
  SubstitutionModelSet* clone() const { return new SubstitutionModelSet(*this); }

  const Alphabet* getAlphabet() const { return alphabet_; }
  size_t getNumberOfModels() const { return models_.size(); }
  size_t getNumberOfStates() const { return models_.empty() ? 0 : models_[0]->getNumberOfStates(); }
  SubstitutionModel* getModel(size_t i) { return models_.at(i).get(); }
  const SubstitutionModel* getModel(size_t i) const { return models_.at(i).get(); }
  size_t getModelIndexForNode(int nodeId) const {
    auto it = modelOfNode_.find(nodeId);
    if (it == modelOfNode_.end()) throw Exception("SubstitutionModelSet::getModelIndexForNode: no model for node " + std::to_string(nodeId));
    return it->second;
  }
  const SubstitutionModel* getModelForNode(int nodeId) const { return models_[getModelIndexForNode(nodeId)].get(); }
  const std::vector<int>& getNodesWithModel(size_t i) const { return nodesOfModel_.at(i); }
  // nodes whose model carries `name` or one of its aliases (SubstitutionModelSet.cpp:110-130)
  std::vector<int> getNodesWithParameter(const std::string& name) const;
  Vdouble getRootFrequencies() const {
    return rootFreqs_ ? rootFreqs_->getFrequencies() : models_.at(0)->getFrequencies();
  }
  bool isStationary() const { return !rootFreqs_; }
  ParameterList getRootFrequenciesParameters() const {
    return rootFreqs_ ? rootFreqs_->getParameters() : ParameterList();
  }
  // every parameter but the root frequencies' (SubstitutionModelSet.h:457-466)
  ParameterList getNodeParameters() const;
  ParameterList getModelParameters() const { return getNodeParameters(); }
  // the parameters that are not aliases of another one
  ParameterList getIndependentParameters() const override;
  std::vector<std::string> getAlias(const std::string& name) const;
  // true when every non-root node of `tree` has a model
  bool isFullySetUpFor(const Tree& tree) const;

  // Build-up API
  void setRootFrequencies(FrequencySet* rootFreqs);
  void addModel(SubstitutionModel* model, const std::vector<int>& nodesId);
  // p2 follows p1 from now on (bpp-core AbstractParameterAliasable::aliasParameters)
  void aliasParameters(const std::string& p1, const std::string& p2);
  bool matchParametersValues(const ParameterList& pl) override;
  void setParametersValues(const ParameterList& pl) override;
  void fireParameterChanged(const ParameterList& pl) override;
  // what the last fireParameterChanged changed: model indices whose parameters moved (their
  // eigen-systems were recomputed) and whether the root frequencies moved
  const std::vector<size_t>& getLastChangedModels() const { return lastChangedModels_; }
  bool getLastRootFrequenciesChanged() const { return lastRootFreqsChanged_; }
};

struct SubstitutionModelSetTools {
  // One clone of `model` per branch of `tree` (every node except the root); model
  // parameters listed in globalParameterNames are shared.  rootFreqs is owned by the set.
  static SubstitutionModelSet* createNonHomogeneousModelSet(
      SubstitutionModel* model, FrequencySet* rootFreqs, const Tree* tree,
      const std::map<std::string, std::string>& aliasFreqNames,
      std::map<std::string, std::vector<Vint> >& globalParameterNames);
  static SubstitutionModelSet* createHomogeneousModelSet(SubstitutionModel* model, FrequencySet* rootFreqs,
                                                         const Tree* tree);
};

}  // namespace bpp

#endif
