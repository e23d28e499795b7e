// Non-homogeneous model sets: one model per branch, shared ("global") parameters,
// root frequencies.  After Model/SubstitutionModelSet.h (getModelForNode :329-341,
// getRootFrequencies :429-435) and SubstitutionModelSetTools::createNonHomogeneousModelSet
// (Model/SubstitutionModelSetTools.cpp:81-175): per-model parameter names carry the
// suffix "_<k>" (k = 1-based model index), global ones keep the model's name.
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
  std::vector<std::string> globalNames_;  // model parameter names shared by all models

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
  Vdouble getRootFrequencies() const {
    return rootFreqs_ ? rootFreqs_->getFrequencies() : models_.at(0)->getFrequencies();
  }
  bool isStationary() const { return !rootFreqs_; }
  ParameterList getRootFrequenciesParameters() const {
    return rootFreqs_ ? rootFreqs_->getParameters() : ParameterList();
  }
  ParameterList getModelParameters() const;

  // Build-up API
  void setRootFrequencies(FrequencySet* rootFreqs);
  void addModel(SubstitutionModel* model, const std::vector<int>& nodesId, const std::vector<std::string>& globalNames);
  void fireParameterChanged(const ParameterList& pl) override;
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
