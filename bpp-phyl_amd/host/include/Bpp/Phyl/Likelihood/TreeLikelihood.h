// Likelihood classes of the host mirror: the Bio++ TreeLikelihood API surface the
// reference's tests use (Likelihood/TreeLikelihood.h:66-442,
// Likelihood/RHomogeneousTreeLikelihood.h:131-138, RNonHomogeneousTreeLikelihood.h),
// implemented over libplk (include/plk.h).  The hot path
// (computeTransitionProbabilities*, computeTreeLikelihood, getLogLikelihood) runs on
// the GPU; the host keeps parameters, tree, patterns and the dispatch logic of
// fireParameterChanged (Likelihood/RHomogeneousTreeLikelihood.cpp:255-283).
#ifndef BPP_AMD_TREELIKELIHOOD_H
#define BPP_AMD_TREELIKELIHOOD_H

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../App/ApplicationTools.h"
#include "../../Numeric/Prob/DiscreteDistribution.h"
#include "../../Seq/Container/SiteContainer.h"
#include "../Model/Models.h"
#include "../Model/SubstitutionModelSet.h"
#include "../TreeTemplate.h"

struct plk_handle_s;

namespace bpp {

class TreeLikelihood : public AbstractParametrizable {
 public:
  virtual ~TreeLikelihood() {}
  virtual void initialize() = 0;
  virtual bool isInitialized() const = 0;
  virtual double getValue() const = 0;            // -lnL
  virtual double getLogLikelihood() const = 0;
  virtual double getLikelihood() const = 0;
  virtual double getLogLikelihoodForASite(size_t site) const = 0;
  virtual double getLikelihoodForASite(size_t site) const = 0;
  virtual size_t getNumberOfSites() const = 0;
  virtual size_t getNumberOfStates() const = 0;
  virtual size_t getNumberOfClasses() const = 0;
  virtual const Tree& getTree() const = 0;
  virtual ParameterList getBranchLengthsParameters() const = 0;
  virtual ParameterList getSubstitutionModelParameters() const = 0;
  virtual ParameterList getRateDistributionParameters() const = 0;
  // parameters with analytic derivatives (the branch lengths) and the others
  // (Likelihood/TreeLikelihood.h:426-435)
  virtual ParameterList getDerivableParameters() const = 0;
  virtual ParameterList getNonDerivableParameters() const = 0;
  virtual void setParameters(const ParameterList& pl) = 0;
  virtual double f(const ParameterList& pl) = 0;
  virtual double getFirstOrderDerivative(const std::string& variable) const = 0;
  virtual double getSecondOrderDerivative(const std::string& variable) const = 0;
  virtual void enableDerivatives(bool yn) = 0;
  // both analytic branch-length derivatives enabled (PseudoNewton then uses them)
  virtual bool derivativesEnabled() const { return false; }
  virtual void enableFirstOrderDerivatives(bool yn) = 0;
  virtual void enableSecondOrderDerivatives(bool yn) = 0;
};

// Common engine plumbing of the R-likelihoods: tree copy, node order, root site
// patterns, the libplk handle and the postorder op list.
class AbstractPlkTreeLikelihood : public virtual TreeLikelihood {
 protected:
  TreeTemplate<Node>* tree_ = nullptr;
  std::vector<Node*> nodes_;                 // postorder minus root (BrLen<i> = nodes_[i])
  DiscreteDistribution* rateDistribution_;   // not owned
  size_t nbClasses_ = 1, nbStates_ = 0;
  // data
  std::unique_ptr<SiteContainer> data_;
  size_t nbSites_ = 0, nbDistinctSites_ = 0;
  std::vector<size_t> rootPatternLinks_;     // site -> pattern
  std::vector<unsigned int> rootWeights_;    // pattern -> number of sites
  std::vector<std::vector<int> > patternStates_;  // [tip engine index][pattern]
  // engine mapping: tips first, internal nodes after
  std::map<const Node*, int> engineIndex_;
  int nTips_ = 0, nInternal_ = 0, rootEngine_ = -1;
  std::vector<int> opParent_, opFlags_;
  std::vector<std::vector<int> > opChildren_;
  plk_handle_s* engine_ = nullptr;
  bool usePatterns_ = true;
  bool verbose_ = true;
  bool initialized_ = false;
  int scalingMode_ = -1;  // setUnderflowScaling: 1 on, 0 off, -1 unscaled first with an exact fallback
  bool scaledNow_ = false;   // scalingMode_ -1: an evaluation flagged underflow, the engine rescales since
  size_t engineModels_ = 1;  // createEngine's arguments (kept for the fallback's new engine)
  bool engineGuard_ = true;
  bool engineScaled_ = false;  // the current engine was created with PLK_FLAG_SCALING
  bool incremental_ = true;
  bool compressed_ = false;  // usePatterns: PLK_FLAG_SUBTREE_PATTERNS on the engine
  bool allDirty_ = true;     // next fireParameterChanged recomputes every P(t) (initialize)
  // fused lnL-only traversal (PLK_FLAG_LNL_ONLY, the benched kernels): interior partials stay
  // in registers, so every evaluation is one full traversal launch and derivatives
  // recompute the partials on demand
  bool lnlOnly_ = false;
  // per engine node: dP / d2P older than P (evaluations upload P only; the derivative
  // calls bring them up to date first)
  mutable std::vector<char> derivStale_;
  size_t maxSons_ = 0;
  bool derivFirst_ = true, derivSecond_ = true;
  unsigned extraFlags_ = 0;                  // plk_create flags of the subclass (PLK_FLAG_DOUBLE_RECURSIVE)
  // double-recursive derivative cache: every branch from one plk_all_branch_derivatives call,
  // valid until the next traversal (indexed by engine node)
  mutable std::vector<double> drD1_, drD2_;
  mutable bool drValid_ = false;
  double minimumBrLen_ = 0.000001, maximumBrLen_ = 10000.;
  std::shared_ptr<IntervalConstraint> brLenConstraint_;
  ParameterList brLenParameters_;
  std::vector<std::string> brLenNames_;      // "BrLen<i>" of nodes_[i]
  std::vector<long> brLenPos_;               // their positions in parameters_ (checked by name)
  std::vector<int> engineById_;              // engine index by node id (-1: none; engineIndex_ is the reference)
  int engineOf(const Node* n) const {
    const int id = n->getId();
    if (id >= 0 && (size_t)id < engineById_.size() && engineById_[(size_t)id] >= 0 &&
        nodeById_[(size_t)id] == n)
      return engineById_[(size_t)id];
    return engineIndex_.at(n);
  }
  std::vector<const Node*> nodeById_;
  mutable double minusLogLik_ = -1.;
  mutable std::vector<double> siteLnl_;      // per pattern (fetched lazily)
  mutable bool siteLnlValid_ = false;
  Vdouble rootFreqs_;

  AbstractPlkTreeLikelihood(const Tree& tree, DiscreteDistribution* rDist, bool checkRooted, bool verbose,
                            bool usePatterns);
  AbstractPlkTreeLikelihood(const AbstractPlkTreeLikelihood&) = delete;
  AbstractPlkTreeLikelihood& operator=(const AbstractPlkTreeLikelihood&) = delete;

  void buildEngineLayout();
  void setDataImpl(const SiteContainer& sites, const Alphabet* alphabet, const SubstitutionModel& model);
  void createEngine(size_t nModels, bool nonNegGuard);
  // the subclass's uploads after createEngine: tip codes, code table and weights (uploadData);
  // eigen-systems, rates and root frequencies (uploadModels)
  virtual void uploadData() = 0;
  virtual void uploadModels() = 0;
  // scalingMode_ -1: the engine flagged a site likelihood below 2^-255 (plk_root_underflow), so
  // a rescaling engine could differ: re-create the engine with PLK_FLAG_SCALING, re-upload and
  // re-evaluate every branch (from then on every evaluation is scaled)
  void switchToScaledEngine();
  bool underflowed() const;
  virtual void initBranchLengthsParameters();
  // set the nodes' lengths from the parameters; returns the nodes whose length changed
  virtual std::vector<const Node*> applyBranchLengths();
  // Upload transition matrices for the given branches (nodes) of model m(node).
  void updatePmatrices(const std::vector<const Node*>& nodes);
  virtual int modelIndexForNode(const Node*) const { return 0; }
  // the model behind engine model index m (host P(t) for a model whose eigen-system failed)
  virtual const SubstitutionModel* modelForIndex(int m) const = 0;
  bool hostPInUse() const;  // a branch's model has no device P(t) (Taylor branch of getPij_t)
  void uploadEigen(int modelIndex, const SubstitutionModel& model);
  void uploadRates();
  void computeTreeLikelihood(const std::vector<const Node*>* changed = nullptr);
  // One evaluation: P(t) of `pnodes`, the traversal (full, or the ancestors of `pnodes`
  // when `incremental` and the engine keeps every partial), the root reduction -- one
  // plk_evaluate call (Likelihood/RHomogeneousTreeLikelihood.cpp:255-283 as one launch
  // sequence); sets minusLogLik_.
  void evaluateTree(const std::vector<const Node*>& pnodes, bool incremental);
  // dP / d2P of every branch whose P(t) changed since they were last computed
  void refreshDerivativeMatrices() const;
  double reduceRoot() const;
  void fetchSiteLnl() const;
  void check(int rc, const char* what) const;
  virtual bool analyticDerivatives(const std::string& variable, double* d1, double* d2) const;
  void uploadRootFrequencies(const Vdouble& pi);
  // evaluation bookkeeping (see EvaluationStats)
  struct EvaluationStats {
    size_t evaluations = 0;      // fireParameterChanged calls that evaluated lnL
    size_t eigenUploads = 0;     // eigen-systems handed to the engine
    size_t pmatBranches = 0;     // branches whose P(t) was recomputed
    size_t fullTraversals = 0;   // traversals over every internal node
    size_t scaledFallbacks = 0;  // unscaled evaluations redone on a rescaling engine (0 or 1)
  };
  EvaluationStats stats_;

 public:
  ~AbstractPlkTreeLikelihood() override;
  bool isInitialized() const override { return initialized_; }
  double getValue() const override;
  double getLogLikelihood() const override;
  double getLikelihood() const override;
  double getLogLikelihoodForASite(size_t site) const override;
  double getLikelihoodForASite(size_t site) const override;
  size_t getNumberOfSites() const override { return nbSites_; }
  size_t getNumberOfDistinctSites() const { return nbDistinctSites_; }
  size_t getNumberOfStates() const override { return nbStates_; }
  size_t getNumberOfClasses() const override { return nbClasses_; }
  const Tree& getTree() const override { return *tree_; }
  ParameterList getBranchLengthsParameters() const override;
  ParameterList getRateDistributionParameters() const override;
  ParameterList getDerivableParameters() const override { return getBranchLengthsParameters(); }
  ParameterList getNonDerivableParameters() const override;
  void setParameters(const ParameterList& pl) override;
  double f(const ParameterList& pl) override {
    setParameters(pl);
    return getValue();
  }
  double getFirstOrderDerivative(const std::string& variable) const override;
  double getSecondOrderDerivative(const std::string& variable) const override;
  void enableDerivatives(bool yn) override { derivFirst_ = derivSecond_ = yn; }
  bool derivativesEnabled() const override { return derivFirst_ && derivSecond_; }
  void enableFirstOrderDerivatives(bool yn) override { derivFirst_ = yn; }
  void enableSecondOrderDerivatives(bool yn) override { derivSecond_ = yn; }
  const std::vector<unsigned int>& getWeights() const { return rootWeights_; }
  size_t getRootArrayPosition(size_t site) const { return rootPatternLinks_[site]; }
  // Exact power-of-two rescaling of partials (a deviation from the reference, which
  // has none and underflows on large trees); bit-identical when it never triggers.  By
  // default every evaluation runs unscaled first -- the faster kernels, one class per wave on
  // cfg2 -- and the engine reports whether any site likelihood fell below 2^-255
  // (plk_root_underflow, include/plk.h: otherwise no rescale could have fired, and the result
  // is bitwise the scaled one); on the first such evaluation the engine is re-created with
  // rescaling and the evaluation redone, and it stays scaled.  setUnderflowScaling(true / false)
  // forces it on / off (off: the reference's arithmetic, which may underflow); a call after
  // the data are set re-creates the engine when the choice changes it (and re-evaluates an
  // initialized object).
  void setUnderflowScaling(bool yn);
  bool underflowScalingActive() const { return scalingMode_ == 1 || (scalingMode_ < 0 && scaledNow_); }
  // Branch-length-only changes re-evaluate just the ancestors of the changed branches
  // (default); false restores the reference's full traversal on every change.
  void setIncrementalRecompute(bool yn) { incremental_ = yn; }
  // Branch-length bounds (AbstractHomogeneousTreeLikelihood.h:248-264): the constraint of
  // every branch-length parameter; the parameters are rebuilt from the tree
  virtual void setMinimumBranchLength(double minimum);
  virtual void setMaximumBranchLength(double maximum);
  double getMinimumBranchLength() const { return minimumBrLen_; }
  double getMaximumBranchLength() const { return maximumBrLen_; }
  // Partial likelihoods of a node in the reference's [pattern][class][state] order.
  VVVdouble getLikelihoodArray(int nodeId) const;
  plk_handle_s* getEngine() const { return engine_; }
  // what the evaluations since construction did on the engine (host counters, no device call)
  const EvaluationStats& getEvaluationStats() const { return stats_; }
};

class RHomogeneousTreeLikelihood : public AbstractPlkTreeLikelihood {
  SubstitutionModel* model_;  // not owned

 protected:
  void uploadData() override;
  void uploadModels() override;

 public:
  RHomogeneousTreeLikelihood(const Tree& tree, SubstitutionModel* model, DiscreteDistribution* rDist,
                             bool checkRooted = true, bool verbose = true, bool usePatterns = true);
  RHomogeneousTreeLikelihood(const Tree& tree, const SiteContainer& data, SubstitutionModel* model,
                             DiscreteDistribution* rDist, bool checkRooted = true, bool verbose = true,
                             bool usePatterns = true);
  void setData(const SiteContainer& sites);
  void initialize() override;
  void fireParameterChanged(const ParameterList& params) override;
  ParameterList getSubstitutionModelParameters() const override;
  const SubstitutionModel* getModel() const { return model_; }
  SubstitutionModel* getModel() { return model_; }
  const SubstitutionModel* modelForIndex(int) const override { return model_; }
  void computeAllTransitionProbabilities();
};

// Likelihood/DRHomogeneousTreeLikelihood.h: same likelihood, derivatives of all branches
// from one double-recursive pass on the device (plk_all_branch_derivatives) instead of one
// path traversal per branch; getFirstOrderDerivative / getSecondOrderDerivative then read
// the per-branch values computed after the last parameter change
// (DRHomogeneousTreeLikelihood.cpp:287-456).
class DRHomogeneousTreeLikelihood : public RHomogeneousTreeLikelihood {
 public:
  DRHomogeneousTreeLikelihood(const Tree& tree, SubstitutionModel* model, DiscreteDistribution* rDist,
                              bool checkRooted = true, bool verbose = true);
  DRHomogeneousTreeLikelihood(const Tree& tree, const SiteContainer& data, SubstitutionModel* model,
                              DiscreteDistribution* rDist, bool checkRooted = true, bool verbose = true);
};

// Likelihood/RNonHomogeneousTreeLikelihood.h: rooted tree, one model per branch from a
// SubstitutionModelSet.  With reparametrizeRoot the two root branches are parametrised
// as BrLenRoot (their sum) and RootPosition (root1's share), as
// AbstractNonHomogeneousTreeLikelihood.cpp:312-330, 377-389.
class RNonHomogeneousTreeLikelihood : public AbstractPlkTreeLikelihood {
  SubstitutionModelSet* modelSet_;  // not owned
  std::map<int, int> modelOfNodeId_;
  std::map<int, const Node*> idToNode_;
  bool reparametrizeRoot_ = false;
  int root1_ = -1, root2_ = -1;       // ids of the root's first two sons

  int modelIndexForNode(const Node* n) const override;
  const SubstitutionModel* modelForIndex(int m) const override;

 protected:
  // engine flags of a subclass (DRNonHomogeneousTreeLikelihood) must be known before setData
  RNonHomogeneousTreeLikelihood(const Tree& tree, const SiteContainer& data, SubstitutionModelSet* modelSet,
                                DiscreteDistribution* rDist, bool verbose, bool usePatterns, bool reparametrizeRoot,
                                unsigned extraFlags);
  void initBranchLengthsParameters() override;
  std::vector<const Node*> applyBranchLengths() override;
  bool analyticDerivatives(const std::string& variable, double* d1, double* d2) const override;
  void uploadData() override;
  void uploadModels() override;

 public:
  RNonHomogeneousTreeLikelihood(const Tree& tree, const SiteContainer& data, SubstitutionModelSet* modelSet,
                                DiscreteDistribution* rDist, bool verbose = true, bool usePatterns = true,
                                bool reparametrizeRoot = false);
  void setData(const SiteContainer& sites);
  void initialize() override;
  void fireParameterChanged(const ParameterList& params) override;
  ParameterList getSubstitutionModelParameters() const override;
  const SubstitutionModelSet* getSubstitutionModelSet() const { return modelSet_; }
  SubstitutionModelSet* getSubstitutionModelSet() { return modelSet_; }
  bool isRootReparametrized() const { return reparametrizeRoot_; }
  void computeAllTransitionProbabilities();
};

// Likelihood/DRNonHomogeneousTreeLikelihood.h:114-120: the NH likelihood with every branch's
// derivatives from one double-recursive pass (plk_all_branch_derivatives)
class DRNonHomogeneousTreeLikelihood : public RNonHomogeneousTreeLikelihood {
 public:
  DRNonHomogeneousTreeLikelihood(const Tree& tree, const SiteContainer& data, SubstitutionModelSet* modelSet,
                                 DiscreteDistribution* rDist, bool verbose = true, bool reparametrizeRoot = false);
};

}  // namespace bpp

#endif
