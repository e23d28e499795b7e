// Host mirror: R-likelihood classes over libplk.
//
// What stays on the host (as in the reference): parameters and their dispatch
// (fireParameterChanged, Likelihood/RHomogeneousTreeLikelihood.cpp:255-283), the
// tree copy / unroot / postorder node list (Likelihood/AbstractHomogeneousTreeLikelihood.cpp:140-166),
// root site patterns (SitePatterns.cpp:51-100), model eigen-systems.
// What runs on the MI355X: every branch transition matrix (plk_update_pmatrices),
// the full postorder traversal (plk_update_partials) and the root reduction
// (plk_root_loglik).  Only one scalar comes back per evaluation.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

#include "Bpp/App/ApplicationTools.h"
#include "Bpp/Phyl/Likelihood/TreeLikelihood.h"
#include "plk.h"

namespace bpp {

namespace {
int deviceFromEnv() {
  const char* e = std::getenv("BPP_AMD_DEVICE");
  return e ? std::atoi(e) : 0;
}

// BPP_AMD_DEVICES=0,1,2,...: shard the site patterns over these devices (plk_create_multi);
// empty: one device (BPP_AMD_DEVICE, default 0)
std::vector<int> devicesFromEnv() {
  std::vector<int> d;
  const char* e = std::getenv("BPP_AMD_DEVICES");
  if (!e) return d;
  std::string s(e);
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    if (j > i) d.push_back(std::atoi(s.substr(i, j - i).c_str()));
    i = j + 1;
  }
  return d;
}
}  // namespace

void AbstractPlkTreeLikelihood::check(int rc, const char* what) const {
  if (rc != PLK_OK) throw DeviceException(rc, std::string(what) + ": " + plk_last_error(engine_));
}

AbstractPlkTreeLikelihood::AbstractPlkTreeLikelihood(const Tree& tree, DiscreteDistribution* rDist, bool checkRooted,
                                                     bool verbose, bool usePatterns)
    : rateDistribution_(rDist), usePatterns_(usePatterns), verbose_(verbose) {
  if (!rDist) throw NullPointerException("AbstractPlkTreeLikelihood: null rate distribution");
  tree_ = new TreeTemplate<Node>(tree);
  if (checkRooted && tree_->isRooted()) {
    if (verbose) ApplicationTools::displayWarning("Tree has been unrooted.");
    tree_->unroot();
  }
  nodes_ = tree_->getNodes();
  nodes_.pop_back();  // the root is last in postorder
  nbClasses_ = rateDistribution_->getNumberOfCategories();
  brLenConstraint_ = std::make_shared<IntervalConstraint>(minimumBrLen_, maximumBrLen_, true, true);
  buildEngineLayout();
}

AbstractPlkTreeLikelihood::~AbstractPlkTreeLikelihood() {
  if (engine_) plk_destroy(engine_);
  delete tree_;
}

void AbstractPlkTreeLikelihood::buildEngineLayout() {
  std::vector<Node*> all = tree_->getNodes();
  engineIndex_.clear();
  nTips_ = nInternal_ = 0;
  for (Node* n : all)
    if (n->isLeaf()) engineIndex_[n] = nTips_++;
  for (Node* n : all)
    if (!n->isLeaf()) engineIndex_[n] = nTips_ + nInternal_++;
  rootEngine_ = engineIndex_[tree_->getRootNode()];
  engineById_.clear();
  nodeById_.clear();
  for (const auto& kv : engineIndex_) {
    const int id = kv.first->getId();
    if (id < 0 || id > 16 * (int)all.size() + 1024) continue;  // sparse ids stay on the map
    if ((size_t)id >= engineById_.size()) {
      engineById_.resize((size_t)id + 1, -1);
      nodeById_.resize((size_t)id + 1, nullptr);
    }
    if (nodeById_[(size_t)id]) {  // duplicate id: lookups by id are ambiguous
      engineById_[(size_t)id] = -1;
      continue;
    }
    engineById_[(size_t)id] = kv.second;
    nodeById_[(size_t)id] = kv.first;
  }
  opParent_.clear();
  opChildren_.clear();
  opFlags_.clear();
  maxSons_ = 0;
  for (Node* n : all) {
    if (n->isLeaf()) continue;
    maxSons_ = std::max(maxSons_, n->getNumberOfSons());
    for (size_t k = 0; k < n->getNumberOfSons(); k += 3) {
      std::vector<int> ch;
      for (size_t j = k; j < std::min(k + 3, n->getNumberOfSons()); j++) ch.push_back(engineIndex_[n->getSon(j)]);
      opParent_.push_back(engineIndex_[n]);
      opChildren_.push_back(ch);
      opFlags_.push_back(k == 0 ? 0 : PLK_OP_ACCUMULATE);
    }
  }
}

// DRASRTreeLikelihoodData::initLikelihoods (Likelihood/DRASRTreeLikelihoodData.cpp:55-90):
// checks, root site patterns, leaf states.  The engine always evaluates the root
// patterns; per-subtree compression (usePatterns) changes nothing in the result.
void AbstractPlkTreeLikelihood::setDataImpl(const SiteContainer& sites, const Alphabet* alphabet,
                                            const SubstitutionModel& model) {
  if (sites.getNumberOfSequences() == 1) throw Exception("Error, only 1 sequence!");
  if (sites.getNumberOfSequences() == 0) throw Exception("Error, no sequence!");
  if (sites.getAlphabet()->getAlphabetType() != alphabet->getAlphabetType())
    throw AlphabetMismatchException("Data and model must have the same alphabet type.");
  std::vector<const Node*> leaves(nTips_);
  for (auto& kv : engineIndex_)
    if (kv.second < nTips_) leaves[kv.second] = kv.first;
  std::vector<const Sequence*> seqs(nTips_);
  for (int t = 0; t < nTips_; t++) {
    if (!sites.hasSequence(leaves[t]->getName()))
      throw SequenceNotFoundException("Leaf name in tree not found in site container", leaves[t]->getName());
    seqs[t] = &sites.getSequence(leaves[t]->getName());
  }
  nbSites_ = sites.getNumberOfSites();
  // leaf states must be allowed by the model (getInitValue throws BadIntException)
  for (int t = 0; t < nTips_; t++)
    for (size_t i = 0; i < nbSites_; i++) {
      const int s = seqs[t]->getValue(i);
      if (s < 0 || !alphabet->isIntInAlphabet(s)) model.getInitValue(0, s);
    }
  // root patterns (first-occurrence order; SitePatterns sorts, which only permutes them)
  std::unordered_map<std::string, size_t> seen;
  rootPatternLinks_.assign(nbSites_, 0);
  rootWeights_.clear();
  std::vector<size_t> repr;
  std::string key(nTips_ * sizeof(int), '\0');
  for (size_t i = 0; i < nbSites_; i++) {
    for (int t = 0; t < nTips_; t++) {
      const int s = seqs[t]->getValue(i);
      std::memcpy(&key[t * sizeof(int)], &s, sizeof(int));
    }
    auto it = seen.find(key);
    if (it == seen.end()) {
      it = seen.emplace(key, rootWeights_.size()).first;
      rootWeights_.push_back(0);
      repr.push_back(i);
    }
    rootPatternLinks_[i] = it->second;
    rootWeights_[it->second]++;
  }
  nbDistinctSites_ = rootWeights_.size();
  patternStates_.assign(nTips_, std::vector<int>(nbDistinctSites_));
  for (int t = 0; t < nTips_; t++)
    for (size_t p = 0; p < nbDistinctSites_; p++) patternStates_[t][p] = seqs[t]->getValue(repr[p]);
  data_.reset(sites.clone());
  nbStates_ = model.getNumberOfStates();
  initialized_ = false;
  scaledNow_ = false;  // new data: unscaled first again
}

void AbstractPlkTreeLikelihood::createEngine(size_t nModels, bool nonNegGuard) {
  if (engine_) {
    plk_destroy(engine_);
    engine_ = nullptr;
  }
  // Exact power-of-two rescaling when forced, or after an unscaled evaluation flagged underflow
  // (setUnderflowScaling, switchToScaledEngine)
  engineModels_ = nModels;
  engineGuard_ = nonNegGuard;
  const bool scaling = underflowScalingActive();
  engineScaled_ = scaling;
  unsigned flags = (scaling ? (unsigned)PLK_FLAG_SCALING : 0u) | (nonNegGuard ? (unsigned)PLK_FLAG_NONNEG_GUARD : 0u) |
                   extraFlags_;
  // usePatterns (the reference default): per-subtree site-pattern compression on the device
  // (DRASRTreeLikelihoodData.cpp:218-332, PLK_FLAG_SUBTREE_PATTERNS); not for the double-
  // recursive classes (their data class has no compression either, DRASDRTreeLikelihoodData);
  // BPP_AMD_USE_PATTERNS=0 switches it off
  compressed_ = usePatterns_ && !(extraFlags_ & PLK_FLAG_DOUBLE_RECURSIVE);
  if (const char* e = std::getenv("BPP_AMD_USE_PATTERNS"))
    if (e[0] == '0') compressed_ = false;
  // Shapes the fused tree kernels serve (4 states with 1, 2 or 4 classes: plk_jit_tree4;
  // 20 states, up to 4 classes: plk_jit_treeM; 64 states, 1 class: treeM) run lnL-only:
  // one launch per evaluation with the partials in registers, faster than the per-subtree
  // compression at every size measured (cfg2: 0.14 vs 0.36 ms), so compression is kept for
  // the other shapes.  BPP_AMD_FUSED=0 turns this off.
  const size_t S = nbStates_, C = nbClasses_;
  lnlOnly_ = (S == 4 && (C == 1 || C == 2 || C == 4)) || (S == 20 && C <= 4) || (S == 64 && C == 1);
  if (const char* e = std::getenv("BPP_AMD_FUSED"))
    if (e[0] == '0') lnlOnly_ = false;
  if (lnlOnly_) {
    compressed_ = false;
    flags |= PLK_FLAG_LNL_ONLY;
  }
  if (compressed_) flags |= PLK_FLAG_SUBTREE_PATTERNS;
  plk_handle h = nullptr;
  const std::vector<int> devs = devicesFromEnv();
  int rc = devs.empty() ? plk_create(deviceFromEnv(), (int)nbStates_, (int)nbClasses_, (int64_t)nbDistinctSites_, nTips_,
                                     nInternal_, (int)nModels, flags, &h)
                        : plk_create_multi(devs.data(), (int)devs.size(), (int)nbStates_, (int)nbClasses_,
                                           (int64_t)nbDistinctSites_, nTips_, nInternal_, (int)nModels, flags, &h);
  if (rc != PLK_OK) throw DeviceException(rc, std::string("plk_create: ") + plk_last_error(nullptr));
  engine_ = h;
  derivStale_.assign((size_t)(nTips_ + nInternal_), 1);
}

void AbstractPlkTreeLikelihood::initBranchLengthsParameters() {
  brLenParameters_.reset();
  for (size_t i = 0; i < nodes_.size(); i++) {
    double d = minimumBrLen_;
    if (!nodes_[i]->hasDistanceToFather()) {
      if (verbose_)
        ApplicationTools::displayWarning("Missing branch length " + std::to_string(i) + ". Value is set to " +
                                         std::to_string(minimumBrLen_));
      nodes_[i]->setDistanceToFather(minimumBrLen_);
    } else {
      d = nodes_[i]->getDistanceToFather();
      if (d < minimumBrLen_) {
        nodes_[i]->setDistanceToFather(minimumBrLen_);
        d = minimumBrLen_;
      }
      if (d > maximumBrLen_) {
        nodes_[i]->setDistanceToFather(maximumBrLen_);
        d = maximumBrLen_;
      }
    }
    brLenParameters_.addParameter(Parameter("BrLen" + std::to_string(i), d, brLenConstraint_));
  }
}

void AbstractPlkTreeLikelihood::setMinimumBranchLength(double minimum) {
  if (minimum > maximumBrLen_)
    throw Exception("AbstractHomogeneousTreeLikelihood::setMinimumBranchLength. Minimum branch length sould be lower "
                    "than the maximum one: " + TextTools::toString(maximumBrLen_));
  minimumBrLen_ = minimum;
  brLenConstraint_ = std::make_shared<IntervalConstraint>(minimumBrLen_, maximumBrLen_, true, true);
  initBranchLengthsParameters();
}

void AbstractPlkTreeLikelihood::setMaximumBranchLength(double maximum) {
  if (maximum < minimumBrLen_)
    throw Exception("AbstractHomogeneousTreeLikelihood::setMaximumBranchLength. Maximum branch length sould be higher "
                    "than the minimum one: " + TextTools::toString(minimumBrLen_));
  maximumBrLen_ = maximum;
  brLenConstraint_ = std::make_shared<IntervalConstraint>(minimumBrLen_, maximumBrLen_, true, true);
  initBranchLengthsParameters();
}

std::vector<const Node*> AbstractPlkTreeLikelihood::applyBranchLengths() {
  std::vector<const Node*> changed;
  if (brLenNames_.size() != nodes_.size()) {
    brLenNames_.clear();
    for (size_t i = 0; i < nodes_.size(); i++) brLenNames_.push_back("BrLen" + std::to_string(i));
    brLenPos_.assign(nodes_.size(), -1);
  }
  const ParameterList& pl = parameters_;
  for (size_t i = 0; i < nodes_.size(); i++) {
    const long k = pl.indexOf(brLenNames_[i], (size_t)brLenPos_[i]);
    brLenPos_[i] = k;
    if (k < 0) continue;
    const double v = pl[(size_t)k].getValue();
    if (!nodes_[i]->hasDistanceToFather() || nodes_[i]->getDistanceToFather() != v) {
      nodes_[i]->setDistanceToFather(v);
      changed.push_back(nodes_[i]);
    }
  }
  return changed;
}

void AbstractPlkTreeLikelihood::uploadEigen(int m, const SubstitutionModel& model) {
  const size_t S = nbStates_;
  std::vector<double> lam(S);
  for (size_t k = 0; k < S; k++) lam[k] = model.getEigenValues()[k] * model.getRate();
  check(plk_set_eigen(engine_, m, model.getColumnRightEigenVectors().data(), model.getRowLeftEigenVectors().data(),
                      lam.data()),
        "plk_set_eigen");
  stats_.eigenUploads++;
}

void AbstractPlkTreeLikelihood::uploadRootFrequencies(const Vdouble& pi) {
  rootFreqs_ = pi;
  check(plk_set_root_frequencies(engine_, rootFreqs_.data()), "plk_set_root_frequencies");
}

void AbstractPlkTreeLikelihood::uploadRates() {
  check(plk_set_category_rates(engine_, rateDistribution_->getCategories().data(),
                               rateDistribution_->getProbabilities().data()),
        "plk_set_category_rates");
}

void AbstractPlkTreeLikelihood::updatePmatrices(const std::vector<const Node*>& nodes) {
  if (nodes.empty()) return;
  stats_.pmatBranches += nodes.size();
  std::vector<int32_t> br, mod;
  std::vector<double> t;
  for (const Node* n : nodes) {
    br.push_back(engineIndex_.at(n));
    mod.push_back(modelIndexForNode(n));
    t.push_back(n->getDistanceToFather());
  }
  // a model whose eigen-system failed its check (SubstitutionModel::checkEigen) has no
  // device path: its branches get host P(t . r_c) from the Taylor branch of getPij_t
  // (plk_set_pmatrix; derivatives of those branches are then numerical)
  {
    size_t k = 0;
    const Vdouble& rates = rateDistribution_->getCategories();
    std::vector<double> P(nbClasses_ * nbStates_ * nbStates_);
    for (size_t i = 0; i < br.size(); i++) {
      const SubstitutionModel* m = modelForIndex(mod[i]);
      if (m && m->needsHostPij()) {
        for (size_t c = 0; c < nbClasses_; c++) {
          const RowMatrix<double>& Pc = m->getPij_t(t[i] * rates[c]);
          std::copy(Pc.data(), Pc.data() + nbStates_ * nbStates_, P.begin() + c * nbStates_ * nbStates_);
        }
        check(plk_set_pmatrix(engine_, br[i], P.data()), "plk_set_pmatrix");
      } else {
        br[k] = br[i];
        mod[k] = mod[i];
        t[k] = t[i];
        k++;
      }
    }
    br.resize(k);
    mod.resize(k);
    t.resize(k);
    if (br.empty()) return;
  }
  // P only: dP and d2P (which the reference computes with every P,
  // AbstractHomogeneousTreeLikelihood.cpp:375-413) follow when a derivative is requested
  check(plk_update_pmatrices(engine_, (int)br.size(), br.data(), mod.data(), t.data(), PLK_DERIV_P),
        "plk_update_pmatrices");
  for (int b : br) derivStale_[(size_t)b] = 1;
}

void AbstractPlkTreeLikelihood::refreshDerivativeMatrices() const {
  std::vector<int32_t> br, mod;
  std::vector<double> t;
  for (const Node* n : nodes_) {
    const int e = engineIndex_.at(n);
    if (!derivStale_[(size_t)e]) continue;
    const SubstitutionModel* m = modelForIndex(modelIndexForNode(n));
    if (m && m->needsHostPij()) continue;  // host P(t): numerical derivatives
    br.push_back(e);
    mod.push_back(modelIndexForNode(n));
    t.push_back(n->getDistanceToFather());
  }
  if (br.empty()) return;
  check(plk_update_pmatrices(engine_, (int)br.size(), br.data(), mod.data(), t.data(),
                             PLK_DERIV_P | PLK_DERIV_DP | PLK_DERIV_D2P),
        "plk_update_pmatrices");
  for (int b : br) derivStale_[(size_t)b] = 0;
}

void AbstractPlkTreeLikelihood::evaluateTree(const std::vector<const Node*>& pnodes, bool incremental) {
  stats_.pmatBranches += pnodes.size();
  // host P(t) (a model whose eigen-system failed its check) goes up first
  std::vector<int32_t> br, mod;
  std::vector<double> t;
  {
    const Vdouble& rates = rateDistribution_->getCategories();
    std::vector<double> P(nbClasses_ * nbStates_ * nbStates_);
    for (const Node* n : pnodes) {
      const int e = engineOf(n), mi = modelIndexForNode(n);
      const SubstitutionModel* m = modelForIndex(mi);
      if (m && m->needsHostPij()) {
        for (size_t c = 0; c < nbClasses_; c++) {
          const RowMatrix<double>& Pc = m->getPij_t(n->getDistanceToFather() * rates[c]);
          std::copy(Pc.data(), Pc.data() + nbStates_ * nbStates_, P.begin() + c * nbStates_ * nbStates_);
        }
        check(plk_set_pmatrix(engine_, e, P.data()), "plk_set_pmatrix");
      } else {
        br.push_back(e);
        mod.push_back(mi);
        t.push_back(n->getDistanceToFather());
      }
    }
  }
  // the op list: every internal node, or the ancestors of the changed branches when the
  // engine keeps all partials in HBM (not lnL-only, not compressed)
  std::vector<char> need;
  if (incremental && incremental_ && !compressed_ && !lnlOnly_) {
    need.assign((size_t)(nTips_ + nInternal_), 0);
    for (const Node* n : pnodes)
      for (const Node* p = n->getFather(); p; p = p->getFather()) {
        char& f = need[(size_t)engineOf(p)];
        if (f) break;
        f = 1;
      }
  }
  std::vector<plk_op> ops;
  ops.reserve(opParent_.size());
  for (size_t i = 0; i < opParent_.size(); i++) {
    if (!need.empty() && !need[(size_t)opParent_[i]]) continue;
    ops.emplace_back();
    plk_op& o = ops.back();
    o.parent = opParent_[i];
    o.n_children = (int)opChildren_[i].size();
    for (size_t k = 0; k < 3; k++) o.child[k] = k < opChildren_[i].size() ? opChildren_[i][k] : -1;
    o.flags = opFlags_[i];
  }
  drValid_ = false;
  siteLnlValid_ = false;
  stats_.evaluations++;
  if (need.empty()) stats_.fullTraversals++;
  for (int b : br) derivStale_[(size_t)b] = 1;
  if (ops.empty()) {
    check(plk_update_pmatrices(engine_, (int)br.size(), br.data(), mod.data(), t.data(), PLK_DERIV_P),
          "plk_update_pmatrices");
    minusLogLik_ = -reduceRoot();
    if (underflowed()) switchToScaledEngine();
    return;
  }
  double lnl = 0.;
  check(plk_evaluate(engine_, (int)br.size(), br.data(), mod.data(), t.data(), ops.data(), (int)ops.size(),
                     rootEngine_, &lnl, nullptr),
        "plk_evaluate");
  minusLogLik_ = -lnl;
  if (underflowed()) switchToScaledEngine();
}

// plk_root_underflow after an unscaled evaluation in the default mode (include/plk.h: a 0 proves
// the rescaling engine would have returned bitwise the same lnL)
bool AbstractPlkTreeLikelihood::underflowed() const {
  if (scalingMode_ >= 0 || scaledNow_) return false;
  int flag = 0;
  check(plk_root_underflow(engine_, &flag), "plk_root_underflow");
  return flag != 0;
}

void AbstractPlkTreeLikelihood::setUnderflowScaling(bool yn) {
  scalingMode_ = yn ? 1 : 0;
  scaledNow_ = false;
  if (!engine_ || engineScaled_ == underflowScalingActive()) return;
  createEngine(engineModels_, engineGuard_);
  uploadData();
  allDirty_ = true;
  if (initialized_) fireParameterChanged(getParameters());
}

void AbstractPlkTreeLikelihood::switchToScaledEngine() {
  scaledNow_ = true;
  stats_.scaledFallbacks++;
  createEngine(engineModels_, engineGuard_);
  uploadData();
  uploadModels();
  evaluateTree(std::vector<const Node*>(nodes_.begin(), nodes_.end()), false);
}

// Full postorder traversal (Likelihood/RHomogeneousTreeLikelihood.cpp:795-798), or,
// when only branch lengths changed, the traversal restricted to the ancestors of
// the changed branches: every other partial is still resident in HBM and the engine
// LOADs it (the reference always re-traverses, :280).  Same per-node arithmetic, so
// the result is bit-identical to a full traversal.
void AbstractPlkTreeLikelihood::computeTreeLikelihood(const std::vector<const Node*>* changed) {
  std::vector<char> need;
  // a compressed traversal rebuilds every node from its subtree's patterns, an lnL-only
  // one keeps no partials: both always full
  if (changed && incremental_ && !compressed_ && !lnlOnly_) {
    need.assign((size_t)(nTips_ + nInternal_), 0);
    for (const Node* n : *changed)
      for (const Node* p = n->getFather(); p; p = p->getFather()) {
        char& f = need[(size_t)engineIndex_.at(p)];
        if (f) break;  // the rest of the path is already marked
        f = 1;
      }
  }
  std::vector<plk_op> ops;
  ops.reserve(opParent_.size());
  for (size_t i = 0; i < opParent_.size(); i++) {
    if (!need.empty() && !need[(size_t)opParent_[i]]) continue;
    ops.emplace_back();
    plk_op& o = ops.back();
    o.parent = opParent_[i];
    o.n_children = (int)opChildren_[i].size();
    for (size_t k = 0; k < 3; k++) o.child[k] = k < opChildren_[i].size() ? opChildren_[i][k] : -1;
    o.flags = opFlags_[i];
  }
  drValid_ = false;
  stats_.evaluations++;
  if (need.empty()) stats_.fullTraversals++;
  if (ops.empty()) {
    siteLnlValid_ = false;
    return;
  }
  check(plk_update_partials(engine_, ops.data(), (int)ops.size()), "plk_update_partials");
  siteLnlValid_ = false;
}

double AbstractPlkTreeLikelihood::reduceRoot() const {
  double lnl = 0.;
  check(plk_root_loglik(engine_, rootEngine_, &lnl, nullptr, nullptr), "plk_root_loglik");
  return lnl;
}

void AbstractPlkTreeLikelihood::fetchSiteLnl() const {
  if (siteLnlValid_) return;
  siteLnl_.resize(nbDistinctSites_);
  double lnl = 0.;
  check(plk_root_loglik(engine_, rootEngine_, &lnl, siteLnl_.data(), nullptr), "plk_root_loglik");
  siteLnlValid_ = true;
}

double AbstractPlkTreeLikelihood::getValue() const {
  if (!initialized_) throw Exception("TreeLikelihood::getValue(). Instance is not initialized.");
  return minusLogLik_;
}

double AbstractPlkTreeLikelihood::getLogLikelihood() const { return -getValue(); }

double AbstractPlkTreeLikelihood::getLikelihood() const {
  double l = 1.;
  for (size_t i = 0; i < nbSites_; i++) l *= getLikelihoodForASite(i);
  return l;
}

double AbstractPlkTreeLikelihood::getLogLikelihoodForASite(size_t site) const {
  fetchSiteLnl();
  return siteLnl_.at(rootPatternLinks_.at(site));
}

double AbstractPlkTreeLikelihood::getLikelihoodForASite(size_t site) const {
  return std::exp(getLogLikelihoodForASite(site));
}

ParameterList AbstractPlkTreeLikelihood::getBranchLengthsParameters() const {
  if (!initialized_) throw Exception("getBranchLengthsParameters(). Object is not initialized.");
  return brLenParameters_.getCommonParametersWith(getParameters());
}

ParameterList AbstractPlkTreeLikelihood::getNonDerivableParameters() const {
  ParameterList pl = getSubstitutionModelParameters();
  pl.addParameters(getRateDistributionParameters());
  return pl;
}

ParameterList AbstractPlkTreeLikelihood::getRateDistributionParameters() const {
  if (!initialized_) throw Exception("getRateDistributionParameters(). Object is not initialized.");
  return rateDistribution_->getIndependentParameters().getCommonParametersWith(getParameters());
}

void AbstractPlkTreeLikelihood::setParameters(const ParameterList& pl) { setParametersValues(pl); }

VVVdouble AbstractPlkTreeLikelihood::getLikelihoodArray(int nodeId) const {
  const Node* node = tree_->getNode(nodeId);
  const int e = engineIndex_.at(node);
  VVVdouble out(nbDistinctSites_, VVdouble(nbClasses_, Vdouble(nbStates_)));
  if (e < nTips_) {
    throw Exception("getLikelihoodArray: leaf arrays are held as state codes on the device");
  }
  std::vector<double> buf(nbDistinctSites_ * nbClasses_ * nbStates_);
  check(plk_get_partials(engine_, e, buf.data()), "plk_get_partials");
  for (size_t i = 0; i < nbDistinctSites_; i++)
    for (size_t c = 0; c < nbClasses_; c++)
      for (size_t s = 0; s < nbStates_; s++) out[i][c][s] = buf[(i * nbClasses_ + c) * nbStates_ + s];
  return out;
}

// Branch-length derivatives: analytic on the device (plk_branch_derivatives, the
// dL / d2L propagation of Likelihood/RHomogeneousTreeLikelihood.cpp:346-541, 596-791)
// for every model; central differences of the device log-likelihood only if the
// engine reports PLK_ERR_UNSUPPORTED (per-subtree pattern compression).
// some branch's model currently has no device P(t) (its eigen-system failed its check:
// host Taylor P(t), no dP / d2P on the device); asked per derivative, so a model that
// recovers a valid eigen-system gets analytic derivatives back
bool AbstractPlkTreeLikelihood::hostPInUse() const {
  for (const Node* n : nodes_) {
    const SubstitutionModel* m = modelForIndex(modelIndexForNode(n));
    if (m && m->needsHostPij()) return true;
  }
  return false;
}

bool AbstractPlkTreeLikelihood::analyticDerivatives(const std::string& variable, double* d1, double* d2) const {
  if (!(derivFirst_ || derivSecond_) || hostPInUse()) return false;
  if (variable.size() <= 5 || variable.find_first_not_of("0123456789", 5) != std::string::npos)
    throw Exception("analyticDerivatives: not a branch-length parameter: " + variable);
  const Node* n = nodes_.at(TextTools::to<size_t>(variable.substr(5)));
  refreshDerivativeMatrices();
  if (extraFlags_ & PLK_FLAG_DOUBLE_RECURSIVE) {
    if (!drValid_) {
      const size_t nn = (size_t)(nTips_ + nInternal_);
      drD1_.assign(nn, 0.);
      drD2_.assign(nn, 0.);
      check(plk_all_branch_derivatives(engine_, drD1_.data(), drD2_.data()), "plk_all_branch_derivatives");
      drValid_ = true;
    }
    *d1 = drD1_[(size_t)engineIndex_.at(n)];
    *d2 = drD2_[(size_t)engineIndex_.at(n)];
    return true;
  }
  const int rc = plk_branch_derivatives(engine_, engineIndex_.at(n), d1, d2);
  if (rc == PLK_ERR_UNSUPPORTED) return false;
  check(rc, "plk_branch_derivatives");
  return true;
}

double AbstractPlkTreeLikelihood::getFirstOrderDerivative(const std::string& variable) const {
  if (!parameters_.hasParameter(variable)) throw ParameterNotFoundException("getFirstOrderDerivative().", variable);
  if (!getDerivableParameters().hasParameter(variable))
    throw Exception("Derivatives are only implemented for branch length parameters.");
  double d1, d2;
  if (analyticDerivatives(variable, &d1, &d2)) return -d1;
  AbstractPlkTreeLikelihood* self = const_cast<AbstractPlkTreeLikelihood*>(this);
  const double t = parameters_.getParameterValue(variable);
  const double h = 1e-5 * std::max(t, 1e-3);
  ParameterList pl = parameters_.createSubList(std::vector<std::string>(1, variable));
  // both points inside the parameter's own constraint (BrLen<i>: [min, max] branch length,
  // RootPosition: (0, 1)); one-sided at a bound
  double tp = t + h, tm = t - h;
  if (pl[0].hasConstraint()) {
    const Constraint& c = *pl[0].getConstraint();
    if (!c.isCorrect(tp)) tp = t;
    if (!c.isCorrect(tm)) tm = t;
  }
  if (tp == tm) throw Exception("getFirstOrderDerivative: no room for a difference in " + variable);
  pl[0].setValue(tp);
  self->setParameters(pl);
  const double fp = minusLogLik_;
  pl[0].setValue(tm);
  self->setParameters(pl);
  const double fm = minusLogLik_;
  pl[0].setValue(t);
  self->setParameters(pl);
  return (fp - fm) / (tp - tm);
}

double AbstractPlkTreeLikelihood::getSecondOrderDerivative(const std::string& variable) const {
  if (!parameters_.hasParameter(variable)) throw ParameterNotFoundException("getSecondOrderDerivative().", variable);
  if (!getDerivableParameters().hasParameter(variable))
    throw Exception("Derivatives are only implemented for branch length parameters.");
  double d1, d2;
  if (analyticDerivatives(variable, &d1, &d2)) return -d2;
  AbstractPlkTreeLikelihood* self = const_cast<AbstractPlkTreeLikelihood*>(this);
  const double t = parameters_.getParameterValue(variable);
  const double h = 1e-4 * std::max(t, 1e-2);
  ParameterList pl = parameters_.createSubList(std::vector<std::string>(1, variable));
  const double f0 = minusLogLik_;
  // three equally spaced points inside the parameter's own constraint: centred, or shifted
  // one step in when t +- h leaves it (one-sided second difference at a bound)
  double x0 = t - h;
  if (pl[0].hasConstraint()) {
    const Constraint& c = *pl[0].getConstraint();
    if (!c.isCorrect(t - h)) x0 = t;
    else if (!c.isCorrect(t + h)) x0 = t - 2. * h;
    if (!c.isCorrect(x0) || !c.isCorrect(x0 + 2. * h))
      throw Exception("getSecondOrderDerivative: no room for a difference in " + variable);
  }
  double f[3];
  for (int k = 0; k < 3; k++) {
    const double x = x0 + k * h;
    if (x == t) {
      f[k] = f0;
      continue;
    }
    pl[0].setValue(x);
    self->setParameters(pl);
    f[k] = minusLogLik_;
  }
  pl[0].setValue(t);
  self->setParameters(pl);
  return (f[2] - 2. * f[1] + f[0]) / (h * h);
}

// ---------------------------------------------------------------------------
// RHomogeneousTreeLikelihood
// ---------------------------------------------------------------------------

RHomogeneousTreeLikelihood::RHomogeneousTreeLikelihood(const Tree& tree, SubstitutionModel* model,
                                                       DiscreteDistribution* rDist, bool checkRooted, bool verbose,
                                                       bool usePatterns)
    : AbstractPlkTreeLikelihood(tree, rDist, checkRooted, verbose, usePatterns), model_(model) {
  if (!model) throw NullPointerException("RHomogeneousTreeLikelihood: null model");
  nbStates_ = model->getNumberOfStates();
}

RHomogeneousTreeLikelihood::RHomogeneousTreeLikelihood(const Tree& tree, const SiteContainer& data,
                                                       SubstitutionModel* model, DiscreteDistribution* rDist,
                                                       bool checkRooted, bool verbose, bool usePatterns)
    : RHomogeneousTreeLikelihood(tree, model, rDist, checkRooted, verbose, usePatterns) {
  setData(data);
}

void RHomogeneousTreeLikelihood::setData(const SiteContainer& sites) {
  if (verbose_) ApplicationTools::displayTask("Initializing data structure");
  setDataImpl(sites, model_->getAlphabet(), *model_);
  createEngine(1, true);
  uploadData();
  if (verbose_) {
    ApplicationTools::displayTaskDone();
    ApplicationTools::displayResult("Number of distinct sites", nbDistinctSites_);
  }
}

// leaf codes and init values (getInitValue), pattern weights
void RHomogeneousTreeLikelihood::uploadData() {
  const Alphabet* a = model_->getAlphabet();
  const int nc = a->getNumberOfCodes();
  std::vector<double> table((size_t)nc * nbStates_);
  for (int c = 0; c < nc; c++)
    for (size_t s = 0; s < nbStates_; s++) table[c * nbStates_ + s] = model_->getInitValue(s, c);
  check(plk_set_code_table(engine_, nc, table.data()), "plk_set_code_table");
  std::vector<uint8_t> codes(nbDistinctSites_);
  for (int t = 0; t < nTips_; t++) {
    for (size_t p = 0; p < nbDistinctSites_; p++) codes[p] = (uint8_t)patternStates_[t][p];
    check(plk_set_tip_codes(engine_, t, codes.data()), "plk_set_tip_codes");
  }
  std::vector<double> w(rootWeights_.begin(), rootWeights_.end());
  check(plk_set_pattern_weights(engine_, w.data()), "plk_set_pattern_weights");
}

void RHomogeneousTreeLikelihood::uploadModels() {
  uploadEigen(0, *model_);
  uploadRates();
  uploadRootFrequencies(model_->getFrequencies());
}

void RHomogeneousTreeLikelihood::initialize() {
  if (initialized_) throw Exception("RHomogeneousTreeLikelihood::initialize(). Object is already initialized.");
  allDirty_ = true;
  if (!data_) throw Exception("RHomogeneousTreeLikelihood::initialize(). Data are no set.");
  resetParameters_();
  initBranchLengthsParameters();
  addParameters_(brLenParameters_);
  addParameters_(model_->getIndependentParameters());
  addParameters_(rateDistribution_->getIndependentParameters());
  initialized_ = true;
  fireParameterChanged(getParameters());
}

ParameterList RHomogeneousTreeLikelihood::getSubstitutionModelParameters() const {
  if (!initialized_) throw Exception("getSubstitutionModelParameters(). Object is not initialized.");
  return model_->getParameters().getCommonParametersWith(getParameters());
}

void RHomogeneousTreeLikelihood::computeAllTransitionProbabilities() {
  uploadEigen(0, *model_);
  uploadRates();
  std::vector<const Node*> all(nodes_.begin(), nodes_.end());
  updatePmatrices(all);
  uploadRootFrequencies(model_->getFrequencies());
}

// Likelihood/RHomogeneousTreeLikelihood.cpp:255-283: a model or rate-distribution change
// recomputes every P(t); otherwise only the branches whose length changed get a new P(t),
// and only their ancestors are re-traversed (the reference always re-traverses, :280).
// Changes are detected by value, so a caller that hands over every parameter (as the
// optimisers do) recomputes only what moved.
void RHomogeneousTreeLikelihood::fireParameterChanged(const ParameterList&) {
  if (!initialized_) throw Exception("RHomogeneousTreeLikelihood::fireParameterChanged(). Object not initialized.");
  const std::vector<const Node*> changed = applyBranchLengths();
  const bool modelChanged = model_->matchParametersValues(getParameters());
  const bool rateChanged = rateDistribution_->matchParametersValues(getParameters());
  if (allDirty_ || modelChanged || rateChanged) {
    allDirty_ = false;
    uploadModels();
    evaluateTree(std::vector<const Node*>(nodes_.begin(), nodes_.end()), false);
  } else {
    evaluateTree(changed, true);
  }
}

// ---------------------------------------------------------------------------
// DRHomogeneousTreeLikelihood (Likelihood/DRHomogeneousTreeLikelihood.h): the engine keeps
// an upper vector per branch (PLK_FLAG_DOUBLE_RECURSIVE)
// ---------------------------------------------------------------------------

DRHomogeneousTreeLikelihood::DRHomogeneousTreeLikelihood(const Tree& tree, SubstitutionModel* model,
                                                         DiscreteDistribution* rDist, bool checkRooted, bool verbose)
    : RHomogeneousTreeLikelihood(tree, model, rDist, checkRooted, verbose, true) {
  extraFlags_ = PLK_FLAG_DOUBLE_RECURSIVE;
}

DRHomogeneousTreeLikelihood::DRHomogeneousTreeLikelihood(const Tree& tree, const SiteContainer& data,
                                                         SubstitutionModel* model, DiscreteDistribution* rDist,
                                                         bool checkRooted, bool verbose)
    : DRHomogeneousTreeLikelihood(tree, model, rDist, checkRooted, verbose) {
  setData(data);
}

// ---------------------------------------------------------------------------
// RNonHomogeneousTreeLikelihood (rooted; one eigen-system per branch model)
// ---------------------------------------------------------------------------

RNonHomogeneousTreeLikelihood::RNonHomogeneousTreeLikelihood(const Tree& tree, const SiteContainer& data,
                                                             SubstitutionModelSet* modelSet,
                                                             DiscreteDistribution* rDist, bool verbose,
                                                             bool usePatterns, bool reparametrizeRoot)
    : RNonHomogeneousTreeLikelihood(tree, data, modelSet, rDist, verbose, usePatterns, reparametrizeRoot, 0u) {}

DRNonHomogeneousTreeLikelihood::DRNonHomogeneousTreeLikelihood(const Tree& tree, const SiteContainer& data,
                                                               SubstitutionModelSet* modelSet,
                                                               DiscreteDistribution* rDist, bool verbose,
                                                               bool reparametrizeRoot)
    : RNonHomogeneousTreeLikelihood(tree, data, modelSet, rDist, verbose, true, reparametrizeRoot,
                                    PLK_FLAG_DOUBLE_RECURSIVE) {}

RNonHomogeneousTreeLikelihood::RNonHomogeneousTreeLikelihood(const Tree& tree, const SiteContainer& data,
                                                             SubstitutionModelSet* modelSet,
                                                             DiscreteDistribution* rDist, bool verbose,
                                                             bool usePatterns, bool reparametrizeRoot,
                                                             unsigned extraFlags)
    : AbstractPlkTreeLikelihood(tree, rDist, false, verbose, usePatterns), modelSet_(modelSet),
      reparametrizeRoot_(reparametrizeRoot) {
  if (!modelSet) throw NullPointerException("RNonHomogeneousTreeLikelihood: null model set");
  extraFlags_ = extraFlags;
  nbStates_ = modelSet->getNumberOfStates();
  // AbstractNonHomogeneousTreeLikelihood::init_ (:160-185)
  const Node* root = tree_->getRootNode();
  if (root->getNumberOfSons() < 2) throw Exception("RNonHomogeneousTreeLikelihood: the root must have two sons");
  root1_ = root->getSon(0)->getId();
  root2_ = root->getSon(1)->getId();
  for (const Node* n : nodes_) {
    modelOfNodeId_[n->getId()] = (int)modelSet_->getModelIndexForNode(n->getId());
    idToNode_[n->getId()] = n;
  }
  setData(data);
}

int RNonHomogeneousTreeLikelihood::modelIndexForNode(const Node* n) const { return modelOfNodeId_.at(n->getId()); }
const SubstitutionModel* RNonHomogeneousTreeLikelihood::modelForIndex(int m) const {
  return modelSet_->getModel((size_t)m);
}

void RNonHomogeneousTreeLikelihood::setData(const SiteContainer& sites) {
  const SubstitutionModel& m0 = *modelSet_->getModel(0);
  setDataImpl(sites, modelSet_->getAlphabet(), m0);
  createEngine(modelSet_->getNumberOfModels(), false);
  uploadData();
}

void RNonHomogeneousTreeLikelihood::uploadData() {
  const SubstitutionModel& m0 = *modelSet_->getModel(0);
  const Alphabet* a = modelSet_->getAlphabet();
  const int nc = a->getNumberOfCodes();
  std::vector<double> table((size_t)nc * nbStates_);
  for (int c = 0; c < nc; c++)
    for (size_t s = 0; s < nbStates_; s++) table[c * nbStates_ + s] = m0.getInitValue(s, c);
  check(plk_set_code_table(engine_, nc, table.data()), "plk_set_code_table");
  std::vector<uint8_t> codes(nbDistinctSites_);
  for (int t = 0; t < nTips_; t++) {
    for (size_t p = 0; p < nbDistinctSites_; p++) codes[p] = (uint8_t)patternStates_[t][p];
    check(plk_set_tip_codes(engine_, t, codes.data()), "plk_set_tip_codes");
  }
  std::vector<double> w(rootWeights_.begin(), rootWeights_.end());
  check(plk_set_pattern_weights(engine_, w.data()), "plk_set_pattern_weights");
}

// AbstractNonHomogeneousTreeLikelihood::initBranchLengthsParameters (:343-390): the root's
// two branches become BrLenRoot = l1 + l2 and RootPosition = l1 / (l1 + l2)
void RNonHomogeneousTreeLikelihood::initBranchLengthsParameters() {
  if (!reparametrizeRoot_) {
    AbstractPlkTreeLikelihood::initBranchLengthsParameters();
    return;
  }
  AbstractPlkTreeLikelihood::initBranchLengthsParameters();
  double l1 = 0., l2 = 0.;
  ParameterList kept;
  for (size_t i = 0; i < nodes_.size(); i++) {
    const int id = nodes_[i]->getId();
    const Parameter& p = brLenParameters_[i];
    if (id == root1_)
      l1 = p.getValue();
    else if (id == root2_)
      l2 = p.getValue();
    else
      kept.addParameter(p);
  }
  brLenParameters_ = kept;
  brLenParameters_.addParameter(Parameter("BrLenRoot", l1 + l2, brLenConstraint_));
  brLenParameters_.addParameter(Parameter("RootPosition", l1 / (l1 + l2), Parameter::PROP_CONSTRAINT_EX));
}

// AbstractNonHomogeneousTreeLikelihood::applyParameters (:312-335)
std::vector<const Node*> RNonHomogeneousTreeLikelihood::applyBranchLengths() {
  std::vector<const Node*> changed = AbstractPlkTreeLikelihood::applyBranchLengths();
  if (!reparametrizeRoot_) return changed;
  const double len = parameters_.getParameterValue("BrLenRoot");
  const double pos = parameters_.getParameterValue("RootPosition");
  for (const Node* n : nodes_) {
    const int id = n->getId();
    if (id != root1_ && id != root2_) continue;
    const double v = id == root1_ ? len * pos : len * (1. - pos);
    Node* m = const_cast<Node*>(n);
    if (!m->hasDistanceToFather() || m->getDistanceToFather() != v) {
      m->setDistanceToFather(v);
      changed.push_back(n);
    }
  }
  return changed;
}

// BrLenRoot and RootPosition move both root branches: one directional derivative on the
// device (plk_root_pair_derivatives), as computeTreeDLikelihood / computeTreeD2Likelihood do
// for them (RNonHomogeneousTreeLikelihood.cpp:391-560, 862-1100)
bool RNonHomogeneousTreeLikelihood::analyticDerivatives(const std::string& variable, double* d1, double* d2) const {
  if (!reparametrizeRoot_ || (variable != "BrLenRoot" && variable != "RootPosition"))
    return AbstractPlkTreeLikelihood::analyticDerivatives(variable, d1, d2);
  if (!(derivFirst_ || derivSecond_) || hostPInUse()) return false;
  const double len = parameters_.getParameterValue("BrLenRoot");
  const double pos = parameters_.getParameterValue("RootPosition");
  const double alpha = variable == "BrLenRoot" ? pos : len;
  const double beta = variable == "BrLenRoot" ? 1. - pos : -len;
  const int a = engineIndex_.at(idToNode_.at(root1_)), b = engineIndex_.at(idToNode_.at(root2_));
  refreshDerivativeMatrices();
  const int rc = plk_root_pair_derivatives(engine_, a, b, alpha, beta, d1, d2);
  if (rc == PLK_ERR_UNSUPPORTED) return false;
  check(rc, "plk_root_pair_derivatives");
  return true;
}

void RNonHomogeneousTreeLikelihood::initialize() {
  if (initialized_) throw Exception("RNonHomogeneousTreeLikelihood::initialize(). Object is already initialized.");
  allDirty_ = true;
  // AbstractNonHomogeneousTreeLikelihood::initParameters (:290-306)
  resetParameters_();
  initBranchLengthsParameters();
  addParameters_(brLenParameters_);
  addParameters_(modelSet_->getIndependentParameters());
  addParameters_(rateDistribution_->getIndependentParameters());
  initialized_ = true;
  fireParameterChanged(getParameters());
}

ParameterList RNonHomogeneousTreeLikelihood::getSubstitutionModelParameters() const {
  if (!initialized_) throw Exception("getSubstitutionModelParameters(). Object is not initialized.");
  return modelSet_->getParameters().getCommonParametersWith(getParameters());
}

void RNonHomogeneousTreeLikelihood::uploadModels() {
  for (size_t m = 0; m < modelSet_->getNumberOfModels(); m++) uploadEigen((int)m, *modelSet_->getModel(m));
  uploadRates();
  uploadRootFrequencies(modelSet_->getRootFrequencies());
}

void RNonHomogeneousTreeLikelihood::computeAllTransitionProbabilities() {
  for (size_t m = 0; m < modelSet_->getNumberOfModels(); m++) uploadEigen((int)m, *modelSet_->getModel(m));
  uploadRates();
  std::vector<const Node*> all(nodes_.begin(), nodes_.end());
  updatePmatrices(all);
  uploadRootFrequencies(modelSet_->getRootFrequencies());
}

// Likelihood/RNonHomogeneousTreeLikelihood.cpp:259-311: a rate-distribution change
// recomputes every P(t); otherwise the branches of the models whose parameters moved
// (getNodesWithParameter, through the aliases) get a new eigen-system and P(t), as do
// the branches whose length moved, and the root frequencies follow the model set.  Only
// the ancestors of those branches are re-traversed (the reference re-traverses everything).
void RNonHomogeneousTreeLikelihood::fireParameterChanged(const ParameterList&) {
  if (!initialized_) throw Exception("RNonHomogeneousTreeLikelihood::fireParameterChanged(). Object not initialized.");
  std::vector<const Node*> changed = applyBranchLengths();
  const bool setChanged = modelSet_->matchParametersValues(getParameters());
  const bool rateChanged = rateDistribution_->matchParametersValues(getParameters());
  if (allDirty_ || rateChanged) {
    allDirty_ = false;
    uploadModels();
    evaluateTree(std::vector<const Node*>(nodes_.begin(), nodes_.end()), false);
    return;
  }
  if (setChanged) {
    for (size_t m : modelSet_->getLastChangedModels()) {
      uploadEigen((int)m, *modelSet_->getModel(m));
      for (int id : modelSet_->getNodesWithModel(m)) {
        auto it = idToNode_.find(id);
        if (it != idToNode_.end() && std::find(changed.begin(), changed.end(), it->second) == changed.end())
          changed.push_back(it->second);
      }
    }
    if (modelSet_->getLastRootFrequenciesChanged()) uploadRootFrequencies(modelSet_->getRootFrequencies());
  }
  evaluateTree(changed, true);
}

}  // namespace bpp
