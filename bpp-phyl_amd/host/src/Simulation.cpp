// Host mirror: NonHomogeneousSequenceSimulator (see the header).
#include "Bpp/Phyl/Simulation/NonHomogeneousSequenceSimulator.h"

#include "Bpp/Numeric/Random/RandomTools.h"
#include "Bpp/Phyl/Model/SubstitutionModelSet.h"

namespace bpp {

NonHomogeneousSequenceSimulator::NonHomogeneousSequenceSimulator(const SubstitutionModelSet* modelSet,
                                                                 const DiscreteDistribution* rate, const Tree* tree)
    : modelSet_(modelSet), alphabet_(modelSet ? modelSet->getAlphabet() : nullptr), rate_(rate) {
  if (!modelSet || !rate || !tree) throw NullPointerException("NonHomogeneousSequenceSimulator: null argument");
  const TreeTemplate<Node>* tt = dynamic_cast<const TreeTemplate<Node>*>(tree);
  if (!tt) throw Exception("NonHomogeneousSequenceSimulator: unsupported tree implementation");
  if (!modelSet->isFullySetUpFor(*tree))
    throw Exception("NonHomogeneousSequenceSimulator(constructor). Model set is not fully specified.");
  tree_.reset(new TreeTemplate<Node>(*tt));
  init();
}

NonHomogeneousSequenceSimulator::NonHomogeneousSequenceSimulator(const SubstitutionModel* model,
                                                                 const DiscreteDistribution* rate, const Tree* tree)
    : modelSet_(nullptr), alphabet_(model ? model->getAlphabet() : nullptr), rate_(rate) {
  if (!model || !rate || !tree) throw NullPointerException("NonHomogeneousSequenceSimulator: null argument");
  const TreeTemplate<Node>* tt = dynamic_cast<const TreeTemplate<Node>*>(tree);
  if (!tt) throw Exception("NonHomogeneousSequenceSimulator: unsupported tree implementation");
  FixedFrequencySet* f = new FixedFrequencySet(model->getAlphabet(), model->getFrequencies());
  f->setNamespace("anc.");
  ownModelSet_.reset(SubstitutionModelSetTools::createHomogeneousModelSet(model->clone(), f, tt));
  modelSet_ = ownModelSet_.get();
  tree_.reset(new TreeTemplate<Node>(*tt));
  init();
}

// :110-160: cumulative P(t . r_c) rows per branch and class
void NonHomogeneousSequenceSimulator::init() {
  nbClasses_ = rate_->getNumberOfCategories();
  nbStates_ = modelSet_->getNumberOfStates();
  leaves_.clear();
  for (const Node* n : tree_->getNodes())
    if (n->isLeaf()) leaves_.push_back(n);
  outputInternalSequences(outputInternalSequences_);
  cumpxy_.clear();
  for (const Node* n : tree_->getNodes()) {
    if (n == tree_->getRootNode()) continue;
    const SubstitutionModel* m = modelSet_->getModelForNode(n->getId());
    const double d = n->getDistanceToFather();
    VVVdouble& cum = cumpxy_[n->getId()];
    cum.assign(nbClasses_, VVdouble(nbStates_, Vdouble(nbStates_)));
    for (size_t c = 0; c < nbClasses_; c++) {
      const RowMatrix<double>& P = m->getPij_t(d * rate_->getCategory(c));
      for (size_t x = 0; x < nbStates_; x++) {
        cum[c][x][0] = P(x, 0);
        for (size_t y = 1; y < nbStates_; y++) cum[c][x][y] = cum[c][x][y - 1] + P(x, y);
      }
    }
  }
}

void NonHomogeneousSequenceSimulator::outputInternalSequences(bool yn) {
  outputInternalSequences_ = yn;
  seqNames_.clear();
  if (yn) {
    for (const Node* n : tree_->getNodes())
      seqNames_.push_back(n->isLeaf() ? n->getName() : std::to_string(n->getId()));
  } else {
    for (const Node* n : leaves_) seqNames_.push_back(n->getName());
  }
}

// :306-353: root states from the root frequencies (first state whose cumulative
// probability reaches r), then one rate class per site
SiteContainer* NonHomogeneousSequenceSimulator::simulate(size_t numberOfSites) const {
  const Vdouble freqs = modelSet_->getRootFrequencies();
  std::vector<size_t> root(numberOfSites, 0);
  for (size_t j = 0; j < numberOfSites; j++) {
    const double r = RandomTools::giveRandomNumberBetweenZeroAndEntry(1.);
    double cum = 0.;
    for (size_t i = 0; i < nbStates_; i++) {
      cum += freqs[i];
      if (r <= cum) {
        root[j] = i;
        break;
      }
    }
  }
  std::vector<size_t> classes(numberOfSites);
  for (size_t j = 0; j < numberOfSites; j++)
    classes[j] = RandomTools::giveIntRandomNumberBetweenZeroAndEntry<size_t>(nbClasses_);
  return multipleEvolve(root, classes);
}

// :463-483, 519-534: every site's child state from the cumulative row of its class and
// parent state, branches in preorder
void NonHomogeneousSequenceSimulator::multipleEvolve(const Node* node, const std::vector<size_t>& rateClasses,
                                                     std::map<int, std::vector<size_t> >& states) const {
  const std::vector<size_t>& in = states.at(node->getFather()->getId());
  std::vector<size_t>& out = states[node->getId()];
  out.assign(in.size(), 0);
  const VVVdouble& cum = cumpxy_.at(node->getId());
  for (size_t i = 0; i < in.size(); i++) {
    const Vdouble& row = cum[rateClasses[i]][in[i]];
    const double r = RandomTools::giveRandomNumberBetweenZeroAndEntry(1.);
    for (size_t y = 0; y < nbStates_; y++)
      if (r < row[y]) {
        out[i] = y;
        break;
      }
  }
  for (size_t k = 0; k < node->getNumberOfSons(); k++) multipleEvolve(node->getSon(k), rateClasses, states);
}

SiteContainer* NonHomogeneousSequenceSimulator::multipleEvolve(const std::vector<size_t>& initialStateIndices,
                                                               const std::vector<size_t>& rateClasses) const {
  if (rateClasses.size() != initialStateIndices.size())
    throw Exception("NonHomogeneousSequenceSimulator::multipleEvolve: one rate class per site is needed");
  std::map<int, std::vector<size_t> > states;
  const Node* root = tree_->getRootNode();
  states[root->getId()] = initialStateIndices;
  for (size_t k = 0; k < root->getNumberOfSons(); k++) multipleEvolve(root->getSon(k), rateClasses, states);
  VectorSiteContainer* sites = new VectorSiteContainer(alphabet_);
  std::vector<const Node*> out;
  if (outputInternalSequences_) {
    for (const Node* n : tree_->getNodes()) out.push_back(n);
  } else {
    out = leaves_;
  }
  for (size_t i = 0; i < out.size(); i++) {
    const std::vector<size_t>& s = states.at(out[i]->getId());
    std::vector<int> content(s.begin(), s.end());
    sites->addSequence(BasicSequence(seqNames_[i], content, alphabet_));
  }
  return sites;
}

}  // namespace bpp
