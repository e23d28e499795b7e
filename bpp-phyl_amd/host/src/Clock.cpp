// Host mirror: RHomogeneousClockTreeLikelihood (see its header).  Only the parametrisation
// differs from RHomogeneousTreeLikelihood: the node heights are the parameters and the
// branch lengths derived from them feed the same device evaluation.
#include "Bpp/Phyl/Likelihood/RHomogeneousClockTreeLikelihood.h"

#include <algorithm>
#include <map>

namespace bpp {

RHomogeneousClockTreeLikelihood::RHomogeneousClockTreeLikelihood(const Tree& tree, SubstitutionModel* model,
                                                                 DiscreteDistribution* rDist, bool, bool verbose)
    : RHomogeneousTreeLikelihood(tree, model, rDist, false, verbose, true) {
  init_();
}

RHomogeneousClockTreeLikelihood::RHomogeneousClockTreeLikelihood(const Tree& tree, const SiteContainer& data,
                                                                 SubstitutionModel* model, DiscreteDistribution* rDist,
                                                                 bool, bool verbose)
    : RHomogeneousTreeLikelihood(tree, data, model, rDist, false, verbose, true) {
  init_();
}

void RHomogeneousClockTreeLikelihood::init_() {
  if (!tree_->isRooted()) throw Exception("RHomogeneousClockTreeLikelihood::init_(). Tree is unrooted!");
  if (TreeTemplateTools::isMultifurcating(*tree_->getRootNode()))
    throw Exception("HomogeneousClockTreeLikelihood::init_(). Tree is multifurcating.");
  setMinimumBranchLength(0.);
}

// RHomogeneousClockTreeLikelihood.cpp:110-145: missing or too short branches are set to the
// minimum, then TotalHeight = h(root) and HeightP<id> = h(v) / h(father(v)) per internal
// non-root node, in postorder
void RHomogeneousClockTreeLikelihood::initBranchLengthsParameters() {
  for (size_t i = 0; i < nodes_.size(); i++) {
    Node* n = nodes_[i];
    if (!n->hasDistanceToFather()) {
      if (verbose_)
        ApplicationTools::displayWarning("Missing branch length " + TextTools::toString(i) + ". Value is set to " +
                                         TextTools::toString(minimumBrLen_));
      n->setDistanceToFather(minimumBrLen_);
    } else if (n->getDistanceToFather() < minimumBrLen_) {
      if (verbose_)
        ApplicationTools::displayWarning("Branch length " + TextTools::toString(i) + " is too small: " +
                                         TextTools::toString(n->getDistanceToFather()) + ". Value is set to " +
                                         TextTools::toString(minimumBrLen_));
      n->setDistanceToFather(minimumBrLen_);
    }
  }
  brLenParameters_.reset();
  std::map<const Node*, double> heights;
  const Node* root = tree_->getRootNode();
  TreeTemplateTools::getHeights(*root, heights);
  brLenParameters_.addParameter(Parameter("TotalHeight", heights[root], brLenConstraint_));
  heightNames_.clear();
  for (size_t i = 0; i < nodes_.size(); i++) {
    const Node* n = nodes_[i];
    if (n->isLeaf()) continue;
    const std::string& name = heightNames_[n] = "HeightP" + TextTools::toString(n->getId());
    brLenParameters_.addParameter(
        Parameter(name, heights[n] / heights[n->getFather()], Parameter::PROP_CONSTRAINT_IN));
  }
}

// RHomogeneousClockTreeLikelihood.cpp:150-168: a leaf son hangs at height 0, an internal
// son at HeightP * height; lengths below the minimum are raised to it
void RHomogeneousClockTreeLikelihood::branchLengthsFromHeights(Node* node, double height,
                                                               std::vector<const Node*>& changed) {
  for (size_t k = 0; k < node->getNumberOfSons(); k++) {
    Node* son = node->getSon(k);
    double len, sonHeight = 0.;
    if (son->isLeaf()) {
      len = std::max(minimumBrLen_, height);
    } else {
      sonHeight = parameters_.getParameterValue(heightNames_.at(son)) * height;
      len = std::max(minimumBrLen_, height - sonHeight);
    }
    if (!son->hasDistanceToFather() || son->getDistanceToFather() != len) {
      son->setDistanceToFather(len);
      changed.push_back(son);
    }
    if (!son->isLeaf()) branchLengthsFromHeights(son, sonHeight, changed);
  }
}

// RHomogeneousClockTreeLikelihood::applyParameters (:96-108) for the branch lengths
std::vector<const Node*> RHomogeneousClockTreeLikelihood::applyBranchLengths() {
  std::vector<const Node*> changed;
  branchLengthsFromHeights(tree_->getRootNode(), parameters_.getParameterValue("TotalHeight"), changed);
  return changed;
}

ParameterList RHomogeneousClockTreeLikelihood::getDerivableParameters() const {
  if (!initialized_)
    throw Exception("RHomogeneousClockTreeLikelihood::getDerivableParameters(). Object is not initialized.");
  return ParameterList();
}

ParameterList RHomogeneousClockTreeLikelihood::getNonDerivableParameters() const {
  if (!initialized_)
    throw Exception("RHomogeneousClockTreeLikelihood::getNonDerivableParameters(). Object is not initialized.");
  return getParameters();
}

double RHomogeneousClockTreeLikelihood::getFirstOrderDerivative(const std::string&) const {
  throw Exception("No first order derivative is implemented for this function.");
}

double RHomogeneousClockTreeLikelihood::getSecondOrderDerivative(const std::string&) const {
  throw Exception("No second order derivative is implemented for this function.");
}

}  // namespace bpp
