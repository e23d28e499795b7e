// Trees for the likelihood classes: Node, Tree, TreeTemplate<Node>, TreeTemplateTools.
// Semantics follow the reference where the hot path depends on them:
//   - parenthesisToTree creates nodes recursively and resets ids to the postorder
//     index (TreeTemplateTools.cpp:335-354, TreeTemplateTools.h:354-361);
//   - getNodes() is postorder, sons before their father;
//   - unroot() merges the root's two branches into the non-leaf son
//     (TreeTemplate.h:244-300).
#ifndef BPP_AMD_TREETEMPLATE_H
#define BPP_AMD_TREETEMPLATE_H

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../Exceptions.h"

namespace bpp {

class Node {
  int id_ = 0;
  std::string name_;
  bool hasName_ = false;
  double distance_ = 0.;
  bool hasDistance_ = false;
  Node* father_ = nullptr;
  std::vector<Node*> sons_;

 public:
  Node() {}
  explicit Node(int id) : id_(id) {}
  Node(int id, const std::string& name) : id_(id), name_(name), hasName_(true) {}
  virtual ~Node() {}
  Node(const Node&) = delete;
  Node& operator=(const Node&) = delete;

  int getId() const { return id_; }
  void setId(int id) { id_ = id; }
  bool hasName() const { return hasName_; }
  const std::string& getName() const {
    if (!hasName_) throw NodeNotFoundException("Node::getName: node has no name", std::to_string(id_));
    return name_;
  }
  void setName(const std::string& n) {
    name_ = n;
    hasName_ = true;
  }
  bool hasDistanceToFather() const { return hasDistance_; }
  double getDistanceToFather() const {
    if (!hasDistance_) throw Exception("Node::getDistanceToFather: node " + std::to_string(id_) + " has no length");
    return distance_;
  }
  void setDistanceToFather(double d) {
    distance_ = d;
    hasDistance_ = true;
  }
  void deleteDistanceToFather() { hasDistance_ = false; }
  bool hasFather() const { return father_ != nullptr; }
  Node* getFather() { return father_; }
  const Node* getFather() const { return father_; }
  void setFather(Node* f) { father_ = f; }
  void removeFather() { father_ = nullptr; }
  size_t getNumberOfSons() const { return sons_.size(); }
  Node* getSon(size_t i) { return sons_.at(i); }
  const Node* getSon(size_t i) const { return sons_.at(i); }
  Node* operator[](int i) { return sons_.at((size_t)i); }
  const Node* operator[](int i) const { return sons_.at((size_t)i); }
  bool isLeaf() const { return sons_.empty(); }
  void addSon(Node* s) {
    sons_.push_back(s);
    s->father_ = this;
  }
  void removeSons() {
    for (Node* s : sons_) s->father_ = nullptr;
    sons_.clear();
  }
  void swap(size_t a, size_t b) { std::swap(sons_.at(a), sons_.at(b)); }
  std::vector<Node*>& sons() { return sons_; }
  const std::vector<Node*>& sons() const { return sons_; }
};

class Tree {
 public:
  virtual ~Tree() {}
  virtual Tree* clone() const = 0;
  virtual size_t getNumberOfLeaves() const = 0;
  virtual size_t getNumberOfNodes() const = 0;
  virtual std::vector<std::string> getLeavesNames() const = 0;
  virtual std::vector<int> getNodesId() const = 0;
  virtual bool isRooted() const = 0;
};

template <class N>
class TreeTemplate : public Tree {
  N* root_ = nullptr;

  static N* copySubtree(const N* n) {
    N* m = new N(n->getId());
    if (n->hasName()) m->setName(n->getName());
    if (n->hasDistanceToFather()) m->setDistanceToFather(n->getDistanceToFather());
    for (size_t i = 0; i < n->getNumberOfSons(); i++) m->addSon(copySubtree(n->getSon(i)));
    return m;
  }
  static void destroy(N* n) {
    if (!n) return;
    for (size_t i = 0; i < n->getNumberOfSons(); i++) destroy(n->getSon(i));
    delete n;
  }
  static void postorder(N* n, std::vector<N*>& out) {
    for (size_t i = 0; i < n->getNumberOfSons(); i++) postorder(n->getSon(i), out);
    out.push_back(n);
  }

 public:
  TreeTemplate() {}
  explicit TreeTemplate(N* root) : root_(root) {}
  TreeTemplate(const TreeTemplate& t) : root_(t.root_ ? copySubtree(t.root_) : nullptr) {}
  explicit TreeTemplate(const Tree& t) {
    const TreeTemplate* tt = dynamic_cast<const TreeTemplate*>(&t);
    if (!tt) throw Exception("TreeTemplate(const Tree&): unsupported tree implementation");
    root_ = tt->root_ ? copySubtree(tt->root_) : nullptr;
  }
  TreeTemplate& operator=(const TreeTemplate& t) {
    if (this != &t) {
      destroy(root_);
      root_ = t.root_ ? copySubtree(t.root_) : nullptr;
    }
    return *this;
  }
  ~TreeTemplate() override { destroy(root_); }
  TreeTemplate* clone() const override { return new TreeTemplate(*this); }

  N* getRootNode() { return root_; }
  const N* getRootNode() const { return root_; }
  void setRootNode(N* r) {
    root_ = r;
    if (r) r->removeFather();
  }
  std::vector<N*> getNodes() {
    std::vector<N*> v;
    if (root_) postorder(root_, v);
    return v;
  }
  std::vector<const N*> getNodes() const {
    std::vector<N*> v;
    if (root_) postorder(root_, v);
    return std::vector<const N*>(v.begin(), v.end());
  }
  std::vector<const N*> getLeaves() const {
    std::vector<const N*> out;
    for (const N* n : getNodes())
      if (n->isLeaf()) out.push_back(n);
    return out;
  }
  size_t getNumberOfLeaves() const override { return getLeaves().size(); }
  size_t getNumberOfNodes() const override { return getNodes().size(); }
  std::vector<std::string> getLeavesNames() const override {
    std::vector<std::string> v;
    for (const N* n : getLeaves()) v.push_back(n->getName());
    return v;
  }
  std::vector<int> getNodesId() const override {
    std::vector<int> v;
    for (const N* n : getNodes()) v.push_back(n->getId());
    return v;
  }
  N* getNode(int id) {
    for (N* n : getNodes())
      if (n->getId() == id) return n;
    throw NodeNotFoundException("TreeTemplate::getNode", std::to_string(id));
  }
  const N* getNode(int id) const {
    for (const N* n : getNodes())
      if (n->getId() == id) return n;
    throw NodeNotFoundException("TreeTemplate::getNode", std::to_string(id));
  }
  bool isRooted() const override { return root_ && root_->getNumberOfSons() == 2; }
  void resetNodesId() {
    std::vector<N*> nodes = getNodes();
    for (size_t i = 0; i < nodes.size(); i++) nodes[i]->setId((int)i);
  }
  // TreeTemplate.h:244-300 of the reference.
  bool unroot() {
    if (!isRooted()) throw UnrootedTreeException("Tree::unroot");
    N* son1 = root_->getSon(0);
    N* son2 = root_->getSon(1);
    if (son1->isLeaf() && son2->isLeaf()) return false;
    if (son1->isLeaf()) {
      root_->swap(0, 1);
      son1 = root_->getSon(0);
      son2 = root_->getSon(1);
    }
    if (son1->hasDistanceToFather()) {
      if (son2->hasDistanceToFather())
        son2->setDistanceToFather(son1->getDistanceToFather() + son2->getDistanceToFather());
      else
        son2->setDistanceToFather(son1->getDistanceToFather());
      son1->deleteDistanceToFather();
    }
    root_->removeSons();
    son1->addSon(son2);
    delete root_;
    setRootNode(son1);
    return true;
  }
  void scaleTree(double factor) {
    for (N* n : getNodes())
      if (n->hasDistanceToFather()) n->setDistanceToFather(n->getDistanceToFather() * factor);
  }
};

struct TreeTemplateTools {
  // Newick -> tree; ids reset to the postorder index.
  static TreeTemplate<Node>* parenthesisToTree(const std::string& description, bool bootstrap = true,
                                              const std::string& propertyName = "", bool withId = false,
                                              bool verbose = false);
  static std::string treeToParenthesis(const TreeTemplate<Node>& tree);
  // TreeTemplateTools.cpp:63-76: a node of more than two sons anywhere below `node`
  template <class N>
  static bool isMultifurcating(const N& node) {
    if (node.getNumberOfSons() > 2) return true;
    for (size_t i = 0; i < node.getNumberOfSons(); i++)
      if (isMultifurcating(*node.getSon(i))) return true;
    return false;
  }
  // TreeTemplateTools.cpp:173-186: the height of every node below `node` (the longest path
  // to a leaf); returns the height of `node`
  template <class N>
  static double getHeights(const N& node, std::map<const N*, double>& heights) {
    double d = 0.;
    for (size_t i = 0; i < node.getNumberOfSons(); i++) {
      const N* son = node.getSon(i);
      const double c = getHeights(*son, heights) + son->getDistanceToFather();
      if (c > d) d = c;
    }
    heights[&node] = d;
    return d;
  }
  template <class N>
  static std::vector<const N*> getLeaves(const N& node) {
    std::vector<const N*> out;
    collectLeaves(&node, out);
    return out;
  }

 private:
  template <class N>
  static void collectLeaves(const N* n, std::vector<const N*>& out) {
    if (n->isLeaf()) {
      out.push_back(n);
      return;
    }
    for (size_t i = 0; i < n->getNumberOfSons(); i++) collectLeaves(n->getSon(i), out);
  }
};

}  // namespace bpp

#endif
