// Parameters, constraints and parameter lists with bpp-core 2.4 semantics, as far
// as the likelihood classes and their callers use them.
#ifndef BPP_AMD_PARAMETER_H
#define BPP_AMD_PARAMETER_H

#include <cmath>
#include <iostream>
#include <limits>
#include <memory>
#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>

#include "../Exceptions.h"

namespace bpp {

class Constraint {
 public:
  virtual ~Constraint() {}
  virtual Constraint* clone() const = 0;
  virtual bool isCorrect(double value) const = 0;
  virtual double getAcceptedLimit(double value) const = 0;
  virtual double getLowerBound() const = 0;
  virtual double getUpperBound() const = 0;
  virtual bool strictLowerBound() const = 0;
  virtual bool strictUpperBound() const = 0;
};

class IntervalConstraint : public Constraint {
  double lower_, upper_;
  bool inclLower_, inclUpper_;
  double precision_;

 public:
  IntervalConstraint(double lower, double upper, bool inclLower, bool inclUpper, double precision = 1e-7)
      : lower_(lower), upper_(upper), inclLower_(inclLower), inclUpper_(inclUpper), precision_(precision) {}
  IntervalConstraint* clone() const override { return new IntervalConstraint(*this); }
  bool isCorrect(double v) const override {
    bool lo = inclLower_ ? v >= lower_ : v > lower_;
    bool hi = inclUpper_ ? v <= upper_ : v < upper_;
    return lo && hi;
  }
  double getAcceptedLimit(double v) const override {
    if (!(inclLower_ ? v >= lower_ : v > lower_)) return inclLower_ ? lower_ : lower_ + precision_;
    if (!(inclUpper_ ? v <= upper_ : v < upper_)) return inclUpper_ ? upper_ : upper_ - precision_;
    return v;
  }
  double getLowerBound() const override { return lower_; }
  double getUpperBound() const override { return upper_; }
  bool strictLowerBound() const override { return !inclLower_; }
  bool strictUpperBound() const override { return !inclUpper_; }
};

class Parameter {
  std::string name_;
  double value_;
  std::shared_ptr<Constraint> constraint_;

 public:
  static const std::shared_ptr<IntervalConstraint> R_PLUS;
  static const std::shared_ptr<IntervalConstraint> R_PLUS_STAR;
  static const std::shared_ptr<IntervalConstraint> PROP_CONSTRAINT_IN;
  static const std::shared_ptr<IntervalConstraint> PROP_CONSTRAINT_EX;

  Parameter() : name_(), value_(0.), constraint_() {}
  Parameter(const std::string& name, double value, std::shared_ptr<Constraint> c = nullptr)
      : name_(name), value_(value), constraint_(c) {
    if (constraint_ && !constraint_->isCorrect(value))
      throw ConstraintException("Parameter::Parameter: value out of constraint", name, value);
  }
  const std::string& getName() const { return name_; }
  void setName(const std::string& n) { name_ = n; }
  double getValue() const { return value_; }
  void setValue(double v) {
    if (constraint_ && !constraint_->isCorrect(v))
      throw ConstraintException("Parameter::setValue", name_, v);
    value_ = v;
  }
  bool hasConstraint() const { return (bool)constraint_; }
  std::shared_ptr<Constraint> getConstraint() const { return constraint_; }
  void setConstraint(std::shared_ptr<Constraint> c) { constraint_ = c; }
};

// An ordered list of parameters.  Name lookups go through a name -> position index that
// is rebuilt lazily whenever the list changed (or a parameter was renamed through
// operator[]), so the optimisers' per-evaluation setParameters of every parameter costs
// O(n), not O(n^2) string comparisons; a position hint (lists that share an order, the
// usual case: a sublist handed back to the object it came from) skips the hash.
class ParameterList {
  std::vector<Parameter> params_;
  mutable std::unordered_map<std::string, size_t> index_;
  mutable bool indexValid_ = false;

  long find(const std::string& name) const {
    if (!indexValid_ || index_.size() != params_.size()) rebuild();
    auto it = index_.find(name);
    if (it == index_.end()) return -1;
    if (params_[it->second].getName() != name) {  // renamed through operator[]
      rebuild();
      it = index_.find(name);
      return it == index_.end() ? -1 : (long)it->second;
    }
    return (long)it->second;
  }
  long find(const std::string& name, size_t hint) const {
    if (hint < params_.size() && params_[hint].getName() == name) return (long)hint;
    return find(name);
  }
  void rebuild() const {
    index_.clear();
    for (size_t i = 0; i < params_.size(); i++) index_.emplace(params_[i].getName(), i);  // first wins
    indexValid_ = true;
  }

 public:
  size_t size() const { return params_.size(); }
  const Parameter& operator[](size_t i) const { return params_[i]; }
  Parameter& operator[](size_t i) {
    indexValid_ = false;  // the caller may rename it
    return params_[i];
  }
  std::vector<std::string> getParameterNames() const {
    std::vector<std::string> v;
    for (auto& p : params_) v.push_back(p.getName());
    return v;
  }
  bool hasParameter(const std::string& name) const { return find(name) >= 0; }
  // position of `name` (-1: absent), trying position `hint` first (not in the reference API)
  long indexOf(const std::string& name, size_t hint = (size_t)-1) const { return find(name, hint); }
  size_t whichParameterHasName(const std::string& name) const {
    const long i = find(name);
    if (i < 0) throw ParameterNotFoundException("ParameterList::whichParameterHasName", name);
    return (size_t)i;
  }
  const Parameter& getParameter(const std::string& name) const { return params_[whichParameterHasName(name)]; }
  double getParameterValue(const std::string& name) const { return getParameter(name).getValue(); }
  void addParameter(const Parameter& p) {
    if (hasParameter(p.getName())) throw Exception("ParameterList::addParameter: duplicate " + p.getName());
    params_.push_back(p);
    index_.emplace(p.getName(), params_.size() - 1);
  }
  void addParameters(const ParameterList& pl) {
    for (size_t i = 0; i < pl.size(); i++) addParameter(pl[i]);
  }
  void includeParameters(const ParameterList& pl) {
    for (size_t i = 0; i < pl.size(); i++) {
      const long k = find(pl[i].getName());
      if (k >= 0)
        params_[(size_t)k].setValue(pl[i].getValue());
      else
        addParameter(pl[i]);
    }
  }
  void setParameterValue(const std::string& name, double v) { params_[whichParameterHasName(name)].setValue(v); }
  // Update values of parameters present in both lists; returns true if any changed.
  // `changed` receives the positions that changed (each once).  A much longer `pl` (a
  // model's few parameters matched against a likelihood's whole list) is probed by this
  // list's names instead of walking all of it.
  bool matchParametersValues(const ParameterList& pl, std::vector<size_t>* changed = nullptr) {
    bool any = false;
    std::vector<char> seen;
    auto set = [&](size_t i, double v) {
      Parameter& p = params_[i];
      if (p.getValue() == v) return;
      p.setValue(v);
      any = true;
      if (changed) {
        if (seen.empty()) seen.assign(params_.size(), 0);
        if (!seen[i]) changed->push_back(i);
        seen[i] = 1;
      }
    };
    if (pl.size() > 2 * params_.size()) {
      for (size_t i = 0; i < params_.size(); i++) {
        const long j = pl.find(params_[i].getName());
        if (j >= 0) set(i, pl.params_[(size_t)j].getValue());
      }
      return any;
    }
    size_t hint = 0;
    for (size_t j = 0; j < pl.size(); j++) {
      const long i = find(pl.params_[j].getName(), hint);
      if (i < 0) continue;
      hint = (size_t)i + 1;
      set((size_t)i, pl.params_[j].getValue());
    }
    return any;
  }
  ParameterList getCommonParametersWith(const ParameterList& pl) const {
    ParameterList out;
    for (auto& p : params_)
      if (pl.hasParameter(p.getName())) out.addParameter(p);
    return out;
  }
  ParameterList createSubList(const std::vector<std::string>& names) const {
    ParameterList out;
    for (auto& n : names) out.params_.push_back(getParameter(n));
    return out;
  }
  void deleteParameter(const std::string& name) {
    params_.erase(params_.begin() + whichParameterHasName(name));
    indexValid_ = false;
  }
  void reset() {
    params_.clear();
    index_.clear();
    indexValid_ = true;
  }
  void printParameters(std::ostream& out) const {
    for (auto& p : params_) out << p.getName() << "=" << p.getValue() << std::endl;
  }
};

// Parametrizable objects with a namespace prefix ("T92.", "GTR.", ...).
class Parametrizable {
 public:
  virtual ~Parametrizable() {}
  virtual const ParameterList& getParameters() const = 0;
  virtual bool matchParametersValues(const ParameterList& pl) = 0;
};

class AbstractParametrizable : public virtual Parametrizable {
 protected:
  ParameterList parameters_;
  std::string prefix_;

 public:
  explicit AbstractParametrizable(const std::string& prefix = "") : parameters_(), prefix_(prefix) {}
  virtual ~AbstractParametrizable() {}
  const ParameterList& getParameters() const override { return parameters_; }
  virtual ParameterList getIndependentParameters() const { return parameters_; }
  const std::string& getNamespace() const { return prefix_; }
  virtual void setNamespace(const std::string& prefix) {
    for (size_t i = 0; i < parameters_.size(); i++) {
      std::string n = parameters_[i].getName();
      if (n.compare(0, prefix_.size(), prefix_) == 0) n = n.substr(prefix_.size());
      parameters_[i].setName(prefix + n);
    }
    prefix_ = prefix;
  }
  std::string getParameterNameWithoutNamespace(const std::string& name) const {
    if (name.compare(0, prefix_.size(), prefix_) == 0) return name.substr(prefix_.size());
    return name;
  }
  bool hasParameter(const std::string& name) const { return parameters_.hasParameter(prefix_ + name); }
  const Parameter& getParameter(const std::string& name) const { return parameters_.getParameter(prefix_ + name); }
  double getParameterValue(const std::string& name) const { return parameters_.getParameterValue(prefix_ + name); }
  virtual void setParameterValue(const std::string& name, double v) {
    ParameterList pl;
    Parameter p = parameters_.getParameter(prefix_ + name);
    p.setValue(v);
    pl.addParameter(p);
    matchParametersValues(pl);
  }
  bool matchParametersValues(const ParameterList& pl) override {
    std::vector<size_t> changed;
    bool any = parameters_.matchParametersValues(pl, &changed);
    if (any) {
      ParameterList ch;
      for (size_t i : changed) ch.addParameter(parameters_[i]);
      fireParameterChanged(ch);
    }
    return any;
  }
  virtual void setParametersValues(const ParameterList& pl) {
    parameters_.matchParametersValues(pl);
    fireParameterChanged(pl);
  }
  virtual void fireParameterChanged(const ParameterList&) {}

 protected:
  void addParameter_(const Parameter& p) { parameters_.addParameter(p); }
  void addParameters_(const ParameterList& pl) { parameters_.addParameters(pl); }
  void resetParameters_() { parameters_.reset(); }
};

}  // namespace bpp

#endif
