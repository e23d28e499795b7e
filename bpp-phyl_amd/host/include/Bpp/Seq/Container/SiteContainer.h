// Aligned sequence containers (bpp-seq SiteContainer / VectorSiteContainer subset).
#ifndef BPP_AMD_SITECONTAINER_H
#define BPP_AMD_SITECONTAINER_H

#include <map>
#include <string>
#include <vector>

#include "../Sequence.h"

namespace bpp {

class SiteContainer {
 public:
  virtual ~SiteContainer() {}
  virtual SiteContainer* clone() const = 0;
  virtual const Alphabet* getAlphabet() const = 0;
  virtual size_t getNumberOfSequences() const = 0;
  virtual size_t getNumberOfSites() const = 0;
  virtual std::vector<std::string> getSequencesNames() const = 0;
  virtual const Sequence& getSequence(const std::string& name) const = 0;
  virtual const Sequence& getSequence(size_t i) const = 0;
  virtual bool hasSequence(const std::string& name) const = 0;
  // state of sequence `seq` at site `site`
  int getState(size_t seq, size_t site) const { return getSequence(seq).getValue(site); }
};

class VectorSiteContainer : public SiteContainer {
  const Alphabet* alphabet_;
  std::vector<Sequence> seqs_;
  std::map<std::string, size_t> index_;

 public:
  explicit VectorSiteContainer(const Alphabet* alpha) : alphabet_(alpha) {}
  VectorSiteContainer* clone() const override { return new VectorSiteContainer(*this); }
  void addSequence(const Sequence& s, bool checkNames = true) {
    if (s.getAlphabet()->getAlphabetType() != alphabet_->getAlphabetType())
      throw AlphabetMismatchException("VectorSiteContainer::addSequence");
    if (!seqs_.empty() && s.size() != seqs_[0].size())
      throw Exception("VectorSiteContainer::addSequence: sequence '" + s.getName() + "' does not match the alignment length");
    if (checkNames && index_.count(s.getName())) throw Exception("VectorSiteContainer::addSequence: duplicate name " + s.getName());
    index_[s.getName()] = seqs_.size();
    seqs_.push_back(s);
  }
  const Alphabet* getAlphabet() const override { return alphabet_; }
  size_t getNumberOfSequences() const override { return seqs_.size(); }
  size_t getNumberOfSites() const override { return seqs_.empty() ? 0 : seqs_[0].size(); }
  std::vector<std::string> getSequencesNames() const override {
    std::vector<std::string> v;
    for (auto& s : seqs_) v.push_back(s.getName());
    return v;
  }
  const Sequence& getSequence(const std::string& name) const override {
    auto it = index_.find(name);
    if (it == index_.end()) throw SequenceNotFoundException("VectorSiteContainer::getSequence", name);
    return seqs_[it->second];
  }
  const Sequence& getSequence(size_t i) const override { return seqs_.at(i); }
  bool hasSequence(const std::string& name) const override { return index_.count(name) > 0; }
};

}  // namespace bpp

#endif
