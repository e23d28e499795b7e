// Sequences (bpp-seq BasicSequence) as vectors of alphabet state codes.
#ifndef BPP_AMD_SEQUENCE_H
#define BPP_AMD_SEQUENCE_H

#include <string>
#include <vector>

#include "Alphabet/Alphabet.h"

namespace bpp {

class Sequence {
 protected:
  std::string name_;
  std::vector<int> content_;
  const Alphabet* alphabet_;

 public:
  Sequence(const std::string& name, const std::vector<int>& content, const Alphabet* alpha)
      : name_(name), content_(content), alphabet_(alpha) {}
  virtual ~Sequence() {}
  const std::string& getName() const { return name_; }
  const std::vector<int>& getContent() const { return content_; }
  size_t size() const { return content_.size(); }
  int getValue(size_t i) const { return content_[i]; }
  int operator[](size_t i) const { return content_[i]; }
  const Alphabet* getAlphabet() const { return alphabet_; }
  std::string toString() const {
    std::string s;
    for (int v : content_) s += alphabet_->intToChar(v);
    return s;
  }
};

class BasicSequence : public Sequence {
 public:
  BasicSequence(const std::string& name, const std::string& seq, const Alphabet* alpha)
      : Sequence(name, alpha->encode(seq), alpha) {}
  BasicSequence(const std::string& name, const std::vector<int>& content, const Alphabet* alpha)
      : Sequence(name, content, alpha) {}
};

}  // namespace bpp

#endif
