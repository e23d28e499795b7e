// Alphabets with bpp-seq 12 state integers (the reference gets them from bpp-seq):
//   DNA      A C G T = 0..3, M R W S Y K V H D B N = 4..14, gap = -1
//   Protein  A R N D C Q E G H I L K M F P S T W Y V = 0..19, B Z J X = 20..23, gap = -1
//   Codon    16*n1 + 4*n2 + n3 over ACGT = 0..63 (stop codons included), NNN = 64, gap = -1
// getAlias(state) lists the resolved states a code stands for; the likelihood's leaf
// init is getInitValue(s, state) = [s in getAlias(state)]
// (Model/AbstractSubstitutionModel.cpp:98-112 in the reference).
#ifndef BPP_AMD_ALPHABET_H
#define BPP_AMD_ALPHABET_H

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../Exceptions.h"

namespace bpp {

class Alphabet {
 protected:
  std::vector<std::string> chars_;           // code -> character(s), codes 0..n-1
  std::vector<std::vector<int> > alias_;     // code -> resolved states
  std::map<std::string, int> lookup_;        // character(s) -> code (gap = -1)
  int size_;                                 // number of resolved states
  std::string type_;

 public:
  virtual ~Alphabet() {}
  int getSize() const { return size_; }
  unsigned int getNumberOfStates() const { return (unsigned int)size_; }
  int getNumberOfCodes() const { return (int)chars_.size(); }
  const std::string& getAlphabetType() const { return type_; }
  virtual unsigned int getStateCodingSize() const { return 1; }
  int getGapCharacterCode() const { return -1; }
  bool isIntInAlphabet(int state) const { return state >= -1 && state < (int)chars_.size(); }
  bool isCharInAlphabet(const std::string& c) const { return lookup_.count(c) > 0; }
  int charToInt(const std::string& c) const {
    auto it = lookup_.find(c);
    if (it == lookup_.end()) throw BadCharException(c, "Alphabet::charToInt: unknown character in " + type_);
    return it->second;
  }
  std::string intToChar(int state) const {
    if (state == -1) return "-";
    if (state < 0 || state >= (int)chars_.size()) throw BadIntException(state, "Alphabet::intToChar");
    return chars_[state];
  }
  std::vector<int> getAlias(int state) const {
    if (state < 0 || state >= (int)alias_.size()) throw BadIntException(state, "Alphabet::getAlias");
    return alias_[state];
  }
  bool isUnresolved(int state) const { return state >= size_; }
  int getUnknownCharacterCode() const { return (int)chars_.size() - 1; }
  // Encode a whole sequence string into state codes.
  std::vector<int> encode(const std::string& seq) const {
    std::vector<int> out;
    unsigned int w = getStateCodingSize();
    for (size_t i = 0; i + w <= seq.size(); i += w) {
      std::string c = seq.substr(i, w);
      for (auto& ch : c) ch = (char)toupper((unsigned char)ch);
      out.push_back(charToInt(c));
    }
    return out;
  }
};

class NucleicAlphabet : public Alphabet {
 public:
  NucleicAlphabet() {
    type_ = "DNA alphabet";
    size_ = 4;
    const char* codes = "ACGTMRWSYKVHDBN";
    const char* sets[] = {"A", "C", "G", "T", "AC", "AG", "AT", "CG", "CT", "GT", "ACG", "ACT", "AGT", "CGT", "ACGT"};
    for (int i = 0; i < 15; i++) {
      chars_.push_back(std::string(1, codes[i]));
      lookup_[chars_.back()] = i;
      std::vector<int> a;
      for (const char* p = sets[i]; *p; ++p) a.push_back((int)std::string("ACGT").find(*p));
      alias_.push_back(a);
    }
    lookup_["U"] = 3;
    lookup_["X"] = lookup_["O"] = lookup_["0"] = lookup_["?"] = 14;
    lookup_["-"] = lookup_["."] = -1;
  }
};

class DNA : public NucleicAlphabet {};

class ProteicAlphabet : public Alphabet {
 public:
  ProteicAlphabet() {
    type_ = "Proteic alphabet";
    size_ = 20;
    const std::string aa = "ARNDCQEGHILKMFPSTWYV";
    for (int i = 0; i < 20; i++) {
      chars_.push_back(aa.substr(i, 1));
      lookup_[chars_.back()] = i;
      alias_.push_back(std::vector<int>(1, i));
    }
    const char* extra = "BZJX";
    const char* sets[] = {"ND", "QE", "IL", "ARNDCQEGHILKMFPSTWYV"};
    for (int k = 0; k < 4; k++) {
      chars_.push_back(std::string(1, extra[k]));
      lookup_[chars_.back()] = 20 + k;
      std::vector<int> a;
      for (const char* p = sets[k]; *p; ++p) a.push_back((int)aa.find(*p));
      alias_.push_back(a);
    }
    lookup_["?"] = 23;
    lookup_["-"] = lookup_["."] = lookup_["*"] = -1;
  }
};

class CodonAlphabet : public Alphabet {
  const NucleicAlphabet* nuc_;

 public:
  explicit CodonAlphabet(const NucleicAlphabet* nuc) : nuc_(nuc) {
    type_ = "Codon alphabet";
    size_ = 64;
    const std::string n = "ACGT";
    for (int i = 0; i < 64; i++) {
      chars_.push_back(std::string() + n[i / 16] + n[(i / 4) % 4] + n[i % 4]);
      lookup_[chars_.back()] = i;
      alias_.push_back(std::vector<int>(1, i));
    }
    chars_.push_back("NNN");
    lookup_["NNN"] = 64;
    std::vector<int> all;
    for (int i = 0; i < 64; i++) all.push_back(i);
    alias_.push_back(all);
    lookup_["---"] = -1;
  }
  unsigned int getStateCodingSize() const override { return 3; }
  const NucleicAlphabet* getNucleicAlphabet() const { return nuc_; }
  int getNPosition(int codon, size_t pos) const {
    return pos == 0 ? codon / 16 : (pos == 1 ? (codon / 4) % 4 : codon % 4);
  }
};

// NCBI standard genetic code over the 64-codon alphabet.
class GeneticCode {
 protected:
  std::shared_ptr<CodonAlphabet> owned_;
  const CodonAlphabet* codonAlphabet_;
  std::string aa_;  // amino acid letter per codon, '*' for stops

 public:
  GeneticCode(const CodonAlphabet* ca, const std::string& aa) : codonAlphabet_(ca), aa_(aa) {}
  virtual ~GeneticCode() {}
  const CodonAlphabet* getSourceAlphabet() const { return codonAlphabet_; }
  bool isStop(int codon) const { return aa_[codon] == '*'; }
  char translate(int codon) const { return aa_[codon]; }
  bool areSynonymous(int i, int j) const { return aa_[i] == aa_[j]; }
};

class StandardGeneticCode : public GeneticCode {
 public:
  explicit StandardGeneticCode(const NucleicAlphabet* nuc)
      : GeneticCode(nullptr, "KNKNTTTTRSRSIIMIQHQHPPPPRRRRLLLLEDEDAAAAGGGGVVVV*Y*YSSSS*CWCLFLF") {
    owned_ = std::make_shared<CodonAlphabet>(nuc);
    codonAlphabet_ = owned_.get();
  }
  explicit StandardGeneticCode(const CodonAlphabet* ca)
      : GeneticCode(ca, "KNKNTTTTRSRSIIMIQHQHPPPPRRRRLLLLEDEDAAAAGGGGVVVV*Y*YSSSS*CWCLFLF") {}
};

struct AlphabetTools {
  static const DNA DNA_ALPHABET;
  static const ProteicAlphabet PROTEIN_ALPHABET;
  static bool isNucleicAlphabet(const Alphabet* a) { return a->getAlphabetType() == "DNA alphabet"; }
  static bool isProteicAlphabet(const Alphabet* a) { return a->getAlphabetType() == "Proteic alphabet"; }
  static bool isCodonAlphabet(const Alphabet* a) { return a->getAlphabetType() == "Codon alphabet"; }
};

}  // namespace bpp

#endif
