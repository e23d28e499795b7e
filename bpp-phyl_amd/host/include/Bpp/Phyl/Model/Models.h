// Concrete models used by BASELINE.json's configurations: T92, GTR, LG08, YN98,
// plus the frequency sets the NH path needs.
#ifndef BPP_AMD_MODELS_H
#define BPP_AMD_MODELS_H

#include <memory>

#include "SubstitutionModel.h"

namespace bpp {

// T92 (Model/Nucleotide/T92.cpp:81-187, closed-form P(t) :355-386).
class T92 : public AbstractReversibleSubstitutionModel {
  double kappa_, theta_, k_, r_;

 public:
  T92(const NucleicAlphabet* alpha, double kappa = 1., double theta = 0.5);
  T92* clone() const override { return new T92(*this); }
  std::string getName() const override { return "T92"; }
  bool hasClosedFormPij() const override { return true; }
  void updateMatrices() override;
  const RowMatrix<double>& getPij_t(double d) const override;
  const RowMatrix<double>& getdPij_dt(double d) const override;
  const RowMatrix<double>& getd2Pij_dt2(double d) const override;
};

// GTR in the Bio++ parameterisation (Model/Nucleotide/GTR.cpp:84-124).
class GTR : public AbstractReversibleSubstitutionModel {
 public:
  GTR(const NucleicAlphabet* alpha, double a = 1., double b = 1., double c = 1., double d = 1., double e = 1.,
      double piA = 0.25, double piC = 0.25, double piG = 0.25, double piT = 0.25);
  GTR* clone() const override { return new GTR(*this); }
  std::string getName() const override { return "GTR"; }
  void updateMatrices() override;
};

// L95 (Lobry 1995) strand-symmetric, non-reversible nucleotide model
// (Model/Nucleotide/L95.cpp:56-119): generator from alpha, beta, gamma, kappa, theta,
// frequencies ((1-theta)/2, theta/2, theta/2, (1-theta)/2).  Its eigenvalues can be
// complex: P(t) then takes the block form (SubstitutionModel::getPij_t) on the host.
class L95 : public SubstitutionModel {
  double alpha_, beta_, gamma_, kappa_, theta_;

 public:
  L95(const NucleicAlphabet* alpha, double a = 0.5, double b = 0.5, double g = 0.5, double kappa = 1.,
      double theta = 0.5);
  L95* clone() const override { return new L95(*this); }
  std::string getName() const override { return "L95"; }
  void updateMatrices() override;
};

// LG08 empirical amino-acid model (Model/Protein/LG08.cpp:53-62), fixed frequencies.
class LG08 : public AbstractReversibleSubstitutionModel {
 public:
  explicit LG08(const ProteicAlphabet* alpha);
  LG08* clone() const override { return new LG08(*this); }
  std::string getName() const override { return "LG08"; }
  void updateMatrices() override;
};

// YN98 codon model on the 64-state codon alphabet (stop codons are null states):
// Q_ij = K80(kappa)_{n_i -> n_j} * (omega if non-synonymous) * pi_j for codons that
// differ at one position, 0 otherwise and for stop codons
// (Model/Codon/YN98.cpp:51-78, Model/AbstractWordSubstitutionModel.cpp:355-390,
// Model/Codon/AbstractCodonSubstitutionModel.cpp:174-190,
// Model/Codon/AbstractCodonDistanceSubstitutionModel.cpp:80-88).
class YN98 : public AbstractReversibleSubstitutionModel {
  const GeneticCode* gc_;
  Vdouble codonFreqs_;

 public:
  // codonFreqs: 64 values (stop codons are set to 0 and the rest renormalised);
  // empty = F3X4 with equal nucleotide frequencies.
  YN98(const GeneticCode* gc, const Vdouble& codonFreqs = Vdouble(), double kappa = 1., double omega = 1.);
  YN98* clone() const override { return new YN98(*this); }
  std::string getName() const override { return "YN98"; }
  void updateMatrices() override;
};

// Frequency sets (only what the NH configuration uses).
class FrequencySet : public AbstractParametrizable {
 protected:
  const Alphabet* alphabet_;
  Vdouble freq_;

 public:
  static const std::shared_ptr<IntervalConstraint> FREQUENCE_CONSTRAINT_SMALL;
  FrequencySet(const Alphabet* a, size_t n, const std::string& prefix)
      : AbstractParametrizable(prefix), alphabet_(a), freq_(n, 1. / n) {}
  virtual FrequencySet* clone() const = 0;
  const Vdouble& getFrequencies() const { return freq_; }
  const Alphabet* getAlphabet() const { return alphabet_; }
};

// GC frequency set: pi = ((1-theta)/2, theta/2, theta/2, (1-theta)/2)
// (Model/FrequencySet/NucleotideFrequencySet.h:66).
class GCFrequencySet : public FrequencySet {
 public:
  explicit GCFrequencySet(const NucleicAlphabet* alpha, double theta = 0.5);
  GCFrequencySet* clone() const override { return new GCFrequencySet(*this); }
  void fireParameterChanged(const ParameterList&) override;
};

class FixedFrequencySet : public FrequencySet {
 public:
  FixedFrequencySet(const Alphabet* alpha, const Vdouble& f) : FrequencySet(alpha, f.size(), "Fixed.") { freq_ = f; }
  FixedFrequencySet* clone() const override { return new FixedFrequencySet(*this); }
};

}  // namespace bpp

#endif
