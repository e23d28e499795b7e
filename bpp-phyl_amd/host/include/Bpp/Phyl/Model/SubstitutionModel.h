// Substitution models of the host mirror.  Interface after the reference's
// SubstitutionModel (Model/SubstitutionModel.h:122-602): generator, frequencies,
// eigen-system (getEigenValues / getRowLeftEigenVectors = V^-1 /
// getColumnRightEigenVectors = V, :498-525), getPij_t & derivatives (:233-247),
// getInitValue (:277).  The likelihood classes hand the eigen-system (or, for
// closed-form models, P(t) itself) to libplk, which builds every branch's
// transition matrices on the GPU.
#ifndef BPP_AMD_SUBSTITUTIONMODEL_H
#define BPP_AMD_SUBSTITUTIONMODEL_H

#include <memory>
#include <string>
#include <vector>

#include "../../Numeric/Matrix/Matrix.h"
#include "../../Numeric/NumConstants.h"
#include "../../Numeric/Parameter.h"
#include "../../Numeric/VectorTools.h"
#include "../../Text/TextTools.h"
#include "../../Seq/Alphabet/Alphabet.h"

namespace bpp {

class FrequencySet;

class SubstitutionModel : public AbstractParametrizable {
 protected:
  const Alphabet* alphabet_;
  size_t size_;
  double rate_ = 1.;
  RowMatrix<double> generator_;
  RowMatrix<double> exchangeability_;
  Vdouble freq_;
  Vdouble eigenValues_;
  Vdouble iEigenValues_;                 // imaginary parts (complex pairs: +b, -b)
  RowMatrix<double> leftEigenVectors_;   // V^-1 (rows)
  RowMatrix<double> rightEigenVectors_;  // V (columns)
  bool isDiagonalizable_ = true;
  bool isNonSingular_ = true;
  bool isScalable_ = true;
  mutable RowMatrix<double> pijt_, dpijt_, d2pijt_;
  // powers of the generator for the Taylor branch of getPij_t (singular eigenvectors,
  // Model/AbstractSubstitutionModel.cpp:386-418, 470-492)
  std::vector<RowMatrix<double> > vPowGen_;
  // after the eigen-decomposition: V Lambda V^-1 must give Q back and V V^-1 = I
  // (the reference's isDiagonalizable / isNonSingular checks, :277-330); else Taylor
  void checkEigen();

 public:
  SubstitutionModel(const Alphabet* alpha, size_t size, const std::string& prefix)
      : AbstractParametrizable(prefix), alphabet_(alpha), size_(size), generator_(size, size),
        exchangeability_(size, size), freq_(size, 1. / size), eigenValues_(size, 0.),
        iEigenValues_(size, 0.), leftEigenVectors_(size, size), rightEigenVectors_(size, size), pijt_(size, size), dpijt_(size, size),
        d2pijt_(size, size) {}
  virtual ~SubstitutionModel() {}
  virtual SubstitutionModel* clone() const = 0;
  virtual std::string getName() const = 0;

  const Alphabet* getAlphabet() const { return alphabet_; }
  size_t getNumberOfStates() const { return size_; }
  const Vdouble& getFrequencies() const { return freq_; }
  double freq(size_t i) const { return freq_[i]; }
  const RowMatrix<double>& getGenerator() const { return generator_; }
  const RowMatrix<double>& getExchangeabilityMatrix() const { return exchangeability_; }
  const Vdouble& getEigenValues() const { return eigenValues_; }
  const Vdouble& getIEigenValues() const { return iEigenValues_; }
  const RowMatrix<double>& getRowLeftEigenVectors() const { return leftEigenVectors_; }
  const RowMatrix<double>& getColumnRightEigenVectors() const { return rightEigenVectors_; }
  bool isDiagonalizable() const { return isDiagonalizable_; }
  bool isNonSingular() const { return isNonSingular_; }
  // P(t) from the host (plk_set_pmatrix) instead of the device's real V e^{lambda t} V^-1:
  // the Taylor branch, and complex eigenvalue pairs (the block form of getPij_t)
  bool needsHostPij() const { return !isNonSingular_ || !isDiagonalizable_; }
  double getRate() const { return rate_; }
  void setRate(double r) { rate_ = r; }
  bool isScalable() const { return isScalable_; }
  void setScalable(bool s) { isScalable_ = s; }
  int getAlphabetStateAsInt(size_t i) const { return (int)i; }

  // Closed-form models (T92) expose P(t) directly; the likelihood then hands the
  // host-computed matrices to the engine with plk_set_pmatrix.
  virtual bool hasClosedFormPij() const { return false; }

  // P(t) = V diag(exp(lambda rate t)) V^-1 (Model/AbstractSubstitutionModel.cpp:426-438);
  // complex pairs a +- ib: V B V^-1 with 2x2 blocks e^{a r t} [[cos, sin], [-sin, cos]](b r t)
  // (:440-467), and the derivatives' blocks (:505-537, :581-611)
  virtual const RowMatrix<double>& getPij_t(double t) const;
  virtual const RowMatrix<double>& getdPij_dt(double t) const;
  virtual const RowMatrix<double>& getd2Pij_dt2(double t) const;
  // for tests: replace the eigen-system as a failed decomposition would leave it
  void forceTaylorForTests() {
    isNonSingular_ = false;
    isDiagonalizable_ = false;
    checkEigen();
  }

  // Leaf init value: 1 if resolved state i is in the alias set of `state`
  // (Model/AbstractSubstitutionModel.cpp:98-112); throws BadIntException for gaps.
  double getInitValue(size_t i, int state) const;

  // -sum_i pi_i Q_ii (:645-650) and normalisation to 1 (:686-690)
  double getScale() const;
  void setScale(double scale);
  void normalize() {
    if (isScalable_) setScale(1. / getScale());
  }
  void setDiagonal();

  void fireParameterChanged(const ParameterList&) override { updateMatrices(); }
  virtual void updateMatrices() = 0;

 protected:
  // Eigen-system of the current generator (reversible: symmetric form); strips
  // null (stop) states like Model/AbstractSubstitutionModel.cpp:184-273.
  void computeEigen();
  // Eigen-system of a non-reversible generator (the reference's EigenValue on the
  // generator, :276-281): real eigenvalues and complex pairs, isDiagonalizable_ = no pair
  // (:291-303), isNonSingular_ = one null eigenvalue (:306-372), which is set to 0 exactly.
  void computeEigenGeneral();
  // out = V T V^-1 with T tridiagonal (diagonal dia, T(k,k+1) = up[k], T(k+1,k) = lo[k])
  void blockProduct(const Vdouble& dia, const Vdouble& up, const Vdouble& lo, RowMatrix<double>& out) const;
};

typedef SubstitutionModel TransitionModel;

// Q = S o pi, diagonal, normalise, eigen (Model/AbstractSubstitutionModel.cpp:694-703)
class AbstractReversibleSubstitutionModel : public SubstitutionModel {
 public:
  AbstractReversibleSubstitutionModel(const Alphabet* alpha, size_t size, const std::string& prefix)
      : SubstitutionModel(alpha, size, prefix) {}
  void updateMatrices() override;
};

}  // namespace bpp

#endif
