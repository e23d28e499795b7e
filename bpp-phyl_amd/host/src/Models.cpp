// Host mirror: substitution models (generator, frequencies, eigen-system, P(t)) and
// non-homogeneous model sets.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "Bpp/Phyl/Model/Models.h"
#include "Bpp/Phyl/Model/SubstitutionModelSet.h"

namespace bpp {

#include "lg08_data.inc"

const std::shared_ptr<IntervalConstraint> FrequencySet::FREQUENCE_CONSTRAINT_SMALL =
    std::make_shared<IntervalConstraint>(NumConstants::SMALL(), 1. - NumConstants::SMALL(), true, true);

// ---------------------------------------------------------------------------
// SubstitutionModel
// ---------------------------------------------------------------------------

double SubstitutionModel::getInitValue(size_t i, int state) const {
  if (i >= size_) throw IndexOutOfBoundsException("SubstitutionModel::getInitValue", i, 0, size_ - 1);
  if (state < 0 || !alphabet_->isIntInAlphabet(state))
    throw BadIntException(state, "SubstitutionModel::getInitValue. Character " + alphabet_->intToChar(state) +
                                     " is not allowed in model.");
  for (int s : alphabet_->getAlias(state))
    if (s == (int)i) return 1.;
  return 0.;
}

double SubstitutionModel::getScale() const {
  double s = 0.;
  for (size_t i = 0; i < size_; i++) s += generator_(i, i) * freq_[i];
  return -s;
}

void SubstitutionModel::setScale(double scale) {
  if (!isScalable_) return;
  for (size_t i = 0; i < size_; i++)
    for (size_t j = 0; j < size_; j++) generator_(i, j) *= scale;
  for (double& l : eigenValues_) l *= scale;
  for (double& l : iEigenValues_) l *= scale;  // (Model/AbstractSubstitutionModel.cpp:654-662)
}

void SubstitutionModel::setDiagonal() {
  for (size_t i = 0; i < size_; i++) {
    double lambda = 0.;
    for (size_t j = 0; j < size_; j++)
      if (j != i) lambda += generator_(i, j);
    generator_(i, i) = -lambda;
  }
}

namespace {
// out = V diag(w) Vinv
void eigenProduct(const RowMatrix<double>& V, const Vdouble& w, const RowMatrix<double>& Vi, RowMatrix<double>& out) {
  const size_t n = w.size();
  for (size_t i = 0; i < n; i++)
    for (size_t j = 0; j < n; j++) {
      double s = 0.;
      for (size_t k = 0; k < n; k++) s += V(i, k) * w[k] * Vi(k, j);
      out(i, j) = s;
    }
}
}  // namespace

namespace {
void matMul(const RowMatrix<double>& A, const RowMatrix<double>& B, RowMatrix<double>& out) {
  const size_t n = A.getNumberOfRows();
  RowMatrix<double> r(n, n);
  for (size_t i = 0; i < n; i++)
    for (size_t j = 0; j < n; j++) {
      double s = 0.;
      for (size_t k = 0; k < n; k++) s += A(i, k) * B(k, j);
      r(i, j) = s;
    }
  out = r;
}
}  // namespace

// Model/AbstractSubstitutionModel.cpp:277-330 decide isDiagonalizable / isNonSingular from
// the decomposition; the symmetric form used here is always diagonalizable in exact
// arithmetic, so the check is numerical: the decomposition must reproduce the generator
// and V V^-1 = I to 1e-10 (relative to |Q|).  On failure P(t) comes from the reference's
// truncated Taylor series with scaling and squaring (:386-418, 470-492).
void SubstitutionModel::checkEigen() {
  if (isNonSingular_) {
    double qmax = 0., err = 0.;
    for (size_t i = 0; i < size_; i++)
      for (size_t j = 0; j < size_; j++) qmax = std::max(qmax, std::fabs(generator_(i, j)));
    // the block-diagonal D of the decomposition (complex pairs as 2x2 blocks)
    Vdouble up(size_, 0.);
    for (size_t k = 0; k + 1 < size_; k++)
      if (iEigenValues_[k] != 0. && iEigenValues_[k] == -iEigenValues_[k + 1]) up[k] = iEigenValues_[k];
    for (size_t i = 0; i < size_ && std::isfinite(err); i++)
      for (size_t j = 0; j < size_; j++) {
        double q = 0., id = 0.;
        for (size_t k = 0; k < size_; k++) {
          double dk = eigenValues_[k] * leftEigenVectors_(k, j);
          if (k + 1 < size_) dk += up[k] * leftEigenVectors_(k + 1, j);
          if (k > 0) dk -= up[k - 1] * leftEigenVectors_(k - 1, j);
          q += rightEigenVectors_(i, k) * dk;
          id += rightEigenVectors_(i, k) * leftEigenVectors_(k, j);
        }
        err = std::max(err, std::fabs(q - generator_(i, j)) / std::max(qmax, 1e-300));
        err = std::max(err, std::fabs(id - (i == j ? 1. : 0.)));
        if (!std::isfinite(q) || !std::isfinite(id)) err = INFINITY;
      }
    if (!(err <= 1e-10)) isNonSingular_ = isDiagonalizable_ = false;
  }
  vPowGen_.clear();
  if (!isNonSingular_) {
    // vPowGen_[k] = Q^k / 1 (the factorials are applied in getPij_t), k = 0 .. 30
    vPowGen_.resize(31, RowMatrix<double>(size_, size_));
    for (size_t i = 0; i < size_; i++) vPowGen_[0](i, i) = 1.;
    for (size_t k = 1; k < vPowGen_.size(); k++) matMul(vPowGen_[k - 1], generator_, vPowGen_[k]);
  }
}

const RowMatrix<double>& SubstitutionModel::getPij_t(double t) const {
  if (t == 0.) {
    for (size_t i = 0; i < size_; i++)
      for (size_t j = 0; j < size_; j++) pijt_(i, j) = (i == j) ? 1. : 0.;
    return pijt_;
  }
  if (!isNonSingular_) {
    // exp(r t Q) = (exp(r t / 2^m Q))^(2^m), the inner exponential by 30 Taylor terms
    for (size_t i = 0; i < size_; i++)
      for (size_t j = 0; j < size_; j++) pijt_(i, j) = (i == j) ? 1. : 0.;
    double s = 1., v = rate_ * t;
    size_t m = 0;
    while (v > 0.5) {
      m++;
      v /= 2;
    }
    for (size_t k = 1; k < vPowGen_.size(); k++) {
      s *= v / (double)k;
      for (size_t i = 0; i < size_; i++)
        for (size_t j = 0; j < size_; j++) pijt_(i, j) += s * vPowGen_[k](i, j);
    }
    while (m-- > 0) matMul(pijt_, pijt_, pijt_);
    return pijt_;
  }
  if (!isDiagonalizable_) {  // complex pairs (Model/AbstractSubstitutionModel.cpp:440-467)
    Vdouble dia(size_), up(size_, 0.), lo(size_, 0.);
    const double l = rate_ * t;
    for (size_t i = 0; i < size_; i++) {
      dia[i] = std::exp(eigenValues_[i] * l);
      if (iEigenValues_[i] != 0. && i + 1 < size_) {
        const double s = std::sin(iEigenValues_[i] * l), c = std::cos(iEigenValues_[i] * l);
        up[i] = dia[i] * s;
        lo[i] = -up[i];
        dia[i] *= c;
        dia[i + 1] = dia[i];
        i++;
      }
    }
    blockProduct(dia, up, lo, pijt_);
    return pijt_;
  }
  Vdouble w(size_);
  for (size_t k = 0; k < size_; k++) w[k] = std::exp(eigenValues_[k] * rate_ * t);
  eigenProduct(rightEigenVectors_, w, leftEigenVectors_, pijt_);
  return pijt_;
}

void SubstitutionModel::blockProduct(const Vdouble& dia, const Vdouble& up, const Vdouble& lo,
                                     RowMatrix<double>& out) const {
  const size_t n = size_;
  for (size_t i = 0; i < n; i++)
    for (size_t j = 0; j < n; j++) {
      double s = 0.;
      for (size_t k = 0; k < n; k++) {
        double tk = dia[k] * leftEigenVectors_(k, j);
        if (k + 1 < n) tk += up[k] * leftEigenVectors_(k + 1, j);
        if (k > 0) tk += lo[k - 1] * leftEigenVectors_(k - 1, j);
        s += rightEigenVectors_(i, k) * tk;
      }
      out(i, j) = s;
    }
}

const RowMatrix<double>& SubstitutionModel::getdPij_dt(double t) const {
  if (!isNonSingular_) {  // d/dt exp(r t Q) = r Q exp(r t Q)
    const RowMatrix<double> P = getPij_t(t);
    matMul(generator_, P, dpijt_);
    for (size_t i = 0; i < size_; i++)
      for (size_t j = 0; j < size_; j++) dpijt_(i, j) *= rate_;
    return dpijt_;
  }
  if (!isDiagonalizable_) {  // (:505-537)
    Vdouble dia(size_), up(size_, 0.), lo(size_, 0.);
    const double l = rate_ * t;
    for (size_t i = 0; i < size_; i++) {
      const double e = std::exp(eigenValues_[i] * l);
      if (iEigenValues_[i] != 0. && i + 1 < size_) {
        const double a = eigenValues_[i], b = iEigenValues_[i];
        const double s = std::sin(b * l), c = std::cos(b * l);
        dia[i] = rate_ * (a * c - b * s) * e;
        up[i] = rate_ * (a * s + b * c) * e;
        lo[i] = -up[i];
        dia[i + 1] = dia[i];
        i++;
      } else {
        dia[i] = rate_ * eigenValues_[i] * e;
      }
    }
    blockProduct(dia, up, lo, dpijt_);
    return dpijt_;
  }
  Vdouble w(size_);
  for (size_t k = 0; k < size_; k++) w[k] = rate_ * eigenValues_[k] * std::exp(eigenValues_[k] * rate_ * t);
  eigenProduct(rightEigenVectors_, w, leftEigenVectors_, dpijt_);
  return dpijt_;
}

const RowMatrix<double>& SubstitutionModel::getd2Pij_dt2(double t) const {
  if (!isNonSingular_) {  // r^2 Q^2 exp(r t Q)
    const RowMatrix<double> P = getPij_t(t);
    matMul(vPowGen_[2], P, d2pijt_);
    for (size_t i = 0; i < size_; i++)
      for (size_t j = 0; j < size_; j++) d2pijt_(i, j) *= rate_ * rate_;
    return d2pijt_;
  }
  if (!isDiagonalizable_) {
    // (:581-611), as the reference writes it: the super-diagonal term carries
    // -2ab cos where the exact second derivative of e^{at} sin(bt) has +2ab cos
    Vdouble dia(size_), up(size_, 0.), lo(size_, 0.);
    const double l = rate_ * t, r2 = rate_ * rate_;
    for (size_t i = 0; i < size_; i++) {
      const double e = std::exp(eigenValues_[i] * l);
      if (iEigenValues_[i] != 0. && i + 1 < size_) {
        const double a = eigenValues_[i], b = iEigenValues_[i];
        const double s = std::sin(b * l), c = std::cos(b * l);
        dia[i] = r2 * ((a * a - b * b) * c - 2 * a * b * s) * e;
        up[i] = r2 * ((a * a - b * b) * s - 2 * a * b * c) * e;
        lo[i] = -up[i];
        dia[i + 1] = dia[i];
        i++;
      } else {
        dia[i] = r2 * eigenValues_[i] * eigenValues_[i] * e;
      }
    }
    blockProduct(dia, up, lo, d2pijt_);
    return d2pijt_;
  }
  Vdouble w(size_);
  for (size_t k = 0; k < size_; k++) {
    const double l = rate_ * eigenValues_[k];
    w[k] = l * l * std::exp(eigenValues_[k] * rate_ * t);
  }
  eigenProduct(rightEigenVectors_, w, leftEigenVectors_, d2pijt_);
  return d2pijt_;
}

// Reversible eigen-system via the symmetric form B = D^1/2 Q D^-1/2 (D = diag(pi)):
// B = U L U^T  =>  Q = (D^-1/2 U) L (U^T D^1/2), i.e. V = D^-1/2 U, V^-1 = U^T D^1/2.
// Null states (zero generator row and column: codon stops) are excluded from the
// decomposition and receive unit eigenvectors with eigenvalue 0, placed after the
// live ones (Model/AbstractSubstitutionModel.cpp:184-273).
void SubstitutionModel::computeEigen() {
  std::vector<size_t> live, null;
  for (size_t i = 0; i < size_; i++) {
    bool isNull = std::fabs(generator_(i, i)) < NumConstants::TINY();
    for (size_t j = 0; j < size_ && isNull; j++)
      if (std::fabs(generator_(j, i)) >= NumConstants::TINY()) isNull = false;
    (isNull ? null : live).push_back(i);
  }
  const size_t n = live.size();
  std::vector<double> B(n * n), d, U;
  std::vector<double> sq(n);
  for (size_t a = 0; a < n; a++) sq[a] = std::sqrt(freq_[live[a]]);
  for (size_t a = 0; a < n; a++)
    for (size_t b = 0; b < n; b++) B[a * n + b] = sq[a] * generator_(live[a], live[b]) / sq[b];
  for (size_t a = 0; a < n; a++)
    for (size_t b = a + 1; b < n; b++) {
      const double m = 0.5 * (B[a * n + b] + B[b * n + a]);
      B[a * n + b] = B[b * n + a] = m;
    }
  symmetricEigen(n, B, d, U);
  rightEigenVectors_.resize(size_, size_);
  leftEigenVectors_.resize(size_, size_);
  eigenValues_.assign(size_, 0.);
  size_t nullEig = 0;
  for (size_t k = 0; k < n; k++) {
    eigenValues_[k] = d[k];
    if (std::fabs(d[k]) < std::fabs(d[nullEig])) nullEig = k;
    for (size_t a = 0; a < n; a++) {
      rightEigenVectors_(live[a], k) = U[a * n + k] / sq[a];
      leftEigenVectors_(k, live[a]) = U[a * n + k] * sq[a];
    }
  }
  if (n > 0) eigenValues_[nullEig] = 0.;  // exact stationary eigenvalue (:358-361)
  iEigenValues_.assign(size_, 0.);
  for (size_t s = 0; s < null.size(); s++) {
    rightEigenVectors_(null[s], n + s) = 1.;
    leftEigenVectors_(n + s, null[s]) = 1.;
  }
  isDiagonalizable_ = true;
  isNonSingular_ = true;
  checkEigen();
}

void SubstitutionModel::computeEigenGeneral() {
  const size_t n = size_;
  std::vector<double> A(n * n), wr, wi, V, Vi;
  for (size_t i = 0; i < n; i++)
    for (size_t j = 0; j < n; j++) A[i * n + j] = generator_(i, j);
  isNonSingular_ = isDiagonalizable_ = false;
  eigenValues_.assign(n, 0.);
  iEigenValues_.assign(n, 0.);
  if (generalEigen(n, A, wr, wi, V) && invertMatrix(n, V, Vi)) {
    for (size_t i = 0; i < n; i++) {
      eigenValues_[i] = wr[i];
      iEigenValues_[i] = wi[i];
      for (size_t j = 0; j < n; j++) {
        rightEigenVectors_(i, j) = V[i * n + j];
        leftEigenVectors_(i, j) = Vi[i * n + j];
      }
    }
    isDiagonalizable_ = true;
    for (double b : iEigenValues_)
      if (std::fabs(b) > NumConstants::TINY()) isDiagonalizable_ = false;
    // the null eigenvalue: exactly one with |Re| < fact * SMALL and |Im| < SMALL, fact
    // = 1, 10, 100, 1000 until one is found (:306-316)
    std::vector<size_t> nulls;
    for (double fact = 1.; nulls.empty() && fact <= 1000.; fact *= 10.)
      for (size_t i = 0; i < n; i++)
        if (std::fabs(eigenValues_[i]) < fact * NumConstants::SMALL() &&
            std::fabs(iEigenValues_[i]) < NumConstants::SMALL())
          nulls.push_back(i);
    isNonSingular_ = nulls.size() == 1;
    if (isNonSingular_) eigenValues_[nulls[0]] = iEigenValues_[nulls[0]] = 0.;
  }
  checkEigen();
}

void AbstractReversibleSubstitutionModel::updateMatrices() {
  for (size_t i = 0; i < size_; i++)
    for (size_t j = 0; j < size_; j++) generator_(i, j) = exchangeability_(i, j) * freq_[j];
  setDiagonal();
  normalize();
  computeEigen();
}

// ---------------------------------------------------------------------------
// T92
// ---------------------------------------------------------------------------

T92::T92(const NucleicAlphabet* alpha, double kappa, double theta)
    : AbstractReversibleSubstitutionModel(alpha, 4, "T92."), kappa_(kappa), theta_(theta), k_(0.), r_(0.) {
  addParameter_(Parameter("T92.kappa", kappa, Parameter::R_PLUS_STAR));
  addParameter_(Parameter("T92.theta", theta, FrequencySet::FREQUENCE_CONSTRAINT_SMALL));
  updateMatrices();
}

void T92::updateMatrices() {
  kappa_ = getParameterValue("kappa");
  theta_ = getParameterValue("theta");
  const double th = theta_, ka = kappa_;
  const double piAT = (1. - th) / 2., piCG = th / 2.;
  k_ = (ka + 1.) / 2.;
  r_ = isScalable_ ? 2. / (1. + 2. * th * ka - 2. * th * th * ka) : 1.;
  freq_ = {piAT, piCG, piCG, piAT};
  // unscaled generator (Model/Nucleotide/T92.cpp:100-121), then scaled by r
  const double Qu[4][4] = {{-(1. + th * ka) / 2., th / 2., ka * th / 2., (1. - th) / 2.},
                           {(1. - th) / 2., -(1. + (1. - th) * ka) / 2., th / 2., ka * (1. - th) / 2.},
                           {ka * (1. - th) / 2., th / 2., -(1. + (1. - th) * ka) / 2., (1. - th) / 2.},
                           {(1. - th) / 2., ka * th / 2., th / 2., -(1. + th * ka) / 2.}};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) generator_(i, j) = Qu[i][j] * r_;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) exchangeability_(i, j) = generator_(i, j) / freq_[j];
  // analytic eigen-system (:140-186)
  eigenValues_ = {0., -r_ * (1. + ka) / 2., -r_ * (1. + ka) / 2., -r_};
  const double Vi[4][4] = {{(1. - th) / 2., th / 2., th / 2., (1. - th) / 2.},
                           {0., 1. - th, 0., th - 1.},
                           {th, 0., -th, 0.},
                           {(1. - th) / 2., -th / 2., th / 2., (th - 1.) / 2.}};
  const double V[4][4] = {{1., 0., 1., 1.},
                          {1., 1., 0., -1.},
                          {1., 0., (th - 1.) / th, 1.},
                          {1., th / (th - 1.), 0., -1.}};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      leftEigenVectors_(i, j) = Vi[i][j];
      rightEigenVectors_(i, j) = V[i][j];
    }
}

const RowMatrix<double>& T92::getPij_t(double d) const {
  // closed form, Model/Nucleotide/T92.cpp:355-386
  const double l = rate_ * r_ * d;
  const double e1 = std::exp(-l), e2 = std::exp(-k_ * l);
  const double th = theta_;
  const double piA = (1. - th) / 2., piC = th / 2., piG = th / 2., piT = (1. - th) / 2.;
  const double P[4][4] = {
      {piA * (1. + e1) + th * e2, piC * (1. - e1), piG * (1. + e1) - th * e2, piT * (1. - e1)},
      {piA * (1. - e1), piC * (1. + e1) + (1. - th) * e2, piG * (1. - e1), piT * (1. + e1) - (1. - th) * e2},
      {piA * (1. + e1) - (1. - th) * e2, piC * (1. - e1), piG * (1. + e1) + (1. - th) * e2, piT * (1. - e1)},
      {piA * (1. - e1), piC * (1. + e1) - th * e2, piG * (1. - e1), piT * (1. + e1) + th * e2}};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) pijt_(i, j) = P[i][j];
  return pijt_;
}

const RowMatrix<double>& T92::getdPij_dt(double d) const { return SubstitutionModel::getdPij_dt(d); }
const RowMatrix<double>& T92::getd2Pij_dt2(double d) const { return SubstitutionModel::getd2Pij_dt2(d); }

// ---------------------------------------------------------------------------
// L95 (Model/Nucleotide/L95.cpp:56-119)
// ---------------------------------------------------------------------------

L95::L95(const NucleicAlphabet* alpha, double a, double b, double g, double kappa, double theta)
    : SubstitutionModel(alpha, 4, "L95."), alpha_(a), beta_(b), gamma_(g), kappa_(kappa), theta_(theta) {
  addParameter_(Parameter("L95.alpha", a, Parameter::PROP_CONSTRAINT_IN));
  addParameter_(Parameter("L95.beta", b, Parameter::PROP_CONSTRAINT_IN));
  addParameter_(Parameter("L95.gamma", g, Parameter::PROP_CONSTRAINT_IN));
  addParameter_(Parameter("L95.kappa", kappa, std::make_shared<IntervalConstraint>(0., 1000., false, false, 1e-3)));
  addParameter_(Parameter("L95.theta", theta, std::make_shared<IntervalConstraint>(0., 1., false, false, 1e-3)));
  updateMatrices();
}

void L95::updateMatrices() {
  alpha_ = getParameterValue("alpha");
  beta_ = getParameterValue("beta");
  gamma_ = getParameterValue("gamma");
  kappa_ = getParameterValue("kappa");
  theta_ = getParameterValue("theta");
  const double a = alpha_, b = beta_, g = gamma_, k = kappa_, th = theta_;
  freq_ = {(1. - th) / 2., th / 2., th / 2., (1. - th) / 2.};
  const double Q[4][4] = {{-k * th - g, k * b * th, k * (1. - b) * th, g},
                          {k * a * (1. - th), -k * (1. - th) + g - 1., 1. - g, k * (1. - th) * (1. - a)},
                          {k * (1. - th) * (1. - a), 1. - g, -k * (1. - th) + g - 1., k * a * (1. - th)},
                          {g, k * (1. - b) * th, k * b * th, -k * th - g}};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) generator_(i, j) = Q[i][j];
  setScale(1. / (2. * k * th * (1. - th) + g + th - 2. * th * g));
  // AbstractSubstitutionModel::updateMatrices (:175-418): eigen-system of the generator,
  // then the normalisation to one substitution per unit time
  computeEigenGeneral();
  normalize();
  if (!isNonSingular_) checkEigen();  // the Taylor powers of the normalised generator
}

// ---------------------------------------------------------------------------
// GTR
// ---------------------------------------------------------------------------

GTR::GTR(const NucleicAlphabet* alpha, double a, double b, double c, double d, double e, double piA, double piC,
         double piG, double piT)
    : AbstractReversibleSubstitutionModel(alpha, 4, "GTR.") {
  const double theta = piG + piC;
  addParameter_(Parameter("GTR.a", a, Parameter::R_PLUS_STAR));
  addParameter_(Parameter("GTR.b", b, Parameter::R_PLUS_STAR));
  addParameter_(Parameter("GTR.c", c, Parameter::R_PLUS_STAR));
  addParameter_(Parameter("GTR.d", d, Parameter::R_PLUS_STAR));
  addParameter_(Parameter("GTR.e", e, Parameter::R_PLUS_STAR));
  addParameter_(Parameter("GTR.theta", theta, FrequencySet::FREQUENCE_CONSTRAINT_SMALL));
  addParameter_(Parameter("GTR.theta1", piA / (1. - theta), FrequencySet::FREQUENCE_CONSTRAINT_SMALL));
  addParameter_(Parameter("GTR.theta2", piG / theta, FrequencySet::FREQUENCE_CONSTRAINT_SMALL));
  updateMatrices();
}

void GTR::updateMatrices() {
  const double a = getParameterValue("a"), b = getParameterValue("b"), c = getParameterValue("c");
  const double d = getParameterValue("d"), e = getParameterValue("e");
  const double theta = getParameterValue("theta"), t1 = getParameterValue("theta1"), t2 = getParameterValue("theta2");
  const double pA = t1 * (1. - theta), pC = (1. - t2) * theta, pG = t2 * theta, pT = (1. - t1) * (1. - theta);
  const double p = 2. * (a * pC * pT + b * pA * pT + c * pG * pT + d * pA * pC + e * pC * pG + pA * pG);
  freq_ = {pA, pC, pG, pT};
  // A<->G = 1, a = C<->T, b = A<->T, c = G<->T, d = A<->C, e = C<->G (GTR.cpp:104-120)
  const double S[4][4] = {{0., d, 1., b}, {d, 0., e, a}, {1., e, 0., c}, {b, a, c, 0.}};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) exchangeability_(i, j) = S[i][j] / p;
  AbstractReversibleSubstitutionModel::updateMatrices();
}

// ---------------------------------------------------------------------------
// LG08
// ---------------------------------------------------------------------------

LG08::LG08(const ProteicAlphabet* alpha) : AbstractReversibleSubstitutionModel(alpha, 20, "LG08.") {
  for (int i = 0; i < 20; i++) {
    freq_[i] = kLG08Frequencies[i];
    for (int j = 0; j < 20; j++) exchangeability_(i, j) = kLG08Exchangeability[i][j];
  }
  updateMatrices();
}

void LG08::updateMatrices() { AbstractReversibleSubstitutionModel::updateMatrices(); }

// ---------------------------------------------------------------------------
// YN98
// ---------------------------------------------------------------------------

YN98::YN98(const GeneticCode* gc, const Vdouble& codonFreqs, double kappa, double omega)
    : AbstractReversibleSubstitutionModel(gc->getSourceAlphabet(), 64, "YN98."), gc_(gc), codonFreqs_(codonFreqs) {
  addParameter_(Parameter("YN98.kappa", kappa, Parameter::R_PLUS_STAR));
  addParameter_(Parameter("YN98.omega", omega,
                          std::make_shared<IntervalConstraint>(NumConstants::MILLI(), 999., true, true)));
  if (codonFreqs_.empty()) codonFreqs_.assign(64, 1.);  // F3X4, equal nucleotide frequencies
  double s = 0.;
  for (int i = 0; i < 64; i++) {
    if (gc_->isStop(i)) codonFreqs_[i] = 0.;
    s += codonFreqs_[i];
  }
  for (double& f : codonFreqs_) f /= s;
  updateMatrices();
}

void YN98::updateMatrices() {
  const double kappa = getParameterValue("kappa"), omega = getParameterValue("omega");
  freq_ = codonFreqs_;
  auto isTransition = [](int x, int y) { return (x == 0 && y == 2) || (x == 2 && y == 0) || (x == 1 && y == 3) || (x == 3 && y == 1); };
  for (int i = 0; i < 64; i++)
    for (int j = 0; j < 64; j++) {
      generator_(i, j) = 0.;
      if (i == j || gc_->isStop(i) || gc_->isStop(j)) continue;
      int diff = 0, from = 0, to = 0;
      for (int pos = 0; pos < 3; pos++) {
        const int div = pos == 0 ? 16 : (pos == 1 ? 4 : 1);
        const int a = (i / div) % 4, b = (j / div) % 4;
        if (a != b) {
          diff++;
          from = a;
          to = b;
        }
      }
      if (diff != 1) continue;
      double q = isTransition(from, to) ? kappa : 1.;
      if (!gc_->areSynonymous(i, j)) q *= omega;
      generator_(i, j) = q * freq_[j];
    }
  setDiagonal();
  normalize();
  for (int i = 0; i < 64; i++)
    for (int j = 0; j < 64; j++) exchangeability_(i, j) = freq_[j] > 0. ? generator_(i, j) / freq_[j] : 0.;
  computeEigen();
}

// ---------------------------------------------------------------------------
// Frequency sets
// ---------------------------------------------------------------------------

GCFrequencySet::GCFrequencySet(const NucleicAlphabet* alpha, double theta) : FrequencySet(alpha, 4, "GC.") {
  addParameter_(Parameter("GC.theta", theta, FREQUENCE_CONSTRAINT_SMALL));
  fireParameterChanged(ParameterList());
}

void GCFrequencySet::fireParameterChanged(const ParameterList&) {
  const double th = getParameterValue("theta");
  freq_ = {(1. - th) / 2., th / 2., th / 2., (1. - th) / 2.};
}

// ---------------------------------------------------------------------------
// SubstitutionModelSet
// ---------------------------------------------------------------------------

SubstitutionModelSet::SubstitutionModelSet(const SubstitutionModelSet& s)
    : AbstractParametrizable(s), alphabet_(s.alphabet_), nodesOfModel_(s.nodesOfModel_),
      modelOfNode_(s.modelOfNode_), aliasOf_(s.aliasOf_) {
  for (auto& m : s.models_) models_.push_back(std::shared_ptr<SubstitutionModel>(m->clone()));
  if (s.rootFreqs_) rootFreqs_.reset(s.rootFreqs_->clone());
}

long SubstitutionModelSet::modelIndexOfParameter(const std::string& name) const {
  const size_t u = name.rfind('_');
  if (u == std::string::npos || u + 1 >= name.size()) return -1;
  for (size_t i = u + 1; i < name.size(); i++)
    if (name[i] < '0' || name[i] > '9') return -1;
  const long k = std::atol(name.c_str() + u + 1);
  return (k >= 1 && (size_t)k <= models_.size()) ? k - 1 : -1;
}

void SubstitutionModelSet::setRootFrequencies(FrequencySet* rootFreqs) {
  // the root frequencies' parameters come first (SubstitutionModelSet.h:457-466)
  ParameterList rest;
  for (size_t i = 0; i < parameters_.size(); i++)
    if (!rootFreqs_ || !rootFreqs_->getParameters().hasParameter(parameters_[i].getName()))
      rest.addParameter(parameters_[i]);
  rootFreqs_.reset(rootFreqs);
  resetParameters_();
  if (rootFreqs_) addParameters_(rootFreqs_->getParameters());
  addParameters_(rest);
}

void SubstitutionModelSet::addModel(SubstitutionModel* model, const std::vector<int>& nodesId) {
  const size_t k = models_.size() + 1;
  if (model->getAlphabet()->getAlphabetType() != alphabet_->getAlphabetType())
    throw AlphabetMismatchException("SubstitutionModelSet::addModel: alphabets do not match");
  models_.push_back(std::shared_ptr<SubstitutionModel>(model));
  nodesOfModel_.push_back(nodesId);
  for (int id : nodesId) modelOfNode_[id] = k - 1;
  const ParameterList& pl = model->getParameters();
  for (size_t i = 0; i < pl.size(); i++) {
    Parameter p(pl[i]);
    p.setName(pl[i].getName() + "_" + std::to_string(k));
    addParameter_(p);
  }
}

void SubstitutionModelSet::aliasParameters(const std::string& p1, const std::string& p2) {
  if (!parameters_.hasParameter(p1)) throw ParameterNotFoundException("SubstitutionModelSet::aliasParameters", p1);
  if (!parameters_.hasParameter(p2)) throw ParameterNotFoundException("SubstitutionModelSet::aliasParameters", p2);
  if (p1 == p2) throw Exception("SubstitutionModelSet::aliasParameters: a parameter cannot alias itself: " + p1);
  std::string root = p1;
  while (aliasOf_.count(root)) root = aliasOf_.at(root);
  if (root == p2) throw Exception("SubstitutionModelSet::aliasParameters: cyclic alias " + p1 + " <- " + p2);
  aliasOf_[p2] = p1;
  ParameterList one;
  Parameter q = parameters_.getParameter(p2);
  q.setValue(parameters_.getParameterValue(p1));
  one.addParameter(q);
  matchParametersValues(one);
}

std::vector<std::string> SubstitutionModelSet::getAlias(const std::string& name) const {
  std::vector<std::string> out;
  for (auto& kv : aliasOf_)
    if (kv.second == name) out.push_back(kv.first);
  return out;
}

ParameterList SubstitutionModelSet::getNodeParameters() const {
  ParameterList out;
  ParameterList rf = getRootFrequenciesParameters();
  for (size_t i = 0; i < parameters_.size(); i++)
    if (!rf.hasParameter(parameters_[i].getName())) out.addParameter(parameters_[i]);
  return out;
}

ParameterList SubstitutionModelSet::getIndependentParameters() const {
  ParameterList out;
  for (size_t i = 0; i < parameters_.size(); i++)
    if (!aliasOf_.count(parameters_[i].getName())) out.addParameter(parameters_[i]);
  return out;
}

std::vector<int> SubstitutionModelSet::getNodesWithParameter(const std::string& name) const {
  if (!parameters_.hasParameter(name)) throw ParameterNotFoundException("SubstitutionModelSet::getNodesWithParameter.", name);
  std::vector<int> out;
  std::vector<std::string> names(1, name);
  // the parameter, its aliases, their aliases, ...
  for (size_t i = 0; i < names.size(); i++)
    for (const std::string& a : getAlias(names[i]))
      if (std::find(names.begin(), names.end(), a) == names.end()) names.push_back(a);
  for (const std::string& n : names) {
    const long m = modelIndexOfParameter(n);
    if (m < 0) continue;
    for (int id : nodesOfModel_[(size_t)m])
      if (std::find(out.begin(), out.end(), id) == out.end()) out.push_back(id);
  }
  return out;
}

bool SubstitutionModelSet::isFullySetUpFor(const Tree& tree) const {
  const TreeTemplate<Node>* tt = dynamic_cast<const TreeTemplate<Node>*>(&tree);
  if (!tt) return false;
  for (const Node* n : tt->getNodes())
    if (n != tt->getRootNode() && !modelOfNode_.count(n->getId())) return false;
  return rootFreqs_ ? rootFreqs_->getFrequencies().size() == getNumberOfStates() : true;
}

bool SubstitutionModelSet::matchParametersValues(const ParameterList& pl) {
  std::vector<size_t> changed;
  parameters_.matchParametersValues(pl, &changed);
  // aliases follow their sources (in alias-chain order: repeat until stable)
  for (bool moved = true; moved;) {
    moved = false;
    for (auto& kv : aliasOf_) {
      const double v = parameters_.getParameterValue(kv.second);
      const size_t i = parameters_.whichParameterHasName(kv.first);
      if (parameters_[i].getValue() != v) {
        parameters_[i].setValue(v);
        if (std::find(changed.begin(), changed.end(), i) == changed.end()) changed.push_back(i);
        moved = true;
      }
    }
  }
  if (changed.empty()) return false;
  ParameterList ch;
  for (size_t i : changed) ch.addParameter(parameters_[i]);
  fireParameterChanged(ch);
  return true;
}

void SubstitutionModelSet::setParametersValues(const ParameterList& pl) {
  matchParametersValues(pl);
}

// Each model takes the values of its own "_<k>" parameters; only a model whose values moved
// recomputes its generator and eigen-system (SubstitutionModel::fireParameterChanged).
void SubstitutionModelSet::fireParameterChanged(const ParameterList&) {
  lastChangedModels_.clear();
  for (size_t k = 0; k < models_.size(); k++) {
    ParameterList own;
    const ParameterList& pl = models_[k]->getParameters();
    const std::string suffix = "_" + std::to_string(k + 1);
    for (size_t i = 0; i < pl.size(); i++) {
      const std::string local = pl[i].getName() + suffix;
      if (!parameters_.hasParameter(local)) continue;
      Parameter p(pl[i]);
      p.setValue(parameters_.getParameterValue(local));
      own.addParameter(p);
    }
    if (models_[k]->matchParametersValues(own)) lastChangedModels_.push_back(k);
  }
  lastRootFreqsChanged_ = rootFreqs_ ? rootFreqs_->matchParametersValues(parameters_) : false;
}

namespace {
// ApplicationTools::matchingParameters: a name with '*' wildcards against a list of names
bool wildcardMatch(const std::string& pat, const std::string& s) {
  size_t p = 0, q = 0, star = std::string::npos, mark = 0;
  while (q < s.size()) {
    if (p < pat.size() && pat[p] == s[q]) {
      p++;
      q++;
    } else if (p < pat.size() && pat[p] == '*') {
      star = p++;
      mark = q;
    } else if (star != std::string::npos) {
      p = star + 1;
      q = ++mark;
    } else {
      return false;
    }
  }
  while (p < pat.size() && pat[p] == '*') p++;
  return p == pat.size();
}
}  // namespace

// SubstitutionModelSetTools.cpp:81-175: a clone of the model per non-root node (in
// getNodesId order), global parameters aliased to the first model's copy (or, for a
// parameter given with groups of node ids, to the copy of each group's first node), and
// aliasFreqNames tying root-frequency parameters to model 1's global ones.
SubstitutionModelSet* SubstitutionModelSetTools::createNonHomogeneousModelSet(
    SubstitutionModel* model, FrequencySet* rootFreqs, const Tree* tree,
    const std::map<std::string, std::string>& aliasFreqNames,
    std::map<std::string, std::vector<Vint> >& globalParameterNames) {
  const TreeTemplate<Node>* tt = dynamic_cast<const TreeTemplate<Node>*>(tree);
  if (!tt) throw Exception("createNonHomogeneousModelSet: unsupported tree implementation");
  if (rootFreqs && model->getAlphabet()->getAlphabetType() != rootFreqs->getAlphabet()->getAlphabetType())
    throw AlphabetMismatchException("SubstitutionModelSetTools::createNonHomogeneousModelSet()");
  const std::vector<std::string> modelNames = model->getParameters().getParameterNames();
  std::map<std::string, std::vector<Vint> > globals;
  for (auto& kv : globalParameterNames) {
    bool any = false;
    for (const std::string& n : modelNames)
      if (wildcardMatch(kv.first, n)) {
        globals[n] = kv.second;
        any = true;
      }
    if (!any) throw Exception("SubstitutionModelSetTools::createNonHomogeneousModelSet. Parameter '" + kv.first + "' is not valid.");
  }
  SubstitutionModelSet* set = new SubstitutionModelSet(model->getAlphabet());
  if (rootFreqs) set->setRootFrequencies(rootFreqs);
  std::vector<int> ids = tt->getNodesId();
  ids.erase(std::find(ids.begin(), ids.end(), tt->getRootNode()->getId()));
  for (int id : ids) set->addModel(model->clone(), std::vector<int>(1, id));
  for (const std::string& pname : modelNames) {
    auto g = globals.find(pname);
    if (g == globals.end()) continue;
    auto suffixed = [&](int nodeId) { return pname + "_" + std::to_string(set->getModelIndexForNode(nodeId) + 1); };
    if (g->second.empty()) {
      for (size_t i = 1; i < ids.size(); i++) set->aliasParameters(suffixed(ids[0]), suffixed(ids[i]));
    } else {
      for (const Vint& group : g->second)
        for (size_t i = 1; i < group.size(); i++) set->aliasParameters(suffixed(group[0]), suffixed(group[i]));
    }
  }
  for (auto& kv : aliasFreqNames)
    if (globals.count(kv.second)) set->aliasParameters(kv.second + "_1", kv.first);
  delete model;
  return set;
}

SubstitutionModelSet* SubstitutionModelSetTools::createHomogeneousModelSet(SubstitutionModel* model,
                                                                           FrequencySet* rootFreqs,
                                                                           const Tree* tree) {
  const TreeTemplate<Node>* tt = dynamic_cast<const TreeTemplate<Node>*>(tree);
  if (!tt) throw Exception("createHomogeneousModelSet: unsupported tree implementation");
  std::vector<int> ids = tt->getNodesId();
  ids.erase(std::find(ids.begin(), ids.end(), tt->getRootNode()->getId()));
  SubstitutionModelSet* set = new SubstitutionModelSet(model->getAlphabet());
  if (rootFreqs) set->setRootFrequencies(rootFreqs);
  set->addModel(model, ids);
  return set;
}

}  // namespace bpp
