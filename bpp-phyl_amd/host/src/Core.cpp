// Host mirror: parameters, alphabets, Newick parsing, symmetric eigen-solver and
// the discrete Gamma distribution.
#include <algorithm>
#include <cmath>
#include <complex>
#include <sstream>

#include "Bpp/Numeric/Matrix/Matrix.h"
#include "Bpp/Numeric/Parameter.h"
#include "Bpp/Numeric/Prob/DiscreteDistribution.h"
#include "Bpp/Phyl/Model/RateDistribution/GammaDiscreteRateDistribution.h"
#include "Bpp/Phyl/TreeTemplate.h"
#include "Bpp/Seq/Alphabet/Alphabet.h"
#include "Bpp/Text/TextTools.h"

namespace bpp {

const std::shared_ptr<IntervalConstraint> Parameter::R_PLUS =
    std::make_shared<IntervalConstraint>(0., std::numeric_limits<double>::infinity(), true, false);
const std::shared_ptr<IntervalConstraint> Parameter::R_PLUS_STAR =
    std::make_shared<IntervalConstraint>(0., std::numeric_limits<double>::infinity(), false, false);
const std::shared_ptr<IntervalConstraint> Parameter::PROP_CONSTRAINT_IN =
    std::make_shared<IntervalConstraint>(0., 1., true, true);
const std::shared_ptr<IntervalConstraint> Parameter::PROP_CONSTRAINT_EX =
    std::make_shared<IntervalConstraint>(0., 1., false, false);

const DNA AlphabetTools::DNA_ALPHABET;
const ProteicAlphabet AlphabetTools::PROTEIN_ALPHABET;

// ---------------------------------------------------------------------------
// Newick.  Grammar: subtree = leaf | "(" subtree ("," subtree)* ")" [label] [":" length]
// ---------------------------------------------------------------------------
namespace {

std::vector<std::string> splitTopLevel(const std::string& s) {
  std::vector<std::string> parts;
  int depth = 0;
  size_t start = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '(') depth++;
    else if (s[i] == ')') depth--;
    else if (s[i] == ',' && depth == 0) {
      parts.push_back(s.substr(start, i - start));
      start = i + 1;
    }
  }
  parts.push_back(s.substr(start));
  return parts;
}

Node* parseSubtree(const std::string& desc) {
  std::string d = TextTools::removeSurroundingWhiteSpaces(desc);
  Node* node = new Node();
  std::string tail;
  if (!d.empty() && d[0] == '(') {
    size_t close = d.rfind(')');
    if (close == std::string::npos) throw Exception("Newick: unbalanced parentheses in '" + d + "'");
    for (const std::string& part : splitTopLevel(d.substr(1, close - 1))) node->addSon(parseSubtree(part));
    tail = d.substr(close + 1);
  } else {
    tail = d;
  }
  std::string label = tail;
  size_t colon = tail.rfind(':');
  if (colon != std::string::npos) {
    label = tail.substr(0, colon);
    node->setDistanceToFather(TextTools::toDouble(tail.substr(colon + 1)));
  }
  label = TextTools::removeSurroundingWhiteSpaces(label);
  if (node->isLeaf()) node->setName(label);
  return node;
}

void toNewick(const Node* n, std::ostringstream& o) {
  if (!n->isLeaf()) {
    o << "(";
    for (size_t i = 0; i < n->getNumberOfSons(); i++) {
      if (i) o << ",";
      toNewick(n->getSon(i), o);
    }
    o << ")";
  } else {
    o << n->getName();
  }
  if (n->hasDistanceToFather()) o << ":" << n->getDistanceToFather();
}

}  // namespace

TreeTemplate<Node>* TreeTemplateTools::parenthesisToTree(const std::string& description, bool, const std::string&,
                                                         bool, bool) {
  size_t semi = description.rfind(';');
  if (semi == std::string::npos) throw Exception("TreeTemplateTools::parenthesisToTree(). Bad format: no semi-colon found.");
  std::string content;
  for (char c : description.substr(0, semi))
    if (c != '\n' && c != '\r') content += c;
  TreeTemplate<Node>* tree = new TreeTemplate<Node>(parseSubtree(content));
  tree->resetNodesId();
  return tree;
}

std::string TreeTemplateTools::treeToParenthesis(const TreeTemplate<Node>& tree) {
  std::ostringstream o;
  o.precision(17);
  toNewick(tree.getRootNode(), o);
  o << ";";
  return o.str();
}

// ---------------------------------------------------------------------------
// Symmetric eigen-solver: Householder tridiagonalisation + implicit QL.
// ---------------------------------------------------------------------------
void symmetricEigen(size_t n, const std::vector<double>& Ain, std::vector<double>& d, std::vector<double>& U) {
  std::vector<double> a(Ain);
  auto A = [&](size_t i, size_t j) -> double& { return a[i * n + j]; };
  std::vector<double> e(n, 0.);
  d.assign(n, 0.);
  // Householder reduction: A = Q T Q^T with T tridiagonal (diag d, sub-diagonal e).
  for (size_t i = n - 1; i >= 1; --i) {
    const size_t l = i - 1;
    double h = 0.;
    if (l > 0) {
      double scale = 0.;
      for (size_t k = 0; k <= l; ++k) scale += std::fabs(A(i, k));
      if (scale == 0.) {
        e[i] = A(i, l);
      } else {
        for (size_t k = 0; k <= l; ++k) {
          A(i, k) /= scale;
          h += A(i, k) * A(i, k);
        }
        const double f0 = A(i, l);
        const double g0 = f0 >= 0. ? -std::sqrt(h) : std::sqrt(h);
        e[i] = scale * g0;
        h -= f0 * g0;
        A(i, l) = f0 - g0;
        double f = 0.;
        for (size_t j = 0; j <= l; ++j) {
          A(j, i) = A(i, j) / h;
          double g = 0.;
          for (size_t k = 0; k <= j; ++k) g += A(j, k) * A(i, k);
          for (size_t k = j + 1; k <= l; ++k) g += A(k, j) * A(i, k);
          e[j] = g / h;
          f += e[j] * A(i, j);
        }
        const double hh = f / (h + h);
        for (size_t j = 0; j <= l; ++j) {
          const double fj = A(i, j);
          const double gj = e[j] - hh * fj;
          e[j] = gj;
          for (size_t k = 0; k <= j; ++k) A(j, k) -= (fj * e[k] + gj * A(i, k));
        }
      }
    } else {
      e[i] = A(i, l);
    }
    d[i] = h;
  }
  d[0] = 0.;
  e[0] = 0.;
  // Accumulate the transformations.
  for (size_t i = 0; i < n; ++i) {
    if (d[i] != 0. && i > 0) {
      for (size_t j = 0; j < i; ++j) {
        double g = 0.;
        for (size_t k = 0; k < i; ++k) g += A(i, k) * A(k, j);
        for (size_t k = 0; k < i; ++k) A(k, j) -= g * A(k, i);
      }
    }
    d[i] = A(i, i);
    A(i, i) = 1.;
    for (size_t j = 0; j < i; ++j) A(j, i) = A(i, j) = 0.;
  }
  // Implicit-shift QL on the tridiagonal matrix.
  for (size_t i = 1; i < n; ++i) e[i - 1] = e[i];
  e[n - 1] = 0.;
  for (size_t l = 0; l < n; ++l) {
    int iter = 0;
    size_t m;
    do {
      for (m = l; m + 1 < n; ++m) {
        const double dd = std::fabs(d[m]) + std::fabs(d[m + 1]);
        if (std::fabs(e[m]) <= 1e-15 * dd) break;
      }
      if (m != l) {
        if (iter++ == 100) throw Exception("symmetricEigen: QL iteration did not converge");
        double g = (d[l + 1] - d[l]) / (2. * e[l]);
        double r = std::hypot(g, 1.);
        g = d[m] - d[l] + e[l] / (g + (g >= 0. ? std::fabs(r) : -std::fabs(r)));
        double s = 1., c = 1., p = 0.;
        bool underflow = false;
        for (size_t ii = m; ii-- > l;) {
          double f = s * e[ii];
          const double b = c * e[ii];
          r = std::hypot(f, g);
          e[ii + 1] = r;
          if (r == 0.) {
            d[ii + 1] -= p;
            e[m] = 0.;
            underflow = true;
            break;
          }
          s = f / r;
          c = g / r;
          g = d[ii + 1] - p;
          r = (d[ii] - g) * s + 2. * c * b;
          p = s * r;
          d[ii + 1] = g + p;
          g = c * r - b;
          for (size_t k = 0; k < n; ++k) {
            f = A(k, ii + 1);
            A(k, ii + 1) = s * A(k, ii) + c * f;
            A(k, ii) = c * A(k, ii) - s * f;
          }
        }
        if (underflow) continue;
        d[l] -= p;
        e[l] = g;
        e[m] = 0.;
      }
    } while (m != l);
  }
  U = a;
}

// ---------------------------------------------------------------------------
// Discrete Gamma (bpp-core AbstractDiscreteDistribution::discretize, mean of category)
// ---------------------------------------------------------------------------
double GammaDiscreteDistribution::lnGamma(double x) {
  // Pike & Hill (1966): shift to x >= 7, then Stirling's series.
  double shift = 0.;
  if (x < 7.) {
    double prod = 1.;
    double z = x;
    for (; z < 7.; z += 1.) prod *= z;
    shift = -std::log(prod);
    x = z;
  }
  const double z2 = 1. / (x * x);
  const double series =
      (((-.000595238095238 * z2 + .000793650793651) * z2 - .002777777777778) * z2 + .083333333333333) / x;
  return shift + (x - 0.5) * std::log(x) - x + .918938533204673 + series;
}

double GammaDiscreteDistribution::incompleteGamma(double x, double alpha, double lga) {
  // AS32 (Bhattacharjee 1970): series below the mean, continued fraction above.
  const double tol = 1e-10, big = 1e60;
  if (x == 0.) return 0.;
  if (x < 0. || alpha <= 0.) return -1.;
  const double factor = std::exp(alpha * std::log(x) - x - lga);
  if (x <= 1. || x < alpha) {
    double sum = 1., term = 1., den = alpha;
    do {
      den += 1.;
      term *= x / den;
      sum += term;
    } while (term > tol);
    return sum * factor / alpha;
  }
  double a = 1. - alpha, b = a + x + 1., n = 0.;
  double p0 = 1., p1 = x, p2 = x + 1., p3 = x * b;
  double cf = p2 / p3;
  for (;;) {
    a += 1.;
    b += 2.;
    n += 1.;
    const double an = a * n;
    const double p4 = b * p2 - an * p0;
    const double p5 = b * p3 - an * p1;
    if (p5 != 0.) {
      const double rn = p4 / p5;
      const double dif = std::fabs(cf - rn);
      if (dif <= tol && dif <= tol * rn) return 1. - factor * cf;
      cf = rn;
    }
    p0 = p2;
    p1 = p3;
    p2 = p4;
    p3 = p5;
    if (std::fabs(p4) >= big) {
      p0 /= big;
      p1 /= big;
      p2 /= big;
      p3 /= big;
    }
  }
}

double GammaDiscreteDistribution::qChisq(double prob, double v) {
  // AS91 (Best & Roberts 1975): starting approximation, then a 7-term Taylor
  // correction iterated to relative change 0.5e-6.
  const double eps = .5e-6, ln2 = .6931471805;
  if (prob < 1e-6) return 0.;
  if (prob > 1. - 1e-6) return 9999.;
  if (v <= 0.) return -1.;
  const double g = lnGamma(v / 2.);
  const double xx = v / 2., c = xx - 1.;
  double ch;
  if (v < -1.24 * std::log(prob)) {
    ch = std::pow(prob * xx * std::exp(g + xx * ln2), 1. / xx);
    if (ch < eps) return ch;
  } else if (v <= .32) {
    ch = 0.4;
    const double a = std::log(1. - prob);
    double q;
    do {
      q = ch;
      const double p1 = 1. + ch * (4.67 + ch);
      const double p2 = ch * (6.73 + ch * (6.66 + ch));
      const double t = -0.5 + (4.67 + 2. * ch) / p1 - (6.73 + ch * (13.32 + 3. * ch)) / p2;
      ch -= (1. - std::exp(a + g + .5 * ch + c * ln2) * p2 / p1) / t;
    } while (std::fabs(q / ch - 1.) > .01);
  } else {
    // Wilson-Hilferty start from the normal quantile (AS111)
    const double pl = prob < 0.5 ? prob : 1. - prob;
    const double y = std::sqrt(std::log(1. / (pl * pl)));
    double z = y + ((((y * -.453642210148e-4 + -.0204231210245) * y + -.342242088547) * y + -1.) * y +
                    -.322232431088) /
                       ((((y * .0038560700634 + .103537752850) * y + .531103462366) * y + .588581570495) * y +
                        .0993484626060);
    if (prob < 0.5) z = -z;
    const double p1 = 0.222222 / v;
    ch = v * std::pow(z * std::sqrt(p1) + 1. - p1, 3.);
    if (ch > 2.2 * v + 6.) ch = -2. * (std::log(1. - prob) - c * std::log(.5 * ch) + g);
  }
  double q;
  do {
    q = ch;
    const double p1 = .5 * ch;
    const double ig = incompleteGamma(p1, xx, g);
    if (ig < 0.) return -1.;
    const double t = (prob - ig) * std::exp(xx * ln2 + g + p1 - c * std::log(ch));
    const double b = t / ch;
    const double a = 0.5 * t - b * c;
    const double s1 = (210. + a * (140. + a * (105. + a * (84. + a * (70. + 60. * a))))) / 420.;
    const double s2 = (420. + a * (735. + a * (966. + a * (1141. + 1278. * a)))) / 2520.;
    const double s3 = (210. + a * (462. + a * (707. + 932. * a))) / 2520.;
    const double s4 = (252. + a * (672. + 1182. * a) + c * (294. + a * (889. + 1740. * a))) / 5040.;
    const double s5 = (84. + 264. * a + c * (175. + 606. * a)) / 2520.;
    const double s6 = (120. + c * (346. + 127. * c)) / 5040.;
    ch += t * (1. + 0.5 * t * s1 - b * c * (s1 - b * (s2 - b * (s3 - b * (s4 - b * (s5 - b * s6))))));
  } while (std::fabs(q / ch - 1.) > eps);
  return ch;
}

GammaDiscreteDistribution::GammaDiscreteDistribution(size_t n, double alpha, double beta, const std::string& prefix)
    : DiscreteDistribution(prefix), n_(n) {
  addParameter_(Parameter(prefix + "alpha", alpha, std::make_shared<IntervalConstraint>(0.0001, 1e6, true, true)));
  addParameter_(Parameter(prefix + "beta", beta, std::make_shared<IntervalConstraint>(0.0001, 1e6, true, true)));
  discretize();
}

void GammaDiscreteDistribution::discretize() {
  const double alpha = getParameterValue("alpha");
  const double beta = hasParameter("beta") ? getParameterValue("beta") : alpha;
  values_.assign(n_, 0.);
  probs_.assign(n_, 1. / (double)n_);
  if (n_ == 1) {
    values_[0] = alpha / beta;
    return;
  }
  const double lgA1 = lnGamma(alpha + 1.);
  double prev = 0.;  // Expectation(0)
  for (size_t i = 0; i + 1 < n_; ++i) {
    const double bound = qChisq((double)(i + 1) / (double)n_, 2. * alpha) / (2. * beta);
    const double cur = incompleteGamma(beta * bound, alpha + 1., lgA1) * alpha / beta;
    values_[i] = (cur - prev) * (double)n_;
    prev = cur;
  }
  values_[n_ - 1] = (alpha / beta - prev) * (double)n_;
}

GammaDiscreteRateDistribution::GammaDiscreteRateDistribution(size_t n, double alpha)
    : GammaDiscreteDistribution(n, alpha, alpha, "Gamma.") {
  // beta is tied to alpha (mean rate 1): only alpha is a free parameter
  parameters_.deleteParameter("Gamma.beta");
  discretize();
}

void GammaDiscreteRateDistribution::fireParameterChanged(const ParameterList&) { discretize(); }

}  // namespace bpp

namespace bpp {

// ---------------------------------------------------------------------------
// General real eigen-solver (non-reversible generators).
// ---------------------------------------------------------------------------
namespace {
typedef std::complex<double> cd;

// Solve M x = b in place (complex LU with partial pivoting); a zero pivot is replaced by
// `tiny` (inverse iteration wants the near-singular solve).
void complexSolve(size_t n, std::vector<cd> M, std::vector<cd>& b, double tiny) {
  std::vector<size_t> piv(n);
  for (size_t k = 0; k < n; k++) {
    size_t p = k;
    for (size_t i = k + 1; i < n; i++)
      if (std::abs(M[i * n + k]) > std::abs(M[p * n + k])) p = i;
    if (p != k) {
      for (size_t j = 0; j < n; j++) std::swap(M[k * n + j], M[p * n + j]);
      std::swap(b[k], b[p]);
    }
    if (std::abs(M[k * n + k]) < tiny) M[k * n + k] = tiny;
    for (size_t i = k + 1; i < n; i++) {
      const cd f = M[i * n + k] / M[k * n + k];
      if (f == cd(0.)) continue;
      for (size_t j = k; j < n; j++) M[i * n + j] -= f * M[k * n + j];
      b[i] -= f * b[k];
    }
  }
  for (size_t k = n; k-- > 0;) {
    cd s = b[k];
    for (size_t j = k + 1; j < n; j++) s -= M[k * n + j] * b[j];
    b[k] = s / M[k * n + k];
  }
}

// Eigenvalues of the n x n complex matrix H (row-major, overwritten): Householder reduction
// to upper Hessenberg form, then single-shift QR with Wilkinson shifts and deflation.
bool complexEigenvalues(size_t n, std::vector<cd>& H, std::vector<cd>& w) {
  auto h = [&](size_t i, size_t j) -> cd& { return H[i * n + j]; };
  for (size_t k = 0; k + 2 < n; k++) {
    double norm = 0.;
    for (size_t i = k + 1; i < n; i++) norm += std::norm(h(i, k));
    norm = std::sqrt(norm);
    if (norm == 0.) continue;
    std::vector<cd> v(n, 0.);
    const cd x0 = h(k + 1, k);
    const cd alpha = (std::abs(x0) > 0. ? -x0 / std::abs(x0) : cd(-1.)) * norm;
    for (size_t i = k + 1; i < n; i++) v[i] = h(i, k);
    v[k + 1] -= alpha;
    double vn = 0.;
    for (size_t i = k + 1; i < n; i++) vn += std::norm(v[i]);
    if (vn == 0.) continue;
    // H <- (I - 2 v v^H / |v|^2) H (I - 2 v v^H / |v|^2)
    for (size_t j = 0; j < n; j++) {
      cd s = 0.;
      for (size_t i = k + 1; i < n; i++) s += std::conj(v[i]) * h(i, j);
      s *= 2. / vn;
      for (size_t i = k + 1; i < n; i++) h(i, j) -= v[i] * s;
    }
    for (size_t i = 0; i < n; i++) {
      cd s = 0.;
      for (size_t j = k + 1; j < n; j++) s += h(i, j) * v[j];
      s *= 2. / vn;
      for (size_t j = k + 1; j < n; j++) h(i, j) -= s * std::conj(v[j]);
    }
    for (size_t i = k + 2; i < n; i++) h(i, k) = 0.;
  }
  const double eps = 2.220446049250313e-16;
  size_t hi = n ? n - 1 : 0;
  int iter = 0, total = 0;
  while (n && hi > 0) {
    size_t l = hi;
    while (l > 0) {
      const double s = std::abs(h(l - 1, l - 1)) + std::abs(h(l, l));
      if (std::abs(h(l, l - 1)) <= eps * (s > 0. ? s : 1.)) {
        h(l, l - 1) = 0.;
        break;
      }
      l--;
    }
    if (l == hi) {  // h(hi, hi) is an eigenvalue
      hi--;
      iter = 0;
      continue;
    }
    if (++total > 200 * (int)n) return false;
    const cd a = h(hi - 1, hi - 1), b = h(hi - 1, hi), c = h(hi, hi - 1), d = h(hi, hi);
    cd mu;
    if (++iter % 12 == 0) {
      mu = d + std::abs(c);  // exceptional shift
    } else {
      const cd tr = a + d, disc = std::sqrt(tr * tr / 4. - (a * d - b * c));
      const cd m1 = tr / 2. + disc, m2 = tr / 2. - disc;
      mu = std::abs(m1 - d) < std::abs(m2 - d) ? m1 : m2;
    }
    for (size_t j = l; j <= hi; j++) h(j, j) -= mu;
    std::vector<cd> cs(hi - l), sn(hi - l);
    for (size_t k = l; k < hi; k++) {  // H - mu I = Q R (Givens on rows k, k+1)
      const cd x = h(k, k), y = h(k + 1, k);
      const double r = std::sqrt(std::norm(x) + std::norm(y));
      const cd cc = r > 0. ? x / r : cd(1.), ss = r > 0. ? y / r : cd(0.);
      cs[k - l] = cc;
      sn[k - l] = ss;
      for (size_t j = k; j < n; j++) {
        const cd u = h(k, j), v = h(k + 1, j);
        h(k, j) = std::conj(cc) * u + std::conj(ss) * v;
        h(k + 1, j) = -ss * u + cc * v;
      }
    }
    for (size_t k = l; k < hi; k++) {  // R Q (the rotations' adjoints on columns k, k+1)
      const cd cc = cs[k - l], ss = sn[k - l];
      const size_t rmax = std::min(k + 2, hi);
      for (size_t i = 0; i <= rmax; i++) {
        const cd u = h(i, k), v = h(i, k + 1);
        h(i, k) = u * cc + v * ss;
        h(i, k + 1) = -u * std::conj(ss) + v * std::conj(cc);
      }
    }
    for (size_t j = l; j <= hi; j++) h(j, j) += mu;
  }
  w.resize(n);
  for (size_t i = 0; i < n; i++) w[i] = h(i, i);
  return true;
}
}  // namespace

bool invertMatrix(size_t n, const std::vector<double>& A, std::vector<double>& Ainv) {
  std::vector<double> M(A);
  Ainv.assign(n * n, 0.);
  for (size_t i = 0; i < n; i++) Ainv[i * n + i] = 1.;
  double amax = 0.;
  for (double x : A) amax = std::max(amax, std::fabs(x));
  for (size_t k = 0; k < n; k++) {
    size_t p = k;
    for (size_t i = k + 1; i < n; i++)
      if (std::fabs(M[i * n + k]) > std::fabs(M[p * n + k])) p = i;
    if (!(std::fabs(M[p * n + k]) > 1e-14 * amax)) return false;
    if (p != k)
      for (size_t j = 0; j < n; j++) {
        std::swap(M[k * n + j], M[p * n + j]);
        std::swap(Ainv[k * n + j], Ainv[p * n + j]);
      }
    const double piv = M[k * n + k];
    for (size_t j = 0; j < n; j++) {
      M[k * n + j] /= piv;
      Ainv[k * n + j] /= piv;
    }
    for (size_t i = 0; i < n; i++) {
      if (i == k) continue;
      const double f = M[i * n + k];
      if (f == 0.) continue;
      for (size_t j = 0; j < n; j++) {
        M[i * n + j] -= f * M[k * n + j];
        Ainv[i * n + j] -= f * Ainv[k * n + j];
      }
    }
  }
  return true;
}

bool generalEigen(size_t n, const std::vector<double>& A, std::vector<double>& wr, std::vector<double>& wi,
                  std::vector<double>& V) {
  std::vector<cd> H(A.begin(), A.end()), w;
  if (!complexEigenvalues(n, H, w)) return false;
  double anorm = 0.;
  for (double x : A) anorm = std::max(anorm, std::fabs(x));
  if (anorm == 0.) anorm = 1.;
  const double imTol = 1e-10 * anorm;
  for (cd& z : w)
    if (std::fabs(z.imag()) <= imTol) z = cd(z.real(), 0.);
  // order: the Schur diagonal's, each complex pair as (a + ib, a - ib), b > 0
  std::vector<char> used(n, 0);
  std::vector<cd> order;
  for (size_t i = 0; i < n; i++) {
    if (used[i]) continue;
    used[i] = 1;
    if (w[i].imag() == 0.) {
      order.push_back(w[i]);
      continue;
    }
    size_t best = n;
    for (size_t j = 0; j < n; j++)
      if (!used[j] && w[j].imag() != 0. &&
          (best == n || std::abs(w[j] - std::conj(w[i])) < std::abs(w[best] - std::conj(w[i]))))
        best = j;
    if (best == n) return false;  // an unpaired complex eigenvalue of a real matrix
    used[best] = 1;
    // the pair's two computed members, averaged into an exact conjugate pair
    const cd zm(0.5 * (w[i].real() + w[best].real()), 0.5 * (std::fabs(w[i].imag()) + std::fabs(w[best].imag())));
    order.push_back(zm);
    order.push_back(std::conj(zm));
  }
  wr.assign(n, 0.);
  wi.assign(n, 0.);
  V.assign(n * n, 0.);
  std::vector<std::vector<cd> > found;  // eigenvectors so far (repeated eigenvalues deflate)
  std::vector<cd> foundVal;
  unsigned seed = 12345;
  auto rnd = [&]() {
    seed = seed * 1103515245u + 12345u;
    return 0.5 + (double)((seed >> 8) & 0xffff) / 65536.;
  };
  for (size_t k = 0; k < n; k++) {
    const cd lam = order[k];
    wr[k] = lam.real();
    wi[k] = lam.imag();
    if (lam.imag() < 0.) continue;  // second of a pair: its columns were written with the first
    std::vector<cd> M(n * n);
    for (size_t i = 0; i < n; i++)
      for (size_t j = 0; j < n; j++) M[i * n + j] = cd(A[i * n + j]) - (i == j ? lam : cd(0.));
    std::vector<cd> x(n);
    for (size_t i = 0; i < n; i++) x[i] = cd(rnd(), 0.);
    for (int it = 0; it < 4; it++) {
      complexSolve(n, M, x, 1e-14 * anorm);
      for (size_t f = 0; f < found.size(); f++) {  // deflate against vectors of the same eigenvalue
        if (std::abs(foundVal[f] - lam) > 1e-8 * anorm) continue;
        cd dot = 0.;
        double nn = 0.;
        for (size_t i = 0; i < n; i++) {
          dot += std::conj(found[f][i]) * x[i];
          nn += std::norm(found[f][i]);
        }
        for (size_t i = 0; i < n; i++) x[i] -= dot / nn * found[f][i];
      }
      size_t p = 0;
      for (size_t i = 1; i < n; i++)
        if (std::abs(x[i]) > std::abs(x[p])) p = i;
      const cd s = x[p];
      if (std::abs(s) == 0. || !std::isfinite(std::abs(s))) return false;
      for (size_t i = 0; i < n; i++) x[i] /= s;  // largest component 1 (real for a real eigenvalue)
    }
    found.push_back(x);
    foundVal.push_back(lam);
    if (lam.imag() == 0.) {
      for (size_t i = 0; i < n; i++) V[i * n + k] = x[i].real();
    } else {
      if (k + 1 >= n) return false;
      for (size_t i = 0; i < n; i++) {
        V[i * n + k] = x[i].real();
        V[i * n + k + 1] = x[i].imag();
      }
    }
  }
  return true;
}

}  // namespace bpp
