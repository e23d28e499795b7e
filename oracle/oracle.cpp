// oracle/oracle.cpp -- CPU restatement of bpp-phyl's Felsenstein-pruning hot path.
//
// TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this library, and only as the checker / the timed
// CPU baseline.  The product path (libplk + the Bio++ host mirror) never links it.
//
// The reference (bpp-phyl 2.4.1 fork) cannot be compiled here: it needs bpp-core
// 2.4.1 and bpp-seq 12.0.0, neither of which is on the filesystem.
// This file therefore restates, with the reference's own data layout (nested
// std::vector [site][class][state]) and loop order, the functions below.  Every
// function cites the reference file:line it follows (paths relative to
// /root/reference/src/Bpp/Phyl/).  Third-party arithmetic that lives in bpp-core
// (discrete Gamma, lnGamma, incomplete gamma, chi2 quantile) is restated from the
// published algorithms bpp-core uses (Pike & Hill 1966; Bhattacharjee 1970 AS32;
// Best & Roberts 1975 AS91; Beasley & Springer 1977 AS111).
//
// Pinning: T92+Gamma4 on the test_likelihood.cpp inputs must give the reference
// golden 85.030942031997312824 (test/test_likelihood.cpp:108) and the clock case
// 94.3957 (test/test_likelihood_clock.cpp:115); see tests/test_oracle_golden.py.
//
// Compiled with g++ -std=c++11 -O2 -g, the reference's RelWithDebInfo default
// (CMakeLists.txt:12-17); single-threaded like the reference.

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

typedef std::vector<double> Vdouble;
typedef std::vector<Vdouble> VVdouble;
typedef std::vector<VVdouble> VVVdouble;

namespace {

// ---------------------------------------------------------------------------
// bpp-core RandomTools restatements (used by GammaDiscreteDistribution,
// M/RateDistribution/GammaDiscreteRateDistribution.h:48-60).
// ---------------------------------------------------------------------------

// ln Gamma(x): Pike & Hill (1966) with Stirling series after shifting x >= 7.
double lnGamma(double alpha) {
  double x = alpha, f = 0., z;
  if (x < 7.) {
    f = 1.;
    z = x - 1.;
    while (++z < 7.) f *= z;
    x = z;
    f = -std::log(f);
  }
  z = 1. / (x * x);
  return f + (x - 0.5) * std::log(x) - x + .918938533204673 +
         (((-.000595238095238 * z + .000793650793651) * z - .002777777777778) * z +
          .083333333333333) / x;
}

// Regularised lower incomplete gamma I(x, p), AS32 (series for x<=1 or x<p,
// continued fraction otherwise), accuracy 1e-10 as in bpp-core.
double incompleteGamma(double x, double p, double g) {
  const double accurate = 1e-10, overflow = 1e60;
  double factor, gin, rn, a, b, an, dif, term, pn[6];
  if (x == 0.) return 0.;
  if (x < 0. || p <= 0.) return -1.;
  factor = std::exp(p * std::log(x) - x - g);
  if (x > 1. && x >= p) {
    // continued fraction
    a = 1. - p;
    b = a + x + 1.;
    term = 0.;
    pn[0] = 1.;
    pn[1] = x;
    pn[2] = x + 1.;
    pn[3] = x * b;
    gin = pn[2] / pn[3];
    for (;;) {
      a += 1.;
      b += 2.;
      term += 1.;
      an = a * term;
      for (int i = 0; i < 2; i++) pn[i + 4] = b * pn[i + 2] - an * pn[i];
      if (pn[5] != 0.) {
        rn = pn[4] / pn[5];
        dif = std::fabs(gin - rn);
        if (dif <= accurate && dif <= accurate * rn) {
          return 1. - factor * gin;
        }
        gin = rn;
      }
      for (int i = 0; i < 4; i++) pn[i] = pn[i + 2];
      if (std::fabs(pn[4]) >= overflow)
        for (int i = 0; i < 4; i++) pn[i] /= overflow;
    }
  }
  // series expansion
  gin = 1.;
  term = 1.;
  rn = p;
  do {
    rn += 1.;
    term *= x / rn;
    gin += term;
  } while (term > accurate);
  return gin * factor / p;
}

// Standard normal quantile, AS111 (Beasley & Springer 1977) rational form.
double qNorm(double prob) {
  const double a0 = -.322232431088, a1 = -1., a2 = -.342242088547, a3 = -.0204231210245;
  const double a4 = -.453642210148e-4, b0 = .0993484626060, b1 = .588581570495;
  const double b2 = .531103462366, b3 = .103537752850, b4 = .0038560700634;
  double p = prob, p1 = (p < 0.5 ? p : 1. - p);
  if (p1 < 1e-20) return -9999.;
  double y = std::sqrt(std::log(1. / (p1 * p1)));
  double z = y + ((((y * a4 + a3) * y + a2) * y + a1) * y + a0) /
                     ((((y * b4 + b3) * y + b2) * y + b1) * y + b0);
  return p < 0.5 ? -z : z;
}

// Chi-square quantile, AS91 (Best & Roberts 1975), convergence e = 0.5e-6.
double qChisq(double prob, double v) {
  const double e = .5e-6, aa = .6931471805, small = 1e-6;
  double p = prob, g, xx, c, ch, a = 0., q = 0., p1 = 0., p2 = 0., t = 0., x = 0., b = 0.;
  double s1, s2, s3, s4, s5, s6;
  if (p < small) return 0.;
  if (p > 1. - small) return 9999.;
  if (v <= 0.) return -1.;
  g = lnGamma(v / 2.);
  xx = v / 2.;
  c = xx - 1.;
  if (v < -1.24 * std::log(p)) {
    ch = std::pow((p * xx * std::exp(g + xx * aa)), 1. / xx);
    if (ch - e < 0.) return ch;
  } else if (v <= .32) {
    ch = 0.4;
    a = std::log(1. - p);
    do {
      q = ch;
      p1 = 1. + ch * (4.67 + ch);
      p2 = ch * (6.73 + ch * (6.66 + ch));
      t = -0.5 + (4.67 + 2. * ch) / p1 - (6.73 + ch * (13.32 + 3. * ch)) / p2;
      ch -= (1. - std::exp(a + g + .5 * ch + c * aa) * p2 / p1) / t;
    } while (std::fabs(q / ch - 1.) - .01 > 0.);
  } else {
    x = qNorm(p);
    p1 = 0.222222 / v;
    ch = v * std::pow((x * std::sqrt(p1) + 1. - p1), 3.0);
    if (ch > 2.2 * v + 6.) ch = -2. * (std::log(1. - p) - c * std::log(.5 * ch) + g);
  }
  do {
    q = ch;
    p1 = .5 * ch;
    t = incompleteGamma(p1, xx, g);
    if (t < 0.) return -1.;
    p2 = p - t;
    t = p2 * std::exp(xx * aa + g + p1 - c * std::log(ch));
    b = t / ch;
    a = 0.5 * t - b * c;
    s1 = (210. + a * (140. + a * (105. + a * (84. + a * (70. + 60. * a))))) / 420.;
    s2 = (420. + a * (735. + a * (966. + a * (1141. + 1278. * a)))) / 2520.;
    s3 = (210. + a * (462. + a * (707. + 932. * a))) / 2520.;
    s4 = (252. + a * (672. + 1182. * a) + c * (294. + a * (889. + 1740. * a))) / 5040.;
    s5 = (84. + 264. * a + c * (175. + 606. * a)) / 2520.;
    s6 = (120. + c * (346. + 127. * c)) / 5040.;
    ch += t * (1. + 0.5 * t * s1 - b * c * (s1 - b * (s2 - b * (s3 - b * (s4 - b * (s5 - b * s6))))));
  } while (std::fabs(q / ch - 1.) > e);
  return ch;
}

double qGamma(double prob, double alpha, double beta) { return qChisq(prob, 2. * alpha) / (2. * beta); }
double pGamma(double x, double alpha, double beta) {
  if (std::isinf(x)) return 1.;
  return incompleteGamma(beta * x, alpha, lnGamma(alpha));
}

// ---------------------------------------------------------------------------
// Substitution models
// ---------------------------------------------------------------------------

// Symmetric Jacobi eigen-decomposition (cyclic sweeps).  A is n x n row-major,
// destroyed; on exit d holds eigenvalues, U (row-major) the eigenvectors as
// columns.  Independent of the product's Householder/QL solver on purpose.
void jacobiEigen(int n, std::vector<double>& A, std::vector<double>& d, std::vector<double>& U) {
  U.assign((size_t)n * n, 0.);
  for (int i = 0; i < n; i++) U[(size_t)i * n + i] = 1.;
  for (int sweep = 0; sweep < 100; sweep++) {
    double off = 0.;
    for (int p = 0; p < n; p++)
      for (int q = p + 1; q < n; q++) off += A[(size_t)p * n + q] * A[(size_t)p * n + q];
    if (off < 1e-300) break;
    for (int p = 0; p < n; p++) {
      for (int q = p + 1; q < n; q++) {
        double apq = A[(size_t)p * n + q];
        if (std::fabs(apq) < 1e-300) continue;
        double app = A[(size_t)p * n + p], aqq = A[(size_t)q * n + q];
        double theta = (aqq - app) / (2. * apq);
        double t = (theta >= 0. ? 1. : -1.) / (std::fabs(theta) + std::sqrt(theta * theta + 1.));
        double c = 1. / std::sqrt(t * t + 1.), s = t * c;
        for (int k = 0; k < n; k++) {
          double akp = A[(size_t)k * n + p], akq = A[(size_t)k * n + q];
          A[(size_t)k * n + p] = c * akp - s * akq;
          A[(size_t)k * n + q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; k++) {
          double apk = A[(size_t)p * n + k], aqk = A[(size_t)q * n + k];
          A[(size_t)p * n + k] = c * apk - s * aqk;
          A[(size_t)q * n + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; k++) {
          double ukp = U[(size_t)k * n + p], ukq = U[(size_t)k * n + q];
          U[(size_t)k * n + p] = c * ukp - s * ukq;
          U[(size_t)k * n + q] = s * ukp + c * ukq;
        }
      }
    }
  }
  d.resize(n);
  for (int i = 0; i < n; i++) d[i] = A[(size_t)i * n + i];
}

}  // namespace

extern "C" {

// Discrete Gamma(alpha, beta=alpha) with mean-of-category values and equal
// probabilities -- bpp-core AbstractDiscreteDistribution::discretize as used by
// M/RateDistribution/GammaDiscreteRateDistribution.h:52-56.
int orc_gamma_rates(int n, double alpha, double* rates, double* probs) {
  if (n < 1 || alpha <= 0.) return -1;
  if (n == 1) {
    rates[0] = 1.;
    probs[0] = 1.;
    return 0;
  }
  const double beta = alpha;
  std::vector<double> bounds(n - 1);
  double ec = 1. / n;
  for (int i = 1; i < n; i++) bounds[i - 1] = qGamma(i * ec, alpha, beta);
  // Expectation(x) = pGamma(x, alpha + 1, beta) * alpha / beta
  double a = 0.;
  for (int i = 0; i < n - 1; i++) {
    double b = pGamma(bounds[i], alpha + 1., beta) * alpha / beta;
    rates[i] = (b - a) * n;
    a = b;
  }
  rates[n - 1] = (alpha / beta - a) * n;
  for (int i = 0; i < n; i++) probs[i] = 1. / n;
  return 0;
}

// T92 closed-form P(t) -- M/Nucleotide/T92.cpp:81-110 (parameters) and :355-386.
void orc_t92_pij(double kappa, double theta, double t, double* P) {
  double piA = (1. - theta) / 2., piC = theta / 2., piG = theta / 2., piT = (1. - theta) / 2.;
  double k = (kappa + 1.) / 2.;
  double r = 2. / (1. + 2. * theta * kappa - 2. * theta * theta * kappa);
  double l = 1. * r * t;  // rate_ == 1
  double e1 = std::exp(-l), e2 = std::exp(-k * l);
  double p[16] = {
      piA * (1. + e1) + theta * e2,        piC * (1. - e1), piG * (1. + e1) - theta * e2,        piT * (1. - e1),
      piA * (1. - e1), piC * (1. + e1) + (1. - theta) * e2, piG * (1. - e1), piT * (1. + e1) - (1. - theta) * e2,
      piA * (1. + e1) - (1. - theta) * e2, piC * (1. - e1), piG * (1. + e1) + (1. - theta) * e2, piT * (1. - e1),
      piA * (1. - e1), piC * (1. + e1) - theta * e2,        piG * (1. - e1), piT * (1. + e1) + theta * e2};
  std::memcpy(P, p, sizeof(p));
}

void orc_t92_freqs(double theta, double* pi) {
  pi[0] = (1. - theta) / 2.;
  pi[1] = theta / 2.;
  pi[2] = theta / 2.;
  pi[3] = (1. - theta) / 2.;
}

// Reversible generator from exchangeabilities: Q_ij = S_ij * pi_j (i != j),
// diagonal = -row sum, normalised so that -sum_i pi_i Q_ii = 1.
// M/AbstractSubstitutionModel.cpp:694-703 (hadamardMult, setDiagonal, normalize)
// with :645-690 (getScale / setScale).
void orc_reversible_generator(int S, const double* exch, const double* pi, double* Q) {
  for (int i = 0; i < S; i++)
    for (int j = 0; j < S; j++) Q[i * S + j] = exch[i * S + j] * pi[j];
  for (int i = 0; i < S; i++) {
    double lambda = 0.;
    for (int j = 0; j < S; j++)
      if (j != i) lambda += Q[i * S + j];
    Q[i * S + i] = -lambda;
  }
  double scale = 0.;
  for (int i = 0; i < S; i++) scale += Q[i * S + i] * pi[i];
  scale = -scale;
  for (int i = 0; i < S * S; i++) Q[i] *= 1. / scale;
}

// GTR exchangeabilities and frequencies -- M/Nucleotide/GTR.cpp:84-124.
void orc_gtr_model(double a, double b, double c, double d, double e, double theta, double theta1,
                   double theta2, double* exch, double* pi) {
  double piA = theta1 * (1. - theta), piC = (1. - theta2) * theta, piG = theta2 * theta,
         piT = (1. - theta1) * (1. - theta);
  double p = 2. * (a * piC * piT + b * piA * piT + c * piG * piT + d * piA * piC + e * piC * piG + piA * piG);
  pi[0] = piA;
  pi[1] = piC;
  pi[2] = piG;
  pi[3] = piT;
  double E[16] = {(-b * piT - piG - d * piC) / (piA * p), d / p, 1. / p, b / p,
                  d / p, (-a * piT - e * piG - d * piA) / (piC * p), e / p, a / p,
                  1. / p, e / p, (-c * piT - e * piC - piA) / (piG * p), c / p,
                  b / p, a / p, c / p, (-c * piG - a * piC - b * piA) / (piT * p)};
  std::memcpy(exch, E, sizeof(E));
}

// P(t) = exp(Q t) for a reversible generator: symmetrise B = D^1/2 Q D^-1/2,
// Jacobi-diagonalise, P = D^-1/2 U exp(L t) U^T D^1/2.  States with pi == 0 and
// a null generator row/column (codon stop states) are stripped and get identity
// rows, as M/AbstractSubstitutionModel.cpp:184-273 does.  Equivalent to the
// reference's V diag(exp(lambda t)) V^-1 (:436-438).
int orc_reversible_pij(int S, const double* Q, const double* pi, double t, double* P) {
  std::vector<int> live;
  for (int i = 0; i < S; i++) {
    bool null = std::fabs(Q[i * S + i]) < 1e-12;
    for (int j = 0; j < S && null; j++)
      if (std::fabs(Q[j * S + i]) >= 1e-12) null = false;
    if (!null) live.push_back(i);
  }
  int n = (int)live.size();
  std::vector<double> B((size_t)n * n), d, U;
  for (int a = 0; a < n; a++)
    for (int b = 0; b < n; b++) {
      int i = live[a], j = live[b];
      B[(size_t)a * n + b] = std::sqrt(pi[i]) * Q[i * S + j] / std::sqrt(pi[j]);
    }
  // exact symmetrisation against rounding
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++) {
      double m = 0.5 * (B[(size_t)a * n + b] + B[(size_t)b * n + a]);
      B[(size_t)a * n + b] = B[(size_t)b * n + a] = m;
    }
  jacobiEigen(n, B, d, U);
  for (int i = 0; i < S * S; i++) P[i] = 0.;
  for (int i = 0; i < S; i++) P[i * S + i] = 1.;
  if (t == 0.) return 0;
  std::vector<double> ex(n);
  for (int k = 0; k < n; k++) ex[k] = std::exp(d[k] * t);
  for (int a = 0; a < n; a++)
    for (int b = 0; b < n; b++) {
      double s = 0.;
      for (int k = 0; k < n; k++) s += U[(size_t)a * n + k] * ex[k] * U[(size_t)b * n + k];
      int i = live[a], j = live[b];
      P[i * S + j] = s * std::sqrt(pi[j]) / std::sqrt(pi[i]);
    }
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Tree likelihood: DRASRTreeLikelihoodData + RHomogeneousTreeLikelihood
// ---------------------------------------------------------------------------

namespace {

struct OTree {
  int n_nodes, root;
  std::vector<std::vector<int> > sons;
  std::vector<int> leaf_row;  // row in the state matrix, -1 for internal nodes
};

// Site pattern compression: sort columns by content, merge identical ones
// (SitePatterns.cpp:51-100).  cols[i] is the column string of site i.
struct Patterns {
  std::vector<size_t> sites;    // representative original site of each pattern
  std::vector<unsigned> weights;
  std::vector<size_t> indices;  // site -> pattern
};

Patterns makePatterns(const std::vector<std::string>& cols) {
  Patterns P;
  size_t n = cols.size();
  std::vector<size_t> order(n);
  for (size_t i = 0; i < n; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return cols[a] < cols[b]; });
  P.indices.resize(n);
  if (n == 0) return P;
  P.indices[order[0]] = 0;
  P.sites.push_back(order[0]);
  P.weights.push_back(1);
  size_t cur = 0;
  for (size_t k = 1; k < n; k++) {
    if (cols[order[k]] == cols[P.sites[cur]]) {
      P.weights[cur]++;
    } else {
      P.sites.push_back(order[k]);
      P.weights.push_back(1);
      cur++;
    }
    P.indices[order[k]] = cur;
  }
  return P;
}

struct OLik {
  const OTree* tree;
  int S, C;
  std::vector<VVVdouble> lik;                              // per node [site][class][state]
  std::vector<std::map<int, std::vector<size_t> > > links;  // patternLinks_[node][son]
  std::vector<std::vector<int> > nscale;                   // per node per site (scaling only)
  std::vector<size_t> rootLinks;
  std::vector<unsigned> rootWeights;
  std::map<int, VVVdouble> pxy;
  bool scaling;
};

// Leaves of the subtree in getLeaves order (depth-first, sons in order).
void subtreeLeaves(const OTree& t, int node, std::vector<int>& out) {
  if (t.sons[node].empty()) {
    out.push_back(node);
    return;
  }
  for (size_t i = 0; i < t.sons[node].size(); i++) subtreeLeaves(t, t.sons[node][i], out);
}

void resetArray(VVVdouble& a, size_t nSites, int C, int S) {
  a.resize(nSites);
  for (size_t i = 0; i < nSites; i++) {
    a[i].resize(C);
    for (int c = 0; c < C; c++) a[i][c].assign(S, 1.);
  }
}

int initLeaf(OLik& L, int node, const std::vector<int>& siteIdx, const int* states, int nSitesAll,
             int nCodes, const double* initValues) {
  VVVdouble& a = L.lik[node];
  int row = L.tree->leaf_row[node];
  for (size_t i = 0; i < siteIdx.size(); i++) {
    int state = states[(size_t)row * nSitesAll + siteIdx[i]];
    // AbstractTransitionModel::getInitValue throws BadIntException for gaps /
    // unknown codes (M/AbstractSubstitutionModel.cpp:98-112).
    if (state < 0 || state >= nCodes) return -2;
    for (int c = 0; c < L.C; c++)
      for (int s = 0; s < L.S; s++) a[i][c][s] = initValues[(size_t)state * L.S + s];
  }
  return 0;
}

// Flat initialisation: DRASRTreeLikelihoodData.cpp:120-214 -- every node holds
// the root's distinct patterns, links are identities.
int initFlat(OLik& L, int node, const std::vector<int>& siteIdx, const int* states, int nSitesAll,
             int nCodes, const double* initValues) {
  resetArray(L.lik[node], siteIdx.size(), L.C, L.S);
  if (L.tree->sons[node].empty()) return initLeaf(L, node, siteIdx, states, nSitesAll, nCodes, initValues);
  for (size_t l = 0; l < L.tree->sons[node].size(); l++) {
    int son = L.tree->sons[node][l];
    int rc = initFlat(L, son, siteIdx, states, nSitesAll, nCodes, initValues);
    if (rc) return rc;
    std::vector<size_t>& lk = L.links[node][son];
    lk.resize(siteIdx.size());
    for (size_t i = 0; i < siteIdx.size(); i++) lk[i] = i;
  }
  return 0;
}

// Per-subtree pattern compression: DRASRTreeLikelihoodData.cpp:218-332.
// siteIdx = original site of each row of the parent's (compressed) container.
// Returns the subtree's patterns (indices relative to the parent's rows).
int initWithPatterns(OLik& L, int node, const std::vector<int>& siteIdx, const int* states, int nSitesAll,
                     int nCodes, const double* initValues, Patterns& out) {
  std::vector<int> leaves;
  subtreeLeaves(*L.tree, node, leaves);
  std::vector<std::string> cols(siteIdx.size());
  for (size_t i = 0; i < siteIdx.size(); i++) {
    std::string& s = cols[i];
    s.resize(leaves.size() * sizeof(int));
    for (size_t k = 0; k < leaves.size(); k++) {
      int v = states[(size_t)L.tree->leaf_row[leaves[k]] * nSitesAll + siteIdx[i]];
      std::memcpy(&s[k * sizeof(int)], &v, sizeof(int));
    }
  }
  out = makePatterns(cols);
  std::vector<int> sub(out.sites.size());
  for (size_t i = 0; i < out.sites.size(); i++) sub[i] = siteIdx[out.sites[i]];
  resetArray(L.lik[node], sub.size(), L.C, L.S);
  if (L.tree->sons[node].empty()) return initLeaf(L, node, sub, states, nSitesAll, nCodes, initValues);
  for (size_t l = 0; l < L.tree->sons[node].size(); l++) {
    int son = L.tree->sons[node][l];
    Patterns sp;
    int rc = initWithPatterns(L, son, sub, states, nSitesAll, nCodes, initValues, sp);
    if (rc) return rc;
    L.links[node][son] = sp.indices;
  }
  return 0;
}

const double kScaleUp = 115792089237316195423570985008687907853269984665640564039457584007913129639936.;  // 2^256
const double kScaleThreshold = 1. / kScaleUp;                                                                 // 2^-256

// RHomogeneousTreeLikelihood::computeSubtreeLikelihood, L/RHomogeneousTreeLikelihood.cpp:802-863
// (identical to the NH twin L/RNonHomogeneousTreeLikelihood.cpp:1286-1350).
// The optional power-of-two rescaling (scaling == true) is a documented
// deviation: the reference has none and underflows on big trees.
void computeSubtreeLikelihood(OLik& L, int node) {
  const std::vector<int>& sons = L.tree->sons[node];
  if (sons.empty()) return;
  VVVdouble* likNode = &L.lik[node];
  size_t nbSites = likNode->size();
  for (size_t i = 0; i < nbSites; i++)
    for (int c = 0; c < L.C; c++)
      for (int x = 0; x < L.S; x++) (*likNode)[i][c][x] = 1.;
  if (L.scaling) L.nscale[node].assign(nbSites, 0);
  for (size_t l = 0; l < sons.size(); l++) {
    int son = sons[l];
    computeSubtreeLikelihood(L, son);
    VVVdouble* pxySon = &L.pxy[son];
    std::vector<size_t>* links = &L.links[node][son];
    VVVdouble* likSon = &L.lik[son];
    for (size_t i = 0; i < nbSites; i++) {
      VVdouble* likSon_i = &(*likSon)[(*links)[i]];
      VVdouble* likNode_i = &(*likNode)[i];
      for (int c = 0; c < L.C; c++) {
        Vdouble* likSon_i_c = &(*likSon_i)[c];
        Vdouble* likNode_i_c = &(*likNode_i)[c];
        VVdouble* pxySon_c = &(*pxySon)[c];
        for (int x = 0; x < L.S; x++) {
          Vdouble* pxySon_c_x = &(*pxySon_c)[x];
          double likelihood = 0;
          for (int y = 0; y < L.S; y++) likelihood += (*pxySon_c_x)[y] * (*likSon_i_c)[y];
          (*likNode_i_c)[x] *= likelihood;
        }
      }
      if (L.scaling && !L.tree->sons[son].empty()) L.nscale[node][i] += L.nscale[son][(*links)[i]];
    }
    // The rescale runs after every third son and after the last: the engine's ABI takes
    // at most three children per op (a polytomy is several ACCUMULATE ops, each ending
    // with the check), so a wide polytomy's running product is kept above 2^-256 the same way.
    if (L.scaling && ((l + 1) % 3 == 0 || l + 1 == sons.size())) {
      for (size_t i = 0; i < nbSites; i++) {
        double m = 0.;
        for (int c = 0; c < L.C; c++)
          for (int x = 0; x < L.S; x++) m = std::max(m, (*likNode)[i][c][x]);
        if (m > 0. && m < kScaleThreshold) {
          for (int c = 0; c < L.C; c++)
            for (int x = 0; x < L.S; x++) (*likNode)[i][c][x] *= kScaleUp;
          L.nscale[node][i] += 1;
        }
      }
    }
  }
}

// Root reduction: getLogLikelihood / getLogLikelihoodForASite /
// getLikelihoodForASiteForARateClass.
//  - homogeneous (nh == false), L/RHomogeneousTreeLikelihood.cpp:162-216: terms <= 0 are
//    dropped at both levels (the guards at :197-198 and :212-213);
//  - non-homogeneous (nh == true), L/RNonHomogeneousTreeLikelihood.cpp:168-233: every term
//    is added (getLikelihoodForASiteForARateClass :212-221 has no guard), and the site sum
//    l is clamped l < 0 -> 0 before the log (getLogLikelihoodForASite :198-208, clamp :206).
// Both sort the site values and sum from the largest (homogeneous :170-174, NH :168-180).
double rootLogLikForSite(const OLik& L, size_t site, const double* classProbs, const double* rootFreqs, bool nh) {
  size_t p = L.rootLinks[site];
  const VVdouble& la = L.lik[L.tree->root][p];
  double l = 0;
  for (int c = 0; c < L.C; c++) {
    double lc = 0;
    for (int s = 0; s < L.S; s++) {
      double li = la[c][s] * rootFreqs[s];
      if (nh || li > 0) lc += li;
    }
    double li = lc * classProbs[c];
    if (nh || li > 0) l += li;
  }
  if (nh && l < 0) l = 0;
  double r = std::log(l);
  if (L.scaling) r -= L.nscale[L.tree->root][p] * 256. * 0.69314718055994530942;
  return r;
}

}  // namespace

extern "C" {

// Full likelihood evaluation with the reference's data structures.
//   tree: n_nodes, root, son_start[n_nodes+1] / sons[] (ordered), leaf_row[n_nodes]
//   states: [n_leaf_rows][n_sites] integer state codes (bpp alphabet ints)
//   init_values: [n_codes][S] = getInitValue(s, code)
//   pmats: [n_nodes][C][S][S] transition matrices of the branch above each node
//   use_patterns: 1 = per-subtree compression (reference default), 0 = flat
//   scaling: 1 = power-of-two rescaling deviation (see computeSubtreeLikelihood)
//   n_rep: number of computeTreeLikelihood traversals to time (>= 1)
//   out: lnl (= getLogLikelihood()), site_lnl[n_sites] (nullable),
//        t_traversal (seconds per traversal, nullable), t_reduce (nullable)
// Returns 0, or < 0 on error (-2: state code not allowed by the model).
//   nh_root: 0 = the homogeneous root rule (<= 0 terms dropped), 1 = the NH rule (no
//            per-term guard, class sum clamped at 0), see rootLogLikForSite
int orc_tree_loglik_rule(int n_nodes, int root, const int* son_start, const int* sons, const int* leaf_row,
                         int n_sites, const int* states, int S, int C, int n_codes, const double* init_values,
                         const double* pmats, const double* class_probs, const double* root_freqs,
                         int use_patterns, int scaling, int nh_root, int n_rep, double* lnl, double* site_lnl,
                         double* t_traversal, double* t_reduce) {
  OTree T;
  T.n_nodes = n_nodes;
  T.root = root;
  T.sons.resize(n_nodes);
  T.leaf_row.assign(leaf_row, leaf_row + n_nodes);
  for (int i = 0; i < n_nodes; i++) T.sons[i].assign(sons + son_start[i], sons + son_start[i + 1]);
  OLik L;
  L.tree = &T;
  L.S = S;
  L.C = C;
  L.scaling = scaling != 0;
  L.lik.resize(n_nodes);
  L.links.resize(n_nodes);
  L.nscale.resize(n_nodes);
  for (int n = 0; n < n_nodes; n++) {
    if (n == root) continue;
    VVVdouble& p = L.pxy[n];
    p.resize(C);
    for (int c = 0; c < C; c++) {
      p[c].resize(S);
      for (int x = 0; x < S; x++)
        p[c][x].assign(pmats + (((size_t)n * C + c) * S + x) * S, pmats + (((size_t)n * C + c) * S + x + 1) * S);
    }
  }
  // DRASRTreeLikelihoodData::initLikelihoods, L/DRASRTreeLikelihoodData.cpp:55-90
  std::vector<int> all(n_sites);
  for (int i = 0; i < n_sites; i++) all[i] = i;
  int rc;
  if (use_patterns) {
    Patterns rp;
    rc = initWithPatterns(L, root, all, states, n_sites, n_codes, init_values, rp);
    L.rootLinks = rp.indices;
    L.rootWeights = rp.weights;
  } else {
    std::vector<int> leaves;
    subtreeLeaves(T, root, leaves);
    std::vector<std::string> cols(n_sites);
    for (int i = 0; i < n_sites; i++) {
      cols[i].resize(leaves.size() * sizeof(int));
      for (size_t k = 0; k < leaves.size(); k++) {
        int v = states[(size_t)T.leaf_row[leaves[k]] * n_sites + i];
        std::memcpy(&cols[i][k * sizeof(int)], &v, sizeof(int));
      }
    }
    Patterns rp = makePatterns(cols);
    std::vector<int> rows(rp.sites.size());
    for (size_t i = 0; i < rows.size(); i++) rows[i] = (int)rp.sites[i];
    rc = initFlat(L, root, rows, states, n_sites, n_codes, init_values);
    L.rootLinks = rp.indices;
    L.rootWeights = rp.weights;
  }
  if (rc) return rc;
  if (n_rep < 1) n_rep = 1;
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < n_rep; r++) computeSubtreeLikelihood(L, root);  // computeTreeLikelihood :795-798
  auto t1 = std::chrono::steady_clock::now();
  std::vector<double> la(n_sites);
  for (int i = 0; i < n_sites; i++) la[i] = rootLogLikForSite(L, i, class_probs, root_freqs, nh_root != 0);
  if (site_lnl)
    for (int i = 0; i < n_sites; i++) site_lnl[i] = la[i];
  std::sort(la.begin(), la.end());
  double ll = 0;
  for (int i = n_sites; i > 0; i--) ll += la[i - 1];
  auto t2 = std::chrono::steady_clock::now();
  *lnl = ll;
  if (t_traversal) *t_traversal = std::chrono::duration<double>(t1 - t0).count() / n_rep;
  if (t_reduce) *t_reduce = std::chrono::duration<double>(t2 - t1).count();
  return 0;
}

// The homogeneous entry (RHomogeneousTreeLikelihood's root rule).
int orc_tree_loglik(int n_nodes, int root, const int* son_start, const int* sons, const int* leaf_row,
                    int n_sites, const int* states, int S, int C, int n_codes, const double* init_values,
                    const double* pmats, const double* class_probs, const double* root_freqs, int use_patterns,
                    int scaling, int n_rep, double* lnl, double* site_lnl, double* t_traversal,
                    double* t_reduce) {
  return orc_tree_loglik_rule(n_nodes, root, son_start, sons, leaf_row, n_sites, states, S, C, n_codes, init_values,
                              pmats, class_probs, root_freqs, use_patterns, scaling, 0, n_rep, lnl, site_lnl,
                              t_traversal, t_reduce);
}

// Double-recursive branch derivatives, restating DRHomogeneousTreeLikelihood
// (Likelihood/DRHomogeneousTreeLikelihood.cpp): the son-side arrays of every node by the
// postorder recursion (computeSubtreeLikelihoodPostfix :483-541), the father-side array
// of every branch at its father excluding the branch (computeLikelihoodAtNode_ :723-816,
// root frequencies folded in at the root; the father's own father-side array enters
// through pxy of the father, computeLikelihoodFromArrays :868-940), and per branch and
// site dL = sum_c p_c sum_x larray[x] sum_y dpxy[x][y] L_node[y] (computeTreeDLikelihoodAtNode
// :287-328; D2 twin :373-413) divided by the site likelihood.  Flat sites (every column,
// weight 1), no rescaling.  d1[v] = sum_i dL_i / L_i, d2[v] = sum_i (d2L_i / L_i - (dL_i / L_i)^2)
// (getFirstOrderDerivative / getSecondOrderDerivative return the negatives, :340-371, 425-456).
int orc_dr_derivatives(int n_nodes, int root, const int* son_start, const int* sons, const int* leaf_row,
                       int n_sites, const int* states, int S, int C, int n_codes, const double* init_values,
                       const double* pmats, const double* dpmats, const double* d2pmats, const double* class_probs,
                       const double* root_freqs, double* d1, double* d2) {
  std::vector<std::vector<int> > kids(n_nodes);
  std::vector<int> father(n_nodes, -1);
  for (int i = 0; i < n_nodes; i++) {
    kids[i].assign(sons + son_start[i], sons + son_start[i + 1]);
    for (int k : kids[i]) father[k] = i;
  }
  auto P = [&](const double* m, int n, int c, int x, int y) { return m[(((size_t)n * C + c) * S + x) * S + y]; };
  // son-side arrays (postfix), postorder by explicit stack
  std::vector<VVVdouble> down(n_nodes);
  std::vector<int> order;
  {
    std::vector<std::pair<int, size_t> > st(1, std::make_pair(root, (size_t)0));
    while (!st.empty()) {
      const int n = st.back().first;
      if (st.back().second < kids[n].size()) {
        st.push_back(std::make_pair(kids[n][st.back().second++], (size_t)0));
        continue;
      }
      order.push_back(n);
      st.pop_back();
    }
  }
  for (int n : order) {
    VVVdouble& a = down[n];
    a.assign(n_sites, VVdouble(C, Vdouble(S, 1.)));
    if (kids[n].empty()) {
      for (int i = 0; i < n_sites; i++) {
        const int code = states[(size_t)leaf_row[n] * n_sites + i];
        if (code < 0 || code >= n_codes) return -2;
        for (int c = 0; c < C; c++)
          for (int x = 0; x < S; x++) a[i][c][x] = init_values[(size_t)code * S + x];
      }
      continue;
    }
    for (int k : kids[n])
      for (int i = 0; i < n_sites; i++)
        for (int c = 0; c < C; c++)
          for (int x = 0; x < S; x++) {
            double t = 0.;
            for (int y = 0; y < S; y++) t += P(pmats, k, c, x, y) * down[k][i][c][y];
            a[i][c][x] *= t;
          }
  }
  // father-side arrays in preorder: up[v] = array at father(v) excluding v
  std::vector<VVVdouble> up(n_nodes);
  for (auto it = order.rbegin(); it != order.rend(); ++it) {
    const int v = *it;
    if (v == root) continue;
    const int f = father[v];
    VVVdouble& a = up[v];
    a.assign(n_sites, VVdouble(C, Vdouble(S, 1.)));
    for (int s2 : kids[f]) {
      if (s2 == v) continue;
      for (int i = 0; i < n_sites; i++)
        for (int c = 0; c < C; c++)
          for (int x = 0; x < S; x++) {
            double t = 0.;
            for (int y = 0; y < S; y++) t += P(pmats, s2, c, x, y) * down[s2][i][c][y];
            a[i][c][x] *= t;
          }
    }
    for (int i = 0; i < n_sites; i++)
      for (int c = 0; c < C; c++)
        for (int x = 0; x < S; x++) {
          if (f == root) {
            a[i][c][x] *= root_freqs[x];
          } else {
            double t = 0.;
            for (int w = 0; w < S; w++) t += up[f][i][c][w] * P(pmats, f, c, w, x);
            a[i][c][x] *= t;
          }
        }
  }
  for (int v = 0; v < n_nodes; v++) {
    d1[v] = d2[v] = 0.;
    if (v == root) continue;
    for (int i = 0; i < n_sites; i++) {
      double l = 0., dl = 0., d2l = 0.;
      for (int c = 0; c < C; c++) {
        double lc = 0., dlc = 0., d2lc = 0.;
        for (int x = 0; x < S; x++) {
          double t0 = 0., t1 = 0., t2 = 0.;
          for (int y = 0; y < S; y++) {
            t0 += P(pmats, v, c, x, y) * down[v][i][c][y];
            t1 += P(dpmats, v, c, x, y) * down[v][i][c][y];
            t2 += P(d2pmats, v, c, x, y) * down[v][i][c][y];
          }
          lc += t0 * up[v][i][c][x];
          dlc += t1 * up[v][i][c][x];
          d2lc += t2 * up[v][i][c][x];
        }
        l += class_probs[c] * lc;
        dl += class_probs[c] * dlc;
        d2l += class_probs[c] * d2lc;
      }
      d1[v] += dl / l;
      d2[v] += d2l / l - (dl / l) * (dl / l);
    }
  }
  return 0;
}

// Number of distinct root patterns (SitePatterns over all leaves).
int orc_count_patterns(int n_rows, int n_sites, const int* states) {
  std::vector<std::string> cols(n_sites);
  for (int i = 0; i < n_sites; i++) {
    cols[i].resize(n_rows * sizeof(int));
    for (int k = 0; k < n_rows; k++) {
      int v = states[(size_t)k * n_sites + i];
      std::memcpy(&cols[i][k * sizeof(int)], &v, sizeof(int));
    }
  }
  return (int)makePatterns(cols).weights.size();
}

}  // extern "C"
