// ASan + UBSan driver of the oracle (test infrastructure, SURVEY 5 sanitizers): built with
// `make -C oracle asan` together with oracle.cpp, it runs every exported entry point on the
// reference's test_likelihood.cpp case (T92(kappa 3, theta 0.5) + Gamma(4, 1), the 4-taxon
// tree) with and without per-subtree compression and rescaling, plus GTR P(t) through the
// Jacobi path and the DR derivatives, and checks -lnL against the golden 85.030942031997.
// Any sanitizer finding aborts the run (-fno-sanitize-recover).
#include <cmath>
#include <cstdio>
#include <vector>

extern "C" {
int orc_gamma_rates(int n, double alpha, double* rates, double* probs);
void orc_t92_pij(double kappa, double theta, double t, double* P);
void orc_t92_freqs(double theta, double* pi);
void orc_reversible_generator(int S, const double* exch, const double* pi, double* Q);
void orc_gtr_model(double a, double b, double c, double d, double e, double theta, double theta1, double theta2,
                   double* exch, double* pi);
int orc_reversible_pij(int S, const double* Q, const double* pi, double t, double* P);
int orc_tree_loglik(int n_nodes, int root, const int* son_start, const int* sons, const int* leaf_row, int n_sites,
                    const int* states, int S, int C, int n_codes, const double* init_values, const double* pmats,
                    const double* class_probs, const double* root_freqs, int use_patterns, int scaling, int n_rep,
                    double* lnl, double* site_lnl, double* t_traversal, double* t_reduce);
int orc_dr_derivatives(int n_nodes, int root, const int* son_start, const int* sons, const int* leaf_row,
                       int n_sites, const int* states, int S, int C, int n_codes, const double* init_values,
                       const double* pmats, const double* dpmats, const double* d2pmats, const double* class_probs,
                       const double* root_freqs, double* d1, double* d2);
int orc_count_patterns(int n_rows, int n_sites, const int* states);
}

static int failures = 0;
static void check(bool ok, const char* what, double v) {
  std::printf("%s %s (%.15g)\n", ok ? "ok  " : "FAIL", what, v);
  if (!ok) failures++;
}

int main() {
  // ((A:0.01, B:0.02):0.03, C:0.01, D:0.1); A B AB C D root
  const int n_nodes = 6, root = 5;
  const int son_start[] = {0, 0, 0, 2, 2, 2, 5}, sons[] = {0, 1, 2, 3, 4}, leaf_row[] = {0, 1, -1, 2, 3, -1};
  const double brlen[] = {0.01, 0.02, 0.03, 0.01, 0.1, 0.};
  const char* seq[] = {"AAATGGCTGTGCACGTC", "GACTGGATCTGCACGTC", "CTCTGGATGTGCACGTG", "AAATGGCGGTGCGCCTA"};
  const int n_sites = 17, S = 4, C = 4;
  std::vector<int> states(4 * n_sites);
  for (int r = 0; r < 4; r++)
    for (int i = 0; i < n_sites; i++) {
      const char ch = seq[r][i];
      states[r * n_sites + i] = ch == 'A' ? 0 : ch == 'C' ? 1 : ch == 'G' ? 2 : 3;
    }
  std::vector<double> init(16, 0.);
  for (int s = 0; s < 4; s++) init[s * 4 + s] = 1.;
  double rates[4], probs[4], pi[4];
  const int grc = orc_gamma_rates(C, 1.0, rates, probs);
  check(grc == 0 && std::fabs(rates[0] + rates[1] + rates[2] + rates[3] - 4.) < 1e-12, "gamma rates", rates[3]);
  orc_t92_freqs(0.5, pi);
  std::vector<double> pm(n_nodes * C * S * S, 0.), dpm(pm.size(), 0.), d2pm(pm.size(), 0.);
  const double h = 1e-5;
  for (int n = 0; n < n_nodes; n++) {
    if (n == root) continue;
    for (int c = 0; c < C; c++) {
      double* P = &pm[((size_t)n * C + c) * S * S];
      double Pp[16], Pm[16];
      orc_t92_pij(3., 0.5, brlen[n] * rates[c], P);
      orc_t92_pij(3., 0.5, (brlen[n] + h) * rates[c], Pp);
      orc_t92_pij(3., 0.5, (brlen[n] - h) * rates[c], Pm);
      for (int k = 0; k < 16; k++) {
        dpm[((size_t)n * C + c) * 16 + k] = (Pp[k] - Pm[k]) / (2. * h);
        d2pm[((size_t)n * C + c) * 16 + k] = (Pp[k] - 2. * P[k] + Pm[k]) / (h * h);
      }
    }
  }
  for (int up = 0; up < 2; up++)
    for (int sc = 0; sc < 2; sc++) {
      double lnl = 0., tt = 0., tr = 0.;
      std::vector<double> site(n_sites);
      const int rc = orc_tree_loglik(n_nodes, root, son_start, sons, leaf_row, n_sites, states.data(), S, C, 4,
                                     init.data(), pm.data(), probs, pi, up, sc, 2, &lnl, site.data(), &tt, &tr);
      check(rc == 0 && std::fabs(-lnl - 85.030942031997312824) < 1e-9, up ? "lnL usePatterns=1" : "lnL usePatterns=0",
            -lnl);
    }
  std::vector<double> d1(n_nodes), d2(n_nodes);
  const int rc = orc_dr_derivatives(n_nodes, root, son_start, sons, leaf_row, n_sites, states.data(), S, C, 4,
                                    init.data(), pm.data(), dpm.data(), d2pm.data(), probs, pi, d1.data(), d2.data());
  bool fin = rc == 0;
  for (int n = 0; n < n_nodes; n++) fin = fin && std::isfinite(d1[n]) && std::isfinite(d2[n]);
  check(fin, "DR derivatives finite", d1[0]);
  const int np = orc_count_patterns(4, n_sites, states.data());
  check(np == 12, "distinct patterns", np);
  // GTR P(t) through the Jacobi path: rows sum to 1
  double exch[16], gpi[4], Q[16], P[16];
  orc_gtr_model(1.2, 0.4, 0.6, 0.8, 0.5, 0.45, 0.55, 0.5, exch, gpi);
  orc_reversible_generator(4, exch, gpi, Q);
  const int prc = orc_reversible_pij(4, Q, gpi, 0.3, P);
  check(prc == 0, "GTR pij", P[0]);
  double worst = 0.;
  for (int x = 0; x < 4; x++) {
    double s = 0.;
    for (int y = 0; y < 4; y++) s += P[x * 4 + y];
    worst = std::fmax(worst, std::fabs(s - 1.));
  }
  check(worst < 1e-13, "GTR pij rows sum to 1", worst);
  std::printf("%s\n", failures ? "FAILED" : "PASSED");
  return failures ? 1 : 0;
}
