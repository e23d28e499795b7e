// Time the Bio++ drop-in path at a BASELINE configuration's size: the reference API
// (TreeTemplateTools::parenthesisToTree, VectorSiteContainer from a simulated alignment,
// RHomogeneousTreeLikelihood, setParameters(BrLen...) + getValue(),
// Likelihood/RHomogeneousTreeLikelihood.h:131-138, .cpp:255-283) over the host mirror and
// libplk, with every branch length changed per step as bench.py's steps do.  Prints one
// JSON line.
//   bench_mirror <cfg2|cfg3|cfg4> [patterns] [steps] [warmup]
#include <Bpp/App/ApplicationTools.h>
#include <Bpp/Numeric/Prob/GammaDiscreteDistribution.h>
#include <Bpp/Phyl/Likelihood/RHomogeneousTreeLikelihood.h>
#include <Bpp/Phyl/Model/Codon/YN98.h>
#include <Bpp/Phyl/Model/Nucleotide/GTR.h>
#include <Bpp/Phyl/Model/Protein/LG08.h>
#include <Bpp/Phyl/Simulation/NonHomogeneousSequenceSimulator.h>
#include <Bpp/Phyl/TreeTemplate.h>
#include <Bpp/Seq/Alphabet/AlphabetTools.h>
#include <Bpp/Seq/GeneticCode/StandardGeneticCode.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>
#include <string>

#include "plk.h"

using namespace bpp;

// complete balanced binary tree over t0..t{n-1}, branch lengths U(0.01, 0.1)
static std::string balancedNewick(int n, std::mt19937_64& rng) {
  std::uniform_real_distribution<double> u(0.01, 0.1);
  std::vector<std::string> level;
  for (int i = 0; i < n; i++) level.push_back("t" + std::to_string(i));
  auto len = [&]() {
    char b[32];
    std::snprintf(b, sizeof b, ":%.6f", u(rng));
    return std::string(b);
  };
  while (level.size() > 1) {
    std::vector<std::string> next;
    for (size_t i = 0; i + 1 < level.size(); i += 2)
      next.push_back("(" + level[i] + len() + "," + level[i + 1] + len() + ")");
    if (level.size() % 2) next.push_back(level.back());
    level = next;
  }
  return level[0] + ";";
}

int main(int argc, char** argv) {
  const std::string cfg = argc > 1 ? argv[1] : "cfg2";
  const int taxa = cfg == "cfg3" ? 256 : cfg == "cfg4" ? 128 : 64;
  const size_t defP = cfg == "cfg3" ? 200000 : cfg == "cfg4" ? 50000 : 1000000;
  const size_t P = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : defP;
  // 200 steps after 50 warmup: the GPU clock settles (bench.py, profiles/r05/ab_runs.md "window")
  const int steps = argc > 3 ? std::atoi(argv[3]) : 200, warmup = argc > 4 ? std::atoi(argv[4]) : 50;
  ApplicationTools::verbosity() = 0;
  std::mt19937_64 rng(42);
  std::unique_ptr<TreeTemplate<Node> > tree(TreeTemplateTools::parenthesisToTree(balancedNewick(taxa, rng)));
  std::unique_ptr<SubstitutionModel> model;
  std::unique_ptr<DiscreteDistribution> rdist;
  if (cfg == "cfg3") {
    model.reset(new LG08(&AlphabetTools::PROTEIN_ALPHABET));
    rdist.reset(new GammaDiscreteDistribution(4, 0.5, 0.5));
  } else if (cfg == "cfg4") {
    static StandardGeneticCode gc(&AlphabetTools::DNA_ALPHABET);
    model.reset(new YN98(&gc, Vdouble(), 2., 0.3));
    rdist.reset(new ConstantDistribution(1.));
  } else {
    model.reset(new GTR(&AlphabetTools::DNA_ALPHABET, 1.2, 0.4, 0.6, 0.8, 0.5, 0.30, 0.20, 0.25, 0.25));
    rdist.reset(new GammaDiscreteDistribution(4, 0.5, 0.5));
  }
  const auto c0 = std::chrono::steady_clock::now();
  NonHomogeneousSequenceSimulator sim(model.get(), rdist.get(), tree.get());
  std::unique_ptr<SiteContainer> sites(sim.simulate(P));
  const auto c1 = std::chrono::steady_clock::now();
  RHomogeneousTreeLikelihood tl(*tree, *sites, model.get(), rdist.get(), true, false);
  tl.initialize();
  const auto c2 = std::chrono::steady_clock::now();
  // the same likelihood with rescaling forced on: the default (unscaled first, exact fallback)
  // must return its values bitwise (checked after the timed steps)
  std::unique_ptr<RHomogeneousTreeLikelihood> forced(
      new RHomogeneousTreeLikelihood(*tree, *sites, model.get(), rdist.get(), true, false));
  forced->setUnderflowScaling(true);
  forced->initialize();
  sites.reset();
  ParameterList bl = tl.getBranchLengthsParameters();
  std::vector<ParameterList> sets(2, bl);
  for (size_t i = 0; i < bl.size(); i++) sets[1][i].setValue(bl[i].getValue() * 1.01);
  double v = 0.;
  for (int i = 0; i < warmup; i++) {
    tl.setParameters(sets[(i + 1) & 1]);
    v += tl.getValue();
  }
  plk_reset_timing(tl.getEngine());
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < steps; i++) {
    tl.setParameters(sets[(warmup + i + 1) & 1]);
    v += tl.getValue();
  }
  const auto t1 = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count() / steps;
  // host segments of plk_evaluate over the timed steps ([5]: the mirror's own time between
  // evaluations), then the traversal kernel time of the same steps under HIP events
  plk_timing tm;
  plk_get_timing_ex(tl.getEngine(), &tm);
  const double ne = tm.evaluations > 0 ? (double)tm.evaluations : 1.0;
  plk_set_timing(tl.getEngine(), PLK_TIME_PARTIALS | PLK_TIME_PMAT | PLK_TIME_ROOT | PLK_TIME_TABLES);
  plk_reset_timing(tl.getEngine());
  for (int i = 0; i < steps; i++) {
    tl.setParameters(sets[(warmup + steps + i + 1) & 1]);
    v += tl.getValue();
  }
  plk_timing tk;
  plk_get_timing_ex(tl.getEngine(), &tk);
  plk_set_timing(tl.getEngine(), 0);
  const double nk = tk.evaluations > 0 ? (double)tk.evaluations : 1.0;
  int mismatches = 0;
  for (int k = 0; k < 2; k++) {
    tl.setParameters(sets[k]);
    forced->setParameters(sets[k]);
    mismatches += tl.getValue() != forced->getValue();
  }
  forced.reset();
  const size_t D = tl.getNumberOfDistinctSites();
  const int internal = taxa - 2;
  const auto& st = tl.getEvaluationStats();
  std::printf(
      "{\"bench\": \"mirror\", \"config\": \"%s\", \"taxa\": %d, \"sites\": %zu, \"distinct_patterns\": %zu, "
      "\"internal_nodes\": %d, \"steps\": %d, \"warmup\": %d, \"ms_per_step\": %.5f, \"updates_per_s\": %.6g, "
      "\"kernel_path\": \"%s\", \"minus_lnl\": %.12f, \"full_traversals\": %zu, \"evaluations\": %zu, "
      "\"scaled_fallbacks\": %zu, \"scaling_active\": %s, \"bitwise_mismatches_vs_forced_scaling\": %d, "
      "\"simulate_s\": %.2f, \"setup_s\": %.2f, \"checksum\": %.6f, \"host_us_per_eval\": {\"pmat_call\": %.2f, "
      "\"traversal_call\": %.2f, \"blocks_call\": %.2f, \"wait\": %.2f, \"sum\": %.2f, \"caller\": %.2f}, "
      "\"kernel_ms_per_eval\": {\"partials\": %.4f, \"tables\": %.4f, \"pmatrix\": %.4f, \"root\": %.4f}}\n",
      cfg.c_str(), taxa, P, D, internal, steps, warmup, ms, (double)D * internal / (ms * 1e-3),
      plk_kernel_path(tl.getEngine()), tl.getValue(), st.fullTraversals, st.evaluations, st.scaledFallbacks,
      tl.underflowScalingActive() ? "true" : "false", mismatches,
      std::chrono::duration<double>(c1 - c0).count(), std::chrono::duration<double>(c2 - c1).count(), v,
      tm.host_us[0] / ne, tm.host_us[1] / ne, tm.host_us[2] / ne, tm.host_us[3] / ne, tm.host_us[4] / ne,
      tm.host_us[5] / ne, tk.partials_ms / nk, tk.tables_ms / nk, tk.pmat_ms / nk, tk.root_ms / nk);
  return 0;
}
