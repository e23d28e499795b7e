// Drop-in check of the Bio++ API mirror on the MI355X: the same calls the
// reference's test/test_likelihood.cpp and test/test_likelihood_clock.cpp make
// (tree from Newick, DNA site container, T92 + discrete Gamma, RHomogeneousTreeLikelihood,
// initialize / getValue, optimizeTreeScale + optimizeNumericalParameters2), checked
// against the goldens those tests hold.  Exit code 0 = pass (reference convention).
#include <Bpp/Numeric/Prob/GammaDiscreteDistribution.h>
#include <Bpp/Phyl/Likelihood/DRHomogeneousTreeLikelihood.h>
#include <Bpp/Phyl/Likelihood/DRNonHomogeneousTreeLikelihood.h>
#include <Bpp/Phyl/Likelihood/RNonHomogeneousTreeLikelihood.h>
#include <Bpp/Phyl/Model/FrequencySet/NucleotideFrequencySet.h>
#include <Bpp/Phyl/Model/SubstitutionModelSetTools.h>
#include <Bpp/Phyl/Likelihood/RHomogeneousTreeLikelihood.h>
#include <Bpp/Phyl/Model/Nucleotide/GTR.h>
#include <Bpp/Phyl/Model/Nucleotide/L95.h>
#include <Bpp/Phyl/Model/Nucleotide/T92.h>
#include <Bpp/Phyl/Model/RateDistribution/GammaDiscreteRateDistribution.h>
#include <Bpp/Phyl/OptimizationTools.h>
#include <Bpp/Phyl/TreeTemplate.h>
#include <Bpp/Seq/Alphabet/AlphabetTools.h>
#include <Bpp/Seq/Container/VectorSiteContainer.h>

#include <cmath>
#include <functional>
#include <string>

#include "plk.h"
#include <iomanip>
#include <iostream>
#include <memory>

using namespace bpp;

static int failures = 0;

static void expectNear(const char* what, double got, double want, double tol) {
  const bool ok = std::fabs(got - want) <= tol;
  std::cout << std::setprecision(20) << what << " = " << got << " (expected " << want << ", tol " << tol << ") "
            << (ok ? "ok" : "FAIL") << std::endl;
  if (!ok) failures++;
}

// test/test_likelihood.cpp:91-108 inputs and goldens
static void unrootedGammaCase() {
  std::unique_ptr<TreeTemplate<Node> > tree(
      TreeTemplateTools::parenthesisToTree("((A:0.01, B:0.02):0.03,C:0.01,D:0.1);"));
  const NucleicAlphabet* dna = &AlphabetTools::DNA_ALPHABET;
  VectorSiteContainer aln(dna);
  const char* names[] = {"A", "B", "C", "D"};
  const char* seqs[] = {"AAATGGCTGTGCACGTC", "GACTGGATCTGCACGTC", "CTCTGGATGTGCACGTG", "AAATGGCGGTGCGCCTA"};
  for (int i = 0; i < 4; i++) aln.addSequence(BasicSequence(names[i], seqs[i], dna));
  T92 model(dna, 3.);
  GammaDiscreteRateDistribution rdist(4, 1.0);
  RHomogeneousTreeLikelihood tl(*tree, aln, &model, &rdist, true, false);
  tl.initialize();
  expectNear("T92+G4 initial -lnL", tl.getValue(), 85.030942031997312824, 1e-9);
  // the drop-in evaluates through the benched kernel: the fused lnL-only traversal
  {
    const std::string path = plk_kernel_path(tl.getEngine());
    std::cout << "kernel path through the mirror: " << path << (path == "jit_tree4" ? " ok" : " FAIL") << std::endl;
    if (path != "jit_tree4") failures++;
  }
  std::cout << "distinct sites: " << tl.getNumberOfDistinctSites() << " of " << tl.getNumberOfSites() << std::endl;
  // per-site log-likelihoods sum to the total
  double s = 0.;
  for (size_t i = 0; i < tl.getNumberOfSites(); i++) s += tl.getLogLikelihoodForASite(i);
  expectNear("sum of site lnL", s, tl.getLogLikelihood(), 1e-10);
  // branch-length parameters are BrLen<postorder index>, 5 branches once unrooted
  ParameterList bl = tl.getBranchLengthsParameters();
  expectNear("number of BrLen parameters", (double)bl.size(), 5., 0.);
  // analytic dlnL/dBrLen (GPU path propagation) vs a central difference of -lnL; the
  // reference checks its R and DR derivatives against each other to 1e-6
  // (test/test_likelihood.cpp:122-135)
  for (const std::string& name : bl.getParameterNames()) {
    const double d1 = tl.getFirstOrderDerivative(name);
    const double t = tl.getParameters().getParameterValue(name);
    const double h = 1e-6;
    ParameterList one = tl.getParameters().createSubList(std::vector<std::string>(1, name));
    one[0].setValue(t + h);
    const double fp = tl.f(one);
    one[0].setValue(t - h);
    const double fm = tl.f(one);
    one[0].setValue(t);
    tl.f(one);
    expectNear((std::string("dlnL/d") + name).c_str(), d1, (fp - fm) / (2 * h), 1e-6);
  }
  // incremental re-evaluation (ancestors of the changed branch only) is bit-identical
  // to the reference's full traversal
  {
    const ParameterList orig = tl.getParameters();
    const double v0 = tl.getValue();
    RHomogeneousTreeLikelihood full(*tree, aln, &model, &rdist, true, false);
    full.setIncrementalRecompute(false);
    full.initialize();
    for (const std::string& name : bl.getParameterNames()) {
      ParameterList one = tl.getParameters().createSubList(std::vector<std::string>(1, name));
      one[0].setValue(one[0].getValue() * 1.7 + 0.003);
      const double a = tl.f(one), b = full.f(one);
      expectNear((std::string("incremental == full after ") + name).c_str(), a, b, 0.);
    }
    tl.setParameters(orig);
    expectNear("restored", tl.getValue(), v0, 0.);
  }
  OptimizationTools::optimizeTreeScale(&tl);
  std::cout << "after tree scale: " << tl.getValue() << std::endl;
  const ParameterList scaled = tl.getParameters();
  // the reference's default method: PseudoNewton on the device's analytic branch derivatives
  const unsigned int nPN = OptimizationTools::optimizeNumericalParameters2(&tl, tl.getParameters(), 0, 0.000001, 10000, 0, 0);
  std::cout << "PseudoNewton: " << OptimizationTools::lastSteps_ << " steps, " << nPN << " evaluations" << std::endl;
  expectNear("T92+G4 optimised -lnL (PseudoNewton)", tl.getValue(), 65.72293577214308868406, 1e-3);
  // the same optimum from the coordinate Brent search, for comparison of evaluation counts
  RHomogeneousTreeLikelihood tlb(*tree, aln, &model, &rdist, true, false);
  tlb.initialize();
  tlb.setParameters(scaled);
  const unsigned int nBrent = OptimizationTools::optimizeNumericalParameters2(
      &tlb, tlb.getParameters(), 0, 0.000001, 10000, 0, 0, false, false, 0, OptimizationTools::OPTIMIZATION_BRENT);
  std::cout << "Brent: " << nBrent << " evaluations" << std::endl;
  expectNear("T92+G4 optimised -lnL (Brent)", tlb.getValue(), 65.72293577214308868406, 1e-3);
  expectNear("PseudoNewton vs Brent optimum", tl.getValue(), tlb.getValue(), 1e-4);
}

// test/test_likelihood_clock.cpp:99-115: rooted tree kept rooted, constant rate
static void rootedConstantCase() {
  std::unique_ptr<TreeTemplate<Node> > tree(
      TreeTemplateTools::parenthesisToTree("(((A:0.01, B:0.01):0.02,C:0.03):0.01,D:0.04);"));
  const NucleicAlphabet* dna = &AlphabetTools::DNA_ALPHABET;
  VectorSiteContainer aln(dna);
  const char* names[] = {"A", "B", "C", "D"};
  const char* seqs[] = {"AAATGGCTGTGCACGTC", "AACTGGATCTGCATGTC", "ATCTGGACGTGCACGTG", "CAACGGGAGTGCGCCTA"};
  for (int i = 0; i < 4; i++) aln.addSequence(BasicSequence(names[i], seqs[i], dna));
  T92 model(dna, 3.);
  ConstantRateDistribution rdist;
  RHomogeneousTreeLikelihood tl(*tree, aln, &model, &rdist, false, false);
  tl.enableFirstOrderDerivatives(false);
  tl.enableSecondOrderDerivatives(false);
  tl.initialize();
  expectNear("T92 rooted initial -lnL", tl.getValue(), 94.3957, 5e-5);
  // global molecular clock, as test_likelihood_clock.cpp:67 (useClock = true)
  OptimizationTools::optimizeNumericalParameters2(&tl, tl.getParameters(), 0, 0.000001, 10000, 0, 0, false, true, 2,
                                                  OptimizationTools::OPTIMIZATION_NEWTON);
  expectNear("T92 rooted clock-optimised -lnL", tl.getValue(), 71.2657, 1e-3);
}

// test/test_likelihood.cpp:111-135: fitModelHDR with the double-recursive class (same
// goldens), then the R-vs-DR first-derivative comparison at 1e-6 on every branch
static void doubleRecursiveCase() {
  std::unique_ptr<TreeTemplate<Node> > tree(
      TreeTemplateTools::parenthesisToTree("((A:0.01, B:0.02):0.03,C:0.01,D:0.1);"));
  const NucleicAlphabet* dna = &AlphabetTools::DNA_ALPHABET;
  VectorSiteContainer aln(dna);
  const char* names[] = {"A", "B", "C", "D"};
  const char* seqs[] = {"AAATGGCTGTGCACGTC", "GACTGGATCTGCACGTC", "CTCTGGATGTGCACGTG", "AAATGGCGGTGCGCCTA"};
  for (int i = 0; i < 4; i++) aln.addSequence(BasicSequence(names[i], seqs[i], dna));
  {
    T92 model(dna, 3.);
    GammaDiscreteRateDistribution rdist(4, 1.0);
    DRHomogeneousTreeLikelihood tl(*tree, aln, &model, &rdist, true, false);
    tl.initialize();
    expectNear("DR T92+G4 initial -lnL", tl.getValue(), 85.030942031997312824, 1e-9);
    OptimizationTools::optimizeTreeScale(&tl);
    OptimizationTools::optimizeNumericalParameters2(&tl, tl.getParameters(), 0, 0.000001, 10000, 0, 0);
    expectNear("DR T92+G4 optimised -lnL", tl.getValue(), 65.72293577214308868406, 1e-3);
  }
  T92 model(dna, 3.);
  GammaDiscreteRateDistribution rdist(4, 1.0);
  RHomogeneousTreeLikelihood tlsr(*tree, aln, &model, &rdist, true, false);
  tlsr.initialize();
  DRHomogeneousTreeLikelihood tldr(*tree, aln, &model, &rdist, true, false);
  tldr.initialize();
  for (const std::string& name : tlsr.getBranchLengthsParameters().getParameterNames()) {
    expectNear((std::string("R vs DR d1 ") + name).c_str(), tldr.getFirstOrderDerivative(name),
               tlsr.getFirstOrderDerivative(name), 1e-6);
    expectNear((std::string("R vs DR d2 ") + name).c_str(), tldr.getSecondOrderDerivative(name),
               tlsr.getSecondOrderDerivative(name), 1e-6);
  }
}

// Non-homogeneous (test_likelihood_nh.cpp model set: T92 per branch with its own GC
// content): the R and DR classes give the same -lnL and the same branch derivatives
static void nonHomogeneousDrCase() {
  std::unique_ptr<TreeTemplate<Node> > tree(
      TreeTemplateTools::parenthesisToTree("(((A:0.01, B:0.02):0.03,C:0.05):0.01,(D:0.1,E:0.04):0.02);"));
  const NucleicAlphabet* dna = &AlphabetTools::DNA_ALPHABET;
  VectorSiteContainer aln(dna);
  const char* names[] = {"A", "B", "C", "D", "E"};
  const char* seqs[] = {"AAATGGCTGTGCACGTC", "GACTGGATCTGCACGTC", "CTCTGGATGTGCACGTG", "AAATGGCGGTGCGCCTA",
                        "AACTGGATGTGCGCGTA"};
  for (int i = 0; i < 5; i++) aln.addSequence(BasicSequence(names[i], seqs[i], dna));
  std::map<std::string, std::vector<Vint> > globals;
  globals["T92.kappa"] = {};
  std::map<std::string, std::string> alias;
  std::unique_ptr<SubstitutionModelSet> set(SubstitutionModelSetTools::createNonHomogeneousModelSet(
      new T92(dna, 3.), new GCFrequencySet(dna), tree.get(), alias, globals));
  for (size_t k = 0; k < set->getNumberOfModels(); k++)
    set->setParameterValue("T92.theta_" + std::to_string(k + 1), 0.3 + 0.05 * (double)k);
  GammaDiscreteRateDistribution rdist(4, 0.8);
  RNonHomogeneousTreeLikelihood r(*tree, aln, set.get(), &rdist, false);
  r.initialize();
  DRNonHomogeneousTreeLikelihood dr(*tree, aln, set.get(), &rdist, false);
  dr.initialize();
  expectNear("NH R vs DR -lnL", dr.getValue(), r.getValue(), 1e-12);
  for (const std::string& name : r.getBranchLengthsParameters().getParameterNames()) {
    expectNear((std::string("NH R vs DR d1 ") + name).c_str(), dr.getFirstOrderDerivative(name),
               r.getFirstOrderDerivative(name), 1e-6);
    expectNear((std::string("NH R vs DR d2 ") + name).c_str(), dr.getSecondOrderDerivative(name),
               r.getSecondOrderDerivative(name), 1e-6);
  }
}

// a model whose eigen-system fails its check: P(t) from the host Taylor branch
// (Model/AbstractSubstitutionModel.cpp:470-492) handed over with plk_set_pmatrix; the
// likelihood equals the device eigen path's, and the optimiser still converges
static void taylorModelCase() {
  std::unique_ptr<TreeTemplate<Node> > tree(
      TreeTemplateTools::parenthesisToTree("((A:0.01, B:0.02):0.03,C:0.01,D:0.1);"));
  const NucleicAlphabet* dna = &AlphabetTools::DNA_ALPHABET;
  VectorSiteContainer aln(dna);
  const char* names[] = {"A", "B", "C", "D"};
  const char* seqs[] = {"AAATGGCTGTGCACGTC", "GACTGGATCTGCACGTC", "CTCTGGATGTGCACGTG", "AAATGGCGGTGCGCCTA"};
  for (int i = 0; i < 4; i++) aln.addSequence(BasicSequence(names[i], seqs[i], dna));
  GTR eig(dna, 1.2, 0.4, 0.6, 0.8, 0.5, 0.30, 0.20, 0.25, 0.25);
  GTR tay(dna, 1.2, 0.4, 0.6, 0.8, 0.5, 0.30, 0.20, 0.25, 0.25);
  tay.forceTaylorForTests();
  GammaDiscreteRateDistribution rdist(4, 0.7);
  RHomogeneousTreeLikelihood a(*tree, aln, &eig, &rdist, true, false);
  a.initialize();
  RHomogeneousTreeLikelihood b(*tree, aln, &tay, &rdist, true, false);
  b.initialize();
  expectNear("host Taylor P(t) vs device eigen P(t): -lnL", b.getValue(), a.getValue(), 1e-10 * a.getValue());
  ParameterList bl = b.getBranchLengthsParameters();
  expectNear("numerical d1 (host P) vs analytic", b.getFirstOrderDerivative(bl[0].getName()),
             a.getFirstOrderDerivative(bl[0].getName()), 1e-4);
}

// Felsenstein's pruning on the host with the model's own getPij_t (an independent check of
// what the engine computes from host-uploaded P(t))
static double hostPruningLnl(const TreeTemplate<Node>& tree, const SiteContainer& aln, const SubstitutionModel& m,
                             const DiscreteDistribution& rd) {
  const size_t S = m.getNumberOfStates();
  double lnl = 0.;
  for (size_t site = 0; site < aln.getNumberOfSites(); site++) {
    double like = 0.;
    for (size_t c = 0; c < rd.getNumberOfCategories(); c++) {
      const double r = rd.getCategories()[c];
      std::function<std::vector<double>(const Node*)> rec = [&](const Node* n) {
        std::vector<double> L(S, 1.);
        if (n->isLeaf()) {
          const int st = aln.getSequence(n->getName()).getValue(site);
          for (size_t i = 0; i < S; i++) L[i] = m.getInitValue(i, st);
          return L;
        }
        for (size_t k = 0; k < n->getNumberOfSons(); k++) {
          const Node* son = n->getSon(k);
          const std::vector<double> Ls = rec(son);
          const RowMatrix<double> P = m.getPij_t(son->getDistanceToFather() * r);
          for (size_t x = 0; x < S; x++) {
            double s = 0.;
            for (size_t y = 0; y < S; y++) s += P(x, y) * Ls[y];
            L[x] *= s;
          }
        }
        return L;
      };
      const std::vector<double> L = rec(tree.getRootNode());
      double s = 0.;
      for (size_t x = 0; x < S; x++) s += m.freq(x) * L[x];
      like += rd.getProbability(c) * s;
    }
    lnl += std::log(like);
  }
  return -lnl;
}

// A non-reversible model with a complex eigenvalue pair (L95, Model/Nucleotide/L95.cpp):
// P(t) takes the block form of Model/AbstractSubstitutionModel.cpp:440-467 on the host and
// reaches the engine through plk_set_pmatrix; checked against host pruning, against the
// Taylor branch, and its branch-length derivative against a central difference.
static void complexEigenModelCase() {
  std::unique_ptr<TreeTemplate<Node> > tree(
      TreeTemplateTools::parenthesisToTree("((A:0.01, B:0.02):0.03,C:0.01,D:0.1);"));
  const NucleicAlphabet* dna = &AlphabetTools::DNA_ALPHABET;
  VectorSiteContainer aln(dna);
  const char* names[] = {"A", "B", "C", "D"};
  const char* seqs[] = {"AAATGGCTGTGCACGTC", "GACTGGATCTGCACGTC", "CTCTGGATGTGCACGTG", "AAATGGCGGTGCGCCTA"};
  for (int i = 0; i < 4; i++) aln.addSequence(BasicSequence(names[i], seqs[i], dna));
  L95 blk(dna, 0.95, 0.05, 0.9, 5.0, 0.3);
  L95 tay(dna, 0.95, 0.05, 0.9, 5.0, 0.3);
  tay.forceTaylorForTests();
  std::cout << "L95 diagonalizable " << blk.isDiagonalizable() << " nonsingular " << blk.isNonSingular()
            << " imag " << blk.getIEigenValues()[0] << " " << blk.getIEigenValues()[1] << " "
            << blk.getIEigenValues()[2] << " " << blk.getIEigenValues()[3] << std::endl;
  if (blk.isDiagonalizable() || !blk.isNonSingular()) failures++;  // the block form must be in use
  GammaDiscreteRateDistribution rdist(4, 0.7);
  RHomogeneousTreeLikelihood a(*tree, aln, &blk, &rdist, true, false);
  a.initialize();
  RHomogeneousTreeLikelihood b(*tree, aln, &tay, &rdist, true, false);
  b.initialize();
  const double host = hostPruningLnl(*tree, aln, blk, rdist);
  expectNear("L95 block-form P(t) through the engine vs host pruning: -lnL", a.getValue(), host, 1e-12 * host);
  expectNear("L95 block form vs Taylor branch: -lnL", a.getValue(), b.getValue(), 1e-10 * host);
  ParameterList bl = a.getBranchLengthsParameters();
  const std::string v = bl[1].getName();
  const double x = bl[1].getValue(), h = 1e-6;
  ParameterList p = bl;
  p[1].setValue(x + h);
  a.setParameters(p);
  const double fp = a.getValue();
  p[1].setValue(x - h);
  a.setParameters(p);
  const double fm = a.getValue();
  p[1].setValue(x);
  a.setParameters(p);
  expectNear("L95 d(-lnL)/dBrLen vs central difference", a.getFirstOrderDerivative(v), (fp - fm) / (2 * h), 1e-4);
}

// gaps are not allowed by the model: BadIntException like getInitValue
static void gapCase() {
  std::unique_ptr<TreeTemplate<Node> > tree(TreeTemplateTools::parenthesisToTree("((A:0.1,B:0.2):0.1,C:0.3);"));
  const NucleicAlphabet* dna = &AlphabetTools::DNA_ALPHABET;
  VectorSiteContainer aln(dna);
  aln.addSequence(BasicSequence("A", "AC-T", dna));
  aln.addSequence(BasicSequence("B", "ACGT", dna));
  aln.addSequence(BasicSequence("C", "ACGA", dna));
  T92 model(dna, 2.);
  ConstantRateDistribution rdist;
  bool thrown = false;
  try {
    RHomogeneousTreeLikelihood tl(*tree, aln, &model, &rdist, true, false);
  } catch (BadIntException&) {
    thrown = true;
  }
  std::cout << "gap -> BadIntException: " << (thrown ? "ok" : "FAIL") << std::endl;
  if (!thrown) failures++;
}

// Underflow scaling by default on a large tree of very short branches: 150 DNA
// taxa, every branch 1e-6, random sequences -- each site's likelihood is ~1e-600, far below
// the double range, so the default rule must switch the exact power-of-two rescaling on (the
// reference's RHomogeneousTreeLikelihood.cpp sums log site likelihoods without rescaling).
static std::string comb(int lo, int hi) {
  if (hi - lo == 1) return "t" + std::to_string(lo) + ":0.000001";
  const int mid = (lo + hi) / 2;
  return "(" + comb(lo, mid) + "," + comb(mid, hi) + "):0.000001";
}

static void shortBranchScalingCase() {
  const int n = 150, L = 40;
  std::string nwk = comb(0, n);
  nwk = nwk.substr(0, nwk.rfind(':')) + ";";
  std::unique_ptr<TreeTemplate<Node> > tree(TreeTemplateTools::parenthesisToTree(nwk));
  const NucleicAlphabet* dna = &AlphabetTools::DNA_ALPHABET;
  VectorSiteContainer aln(dna);
  unsigned long long x = 12345;
  for (int i = 0; i < n; i++) {
    std::string s;
    for (int j = 0; j < L; j++) {
      x = x * 6364136223846793005ULL + 1442695040888963407ULL;
      s += "ACGT"[(x >> 33) & 3];
    }
    aln.addSequence(BasicSequence("t" + std::to_string(i), s, dna));
  }
  T92 model(dna, 3.);
  GammaDiscreteRateDistribution rdist(4, 0.5);
  RHomogeneousTreeLikelihood def(*tree, aln, &model, &rdist, false, false);
  def.initialize();
  RHomogeneousTreeLikelihood on(*tree, aln, &model, &rdist, false, false);
  on.setUnderflowScaling(true);
  on.initialize();
  const double a = def.getValue(), b = on.getValue();
  std::cout << std::setprecision(17) << "150 taxa, branches 1e-6: default -lnL " << a << ", scaling on " << b
            << ", fallbacks " << def.getEvaluationStats().scaledFallbacks << std::endl;
  if (!std::isfinite(a) || a < 1000.) failures++;
  // the unscaled first evaluation underflows: the default falls back to the rescaling engine
  // once and returns the forced-scaling value bitwise
  if (def.getEvaluationStats().scaledFallbacks != 1 || !def.underflowScalingActive()) failures++;
  if (a != b) {
    std::cout << "FAIL default (fallback) != scaling on, bitwise" << std::endl;
    failures++;
  }
}

// 64 taxa (a balanced tree, branches 0.02-0.1, 300 random DNA sites): no site likelihood comes
// near 2^-255, so the default stays on the unscaled engine -- no fallback -- and every value
// equals the forced-scaling engine's bitwise, through branch-length changes
static void unscaledFirstCase() {
  const int n = 64, L = 300;
  std::string nwk = "t0:0.05";
  {
    std::vector<std::string> level;
    unsigned long long x = 777;
    auto len = [&]() {
      x = x * 6364136223846793005ULL + 1442695040888963407ULL;
      return std::to_string(0.02 + 0.08 * (double)((x >> 33) & 0xffff) / 65536.0);
    };
    for (int i = 0; i < n; i++) level.push_back("t" + std::to_string(i));
    while (level.size() > 1) {
      std::vector<std::string> next;
      for (size_t i = 0; i + 1 < level.size(); i += 2)
        next.push_back("(" + level[i] + ":" + len() + "," + level[i + 1] + ":" + len() + ")");
      level = next;
    }
    nwk = level[0] + ";";
  }
  std::unique_ptr<TreeTemplate<Node> > tree(TreeTemplateTools::parenthesisToTree(nwk));
  const NucleicAlphabet* dna = &AlphabetTools::DNA_ALPHABET;
  VectorSiteContainer aln(dna);
  unsigned long long x = 4242;
  for (int i = 0; i < n; i++) {
    std::string s;
    for (int j = 0; j < L; j++) {
      x = x * 6364136223846793005ULL + 1442695040888963407ULL;
      s += "ACGT"[(x >> 33) & 3];
    }
    aln.addSequence(BasicSequence("t" + std::to_string(i), s, dna));
  }
  GTR model(dna, 1.2, 0.4, 0.6, 0.8, 0.5, 0.30, 0.20, 0.25, 0.25);
  GammaDiscreteRateDistribution rdist(4, 0.5);
  RHomogeneousTreeLikelihood def(*tree, aln, &model, &rdist, true, false);
  def.initialize();
  RHomogeneousTreeLikelihood on(*tree, aln, &model, &rdist, true, false);
  on.setUnderflowScaling(true);
  on.initialize();
  int mismatches = def.getValue() != on.getValue();
  ParameterList bl = def.getBranchLengthsParameters();
  for (int k = 1; k <= 3; k++) {
    for (size_t i = 0; i < bl.size(); i++) bl[i].setValue(bl[i].getValue() * (1.0 + 0.1 * k));
    def.setParameters(bl);
    on.setParameters(bl);
    mismatches += def.getValue() != on.getValue();
  }
  std::cout << std::setprecision(17) << "64 taxa: default -lnL " << def.getValue() << ", scaling on " << on.getValue()
            << ", fallbacks " << def.getEvaluationStats().scaledFallbacks << ", bitwise mismatches " << mismatches
            << std::endl;
  if (mismatches || def.getEvaluationStats().scaledFallbacks != 0 || def.underflowScalingActive()) failures++;
}

// The NH mirror (RNonHomogeneousTreeLikelihood: NH root rule, no non-negative guards) on a
// 64-taxon rooted tree with per-branch T92 theta: unscaled first, no fallback, every value equal
// to the forced-scaling engine's bitwise, through branch-length and model-parameter changes
// (the clear-flag proof on the NH path)
static void unscaledFirstNhCase() {
  const int n = 64, L = 300;
  std::string nwk;
  {
    std::vector<std::string> level;
    unsigned long long x = 991;
    auto len = [&]() {
      x = x * 6364136223846793005ULL + 1442695040888963407ULL;
      return std::to_string(0.02 + 0.08 * (double)((x >> 33) & 0xffff) / 65536.0);
    };
    for (int i = 0; i < n; i++) level.push_back("t" + std::to_string(i));
    while (level.size() > 1) {
      std::vector<std::string> next;
      for (size_t i = 0; i + 1 < level.size(); i += 2)
        next.push_back("(" + level[i] + ":" + len() + "," + level[i + 1] + ":" + len() + ")");
      level = next;
    }
    nwk = level[0] + ";";
  }
  std::unique_ptr<TreeTemplate<Node> > tree(TreeTemplateTools::parenthesisToTree(nwk));
  const NucleicAlphabet* dna = &AlphabetTools::DNA_ALPHABET;
  VectorSiteContainer aln(dna);
  unsigned long long x = 5151;
  for (int i = 0; i < n; i++) {
    std::string s;
    for (int j = 0; j < L; j++) {
      x = x * 6364136223846793005ULL + 1442695040888963407ULL;
      s += "ACGT"[(x >> 33) & 3];
    }
    aln.addSequence(BasicSequence("t" + std::to_string(i), s, dna));
  }
  std::map<std::string, std::vector<Vint> > globals;
  globals["T92.kappa"] = {};
  std::map<std::string, std::string> alias;
  // one model set per likelihood: a set shared by two would report a parameter change only to
  // the first of them (matchParametersValues), as in the reference
  std::unique_ptr<SubstitutionModelSet> sets[2];
  for (auto& set : sets) {
    set.reset(SubstitutionModelSetTools::createNonHomogeneousModelSet(new T92(dna, 3.), new GCFrequencySet(dna),
                                                                       tree.get(), alias, globals));
    for (size_t k = 0; k < set->getNumberOfModels(); k++)
      set->setParameterValue("T92.theta_" + std::to_string(k + 1), 0.3 + 0.4 * (double)(k % 7) / 6.0);
  }
  GammaDiscreteRateDistribution rdist(4, 0.8);
  RNonHomogeneousTreeLikelihood def(*tree, aln, sets[0].get(), &rdist, false);
  def.initialize();
  RNonHomogeneousTreeLikelihood on(*tree, aln, sets[1].get(), &rdist, false);
  on.setUnderflowScaling(true);
  on.initialize();
  int mismatches = def.getValue() != on.getValue();
  ParameterList bl = def.getBranchLengthsParameters();
  for (int k = 1; k <= 3; k++) {
    for (size_t i = 0; i < bl.size(); i++) bl[i].setValue(bl[i].getValue() * (1.0 + 0.1 * k));
    def.setParameters(bl);
    on.setParameters(bl);
    mismatches += def.getValue() != on.getValue();
  }
  // a root-frequency parameter (GC.theta) and a branch model's theta
  for (const char* key : {"GC.theta", "T92.theta_3"}) {
    ParameterList th = def.getParameters();
    for (size_t i = 0; i < th.size(); i++)
      if (th[i].getName() == key) th[i].setValue(0.45);
    def.setParameters(th);
    on.setParameters(th);
    mismatches += def.getValue() != on.getValue();
  }
  std::cout << std::setprecision(17) << "NH 64 taxa: default -lnL " << def.getValue() << ", scaling on "
            << on.getValue() << ", fallbacks " << def.getEvaluationStats().scaledFallbacks << ", bitwise mismatches "
            << mismatches << std::endl;
  if (mismatches || def.getEvaluationStats().scaledFallbacks != 0 || def.underflowScalingActive()) failures++;
}

int main() {
  try {
    unrootedGammaCase();
    rootedConstantCase();
    doubleRecursiveCase();
    nonHomogeneousDrCase();
    taylorModelCase();
    complexEigenModelCase();
    gapCase();
    shortBranchScalingCase();
    unscaledFirstCase();
    unscaledFirstNhCase();
  } catch (Exception& e) {
    std::cerr << e.what() << std::endl;
    return 1;
  }
  std::cout << (failures ? "FAILED" : "PASSED") << std::endl;
  return failures ? 1 : 0;
}
