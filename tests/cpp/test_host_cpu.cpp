// CPU-only checks of the host mirror (no GPU): prints JSON records that
// tests/test_host.py compares with the oracle and the golden fixtures.
#include <Bpp/Phyl/Model/Codon/YN98.h>
#include <Bpp/Phyl/Model/Nucleotide/GTR.h>
#include <Bpp/Phyl/Model/Nucleotide/L95.h>
#include <Bpp/Phyl/Model/Nucleotide/T92.h>
#include <Bpp/Phyl/Model/Protein/LG08.h>
#include <Bpp/Phyl/Model/RateDistribution/GammaDiscreteRateDistribution.h>
#include <Bpp/Phyl/Model/FrequencySet/NucleotideFrequencySet.h>
#include <Bpp/Phyl/Model/SubstitutionModelSet.h>
#include <Bpp/Phyl/Simulation/NonHomogeneousSequenceSimulator.h>
#include <Bpp/Numeric/Prob/GammaDiscreteDistribution.h>
#include <Bpp/Phyl/Likelihood/ClockTreeLikelihood.h>
#include <Bpp/Phyl/OptimizationTools.h>
#include <Bpp/Phyl/TreeTemplate.h>
#include <Bpp/Seq/Alphabet/AlphabetTools.h>

#include <cstdio>
#include <memory>
#include <string>
#include <vector>

using namespace bpp;

// A host-only "likelihood" (no engine) to drive the optimisers on CPU:
// f = sqrt(1 + x^2) + sqrt(1 + y^2) from (10, -7), no analytic derivatives.  Far from the
// minimum the Newton move d1/d2 = x (1 + x^2) overshoots by orders of magnitude, so three
// Felsenstein-Churchill halvings do not help and the fourth correction -- the
// conjugate-gradient search -- has to find the way.
class OvershootLikelihood : public virtual TreeLikelihood {
  TreeTemplate<Node> tree_;
  mutable unsigned evals_ = 0;

 public:
  OvershootLikelihood() : tree_(*std::unique_ptr<TreeTemplate<Node> >(TreeTemplateTools::parenthesisToTree("(a:1,b:1);"))) {
    addParameter_(Parameter("x", 10.));
    addParameter_(Parameter("y", -7.));
  }
  unsigned evaluations() const { return evals_; }
  void initialize() override {}
  bool isInitialized() const override { return true; }
  double getValue() const override {
    evals_++;
    const double x = parameters_.getParameterValue("x"), y = parameters_.getParameterValue("y");
    return std::sqrt(1. + x * x) + std::sqrt(1. + y * y);
  }
  double getLogLikelihood() const override { return -getValue(); }
  double getLikelihood() const override { return std::exp(-getValue()); }
  double getLogLikelihoodForASite(size_t) const override { return -getValue(); }
  double getLikelihoodForASite(size_t) const override { return getLikelihood(); }
  size_t getNumberOfSites() const override { return 1; }
  size_t getNumberOfStates() const override { return 4; }
  size_t getNumberOfClasses() const override { return 1; }
  const Tree& getTree() const override { return tree_; }
  ParameterList getBranchLengthsParameters() const override { return ParameterList(); }
  ParameterList getSubstitutionModelParameters() const override { return parameters_; }
  ParameterList getRateDistributionParameters() const override { return ParameterList(); }
  ParameterList getDerivableParameters() const override { return ParameterList(); }
  ParameterList getNonDerivableParameters() const override { return parameters_; }
  void setParameters(const ParameterList& pl) override { parameters_.matchParametersValues(pl); }
  double f(const ParameterList& pl) override {
    setParameters(pl);
    return getValue();
  }
  double getFirstOrderDerivative(const std::string&) const override { return 0.; }
  double getSecondOrderDerivative(const std::string&) const override { return 0.; }
  void enableDerivatives(bool) override {}
  void enableFirstOrderDerivatives(bool) override {}
  void enableSecondOrderDerivatives(bool) override {}
};

// The same function behind the global-clock interface, for optimizeNumericalParametersWithGlobalClock2
class OvershootClock : public OvershootLikelihood, public DiscreteRatesAcrossSitesClockTreeLikelihood {};

static void printVec(const char* key, const std::vector<double>& v) {
  std::printf("\"%s\": [", key);
  for (size_t i = 0; i < v.size(); i++) std::printf("%s%.17g", i ? ", " : "", v[i]);
  std::printf("]");
}

static void printModel(const char* name, const SubstitutionModel& m, const std::vector<double>& ts) {
  const size_t S = m.getNumberOfStates();
  std::printf("{\"kind\": \"model\", \"name\": \"%s\", \"S\": %zu, ", name, S);
  std::vector<double> Q(m.getGenerator().data(), m.getGenerator().data() + S * S);
  printVec("Q", Q);
  std::printf(", ");
  printVec("pi", m.getFrequencies());
  std::printf(", ");
  printVec("t", ts);
  std::printf(", \"P\": [");
  for (size_t k = 0; k < ts.size(); k++) {
    const RowMatrix<double>& P = m.getPij_t(ts[k]);
    std::vector<double> p(P.data(), P.data() + S * S);
    std::printf("%s[", k ? ", " : "");
    for (size_t i = 0; i < p.size(); i++) std::printf("%s%.17g", i ? ", " : "", p[i]);
    std::printf("]");
  }
  std::printf("], \"P_eigen\": [");
  for (size_t k = 0; k < ts.size(); k++) {
    const RowMatrix<double>& P = m.SubstitutionModel::getPij_t(ts[k]);
    std::vector<double> p(P.data(), P.data() + S * S);
    std::printf("%s[", k ? ", " : "");
    for (size_t i = 0; i < p.size(); i++) std::printf("%s%.17g", i ? ", " : "", p[i]);
    std::printf("]");
  }
  std::printf("]");
  auto mats = [&](const char* key, int which) {
    std::printf(", \"%s\": [", key);
    for (size_t k = 0; k < ts.size(); k++) {
      const RowMatrix<double>& P = which == 1 ? m.getdPij_dt(ts[k]) : m.getd2Pij_dt2(ts[k]);
      std::printf("%s[", k ? ", " : "");
      for (size_t i = 0; i < S * S; i++) std::printf("%s%.17g", i ? ", " : "", P.data()[i]);
      std::printf("]");
    }
    std::printf("]");
  };
  mats("dP", 1);
  mats("d2P", 2);
  std::printf(", \"diagonalizable\": %s, \"nonsingular\": %s, ", m.isDiagonalizable() ? "true" : "false",
              m.isNonSingular() ? "true" : "false");
  printVec("wr", m.getEigenValues());
  std::printf(", ");
  printVec("wi", m.getIEigenValues());
  std::printf(", ");
  printVec("V", std::vector<double>(m.getColumnRightEigenVectors().data(), m.getColumnRightEigenVectors().data() + S * S));
  std::printf(", ");
  printVec("Vi", std::vector<double>(m.getRowLeftEigenVectors().data(), m.getRowLeftEigenVectors().data() + S * S));
  std::printf("}\n");
}

int main() {
  const NucleicAlphabet* dna = &AlphabetTools::DNA_ALPHABET;
  std::vector<double> ts = {1e-6, 0.01, 0.1, 0.5, 2.0, 10.0};
  // gamma rates
  for (double a : {0.2, 0.5, 1.0, 2.0, 7.5}) {
    GammaDiscreteRateDistribution g(4, a);
    std::printf("{\"kind\": \"gamma\", \"alpha\": %.17g, ", a);
    printVec("rates", g.getCategories());
    std::printf("}\n");
  }
  printModel("T92", T92(dna, 3.0, 0.5), ts);
  printModel("T92_k2_t03", T92(dna, 2.0, 0.3), ts);
  printModel("GTR", GTR(dna, 1.2, 0.4, 0.6, 0.8, 0.5, 0.30, 0.20, 0.25, 0.25), ts);
  printModel("LG08", LG08(&AlphabetTools::PROTEIN_ALPHABET), ts);
  {
    // the Taylor branch of getPij_t (a failed eigen-system check): same P(t)
    GTR g(dna, 1.2, 0.4, 0.6, 0.8, 0.5, 0.30, 0.20, 0.25, 0.25);
    g.forceTaylorForTests();
    printModel("GTR_taylor", g, ts);
    LG08 l(&AlphabetTools::PROTEIN_ALPHABET);
    l.forceTaylorForTests();
    printModel("LG08_taylor", l, ts);
  }
  // L95, non-reversible: complex eigenvalue pairs (block form) and a repeated eigenvalue
  printModel("L95_complex", L95(dna, 0.9, 0.1, 0.3, 2.0, 0.4), ts);
  printModel("L95_complex2", L95(dna, 0.95, 0.05, 0.9, 5.0, 0.3), ts);
  printModel("L95_repeated", L95(dna, 0.5, 0.5, 0.5, 1.0, 0.5), ts);
  {
    L95 l(dna, 0.1, 0.9, 0.1, 3.0, 0.6);
    l.setRate(1.7);
    printModel("L95_rate", l, ts);
  }
  StandardGeneticCode gc(dna);
  printModel("YN98", YN98(&gc, std::vector<double>(), 2.0, 0.3), ts);
  // trees: postorder ids, unroot
  const char* newicks[] = {"((A:0.01, B:0.02):0.03,C:0.01,D:0.1);", "(((A:0.01, B:0.01):0.02,C:0.03):0.01,D:0.04);",
                           "((a:1,b:2):3,(c:4,d:5):6);"};
  for (const char* nw : newicks) {
    std::unique_ptr<TreeTemplate<Node> > t(TreeTemplateTools::parenthesisToTree(nw));
    std::printf("{\"kind\": \"tree\", \"newick\": \"%s\", \"rooted\": %s, \"leaves\": [", nw, t->isRooted() ? "true" : "false");
    std::vector<std::string> ln = t->getLeavesNames();
    for (size_t i = 0; i < ln.size(); i++) std::printf("%s\"%s\"", i ? ", " : "", ln[i].c_str());
    std::printf("], \"ids\": [");
    std::vector<int> ids = t->getNodesId();
    for (size_t i = 0; i < ids.size(); i++) std::printf("%s%d", i ? ", " : "", ids[i]);
    std::printf("]");
    if (t->isRooted()) {
      t->unroot();
      std::printf(", \"unrooted\": \"%s\"", TreeTemplateTools::treeToParenthesis(*t).c_str());
    }
    std::printf("}\n");
  }
  // NH model set parameter naming
  std::unique_ptr<TreeTemplate<Node> > t(TreeTemplateTools::parenthesisToTree("((A:0.1,B:0.2):0.3,(C:0.1,D:0.2):0.1);"));
  std::map<std::string, std::vector<Vint> > globals;
  globals["T92.kappa"] = {};
  std::map<std::string, std::string> alias;
  std::unique_ptr<SubstitutionModelSet> set(SubstitutionModelSetTools::createNonHomogeneousModelSet(
      new T92(dna, 3.), new GCFrequencySet(dna), t.get(), alias, globals));
  set->setParameterValue("T92.theta_2", 0.7);
  std::printf("{\"kind\": \"modelset\", \"n\": %zu, \"names\": [", set->getNumberOfModels());
  std::vector<std::string> pn = set->getParameters().getParameterNames();
  for (size_t i = 0; i < pn.size(); i++) std::printf("%s\"%s\"", i ? ", " : "", pn[i].c_str());
  std::printf("], \"independent\": [");
  std::vector<std::string> in = set->getIndependentParameters().getParameterNames();
  for (size_t i = 0; i < in.size(); i++) std::printf("%s\"%s\"", i ? ", " : "", in[i].c_str());
  // the global kappa: changing model 1's copy moves every model; nodes with the parameter
  ParameterList k = set->getParameters().createSubList(std::vector<std::string>(1, "T92.kappa_1"));
  k[0].setValue(2.5);
  set->matchParametersValues(k);
  std::printf("], \"kappa_last\": %.17g, \"changed_models\": %zu, \"kappa_nodes\": %zu, \"theta2_nodes\": [",
              set->getModel(set->getNumberOfModels() - 1)->getParameterValue("kappa"),
              set->getLastChangedModels().size(), set->getNodesWithParameter("T92.kappa_1").size());
  std::vector<int> tn = set->getNodesWithParameter("T92.theta_2");
  for (size_t i = 0; i < tn.size(); i++) std::printf("%s%d", i ? ", " : "", tn[i]);
  std::printf("], \"theta2\": %.17g, \"theta1\": %.17g}\n", set->getModel(1)->getParameterValue("theta"),
              set->getModel(0)->getParameterValue("theta"));
  // NonHomogeneousSequenceSimulator on a rooted cherry with per-branch GC content: the
  // empirical joint distribution of the two leaves against sum_c p_c sum_x pi_x
  // P_a[c][x][i] P_b[c][x][j] (tests/test_host.py)
  {
    std::unique_ptr<TreeTemplate<Node> > ch(TreeTemplateTools::parenthesisToTree("(a:0.15,b:0.4);"));
    std::map<std::string, std::vector<Vint> > g;
    g["T92.kappa"] = {};
    std::unique_ptr<SubstitutionModelSet> ms(SubstitutionModelSetTools::createNonHomogeneousModelSet(
        new T92(dna, 2.), new GCFrequencySet(dna, 0.35), ch.get(), std::map<std::string, std::string>(), g));
    ms->setParameterValue("T92.theta_1", 0.3);
    ms->setParameterValue("T92.theta_2", 0.7);
    GammaDiscreteDistribution rd(4, 0.6, 0.6);
    NonHomogeneousSequenceSimulator sim(ms.get(), &rd, ch.get());
    const size_t n = 200000;
    std::unique_ptr<SiteContainer> sites(sim.simulate(n));
    std::vector<double> emp(16, 0.), want(16, 0.);
    for (size_t i = 0; i < n; i++) emp[sites->getState(0, i) * 4 + sites->getState(1, i)] += 1. / n;
    const Vdouble pi = ms->getRootFrequencies();
    for (size_t c = 0; c < 4; c++) {
      const double r = rd.getCategory(c), pc = rd.getProbability(c);
      RowMatrix<double> Pa = ms->getModelForNode(ch->getRootNode()->getSon(0)->getId())->getPij_t(0.15 * r);
      RowMatrix<double> Pb = ms->getModelForNode(ch->getRootNode()->getSon(1)->getId())->getPij_t(0.4 * r);
      for (int x = 0; x < 4; x++)
        for (int i = 0; i < 4; i++)
          for (int j = 0; j < 4; j++) want[i * 4 + j] += pc * pi[x] * Pa(x, i) * Pb(x, j);
    }
    std::printf("{\"kind\": \"simulator\", \"n\": %zu, \"names\": [\"%s\", \"%s\"], ", n,
                sites->getSequencesNames()[0].c_str(), sites->getSequencesNames()[1].c_str());
    printVec("empirical", emp);
    std::printf(", ");
    printVec("expected", want);
    std::printf("}\n");
  }
  // PseudoNewton with its conjugate-gradient correction
  {
    OvershootLikelihood rl;
    const unsigned n = OptimizationTools::optimizeNumericalParameters2(&rl, rl.getParameters(), 0, 1e-10, 20000, 0, 0);
    std::printf("{\"kind\": \"pn_cg\", \"f\": %.17g, \"x\": %.17g, \"y\": %.17g, \"evals\": %u, \"steps\": %u}\n",
                rl.getValue(), rl.getParameters().getParameterValue("x"), rl.getParameters().getParameterValue("y"), n,
                OptimizationTools::lastSteps_);
  }
  // optimizeNumericalParametersWithGlobalClock2: conjugate gradient over two-point numerical
  // derivatives (the default), and PseudoNewton over three-point ones
  for (const std::string& method : {OptimizationTools::OPTIMIZATION_GRADIENT, OptimizationTools::OPTIMIZATION_NEWTON}) {
    OvershootClock rl;
    const unsigned n = OptimizationTools::optimizeNumericalParametersWithGlobalClock2(&rl, rl.getParameters(), 0, 1e-10,
                                                                                      20000, 0, 0, 1, method);
    std::printf("{\"kind\": \"clock2\", \"method\": \"%s\", \"f\": %.17g, \"x\": %.17g, \"y\": %.17g, \"evals\": %u}\n",
                method.c_str(), rl.getValue(), rl.getParameters().getParameterValue("x"),
                rl.getParameters().getParameterValue("y"), n);
  }
  return 0;
}
