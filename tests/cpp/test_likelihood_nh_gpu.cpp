// Drop-in check of the non-homogeneous Bio++ surface on the MI355X: the calls the
// reference's test/test_likelihood_nh.cpp makes, in its order (header set, GC root
// frequencies, T92 with a global kappa, createNonHomogeneousModelSet, Gamma(4, 1),
// per-branch theta, NonHomogeneousSequenceSimulator::simulate(1000), two
// RNonHomogeneousTreeLikelihood fits (reparametrizeRoot false / true) of the
// substitution-model parameters by OPTIMIZATION_NEWTON, and the same acceptance rule:
// every branch's theta recovered within 0.2 on average over 3 replicates).  Then the
// reference's fitModelNH path (DRNonHomogeneousTreeLikelihood with the root
// reparametrised, tree scale then every parameter) and the engine-side bookkeeping the
// host mirror adds: per-theta evaluations recompute one eigen-system and one branch,
// BrLenRoot / RootPosition derivatives against central differences.  The random numbers
// come from RandomTools' fixed seed.  Exit code 0 = pass.
#include <Bpp/Numeric/Matrix/MatrixTools.h>
#include <Bpp/Seq/Alphabet/AlphabetTools.h>
#include <Bpp/Phyl/TreeTemplate.h>
#include <Bpp/Phyl/Model/Nucleotide/T92.h>
#include <Bpp/Phyl/Model/FrequencySet/NucleotideFrequencySet.h>
#include <Bpp/Phyl/Model/SubstitutionModelSetTools.h>
#include <Bpp/Phyl/Model/RateDistribution/GammaDiscreteRateDistribution.h>
#include <Bpp/Phyl/Simulation/NonHomogeneousSequenceSimulator.h>
#include <Bpp/Phyl/Likelihood/RNonHomogeneousTreeLikelihood.h>
#include <Bpp/Phyl/Likelihood/DRNonHomogeneousTreeLikelihood.h>
#include <Bpp/Phyl/OptimizationTools.h>
#include <Bpp/Numeric/Random/RandomTools.h>
#include <Bpp/Numeric/VectorTools.h>
#include <Bpp/App/ApplicationTools.h>

#include <cmath>
#include <iomanip>
#include <iostream>
#include <memory>

using namespace bpp;
using namespace std;

static int failures = 0;

static void expect(const string& what, bool ok, const string& detail = "") {
  cout << what << (detail.empty() ? "" : ": " + detail) << " " << (ok ? "ok" : "FAIL") << endl;
  if (!ok) failures++;
}

static void expectNear(const string& what, double got, double want, double tol) {
  ostringstream d;
  d << setprecision(12) << got << " (expected " << want << ", tol " << tol << ")";
  expect(what, fabs(got - want) <= tol, d.str());
}

// fitModelNH of the reference test (the DR class with the root reparametrised or not):
// initial value, optimizeTreeScale, then every parameter by the default PseudoNewton
static void fitModelNH(SubstitutionModelSet* model, DiscreteDistribution* rdist, const Tree& tree,
                       const SiteContainer& sites, bool reparam) {
  DRNonHomogeneousTreeLikelihood tl(tree, sites, model, rdist, false, reparam);
  tl.initialize();
  const double v0 = tl.getValue();
  cout << setprecision(20) << "fitModelNH(reparam=" << reparam << ") initial " << v0 << endl;
  OptimizationTools::optimizeTreeScale(&tl);
  const double v1 = tl.getValue();
  OptimizationTools::optimizeNumericalParameters2(&tl, tl.getParameters(), 0, 0.000001, 10000, 0, 0);
  const double v2 = tl.getValue();
  cout << "  after tree scale " << v1 << ", after full optimisation " << v2 << " ("
       << OptimizationTools::lastSteps_ << " PseudoNewton steps)" << endl;
  expect("fitModelNH(reparam=" + to_string(reparam) + ") improves -lnL", v2 <= v1 + 1e-9 && v1 <= v0 + 1e-9);
  if (reparam) {
    ParameterList bl = tl.getBranchLengthsParameters();
    expect("BrLenRoot / RootPosition registered", bl.hasParameter("BrLenRoot") && bl.hasParameter("RootPosition"));
  }
}

// analytic first / second derivatives of the root parameters (plk_root_pair_derivatives)
// against central differences of -lnL
static void rootDerivatives(RNonHomogeneousTreeLikelihood& tl) {
  for (const char* name : {"BrLenRoot", "RootPosition"}) {
    const double d1 = tl.getFirstOrderDerivative(name), d2 = tl.getSecondOrderDerivative(name);
    const double t = tl.getParameters().getParameterValue(name);
    const double h = 1e-5 * max(t, 1e-2);
    ParameterList one = tl.getParameters().createSubList(vector<string>(1, name));
    const double f0 = tl.getValue();
    one[0].setValue(t + h);
    const double fp = tl.f(one);
    one[0].setValue(t - h);
    const double fm = tl.f(one);
    one[0].setValue(t);
    tl.f(one);
    const double n1 = (fp - fm) / (2 * h), n2 = (fp - 2 * f0 + fm) / (h * h);
    expectNear(string("d(-lnL)/d") + name + " analytic vs central difference", d1, n1, 1e-6 * max(1., fabs(n1)));
    expectNear(string("d2(-lnL)/d") + name + "2 analytic vs central difference", d2, n2, 2e-3 * max(1., fabs(n2)));
  }
}

int main() {
  ApplicationTools::verbosity() = 0;
  TreeTemplate<Node>* tree =
      TreeTemplateTools::parenthesisToTree("(((A:0.1, B:0.2):0.3,C:0.1):0.2,(D:0.3,(E:0.2,F:0.05):0.1):0.1);");
  vector<string> seqNames = tree->getLeavesNames();
  vector<int> ids = tree->getNodesId();
  const NucleicAlphabet* alphabet = &AlphabetTools::DNA_ALPHABET;
  FrequencySet* rootFreqs = new GCFrequencySet(alphabet);
  SubstitutionModel* model = new T92(alphabet, 3.);
  std::map<std::string, std::vector<Vint> > globalParameterNames;
  globalParameterNames["T92.kappa"] = {};
  map<string, string> alias;
  SubstitutionModelSet* modelSet =
      SubstitutionModelSetTools::createNonHomogeneousModelSet(model, rootFreqs, tree, alias, globalParameterNames);
  DiscreteDistribution* rdist = new GammaDiscreteRateDistribution(4, 1.0);

  size_t nsites = 1000;
  unsigned int nrep = 3;
  size_t nmodels = modelSet->getNumberOfModels();
  vector<double> thetas(nmodels), thetasEst1(nmodels), thetasEst2(nmodels);
  // the reference's parameter layout: root frequencies first, "_<k>" per model, the global
  // kappa aliased to model 1's (left out of the independent parameters)
  {
    const ParameterList all = modelSet->getParameters(), ind = modelSet->getIndependentParameters();
    expect("model set parameters: GC.theta first", all[0].getName() == "GC.theta");
    expect("model set parameters: T92.kappa_1 independent, T92.kappa_2 an alias",
           ind.hasParameter("T92.kappa_1") && all.hasParameter("T92.kappa_2") && !ind.hasParameter("T92.kappa_2"));
    expect("one model per branch", nmodels == ids.size() - 1, to_string(nmodels));
    expect("kappa reaches every branch", modelSet->getNodesWithParameter("T92.kappa_1").size() == nmodels);
  }
  for (size_t i = 0; i < nmodels; ++i) {
    double theta = RandomTools::giveRandomNumberBetweenZeroAndEntry(0.9) + 0.05;
    cout << "Theta" << i << " set to " << theta << endl;
    modelSet->setParameterValue("T92.theta_" + TextTools::toString(i + 1), theta);
    thetas[i] = theta;
  }
  NonHomogeneousSequenceSimulator simulator(modelSet, rdist, tree);

  size_t evals1 = 0, evals2 = 0;
  for (unsigned int j = 0; j < nrep; j++) {
    OutputStream* profiler = new StlOutputStream(new ofstream("gpurun_out/nh_profile.txt", ios::out));
    OutputStream* messenger = new StlOutputStream(new ofstream("gpurun_out/nh_messages.txt", ios::out));
    unique_ptr<SiteContainer> sites(simulator.simulate(nsites));
    unique_ptr<SubstitutionModelSet> modelSet2(modelSet->clone());
    unique_ptr<SubstitutionModelSet> modelSet3(modelSet->clone());
    RNonHomogeneousTreeLikelihood tl(*tree, *sites.get(), modelSet2.get(), rdist, true, true, false);
    tl.initialize();
    RNonHomogeneousTreeLikelihood tl2(*tree, *sites.get(), modelSet3.get(), rdist, true, true, true);
    tl2.initialize();
    // the two parametrisations describe the same tree: same likelihood
    expectNear("rep " + to_string(j) + ": reparametrised root, same -lnL", tl2.getValue(), tl.getValue(),
               1e-10 * tl.getValue());

    unsigned int c1 = OptimizationTools::optimizeNumericalParameters2(
        &tl, tl.getSubstitutionModelParameters(), 0, 0.0001, 10000, messenger, profiler, false, false, 1,
        OptimizationTools::OPTIMIZATION_NEWTON);
    unsigned int c2 = OptimizationTools::optimizeNumericalParameters2(
        &tl2, tl2.getSubstitutionModelParameters(), 0, 0.0001, 10000, messenger, profiler, false, false, 1,
        OptimizationTools::OPTIMIZATION_NEWTON);
    evals1 += c1;
    evals2 += c2;
    cout << c1 << ": " << tl.getValue() << "\t" << c2 << ": " << tl2.getValue() << endl;
    for (size_t i = 0; i < nmodels; ++i) {
      cout << modelSet2->getModel(i)->getParameter("theta").getValue() << "\t"
           << modelSet3->getModel(i)->getParameter("theta").getValue() << endl;
      thetasEst1[i] += modelSet2->getModel(i)->getParameter("theta").getValue();
      thetasEst2[i] += modelSet3->getModel(i)->getParameter("theta").getValue();
    }
    // engine bookkeeping: one theta moves one model, one eigen-system, one branch
    {
      const auto s0 = tl.getEvaluationStats();
      ParameterList one = tl.getParameters().createSubList(vector<string>(1, "T92.theta_3"));
      one[0].setValue(one[0].getValue() * 0.9);
      tl.setParameters(one);
      const auto s1 = tl.getEvaluationStats();
      expect("rep " + to_string(j) + ": one theta -> one eigen-system, one branch P(t)",
             s1.eigenUploads - s0.eigenUploads == 1 && s1.pmatBranches - s0.pmatBranches == 1,
             to_string(s1.eigenUploads - s0.eigenUploads) + " eigen, " +
                 to_string(s1.pmatBranches - s0.pmatBranches) + " branches");
      ParameterList k = tl.getParameters().createSubList(vector<string>(1, "T92.kappa_1"));
      k[0].setValue(k[0].getValue() * 1.1);
      tl.setParameters(k);
      const auto s2 = tl.getEvaluationStats();
      expect("rep " + to_string(j) + ": global kappa -> every eigen-system",
             s2.eigenUploads - s1.eigenUploads == nmodels, to_string(s2.eigenUploads - s1.eigenUploads));
      cout << "evaluation stats (reparam=false): " << s2.evaluations << " evaluations, " << s2.eigenUploads
           << " eigen uploads, " << s2.pmatBranches << " branch P(t), " << s2.fullTraversals << " full traversals"
           << endl;
    }
    if (j == 0) rootDerivatives(tl2);
    delete profiler;
    delete messenger;
  }
  thetasEst1 /= static_cast<double>(nrep);
  thetasEst2 /= static_cast<double>(nrep);
  cout << "function evaluations: " << evals1 << " (reparam=false), " << evals2 << " (reparam=true)" << endl;
  for (size_t i = 0; i < thetas.size(); ++i) {
    cout << thetas[i] << "\t" << thetasEst1[i] << "\t" << thetasEst2[i] << endl;
    double diff1 = abs(thetas[i] - thetasEst1[i]);
    double diff2 = abs(thetas[i] - thetasEst2[i]);
    expect("theta_" + to_string(i + 1) + " recovered within 0.2 (both parametrisations)", diff1 <= 0.2 && diff2 <= 0.2);
  }
  // a change of the root frequencies only (no model, no branch) re-reduces the root with the
  // new frequencies on every engine path: the lnL-only kernels, the materialising fused
  // traversal (BPP_AMD_FUSED=0; its cached root reduction must not be reused) and the
  // per-subtree-compressed one; checked against a fresh likelihood at the new value
  {
    unique_ptr<SiteContainer> sites(simulator.simulate(nsites));
    for (const char* fused : {"1", "0"})
      for (bool usePatterns : {false, true}) {
        setenv("BPP_AMD_FUSED", fused, 1);
        unique_ptr<SubstitutionModelSet> ms(modelSet->clone());
        RNonHomogeneousTreeLikelihood tl(*tree, *sites, ms.get(), rdist, false, usePatterns, false);
        tl.initialize();
        const double before = tl.getValue();
        ParameterList gc = tl.getParameters().createSubList(vector<string>(1, "GC.theta"));
        gc[0].setValue(gc[0].getValue() < 0.5 ? 0.8 : 0.2);
        tl.setParameters(gc);
        unique_ptr<SubstitutionModelSet> ms2(modelSet->clone());
        ms2->setParameterValue("GC.theta", gc[0].getValue());
        RNonHomogeneousTreeLikelihood fresh(*tree, *sites, ms2.get(), rdist, false, usePatterns, false);
        fresh.initialize();
        const string tag = string("root frequencies only (fused=") + fused + ", usePatterns=" +
                           (usePatterns ? "true" : "false") + ")";
        expect(tag + ": lnL moved", tl.getValue() != before);
        expectNear(tag + ": same -lnL as a fresh likelihood", tl.getValue(), fresh.getValue(),
                   1e-12 * fresh.getValue());
      }
    unsetenv("BPP_AMD_FUSED");
  }
  // the reference's fitModelNH on one more simulated alignment, both root parametrisations
  {
    unique_ptr<SiteContainer> sites(simulator.simulate(nsites));
    for (bool reparam : {false, true}) {
      unique_ptr<SubstitutionModelSet> ms(modelSet->clone());
      fitModelNH(ms.get(), rdist, *tree, *sites, reparam);
    }
  }
  delete tree;
  delete modelSet;
  delete rdist;
  cout << (failures ? "FAILED" : "PASSED") << endl;
  return failures ? 1 : 0;
}
