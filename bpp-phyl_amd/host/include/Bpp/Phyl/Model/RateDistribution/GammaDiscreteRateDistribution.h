// Rate-across-sites distributions (Model/RateDistribution/GammaDiscreteRateDistribution.h:48-60
// and ConstantRateDistribution.h of the reference): Gamma with beta = alpha (mean 1).
#ifndef BPP_AMD_GAMMARATEDIST_H
#define BPP_AMD_GAMMARATEDIST_H
#include "../../../Numeric/Prob/DiscreteDistribution.h"
namespace bpp {
class GammaDiscreteRateDistribution : public GammaDiscreteDistribution {
 public:
  GammaDiscreteRateDistribution(size_t n, double alpha = 1.);
  GammaDiscreteRateDistribution* clone() const override { return new GammaDiscreteRateDistribution(*this); }
  void fireParameterChanged(const ParameterList& pl) override;
};
class ConstantRateDistribution : public ConstantDistribution {
 public:
  ConstantRateDistribution() : ConstantDistribution(1.) {}
  ConstantRateDistribution* clone() const override { return new ConstantRateDistribution(*this); }
};
}  // namespace bpp
#endif
