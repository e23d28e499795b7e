#include "GammaDiscreteRateDistribution.h"
