#include "DiscreteDistribution.h"
