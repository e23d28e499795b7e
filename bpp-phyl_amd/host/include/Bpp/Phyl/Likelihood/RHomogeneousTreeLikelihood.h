#include "TreeLikelihood.h"
