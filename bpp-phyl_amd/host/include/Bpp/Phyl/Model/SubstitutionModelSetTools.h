#include "SubstitutionModelSet.h"
