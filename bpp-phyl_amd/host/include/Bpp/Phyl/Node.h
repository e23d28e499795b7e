#include "TreeTemplate.h"
