#ifndef BPP_AMD_PARAMETERLIST_H
#define BPP_AMD_PARAMETERLIST_H
#include "Parameter.h"
#endif
