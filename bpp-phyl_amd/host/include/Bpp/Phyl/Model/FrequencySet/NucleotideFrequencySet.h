#include "../Models.h"
