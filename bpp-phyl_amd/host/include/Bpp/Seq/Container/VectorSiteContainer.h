#include "SiteContainer.h"
