#include "Alphabet.h"
