#include "../Alphabet/Alphabet.h"
