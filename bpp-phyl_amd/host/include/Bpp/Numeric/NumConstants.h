#ifndef BPP_AMD_NUMCONSTANTS_H
#define BPP_AMD_NUMCONSTANTS_H
#include <limits>
namespace bpp {
struct NumConstants {
  static double TINY() { return 1e-12; }
  static double VERY_TINY() { return 1e-20; }
  static double SMALL() { return 1e-6; }
  static double MILLI() { return 1e-3; }
  static double INF() { return std::numeric_limits<double>::infinity(); }
};
}  // namespace bpp
#endif
