#ifndef BPP_AMD_APPLICATIONTOOLS_H
#define BPP_AMD_APPLICATIONTOOLS_H
#include <iostream>
#include <string>
#include "../Text/TextTools.h"
namespace bpp {
// Console reporting as in bpp-core's ApplicationTools (displayResult / displayTask ...).
struct ApplicationTools {
  static int& verbosity() {
    static int v = 1;
    return v;
  }
  template <class T>
  static void displayResult(const std::string& text, const T& result) {
    if (verbosity() > 0) std::cout << text << ": " << result << std::endl;
  }
  static void displayMessage(const std::string& text) {
    if (verbosity() > 0) std::cout << text << std::endl;
  }
  static void displayWarning(const std::string& text) {
    if (verbosity() > 0) std::cerr << "WARNING!!! " << text << std::endl;
  }
  static void displayTask(const std::string& text, bool = false) {
    if (verbosity() > 0) std::cout << text << "... " << std::flush;
  }
  static void displayTaskDone() {
    if (verbosity() > 0) std::cout << "Done." << std::endl;
  }
};
}  // namespace bpp
#endif
