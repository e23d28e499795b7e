// Bio++-compatible exception family used by the host mirror (the reference gets
// these from bpp-core 2.4.1; see SURVEY.md 8b "Errors").
#ifndef BPP_AMD_EXCEPTIONS_H
#define BPP_AMD_EXCEPTIONS_H

#include <stdexcept>
#include <string>

namespace bpp {

class Exception : public std::exception {
 protected:
  std::string message_;

 public:
  explicit Exception(const std::string& message) : message_(message) {}
  explicit Exception(const char* message) : message_(message) {}
  virtual ~Exception() noexcept {}
  const char* what() const noexcept override { return message_.c_str(); }
  const std::string& message() const { return message_; }
};

class IOException : public Exception {
 public:
  explicit IOException(const std::string& m) : Exception(m) {}
};

class NullPointerException : public Exception {
 public:
  explicit NullPointerException(const std::string& m) : Exception(m) {}
};

class BadIntException : public Exception {
  int badInt_;

 public:
  BadIntException(int badInt, const std::string& m)
      : Exception("BadIntException: " + m + " (" + std::to_string(badInt) + ")"), badInt_(badInt) {}
  int getBadInteger() const { return badInt_; }
};

class BadCharException : public Exception {
 public:
  BadCharException(const std::string& c, const std::string& m) : Exception("BadCharException: " + m + " (" + c + ")") {}
};

class IndexOutOfBoundsException : public Exception {
 public:
  IndexOutOfBoundsException(const std::string& m, size_t badIndex, size_t lo, size_t hi)
      : Exception("IndexOutOfBoundsException: " + m + " " + std::to_string(badIndex) + " not in [" +
                  std::to_string(lo) + ", " + std::to_string(hi) + "]") {}
};

class ParameterNotFoundException : public Exception {
 public:
  ParameterNotFoundException(const std::string& m, const std::string& param)
      : Exception("ParameterNotFoundException: " + m + " (" + param + ")") {}
};

class ConstraintException : public Exception {
 public:
  ConstraintException(const std::string& m, const std::string& param, double value)
      : Exception("ConstraintException: " + m + " (" + param + " = " + std::to_string(value) + ")") {}
};

class SequenceNotFoundException : public Exception {
 public:
  SequenceNotFoundException(const std::string& m, const std::string& id)
      : Exception("SequenceNotFoundException: " + m + " (" + id + ")") {}
};

class AlphabetMismatchException : public Exception {
 public:
  explicit AlphabetMismatchException(const std::string& m) : Exception("AlphabetMismatchException: " + m) {}
};

class UnrootedTreeException : public Exception {
 public:
  explicit UnrootedTreeException(const std::string& m) : Exception("UnrootedTreeException: " + m) {}
};

class NodeNotFoundException : public Exception {
 public:
  NodeNotFoundException(const std::string& m, const std::string& id)
      : Exception("NodeNotFoundException: " + m + " (" + id + ")") {}
};

class ZeroDivisionException : public Exception {
 public:
  explicit ZeroDivisionException(const std::string& m) : Exception("ZeroDivisionException: " + m) {}
};

// Raised when libplk (the MI355X engine under the likelihood classes) reports an error.
class DeviceException : public Exception {
  int code_;

 public:
  DeviceException(int code, const std::string& m)
      : Exception("DeviceException (plk " + std::to_string(code) + "): " + m), code_(code) {}
  int code() const { return code_; }
};

}  // namespace bpp

#endif
