// bpp-core output streams (OutputStream / StlOutputStream subset): the optimisers'
// message and profile channels.  An StlOutputStream owns the std::ostream it wraps.
#ifndef BPP_AMD_OUTPUTSTREAM_H
#define BPP_AMD_OUTPUTSTREAM_H

#include <fstream>
#include <iomanip>
#include <memory>
#include <ostream>
#include <string>

namespace bpp {

class OutputStream {
 protected:
  int precision_ = 6;  // digits of the doubles written (bpp-core AbstractOutputStream default)

 public:
  virtual ~OutputStream() {}
  OutputStream& setPrecision(int digits) {
    precision_ = digits;
    return *this;
  }
  int getPrecision() const { return precision_; }
  virtual OutputStream& operator<<(const std::string& s) = 0;
  virtual OutputStream& operator<<(double d) = 0;
  virtual OutputStream& operator<<(long d) = 0;
  virtual OutputStream& endLine() = 0;
  virtual OutputStream& flush() = 0;
  OutputStream& operator<<(const char* s) { return *this << std::string(s); }
  OutputStream& operator<<(int d) { return *this << (long)d; }
  OutputStream& operator<<(unsigned int d) { return *this << (long)d; }
  OutputStream& operator<<(size_t d) { return *this << (long)d; }
};

class StlOutputStream : public OutputStream {
  std::unique_ptr<std::ostream> stream_;

 public:
  explicit StlOutputStream(std::ostream* stream) : stream_(stream) {}
  using OutputStream::operator<<;
  OutputStream& operator<<(const std::string& s) override {
    if (stream_) *stream_ << s;
    return *this;
  }
  OutputStream& operator<<(double d) override {
    if (stream_) *stream_ << std::setprecision(precision_) << d;
    return *this;
  }
  OutputStream& operator<<(long d) override {
    if (stream_) *stream_ << d;
    return *this;
  }
  OutputStream& endLine() override {
    if (stream_) *stream_ << std::endl;
    return *this;
  }
  OutputStream& flush() override {
    if (stream_) stream_->flush();
    return *this;
  }
};

}  // namespace bpp

#endif
