// Shared helpers for the tk8s native layer (HIP runtime error handling, tiny JSON writer).
//
// The reference (cheapRoc/tritonK8ssupervisor) has no native code at all;
// every native component here is new and exists to validate MI355X workers during bring-up.
#pragma once

#include <cstdint>
#include <cstdio>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

namespace tk8s {

struct HipError : std::runtime_error {
  hipError_t code;
  HipError(const char* expr, hipError_t e, const char* file, int line)
      : std::runtime_error(std::string(file) + ":" + std::to_string(line) + ": " + expr +
                           " failed: " + hipGetErrorString(e)),
        code(e) {}
};

#define TK8S_HIP_CHECK(expr)                                              \
  do {                                                                    \
    hipError_t _tk8s_e = (expr);                                          \
    if (_tk8s_e != hipSuccess)                                            \
      throw ::tk8s::HipError(#expr, _tk8s_e, __FILE__, __LINE__);         \
  } while (0)

// RAII device buffer (hipMalloc / hipFree on the current device).
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t bytes) : bytes_(bytes) {
    if (bytes) TK8S_HIP_CHECK(hipMalloc(&ptr_, bytes));
  }
  ~DeviceBuffer() {
    if (ptr_) (void)hipFree(ptr_);
  }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  DeviceBuffer(DeviceBuffer&& o) noexcept : ptr_(o.ptr_), bytes_(o.bytes_) { o.ptr_ = nullptr; o.bytes_ = 0; }
  void* get() const { return ptr_; }
  size_t bytes() const { return bytes_; }
  template <class T> T* as() const { return static_cast<T*>(ptr_); }

 private:
  void* ptr_ = nullptr;
  size_t bytes_ = 0;
};

// RAII event pair for timing a region on a stream.
class EventTimer {
 public:
  EventTimer() {
    TK8S_HIP_CHECK(hipEventCreate(&start_));
    TK8S_HIP_CHECK(hipEventCreate(&stop_));
  }
  ~EventTimer() {
    (void)hipEventDestroy(start_);
    (void)hipEventDestroy(stop_);
  }
  void start(hipStream_t s) { TK8S_HIP_CHECK(hipEventRecord(start_, s)); }
  void stop(hipStream_t s) { TK8S_HIP_CHECK(hipEventRecord(stop_, s)); }
  // Milliseconds between start and stop (synchronises on stop).
  float elapsed_ms() {
    TK8S_HIP_CHECK(hipEventSynchronize(stop_));
    float ms = 0.f;
    TK8S_HIP_CHECK(hipEventElapsedTime(&ms, start_, stop_));
    return ms;
  }

 private:
  hipEvent_t start_{}, stop_{};
};

// Minimal JSON object writer: enough for flat records and arrays of records.
class Json {
 public:
  Json& kv(const std::string& k, const std::string& v) { key(k); str(v); return *this; }
  Json& kv(const std::string& k, const char* v) { return kv(k, std::string(v)); }
  Json& kv(const std::string& k, double v) { key(k); num(v); return *this; }
  Json& kv(const std::string& k, int64_t v) { key(k); os_ << v; return *this; }
  Json& kv(const std::string& k, uint64_t v) { key(k); os_ << v; return *this; }
  Json& kv(const std::string& k, int v) { return kv(k, static_cast<int64_t>(v)); }
  Json& kv(const std::string& k, unsigned v) { return kv(k, static_cast<uint64_t>(v)); }
  Json& kv(const std::string& k, bool v) { key(k); os_ << (v ? "true" : "false"); return *this; }
  Json& raw(const std::string& k, const std::string& json) { key(k); os_ << json; return *this; }
  std::string str() const { return "{" + os_.str() + "}"; }

  static std::string escape(const std::string& s) {
    std::string o = "\"";
    for (char c : s) {
      switch (c) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\n': o += "\\n"; break;
        case '\t': o += "\\t"; break;
        default:
          if (static_cast<unsigned char>(c) < 0x20) {
            char buf[8];
            std::snprintf(buf, sizeof buf, "\\u%04x", c);
            o += buf;
          } else {
            o += c;
          }
      }
    }
    return o + "\"";
  }
  static std::string array(const std::vector<std::string>& items) {
    std::string o = "[";
    for (size_t i = 0; i < items.size(); ++i) o += (i ? "," : "") + items[i];
    return o + "]";
  }

 private:
  void key(const std::string& k) {
    if (!first_) os_ << ",";
    first_ = false;
    os_ << escape(k) << ":";
  }
  void str(const std::string& v) { os_ << escape(v); }
  void num(double v) {
    char buf[64];
    std::snprintf(buf, sizeof buf, "%.9g", v);
    os_ << buf;
  }
  std::ostringstream os_;
  bool first_ = true;
};

}  // namespace tk8s
