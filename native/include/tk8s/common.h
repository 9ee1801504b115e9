// Shared helpers for the tk8s native layer (HIP runtime error handling, RAII buffers/timers;
// the JSON writer lives in tk8s/json.h so HIP-free code can use it).
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

#include "tk8s/json.h"

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

}  // namespace tk8s
