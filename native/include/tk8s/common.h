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

#include "tk8s/failfast.h"
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

// A bounded wait ran out: the GPU work (or the collective) did not finish in time.
struct GpuTimeout : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Releases a stall kernel armed by a fault point (stream_kernels.hip); a no-op when none is
// armed. Every bounded wait calls it before giving up, so the stalled queue drains.
void gpu_stall_release();

// hipStreamSynchronize under a deadline (TK8S_GPU_SYNC_TIMEOUT_S, default 30 s): the probes'
// kernels are finite, so a wait that runs out means a wedged GPU or a dead link, and the payload
// must report it rather than hang the bring-up.
inline void wait_stream(hipStream_t s, const char* what, double timeout_s = gpu_sync_timeout_s()) {
  hipError_t last = hipSuccess;
  const std::string r = poll_until([&] { return (last = hipStreamQuery(s)) != hipErrorNotReady; }, timeout_s);
  if (!r.empty()) {
    gpu_stall_release();
    throw GpuTimeout(std::string(what) + ": GPU work " + r);
  }
  if (last != hipSuccess) throw HipError(what, last, __FILE__, __LINE__);
}

inline void wait_event(hipEvent_t e, const char* what, double timeout_s = gpu_sync_timeout_s()) {
  hipError_t last = hipSuccess;
  const std::string r = poll_until([&] { return (last = hipEventQuery(e)) != hipErrorNotReady; }, timeout_s);
  if (!r.empty()) {
    gpu_stall_release();
    throw GpuTimeout(std::string(what) + ": GPU work " + r);
  }
  if (last != hipSuccess) throw HipError(what, last, __FILE__, __LINE__);
}

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
  // Milliseconds between start and stop (waits for stop, bounded: wait_event).
  float elapsed_ms(double bound_s = gpu_sync_timeout_s()) {
    wait_event(stop_, "timed region", bound_s);
    float ms = 0.f;
    TK8S_HIP_CHECK(hipEventElapsedTime(&ms, start_, stop_));
    return ms;
  }

 private:
  hipEvent_t start_{}, stop_{};
};

}  // namespace tk8s
