// Development microbenchmark: host-side costs of the first HIP calls on gfx950 (what the
// validation payload pays before any kernel runs). Prints one JSON object of milliseconds.
//   hipcc -O2 --offload-arch=gfx950 -o /tmp/init_costs native/bench/init_costs.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

__global__ void touch(unsigned* p) { p[threadIdx.x] = threadIdx.x; }

// `init_costs null`: first launch on the legacy null stream, before any stream is created —
// does the runtime's own queue come for free, or does it cost what a created stream costs?
static int null_first() {
  auto t0 = clk::now();
  int n = 0;
  (void)hipGetDeviceCount(&n);
  auto t1 = clk::now();
  (void)hipSetDevice(0);
  auto t2 = clk::now();
  void* a = nullptr;
  (void)hipMalloc(&a, 1ull << 30);
  auto t3 = clk::now();
  hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, nullptr, static_cast<unsigned*>(a));
  (void)hipStreamSynchronize(nullptr);
  auto t4 = clk::now();
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  auto t5 = clk::now();
  hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s, static_cast<unsigned*>(a));
  (void)hipStreamSynchronize(s);
  auto t6 = clk::now();
  std::printf("{\"mode\": \"null\", \"get_device_count_ms\": %.3f, \"set_device_ms\": %.3f, \"malloc_1g_ms\": %.3f, "
              "\"null_first_launch_ms\": %.3f, \"stream_after_null_ms\": %.3f, \"stream_launch_ms\": %.3f, \"total_ms\": %.3f}\n",
              ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4), ms(t4, t5), ms(t5, t6), ms(t0, t6));
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'n') return null_first();
  auto t0 = clk::now();
  int n = 0;
  (void)hipGetDeviceCount(&n);
  auto t1 = clk::now();
  (void)hipSetDevice(0);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  auto t2 = clk::now();
  void* a = nullptr;
  (void)hipMalloc(&a, 1ull << 30);
  auto t3 = clk::now();
  hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s, static_cast<unsigned*>(a));
  (void)hipStreamSynchronize(s);
  auto t4 = clk::now();
  void* b = nullptr;
  (void)hipMalloc(&b, 1ull << 30);
  auto t5 = clk::now();
  void* c = nullptr;
  (void)hipMallocAsync(&c, 1ull << 30, s);
  (void)hipStreamSynchronize(s);
  auto t6 = clk::now();
  void* d = nullptr;
  (void)hipMalloc(&d, 64ull << 20);
  auto t7 = clk::now();
  hipStream_t s2;
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  auto t8 = clk::now();
  (void)hipFree(b);
  auto t9 = clk::now();
  std::printf("{\"device_count\": %d, \"get_device_count_ms\": %.3f, \"set_device_stream_ms\": %.3f, "
              "\"malloc_1g_first_ms\": %.3f, \"first_launch_ms\": %.3f, \"malloc_1g_second_ms\": %.3f, "
              "\"malloc_async_1g_ms\": %.3f, \"malloc_64m_ms\": %.3f, \"second_stream_ms\": %.3f, \"free_1g_ms\": %.3f, "
              "\"total_ms\": %.3f}\n",
              n, ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4), ms(t4, t5), ms(t5, t6), ms(t6, t7), ms(t7, t8),
              ms(t8, t9), ms(t0, t9));
  return 0;
}
