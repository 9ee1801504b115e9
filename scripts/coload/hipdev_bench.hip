// (HIPDEV_SAMPLE=1: a 0.25 ms wall-clock sampler over the first stream creation)
// Where a HIP device's first use goes (tk8s-probe's per-device ~20 ms against tk8s-hsaprobe's
// ~9.5 ms of queue + code objects + VRAM): each first call timed on its own.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/time.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

constexpr int kMaxSamples = 20000, kDepth = 48;
static void* g_frames[kMaxSamples][kDepth];
static int g_depth[kMaxSamples];
static volatile int g_n = 0;

static void on_prof(int) {
  const int i = g_n;
  if (i >= kMaxSamples) return;
  g_depth[i] = backtrace(g_frames[i], kDepth);
  g_n = i + 1;
}

static std::string where(void* pc) {
  Dl_info d{};
  if (!dladdr(pc, &d) || !d.dli_fname) return "?";
  std::string lib = d.dli_fname;
  lib = lib.substr(lib.rfind('/') + 1);
  if (d.dli_sname) return lib + ":" + d.dli_sname;
  char buf[64];
  std::snprintf(buf, sizeof buf, "+0x%lx", (unsigned long)((char*)pc - (char*)d.dli_fbase));
  return lib + buf;
}

static void report(const char* file) {
  std::map<std::string, int> leaf, incl;
  for (int i = 0; i < g_n; ++i) {
    // frames 0-1 are the handler and the signal trampoline
    if (g_depth[i] > 2) leaf[where(g_frames[i][2])]++;
    std::map<std::string, int> seen;
    for (int k = 2; k < g_depth[i]; ++k) seen[where(g_frames[i][k])] = 1;
    for (auto& kv : seen) incl[kv.first]++;
  }
  std::vector<std::pair<int, std::string>> a, b;
  for (auto& kv : leaf) a.push_back({kv.second, kv.first});
  for (auto& kv : incl) b.push_back({kv.second, kv.first});
  std::sort(a.rbegin(), a.rend());
  std::sort(b.rbegin(), b.rend());
  std::printf("{\"file\":\"%s\",\"samples\":%d,\"leaf\":[", file, g_n);
  for (size_t i = 0; i < a.size() && i < 25; ++i) std::printf("%s[%d,\"%s\"]", i ? "," : "", a[i].first, a[i].second.c_str());
  std::printf("],\"inclusive\":[");
  for (size_t i = 0; i < b.size() && i < 60; ++i) std::printf("%s[%d,\"%s\"]", i ? "," : "", b[i].first, b[i].second.c_str());
  std::printf("]}\n");
}

__global__ void fill(unsigned* p, size_t n, unsigned v) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) p[i] = v;
}

static double ms(std::chrono::steady_clock::time_point& t) {
  const auto now = std::chrono::steady_clock::now();
  const double r = std::chrono::duration<double, std::milli>(now - t).count();
  t = now;
  return r;
}

int main() {
  auto t = std::chrono::steady_clock::now();
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 3;
  const double init = ms(t);
  (void)hipSetDevice(0);
  const double setdev = ms(t);
  void* p = nullptr;
  if (hipMalloc(&p, size_t(1) << 30) != hipSuccess) return 4;
  const double malloc_ms = ms(t);
  hipStream_t s;
  const bool sample = std::getenv("HIPDEV_SAMPLE") != nullptr;
  if (sample) {
    void* warm[4];
    backtrace(warm, 4);
    struct sigaction sa{};
    sa.sa_handler = on_prof;
    sa.sa_flags = SA_RESTART;
    sigaction(SIGALRM, &sa, nullptr);
    itimerval it{{0, 250}, {0, 250}};
    setitimer(ITIMER_REAL, &it, nullptr);
  }
  t = std::chrono::steady_clock::now();
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const double stream = ms(t);
  if (sample) {
    itimerval off{{0, 0}, {0, 0}};
    setitimer(ITIMER_REAL, &off, nullptr);
    report("stream_create");
  }
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, s, static_cast<unsigned*>(p), size_t(1) << 28, 7u);
  const double launch = ms(t);
  (void)hipStreamSynchronize(s);
  const double sync = ms(t);
  hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, s, static_cast<unsigned*>(p), size_t(1) << 28, 9u);
  (void)hipStreamSynchronize(s);
  const double second = ms(t);
  unsigned h = 0;
  (void)hipMemcpy(&h, p, 4, hipMemcpyDeviceToHost);
  const double memcpy_ms = ms(t);
  hipEvent_t e;
  (void)hipEventCreate(&e);
  const double event = ms(t);
  std::printf("{\"init\":%.2f,\"set_device\":%.2f,\"malloc_1g\":%.2f,\"stream\":%.2f,\"first_launch\":%.2f,"
              "\"first_sync\":%.2f,\"second_kernel\":%.2f,\"first_memcpy\":%.2f,\"event\":%.2f,\"value\":%u}\n",
              init, setdev, malloc_ms, stream, launch, sync, second, memcpy_ms, event, h);
  return 0;
}
