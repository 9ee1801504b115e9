// How long HIP takes to load a code object (hipModuleLoadData + a first hipModuleGetFunction),
// for each file given: the RCCL gfx950 code object (~500 kernels, 108 MB) and synthetic ones.
// Usage: coload_bench KERNEL_NAME_OR_- FILE...   (prints one JSON line per file)
// With COLOAD_SAMPLE=1 a SIGPROF sampler (1 ms of CPU time; COLOAD_SAMPLE=real: SIGALRM, 1 ms of
// wall-clock, which also catches a blocked main thread) records where each load spends its
// CPU time: the innermost frame and every symbol on the stack (inclusive), resolved by dladdr.
#include <dlfcn.h>
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <sys/time.h>

#include <map>
#include <vector>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <algorithm>
#include <cstdlib>
#include <string>

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

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const char* mode = std::getenv("COLOAD_SAMPLE");
  const bool sample = mode != nullptr, real = sample && std::string(mode) == "real";
  auto start_sampler = [&] {
    void* warm[4];
    backtrace(warm, 4);  // loads the unwinder outside the handler
    g_n = 0;
    struct sigaction sa{};
    sa.sa_handler = on_prof;
    sa.sa_flags = SA_RESTART;
    sigaction(real ? SIGALRM : SIGPROF, &sa, nullptr);
    itimerval it{{0, 1000}, {0, 1000}};
    setitimer(real ? ITIMER_REAL : ITIMER_PROF, &it, nullptr);
  };
  auto stop_sampler = [&](const char* what) {
    itimerval off{{0, 0}, {0, 0}};
    setitimer(real ? ITIMER_REAL : ITIMER_PROF, &off, nullptr);
    report(what);
  };
  if (sample) start_sampler();
  auto t = std::chrono::steady_clock::now();
  if (hipInit(0) != hipSuccess || hipSetDevice(0) != hipSuccess) return 3;
  (void)hipFree(nullptr);
  const double init_ms = ms_since(t);
  if (sample) stop_sampler("hip_init");
  std::printf("{\"hip_init_ms\":%.2f}\n", init_ms);
  for (int i = 2; i < argc; ++i) {
    std::ifstream f(argv[i], std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string img = ss.str();
    if (sample) start_sampler();
    t = std::chrono::steady_clock::now();
    hipModule_t m;
    const hipError_t e = hipModuleLoadData(&m, img.data());
    const double load_ms = ms_since(t);
    if (sample) stop_sampler(argv[i]);
    double fn_ms = -1;
    if (e == hipSuccess && std::string(argv[1]) != "-") {
      t = std::chrono::steady_clock::now();
      hipFunction_t fn;
      fn_ms = hipModuleGetFunction(&fn, m, argv[1]) == hipSuccess ? ms_since(t) : -2;
    }
    std::printf("{\"file\":\"%s\",\"bytes\":%zu,\"ok\":%s,\"load_ms\":%.2f,\"get_function_ms\":%.2f}\n", argv[i],
                img.size(), e == hipSuccess ? "true" : "false", load_ms, fn_ms);
    std::fflush(stdout);
  }
  return 0;
}
