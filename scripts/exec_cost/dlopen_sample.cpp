// What libhsa-runtime64 does when it is loaded (exec -> main of anything linking it took ~10 ms
// more than of a plain program on the MI355X host): dlopen it under a 0.25 ms wall-clock sampler.
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


int main(int argc, char** argv) {
  const char* lib = argc > 1 ? argv[1] : "libhsa-runtime64.so.1";
  void* warm[4];
  backtrace(warm, 4);
  struct sigaction sa{};
  sa.sa_handler = on_prof;
  sa.sa_flags = SA_RESTART;
  sigaction(SIGALRM, &sa, nullptr);
  itimerval it{{0, 250}, {0, 250}};
  const auto t = std::chrono::steady_clock::now();
  setitimer(ITIMER_REAL, &it, nullptr);
  void* h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
  itimerval off{{0, 0}, {0, 0}};
  setitimer(ITIMER_REAL, &off, nullptr);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
  report(lib);
  std::printf("{\"dlopen_ms\":%.3f,\"ok\":%s}\n", ms, h ? "true" : "false");
  return h ? 0 : 1;
}
