// hsa_init_breakdown: where the ~47 ms of hsa_init (the burn-in's runtime start, the largest
// part of the bring-up's critical path) goes.
//
// The executable itself defines the libc entry points libhsa-runtime64 calls (ioctl, open/openat,
// fopen, mmap/munmap, read/pread, the sleeps and polls, pthread_create); linked with -rdynamic,
// those definitions win symbol resolution over libc's, time the real call (dlsym RTLD_NEXT) and
// aggregate per kind, per KFD/DRM ioctl number and per path class (sysfs topology, /dev/kfd, DRM
// render node, /proc). CPU time (user/sys) brackets hsa_init too, so "in the kernel" vs "in ROCr's
// own code" is visible. Then: one 64-packet AQL queue, destroy, hsa_shut_down.
//
//   g++ -O2 -std=c++17 -rdynamic -I/opt/rocm/include hsa_init_breakdown.cpp \
//       -L/opt/rocm/lib -lhsa-runtime64 -ldl -lpthread -o hsa_init_breakdown
//
// Host-side only: no kernel is dispatched.
#include <dirent.h>
#include <errno.h>
#include <stdlib.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <poll.h>
#include <pthread.h>
#include <stdarg.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/select.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

double now_ms() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

enum Kind { kIoctl, kOpen, kFopen, kMmap, kMunmap, kRead, kSleep, kPoll, kThread, kClose, kNKinds };
const char* kKindName[kNKinds] = {"ioctl", "open", "fopen", "mmap", "munmap", "read", "sleep", "poll",
                                  "pthread_create", "close"};
std::atomic<long> g_count[kNKinds];
std::atomic<long> g_ns[kNKinds];

// ioctl by (type << 8 | nr)
std::atomic<long> g_ioctl_count[65536];
std::atomic<long> g_ioctl_ns[65536];

// open/fopen by path class
enum PathClass { kSysTopo, kSysOther, kDevKfd, kDevDri, kProc, kOtherPath, kNPaths };
const char* kPathName[kNPaths] = {"sysfs kfd topology", "sysfs other", "/dev/kfd", "/dev/dri", "/proc", "other"};
std::atomic<long> g_path_count[kNPaths];
std::atomic<long> g_path_ns[kNPaths];

struct Slow {
  double ms;
  std::string what;
};
std::mutex g_slow_mu;
std::vector<Slow> g_slow;
std::vector<Slow> g_other;
std::vector<Slow> g_dirs;
std::map<std::string, std::pair<long, double>> g_topo;
std::atomic<long> g_fopen_fail{0};
std::atomic<bool> g_on{false};

void note_slow(double ms, const std::string& what) {
  if (ms < 0.5) return;
  std::lock_guard<std::mutex> l(g_slow_mu);
  g_slow.push_back({ms, what});
}

PathClass classify(const char* p) {
  if (!p) return kOtherPath;
  if (!strncmp(p, "/sys/devices/virtual/kfd", 24) || !strncmp(p, "/sys/class/kfd", 14)) return kSysTopo;
  if (!strncmp(p, "/sys/", 5)) return kSysOther;
  if (!strcmp(p, "/dev/kfd")) return kDevKfd;
  if (!strncmp(p, "/dev/dri", 8)) return kDevDri;
  if (!strncmp(p, "/proc/", 6)) return kProc;
  return kOtherPath;
}

void account(Kind k, double t0) {
  if (!g_on.load(std::memory_order_relaxed)) return;
  long ns = (long)((now_ms() - t0) * 1e6);
  g_count[k]++;
  g_ns[k] += ns;
}

void account_path(Kind k, double t0, const char* path) {
  if (!g_on.load(std::memory_order_relaxed)) return;
  double ms = now_ms() - t0;
  account(k, t0);
  PathClass c = classify(path);
  g_path_count[c]++;
  g_path_ns[c] += (long)(ms * 1e6);
  note_slow(ms, std::string(kKindName[k]) + " " + (path ? path : "?"));
  if (c == kSysTopo && path) {
    std::string pat;
    for (const char* q = path; *q; ++q) {
      if (*q >= '0' && *q <= '9') {
        if (pat.empty() || pat.back() != 'N') pat += 'N';
      } else {
        pat += *q;
      }
    }
    std::lock_guard<std::mutex> l(g_slow_mu);
    auto& e = g_topo[pat];
    e.first++;
    e.second += ms;
  }
  if (c == kOtherPath || c == kProc || c == kSysOther) {
    std::lock_guard<std::mutex> l(g_slow_mu);
    if (g_other.size() < 200) g_other.push_back({ms, path ? path : "?"});
  }
}

template <typename F>
F real(const char* name) {
  return reinterpret_cast<F>(dlsym(RTLD_NEXT, name));
}

}  // namespace

extern "C" {

int ioctl(int fd, unsigned long req, ...) {
  static auto f = real<int (*)(int, unsigned long, void*)>("ioctl");
  va_list ap;
  va_start(ap, req);
  void* arg = va_arg(ap, void*);
  va_end(ap);
  double t0 = now_ms();
  int r = f(fd, req, arg);
  if (g_on.load(std::memory_order_relaxed)) {
    double ms = now_ms() - t0;
    account(kIoctl, t0);
    unsigned idx = ((_IOC_TYPE(req) & 0xff) << 8) | (_IOC_NR(req) & 0xff);
    g_ioctl_count[idx]++;
    g_ioctl_ns[idx] += (long)(ms * 1e6);
    char b[64];
    snprintf(b, sizeof b, "ioctl type %c nr 0x%02x", (char)_IOC_TYPE(req), (unsigned)_IOC_NR(req));
    note_slow(ms, b);
  }
  return r;
}

static int open_common(const char* sym, const char* path, int flags, va_list ap) {
  mode_t mode = 0;
  if (flags & (O_CREAT | O_TMPFILE)) mode = va_arg(ap, mode_t);
  auto f = real<int (*)(const char*, int, mode_t)>(sym);
  double t0 = now_ms();
  int r = f(path, flags, mode);
  account_path(kOpen, t0, path);
  return r;
}

int open(const char* path, int flags, ...) {
  va_list ap;
  va_start(ap, flags);
  int r = open_common("open", path, flags, ap);
  va_end(ap);
  return r;
}

int open64(const char* path, int flags, ...) {
  va_list ap;
  va_start(ap, flags);
  int r = open_common("open64", path, flags, ap);
  va_end(ap);
  return r;
}

int openat(int dirfd, const char* path, int flags, ...) {
  static auto f = real<int (*)(int, const char*, int, mode_t)>("openat");
  mode_t mode = 0;
  va_list ap;
  va_start(ap, flags);
  if (flags & (O_CREAT | O_TMPFILE)) mode = va_arg(ap, mode_t);
  va_end(ap);
  double t0 = now_ms();
  int r = f(dirfd, path, flags, mode);
  account_path(kOpen, t0, path);
  return r;
}

// SKIP_GPU_CACHES=1: an empty file (/dev/null) for the KFD topology's per-node cache property files
static bool gpu_cache_props(const char* p) {
  static const bool skip = getenv("SKIP_GPU_CACHES") && !strcmp(getenv("SKIP_GPU_CACHES"), "1");
  return skip && p && !strncmp(p, "/sys/devices/virtual/kfd/kfd/topology/nodes/", 44) && strstr(p, "/caches/");
}

FILE* fopen(const char* path, const char* mode) {
  static auto f = real<FILE* (*)(const char*, const char*)>("fopen");
  if (gpu_cache_props(path)) return f("/dev/null", mode);  // an empty property file
  double t0 = now_ms();
  FILE* r = f(path, mode);
  account_path(kFopen, t0, path);
  if (!r && g_on.load(std::memory_order_relaxed)) g_fopen_fail++;
  return r;
}

FILE* fopen64(const char* path, const char* mode) {
  static auto f = real<FILE* (*)(const char*, const char*)>("fopen64");
  double t0 = now_ms();
  FILE* r = f(path, mode);
  account_path(kFopen, t0, path);
  return r;
}

void* mmap(void* a, size_t len, int prot, int flags, int fd, off_t off) {
  static auto f = real<void* (*)(void*, size_t, int, int, int, off_t)>("mmap");
  double t0 = now_ms();
  void* r = f(a, len, prot, flags, fd, off);
  if (g_on.load(std::memory_order_relaxed)) {
    account(kMmap, t0);
    char b[96];
    snprintf(b, sizeof b, "mmap %zu MiB fd %d flags 0x%x", len >> 20, fd, flags);
    note_slow(now_ms() - t0, b);
  }
  return r;
}

void* mmap64(void* a, size_t len, int prot, int flags, int fd, off_t off) { return mmap(a, len, prot, flags, fd, off); }

int munmap(void* a, size_t len) {
  static auto f = real<int (*)(void*, size_t)>("munmap");
  double t0 = now_ms();
  int r = f(a, len);
  if (g_on.load(std::memory_order_relaxed)) {
    account(kMunmap, t0);
    char b[64];
    snprintf(b, sizeof b, "munmap %zu MiB", len >> 20);
    note_slow(now_ms() - t0, b);
  }
  return r;
}

ssize_t read(int fd, void* buf, size_t n) {
  static auto f = real<ssize_t (*)(int, void*, size_t)>("read");
  double t0 = now_ms();
  ssize_t r = f(fd, buf, n);
  account(kRead, t0);
  return r;
}

ssize_t pread64(int fd, void* buf, size_t n, off_t off) {
  static auto f = real<ssize_t (*)(int, void*, size_t, off_t)>("pread64");
  double t0 = now_ms();
  ssize_t r = f(fd, buf, n, off);
  account(kRead, t0);
  return r;
}

int close(int fd) {
  static auto f = real<int (*)(int)>("close");
  double t0 = now_ms();
  int r = f(fd);
  if (g_on.load(std::memory_order_relaxed)) {
    account(kClose, t0);
    note_slow(now_ms() - t0, "close");
  }
  return r;
}

// "/sys/devices/system/.../cpu<N>/cache": one CPU's cache directory (what tk8s-hsaprobe hides)
static bool cpu_cache_dir(const char* p) {
  static const char kSys[] = "/sys/devices/system/";
  static const char kTail[] = "/cache";
  if (!p || strncmp(p, kSys, sizeof kSys - 1) != 0) return false;
  size_t n = strlen(p);
  if (n < sizeof kTail || strcmp(p + n - (sizeof kTail - 1), kTail) != 0) return false;
  size_t end = n - (sizeof kTail - 1), i = end;
  while (i > 0 && p[i - 1] >= '0' && p[i - 1] <= '9') --i;
  return i < end && i >= 4 && !strncmp(p + i - 4, "/cpu", 4);
}

// SKIP_NUMA=1: hide /sys/devices/system/node/node<N> from the thunk (what tk8s-hsaprobe does)
DIR* opendir(const char* name) {
  static auto f = real<DIR* (*)(const char*)>("opendir");
  static const bool skip = getenv("SKIP_NUMA") && !strcmp(getenv("SKIP_NUMA"), "1");
  static const char kP[] = "/sys/devices/system/node/node";
  (void)kP;
  const bool hide = skip && cpu_cache_dir(name);
  if (g_on.load(std::memory_order_relaxed)) {
    std::lock_guard<std::mutex> l(g_slow_mu);
    g_dirs.push_back({hide ? 1.0 : 0.0, name ? name : "?"});
  }
  if (hide) {
    errno = ENOENT;
    return nullptr;
  }
  return f(name);
}

int usleep(useconds_t us) {
  static auto f = real<int (*)(useconds_t)>("usleep");
  double t0 = now_ms();
  int r = f(us);
  if (g_on.load(std::memory_order_relaxed)) {
    account(kSleep, t0);
    note_slow(now_ms() - t0, "usleep " + std::to_string(us));
  }
  return r;
}

int nanosleep(const timespec* req, timespec* rem) {
  static auto f = real<int (*)(const timespec*, timespec*)>("nanosleep");
  double t0 = now_ms();
  int r = f(req, rem);
  if (g_on.load(std::memory_order_relaxed)) {
    account(kSleep, t0);
    note_slow(now_ms() - t0, "nanosleep");
  }
  return r;
}

int clock_nanosleep(clockid_t c, int fl, const timespec* req, timespec* rem) {
  static auto f = real<int (*)(clockid_t, int, const timespec*, timespec*)>("clock_nanosleep");
  double t0 = now_ms();
  int r = f(c, fl, req, rem);
  if (g_on.load(std::memory_order_relaxed)) {
    account(kSleep, t0);
    note_slow(now_ms() - t0, "clock_nanosleep");
  }
  return r;
}

int poll(struct pollfd* fds, nfds_t n, int timeout) {
  static auto f = real<int (*)(struct pollfd*, nfds_t, int)>("poll");
  double t0 = now_ms();
  int r = f(fds, n, timeout);
  account(kPoll, t0);
  return r;
}

int pthread_create(pthread_t* t, const pthread_attr_t* a, void* (*fn)(void*), void* arg) {
  static auto f = real<int (*)(pthread_t*, const pthread_attr_t*, void* (*)(void*), void*)>("pthread_create");
  double t0 = now_ms();
  int r = f(t, a, fn, arg);
  if (g_on.load(std::memory_order_relaxed)) {
    account(kThread, t0);
    note_slow(now_ms() - t0, "pthread_create");
  }
  return r;
}

}  // extern "C"

namespace {

double cpu_ms(int who) {
  rusage u;
  getrusage(who, &u);
  return (u.ru_utime.tv_sec + u.ru_stime.tv_sec) * 1e3 + (u.ru_utime.tv_usec + u.ru_stime.tv_usec) / 1e3;
}

void cpu_split(double* user, double* sys) {
  rusage u;
  getrusage(RUSAGE_SELF, &u);
  *user = u.ru_utime.tv_sec * 1e3 + u.ru_utime.tv_usec / 1e3;
  *sys = u.ru_stime.tv_sec * 1e3 + u.ru_stime.tv_usec / 1e3;
}

int count_dir(const std::string& d) {
  DIR* dp = opendir(d.c_str());
  if (!dp) return -1;
  int n = 0;
  while (dirent* e = readdir(dp))
    if (e->d_name[0] != '.') n++;
  closedir(dp);
  return n;
}

hsa_status_t first_gpu(hsa_agent_t a, void* data) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) {
    *static_cast<hsa_agent_t*>(data) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

}  // namespace

int main() {
  // topology volume: nodes, and cache entries per node (what the thunk walks at init)
  std::string topo = "/sys/devices/virtual/kfd/kfd/topology/nodes";
  int nodes = count_dir(topo);
  std::string caches = "[";
  for (int i = 0; i < nodes && i < 64; i++) {
    caches += (i ? "," : "") + std::to_string(count_dir(topo + "/" + std::to_string(i) + "/caches"));
  }
  caches += "]";

  double u0, s0, u1, s1;
  cpu_split(&u0, &s0);
  g_on = true;
  double t0 = now_ms();
  hsa_status_t st = hsa_init();
  double t_init = now_ms() - t0;
  g_on = false;
  cpu_split(&u1, &s1);
  double t_queue = -1, t_shut = -1;
  if (st == HSA_STATUS_SUCCESS) {
    hsa_agent_t gpu{};
    hsa_iterate_agents(first_gpu, &gpu);
    for (int k = 0; k < kNKinds; k++) g_count[k] = 0, g_ns[k] = 0;
    for (unsigned i = 0; i < 65536; i++) g_ioctl_count[i] = 0, g_ioctl_ns[i] = 0;
    {
      std::lock_guard<std::mutex> l(g_slow_mu);
      g_slow.clear();
    }
    g_on = true;  // from here on the accounting is the queue creation's
    double tq = now_ms();
    hsa_queue_t* q = nullptr;
    hsa_status_t qs = hsa_queue_create(gpu, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q);
    t_queue = now_ms() - tq;
    g_on = false;
    if (qs == HSA_STATUS_SUCCESS) hsa_queue_destroy(q);
    double ts = now_ms();
    hsa_shut_down();
    t_shut = now_ms() - ts;
  }

  printf("{\"ok\": %s, \"status\": %d, ", st == HSA_STATUS_SUCCESS ? "true" : "false", (int)st);
  printf("\"hsa_init_ms\": %.3f, \"queue_create_ms\": %.3f, \"shut_down_ms\": %.3f, "
         "\"init_user_ms\": %.1f, \"init_sys_ms\": %.1f, \"topology_nodes\": %d, \"caches_per_node\": %s, ",
         t_init, t_queue, t_shut, u1 - u0, s1 - s0, nodes, caches.c_str());
  printf("\"calls\": {");
  for (int k = 0; k < kNKinds; k++)
    printf("%s\"%s\": [%ld, %.3f]", k ? ", " : "", kKindName[k], g_count[k].load(), g_ns[k].load() / 1e6);
  printf("}, \"paths\": {");
  for (int c = 0; c < kNPaths; c++)
    printf("%s\"%s\": [%ld, %.3f]", c ? ", " : "", kPathName[c], g_path_count[c].load(), g_path_ns[c].load() / 1e6);
  printf("}, \"ioctls\": {");
  std::vector<std::pair<long, unsigned>> io;
  for (unsigned i = 0; i < 65536; i++)
    if (g_ioctl_count[i]) io.push_back({g_ioctl_ns[i].load(), i});
  std::sort(io.rbegin(), io.rend());
  for (size_t j = 0; j < io.size(); j++)
    printf("%s\"%c/0x%02x\": [%ld, %.3f]", j ? ", " : "", (char)(io[j].second >> 8), io[j].second & 0xff,
           g_ioctl_count[io[j].second].load(), io[j].first / 1e6);
  printf("}, \"slowest\": [");
  std::sort(g_slow.begin(), g_slow.end(), [](const Slow& a, const Slow& b) { return a.ms > b.ms; });
  for (size_t j = 0; j < g_slow.size() && j < 20; j++)
    printf("%s[%.3f, \"%s\"]", j ? ", " : "", g_slow[j].ms, g_slow[j].what.c_str());
  printf("], \"topology_patterns\": {");
  {
    bool first = true;
    for (auto& kv : g_topo) {
      printf("%s\"%s\": [%ld, %.3f]", first ? "" : ", ", kv.first.c_str(), kv.second.first, kv.second.second);
      first = false;
    }
  }
  printf("}, \"fopen_failed\": %ld, \"opendir\": [", g_fopen_fail.load());
  for (size_t j = 0; j < g_dirs.size() && j < 100; j++) printf("%s[%d, \"%s\"]", j ? ", " : "", (int)g_dirs[j].ms, g_dirs[j].what.c_str());
  printf("], \"other_paths\": [");
  for (size_t j = 0; j < g_other.size(); j++) printf("%s[%.3f, \"%s\"]", j ? ", " : "", g_other[j].ms, g_other[j].what.c_str());
  printf("]}\n");
  (void)cpu_ms;
  return st == HSA_STATUS_SUCCESS ? 0 : 1;
}
