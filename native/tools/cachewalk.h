// Skip the HSA thunk's per-CPU cache walk at runtime start (hsa_init, also under HIP's first call).
//
// The thunk inside libhsa-runtime64 walks every CPU's cache hierarchy in sysfs when the runtime
// starts: for each CPU it lists .../cpu<M>/cache and then reads index<K>/{shared_cpu_list,level,
// type,size,...}. On the 2-socket MI355X hosts (256 CPUs) that is ~7,600 sysfs files and about
// two thirds of hsa_init's ~47 ms, all of it kernel time (profiles/r2_hsainit/). The tools never
// ask the CPU agent for its caches, so they tell the thunk a CPU has none: the opendir() below
// preempts libc's for libhsa (the executable comes first in symbol lookup; the tools are linked
// with --export-dynamic-symbol=opendir) and answers ENOENT for per-CPU cache directories only --
// what the thunk sees on kernels or VMs that publish no cache information. Every other directory,
// the NUMA node and cpu lists included, is libc's. (Hiding the node directory is not enough: the
// thunk then walks /sys/devices/system/cpu instead, profiles/r2_hsainit/numa_dir_only/.) glibc's
// own internal directory reads do not come through here, and neither do the reads of a process
// that loads the runtime into an interpreter (python's libc comes first there).
//
// TK8S_HSA_CPU_CACHES=1 keeps the walk. Include this from exactly one translation unit of an
// executable (its main file): it defines opendir.
#pragma once

#include <dirent.h>
#include <dlfcn.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>

namespace tk8s::cachewalk {

inline bool g_skip = true;
inline int g_hidden = 0;

// "/sys/devices/system/<...>/cpu<N>/cache": one CPU's cache directory, under either the NUMA
// node (node/node<K>/cpu<N>) or the flat cpu list (cpu/cpu<N>), the two places the thunk looks.
inline bool cpu_cache_dir(const char* p) {
  static const char kSys[] = "/sys/devices/system/";
  static const char kTail[] = "/cache";
  if (!p || std::strncmp(p, kSys, sizeof kSys - 1) != 0) return false;
  const size_t n = std::strlen(p);
  if (n < sizeof kSys + sizeof kTail || std::strcmp(p + n - (sizeof kTail - 1), kTail) != 0) return false;
  const size_t end = n - (sizeof kTail - 1);
  size_t i = end;
  while (i > 0 && p[i - 1] >= '0' && p[i - 1] <= '9') --i;
  return i < end && i >= 4 && std::strncmp(p + i - 4, "/cpu", 4) == 0;
}

// Call at the top of main(), before anything starts the runtime (after a plan's environment).
inline void configure() {
  const char* e = std::getenv("TK8S_HSA_CPU_CACHES");
  g_skip = !(e && std::strcmp(e, "1") == 0);
}

inline const char* mode() { return g_skip ? "skipped" : "kept"; }

}  // namespace tk8s::cachewalk

extern "C" DIR* opendir(const char* name) {
  static auto real = reinterpret_cast<DIR* (*)(const char*)>(dlsym(RTLD_NEXT, "opendir"));
  if (tk8s::cachewalk::g_skip && tk8s::cachewalk::cpu_cache_dir(name)) {
    ++tk8s::cachewalk::g_hidden;
    errno = ENOENT;
    return nullptr;
  }
  return real(name);
}
