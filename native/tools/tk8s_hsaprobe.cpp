// tk8s-hsaprobe: the GPU validation payload on the ROCr (HSA) runtime directly.
//
// Same checks, same kernels and the same JSON as tk8s-probe (N4 HBM write + verify, N5 Philox +
// MD5 tree against the known answer, N7 local copy), minus the HIP layer. The payload is the
// bring-up's critical path (docs/benchmarks.md, profiles/r1_trace/), and most of what HIP adds
// there is start-up, not work (profiles/r1_init_costs/): mapping libamdhip64 (~10 ms), the HIP
// runtime on top of ROCr (~5 ms), and per stream a 16 MiB pinned host buffer next to the
// hardware queue (~10 ms). Here a device costs one AQL queue, one VRAM allocation, two code
// objects and a page of kernel arguments.
//
// Kernels: the very code objects of native/src/stream_kernels.hip and md5_kernels.hip (built
// device-only for gfx950 into lib/tk8s_stream.co and lib/tk8s_md5.co), dispatched with
// hand-written AQL packets. Their explicit arguments follow the AMDGPU kernel ABI (natural
// alignment, in order); the code-object-v5 hidden arguments the HIP kernels read (gridDim ->
// hidden_block_count_*, blockDim -> hidden_group_size_*) are filled at the ABI offsets after
// them. Results (error counters, the tree digest) live in VRAM and are copied into host-visible
// memory by a last kernel, so no SDMA engine and no host-memory atomics are involved.
// Kernel times are GPU timestamps of the dispatches (hsa_amd_profiling_get_dispatch_time).
//
//   tk8s-hsaprobe [--all-devices | --device D | --devices D,D,...] [--gpuinfo] [--hbm-bytes B] [--md5-bytes B]
//                 [--chunk C] [--seed S] [--copy-bytes B] [--iters K] [--mode plain|nontemporal]
//                 [--peers [--peer-bytes B] [--peer-iters K]] [--peers-host]
//                 [--out FILE] [--reuse FILE [--reuse-wait S]] [--release-after]
//
// --release-after: once the result is written, free every device's queue and VRAM and shut the
// runtime down before exiting (by default the process _exits and the driver reclaims it all).
//
// --peers (N7, the xGMI link check before Ready): once every device has passed its own probes,
// each one fills a source buffer with a pattern naming it, grants every other GPU access to it
// (hsa_amd_agents_allow_access, after checking the pool is not NEVER_ALLOWED for that agent),
// and then in round r = 1..n-1 every GPU i pulls from GPU (i + r) mod n with the stream copy
// kernel and verifies the pattern. A round is a permutation, so each directed link carries one
// pull at a time and its GB/s is that link's. Each pull lands in the destination device's JSON
// under "peers" (src_device/dst_device/kernel_gbps/bad_words), the shape tk8s-probe uses; the
// bring-up judges the link matrix (tritonk8ssupervisor_amd/xgmi.py). With one GPU there is no
// pair and the phase costs nothing. --peers-host runs the same pull path from a host-memory
// source (granted the same way): the part of the mechanism a 1-GPU box can exercise.

#include <fcntl.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "args.h"
#include "cachewalk.h"
#include "reuse.h"
#include "tk8s/failfast.h"
#include "tk8s/json.h"

namespace {

using tk8s::Json;

constexpr const char* kKnownDigest256M = "6a21931a145024b03ee4405e01204ce2";
constexpr uint32_t kBlock = 256;     // stream kernels: 4 wave64s (stream_kernels.hip kBlock)
constexpr uint16_t kFillBlock = 128; // the plain HBM fill: one 2-wave block per CU (stream_kernels.hip)
constexpr size_t kMallFlush = size_t(512) << 20;  // 2 x the MI355X's 256 MB Infinity Cache (MALL)
constexpr uint32_t kMd5Block = 256;  // md5_kernels.hip kMd5Block
constexpr uint64_t kWaveChunks = 64;
constexpr uint32_t kFoldBlock = 256;  // md5_kernels.hip kFoldBlock: 1024 nodes -> 1 per block
constexpr int kFoldLevels = 5;
constexpr size_t kAlign = 4096;
constexpr double kHbmPeakGBps = 8000.0;  // MI355X HBM3E, 8 TB/s per GPU

struct HsaError : std::runtime_error {
  HsaError(const char* what, hsa_status_t s) : std::runtime_error(msg(what, s)) {}
  static std::string msg(const char* what, hsa_status_t s) {
    const char* str = nullptr;
    hsa_status_string(s, &str);
    return std::string(what) + ": " + (str ? str : "unknown HSA error");
  }
};

#define HSA_OK(expr)                                   \
  do {                                                 \
    const hsa_status_t s_ = (expr);                    \
    if (s_ != HSA_STATUS_SUCCESS) throw HsaError(#expr, s_); \
  } while (0)

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

size_t align_up(size_t v, size_t a = kAlign) { return (v + a - 1) / a * a; }

std::string hex(const unsigned char* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    s += d[p[i] >> 4];
    s += d[p[i] & 15];
  }
  return s;
}

std::string link_type_name(uint32_t t) {
  switch (t) {
    case HSA_AMD_LINK_INFO_TYPE_HYPERTRANSPORT: return "hypertransport";
    case HSA_AMD_LINK_INFO_TYPE_QPI: return "qpi";
    case HSA_AMD_LINK_INFO_TYPE_PCIE: return "pcie";
    case HSA_AMD_LINK_INFO_TYPE_INFINBAND: return "infiniband";
    case HSA_AMD_LINK_INFO_TYPE_XGMI: return "xgmi";
    default: return "unknown";
  }
}

// ---- agents and pools --------------------------------------------------------------------
struct Gpu {
  hsa_agent_t agent{};
  hsa_amd_memory_pool_t vram{};
  bool has_vram = false;
  std::string name, product, isa;
  uint32_t cus = 0, bdf = 0, domain = 0, wave = 64, clock_mhz = 0, mem_mhz = 0, mem_width = 0, lds = 0;
  uint64_t mem_bytes = 0;
  std::string uuid;
};

struct Host {
  hsa_agent_t cpu{};
  hsa_amd_memory_pool_t kernarg{};
  bool has_kernarg = false;
};

hsa_status_t find_vram(hsa_amd_memory_pool_t pool, void* data) {
  auto* g = static_cast<Gpu*>(data);
  hsa_amd_segment_t seg;
  uint32_t flags = 0;
  bool alloc = false;
  if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
  if (alloc && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && !g->has_vram) {
    g->vram = pool;
    g->has_vram = true;
    size_t sz = 0;
    hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SIZE, &sz);
    g->mem_bytes = sz;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t find_kernarg(hsa_amd_memory_pool_t pool, void* data) {
  auto* h = static_cast<Host*>(data);
  hsa_amd_segment_t seg;
  uint32_t flags = 0;
  bool alloc = false;
  if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
  if (alloc && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !h->has_kernarg) {
    h->kernarg = pool;
    h->has_kernarg = true;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t find_isa(hsa_isa_t isa, void* data) {
  uint32_t len = 0;
  if (hsa_isa_get_info_alt(isa, HSA_ISA_INFO_NAME_LENGTH, &len) == HSA_STATUS_SUCCESS && len) {
    std::string s(len, '\0');
    hsa_isa_get_info_alt(isa, HSA_ISA_INFO_NAME, &s[0]);
    s.resize(std::strlen(s.c_str()));
    *static_cast<std::string*>(data) = s;
  }
  return HSA_STATUS_INFO_BREAK;
}

struct Topology {
  Host host;
  std::vector<Gpu> gpus;
};

hsa_status_t collect_agent(hsa_agent_t agent, void* data) {
  auto* t = static_cast<Topology*>(data);
  hsa_device_type_t type;
  if (hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (type == HSA_DEVICE_TYPE_CPU) {
    if (!t->host.has_kernarg) {
      t->host.cpu = agent;
      hsa_amd_agent_iterate_memory_pools(agent, find_kernarg, &t->host);
    }
    return HSA_STATUS_SUCCESS;
  }
  if (type != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
  Gpu g;
  g.agent = agent;
  char name[64] = {0}, product[64] = {0}, uuid[32] = {0};
  hsa_agent_get_info(agent, HSA_AGENT_INFO_NAME, name);
  hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_PRODUCT_NAME), product);
  hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_UUID), uuid);
  g.name = name;
  g.product = product;
  // HIP's device UUID is the 16 characters after "GPU-"; tk8s-probe prints them hex-encoded.
  const std::string u = uuid;
  const std::string tail = u.rfind("GPU-", 0) == 0 ? u.substr(4) : u;
  g.uuid = hex(reinterpret_cast<const unsigned char*>(tail.data()), std::min<size_t>(tail.size(), 16));
  hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT), &g.cus);
  hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &g.bdf);
  hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &g.domain);
  hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_MAX_CLOCK_FREQUENCY), &g.clock_mhz);
  hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_MEMORY_MAX_FREQUENCY), &g.mem_mhz);
  hsa_agent_get_info(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_MEMORY_WIDTH), &g.mem_width);
  hsa_agent_get_info(agent, HSA_AGENT_INFO_WAVEFRONT_SIZE, &g.wave);
  hsa_agent_iterate_isas(agent, find_isa, &g.isa);
  hsa_amd_agent_iterate_memory_pools(agent, find_vram, &g);
  g.lds = 65536;
  if (g.cus == 0) g.cus = 1;
  t->gpus.push_back(g);
  return HSA_STATUS_SUCCESS;
}

std::string pci_bus_id(const Gpu& g) {
  char b[32];
  std::snprintf(b, sizeof b, "%04x:%02x:%02x.%x", g.domain & 0xffff, (g.bdf >> 8) & 0xff, (g.bdf >> 3) & 0x1f,
                g.bdf & 7);
  return b;
}

std::string gpuinfo_json(const Topology& t) {
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::string> devs, rows;
  for (size_t i = 0; i < t.gpus.size(); ++i) {
    const Gpu& g = t.gpus[i];
    const std::string arch = g.isa.empty() ? g.name : g.isa.substr(g.isa.rfind('-') == std::string::npos ? 0 : g.isa.find("gfx"));
    devs.push_back(Json()
                       .kv("index", static_cast<int>(i))
                       .kv("name", g.product)
                       .kv("arch", arch)
                       .kv("gfx", g.name)
                       .kv("total_mem_bytes", static_cast<uint64_t>(g.mem_bytes))
                       .kv("cu_count", g.cus)
                       .kv("clock_khz", g.clock_mhz * 1000u)
                       .kv("mem_clock_khz", g.mem_mhz * 1000u)
                       .kv("mem_bus_width", g.mem_width)
                       .kv("wavefront_size", g.wave)
                       .kv("lds_per_block_bytes", g.lds)
                       .kv("pci_bus_id", pci_bus_id(g))
                       .kv("uuid", g.uuid)
                       .str());
  }
  for (size_t i = 0; i < t.gpus.size(); ++i) {
    std::vector<std::string> row;
    for (size_t j = 0; j < t.gpus.size(); ++j) {
      if (i == j) {
        row.push_back(Json().kv("type", "self").kv("hops", 0).kv("p2p", true).str());
        continue;
      }
      // i's view of j's memory: hops, link type, and whether i may be granted access
      uint32_t hops = 0;
      hsa_amd_memory_pool_access_t access = HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED;
      std::string type = "unknown";
      if (t.gpus[j].has_vram) {
        hsa_amd_agent_memory_pool_get_info(t.gpus[i].agent, t.gpus[j].vram, HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &access);
        if (hsa_amd_agent_memory_pool_get_info(t.gpus[i].agent, t.gpus[j].vram,
                                               HSA_AMD_AGENT_MEMORY_POOL_INFO_NUM_LINK_HOPS, &hops) == HSA_STATUS_SUCCESS &&
            hops > 0) {
          std::vector<hsa_amd_memory_pool_link_info_t> info(hops);
          if (hsa_amd_agent_memory_pool_get_info(t.gpus[i].agent, t.gpus[j].vram,
                                                 HSA_AMD_AGENT_MEMORY_POOL_INFO_LINK_INFO, info.data()) == HSA_STATUS_SUCCESS)
            type = link_type_name(info[0].link_type);
        }
      }
      row.push_back(Json()
                        .kv("type", type)
                        .kv("hops", static_cast<int>(hops))
                        .kv("p2p", access != HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED)
                        .str());
    }
    rows.push_back(Json::array(row));
  }
  uint16_t major = 0, minor = 0;
  hsa_system_get_info(HSA_SYSTEM_INFO_VERSION_MAJOR, &major);
  hsa_system_get_info(HSA_SYSTEM_INFO_VERSION_MINOR, &minor);
  return Json()
      .kv("ok", true)
      .kv("device_count", static_cast<int>(t.gpus.size()))
      .kv("runtime", "hsa")
      .kv("hsa_version", std::to_string(major) + "." + std::to_string(minor))
      .raw("devices", Json::array(devs))
      .raw("links", Json::array(rows))
      .kv("discovery_ms", ms_since(t0))
      .str();
}

// ---- code objects and kernels -------------------------------------------------------------
std::string exe_dir() {
  char buf[4096];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof buf - 1);
  if (n <= 0) return ".";
  std::string p(buf, static_cast<size_t>(n));
  return p.substr(0, p.rfind('/'));
}

std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + path);
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

struct Kernel {
  uint64_t object = 0;
  uint32_t kernarg_size = 0, group = 0, priv = 0;
  bool found = false;
};

struct KernelSet {
  Kernel fill_plain, fill_nt, verify, philox, copy, md5c, md5, md5f;
  Kernel stall;  // fault injection only (TK8S_FAULTS probe.hang@peers): not required
};

// The stall kernel's release flag (fine-grained host memory every GPU agent may read; the
// stall_kernel of stream_kernels.hip polls it) -- set by every bounded wait that gives up, so a
// stalled queue drains (failfast.h).
std::atomic<uint32_t*> g_stall_flag{nullptr};
void stall_release() {
  if (uint32_t* f = g_stall_flag.load()) __atomic_store_n(f, 1u, __ATOMIC_SEQ_CST);
}

hsa_status_t find_kernels(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t sym, void* data) {
  auto* ks = static_cast<KernelSet*>(data);
  hsa_symbol_kind_t kind;
  if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) != HSA_STATUS_SUCCESS ||
      kind != HSA_SYMBOL_KIND_KERNEL)
    return HSA_STATUS_SUCCESS;
  uint32_t len = 0;
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len);
  std::string name(len, '\0');
  hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &name[0]);
  // Itanium-mangled tk8s:: kernels: match the length-prefixed identifier (+ template args).
  Kernel* k = nullptr;
  if (name.find("15hbm_fill_kernelILb0E") != std::string::npos) k = &ks->fill_plain;
  else if (name.find("15hbm_fill_kernelILb1E") != std::string::npos) k = &ks->fill_nt;
  else if (name.find("18verify_fill_kernel") != std::string::npos) k = &ks->verify;
  else if (name.find("18philox_fill_kernel") != std::string::npos) k = &ks->philox;
  else if (name.find("18stream_copy_kernel") != std::string::npos) k = &ks->copy;
  else if (name.find("27md5_chunks_coalesced_kernel") != std::string::npos) k = &ks->md5c;
  else if (name.find("17md5_chunks_kernel") != std::string::npos) k = &ks->md5;
  else if (name.find("15md5_fold_kernelILi256E") != std::string::npos) k = &ks->md5f;  // kFoldBlock
  else if (name.find("12stall_kernel") != std::string::npos) k = &ks->stall;
  if (!k) return HSA_STATUS_SUCCESS;
  HSA_OK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->object));
  HSA_OK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->kernarg_size));
  HSA_OK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->group));
  HSA_OK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->priv));
  k->found = true;
  return HSA_STATUS_SUCCESS;
}

// Explicit kernel arguments in ABI order (natural alignment), then the code-object-v5 hidden
// block: hidden_block_count_{x,y,z} (u32) at +0, hidden_group_size_{x,y,z} (u16) at +12,
// hidden_remainder_{x,y,z} (u16) at +18, hidden_global_offset_{x,y,z} (u64) at +40,
// hidden_grid_dims (u16) at +64, starting at the explicit size rounded up to 8
// (verified against the code objects' metadata: llvm-readelf --notes lib/tk8s_stream.co).
class KernArgs {
 public:
  explicit KernArgs(uint8_t* dst, uint32_t cap) : p_(dst), cap_(cap) { std::memset(p_, 0, cap_); }
  KernArgs& ptr(const void* v) { return put(&v, 8); }
  KernArgs& u64(uint64_t v) { return put(&v, 8); }
  KernArgs& u32(uint32_t v) { return put(&v, 4); }
  // Kernels that read no hidden argument (the MD5 ones) have a kernarg segment of just their
  // explicit arguments; nothing to fill then.
  void hidden(uint32_t blocks, uint16_t block, uint32_t segment) {
    const uint32_t base = (off_ + 7u) & ~7u;
    if (segment <= base) return;
    if (base + 66 > segment || base + 66 > cap_) throw std::runtime_error("unexpected hidden-argument layout");
    const uint32_t one = 1;
    const uint16_t one16 = 1;
    std::memcpy(p_ + base + 0, &blocks, 4);
    std::memcpy(p_ + base + 4, &one, 4);
    std::memcpy(p_ + base + 8, &one, 4);
    std::memcpy(p_ + base + 12, &block, 2);
    std::memcpy(p_ + base + 14, &one16, 2);
    std::memcpy(p_ + base + 16, &one16, 2);
    std::memcpy(p_ + base + 64, &one16, 2);  // hidden_grid_dims
  }

 private:
  KernArgs& put(const void* v, uint32_t size) {
    off_ = (off_ + size - 1) / size * size;
    if (off_ + size > cap_) throw std::runtime_error("kernarg segment overflow");
    std::memcpy(p_ + off_, v, size);
    off_ += size;
    return *this;
  }
  uint8_t* p_;
  uint32_t cap_;
  uint32_t off_ = 0;
};

// ---- one device ---------------------------------------------------------------------------
struct Config {
  // copy: 1 GiB each way, 8 x the 256 MB Infinity Cache, so its rate is an HBM rate
  size_t hbm = 1ull << 30, md5 = 256ull << 20, copy = 1ull << 30, peer = 32ull << 20;
  uint32_t chunk = 1024;
  uint64_t seed = 0;
  int iters = 5, peer_iters = 2;
  bool nontemporal = false, peers = false, peers_host = false;
};

struct Dispatch {
  const Kernel* k = nullptr;
  unsigned blocks = 1;
  uint16_t block = 1;
  size_t slot = 0;  // offset of its kernel arguments in the (host staging / VRAM) arena
  bool system = false;       // release at system scope: the host (or a peer GPU) reads the result
  bool sys_acquire = false;  // acquire at system scope: it reads memory another agent wrote
  hsa_signal_t sig{};
};

class Device {
 public:
  Device(const Gpu& g, const Host& h, const std::vector<std::string>& code_objects, double freq)
      : g_(g), h_(h), freq_(freq) {
    // The queue first, then the code objects: loading them on a second thread while the queue is
    // created only made the loads wait on the runtime's locks (4.5 ms overlapped vs 0.25 ms after
    // the queue, profiles/r2_hsaprobe_setup); the queue (~9 ms, KFD) is the whole setup cost.
    const auto tq = std::chrono::steady_clock::now();
    uint32_t qmin = 0;
    hsa_agent_get_info(g_.agent, HSA_AGENT_INFO_QUEUE_MIN_SIZE, &qmin);
    HSA_OK(hsa_queue_create(g_.agent, std::max<uint32_t>(qmin, 1024), HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr,
                            UINT32_MAX, UINT32_MAX, &q_));
    HSA_OK(hsa_amd_profiling_set_profiler_enabled(q_, 1));
    queue_ms = ms_since(tq);
    const auto ta = std::chrono::steady_clock::now();
    HSA_OK(hsa_amd_memory_pool_allocate(h_.kernarg, kKernargArena + kStageSlot, 0, reinterpret_cast<void**>(&stage_)));
    HSA_OK(hsa_amd_memory_pool_allocate(h_.kernarg, kHostBytes, 0, reinterpret_cast<void**>(&host_)));
    HSA_OK(hsa_amd_agents_allow_access(1, &g_.agent, nullptr, stage_));
    HSA_OK(hsa_amd_agents_allow_access(1, &g_.agent, nullptr, host_));
    HSA_OK(hsa_amd_memory_pool_allocate(g_.vram, kKernargArena, 0, reinterpret_cast<void**>(&dev_args_)));
    host_alloc_ms = ms_since(ta);
    const auto t = std::chrono::steady_clock::now();
    HSA_OK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe_));
    for (const auto& co : code_objects) {
      hsa_code_object_reader_t r;
      HSA_OK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &r));
      readers_.push_back(r);
      HSA_OK(hsa_executable_load_agent_code_object(exe_, g_.agent, r, nullptr, nullptr));
    }
    HSA_OK(hsa_executable_freeze(exe_, nullptr));
    HSA_OK(hsa_executable_iterate_agent_symbols(exe_, g_.agent, find_kernels, &ks_));
    for (const Kernel* k : {&ks_.fill_plain, &ks_.fill_nt, &ks_.verify, &ks_.philox, &ks_.copy, &ks_.md5c, &ks_.md5,
                             &ks_.md5f})
      if (!k->found) throw std::runtime_error("kernel missing from the code objects");
    code_ms = ms_since(t);
  }

  ~Device() {
    if (vram_) hsa_amd_memory_pool_free(vram_);
    if (dev_args_) hsa_amd_memory_pool_free(dev_args_);
    if (stage_) hsa_amd_memory_pool_free(stage_);
    if (host_) hsa_amd_memory_pool_free(host_);
    if (q_) hsa_queue_destroy(q_);
    hsa_executable_destroy(exe_);
    for (auto r : readers_) hsa_code_object_reader_destroy(r);
  }

  char* vram(size_t bytes) {
    if (vram_bytes_ < bytes) {
      if (vram_) HSA_OK(hsa_amd_memory_pool_free(vram_));
      vram_ = nullptr;
      vram_bytes_ = 0;
      HSA_OK(hsa_amd_memory_pool_allocate(g_.vram, bytes, 0, reinterpret_cast<void**>(&vram_)));
      vram_bytes_ = bytes;
    }
    return vram_;
  }

  unsigned grid_for(size_t items, unsigned per_cu) const {
    const size_t need = (items + kBlock - 1) / kBlock;
    const size_t cap = static_cast<size_t>(g_.cus) * per_cu;
    const size_t gsz = std::min(need, cap);
    return static_cast<unsigned>(gsz ? gsz : 1);
  }

  // Stage one kernel of the current batch; returns its index (for its GPU timestamps).
  // system: the kernel's results are read by the host (system-scope release).
  template <class Fill>
  size_t launch(const Kernel& k, unsigned blocks, uint16_t block, Fill fill, bool system = false,
                bool sys_acquire = false) {
    const size_t slot = align_up(std::max<uint32_t>(k.kernarg_size, 64), 64);
    if (stage_off_ + slot > kKernargArena) sync();  // the arenas are reused after a sync
    KernArgs args(stage_ + stage_off_, static_cast<uint32_t>(slot));
    fill(args);
    args.hidden(blocks, block, k.kernarg_size);
    Dispatch d;
    d.k = &k;
    d.blocks = blocks;
    d.block = block;
    d.slot = stage_off_;
    d.system = system;
    d.sys_acquire = sys_acquire;
    stage_off_ += slot;
    batch_.push_back(d);
    return count_++;
  }

  // Run the batch and wait; keeps the GPU start/end (ns) of each dispatch.
  //
  // Kernel arguments are read by every wave (s_load from kernarg_address). From fine-grained
  // host memory that is one uncached PCIe read per wave -- 16K waves per 1 GiB fill -- and
  // measured (rocprofv3, profiles/r1_hsaprobe/) 9-25 % off every kernel against HIP, which keeps
  // kernel arguments in device memory. So the batch's arguments are staged in host memory, one
  // small copy kernel (its own few arguments read from the host) moves them into a VRAM arena,
  // and the batch's packets point there.
  // bound_s <= 0: the general GPU bound (TK8S_GPU_SYNC_TIMEOUT_S, 30 s)
  void sync(double bound_s = 0) {
    if (batch_.empty()) return;
    const size_t bytes = align_up(stage_off_, 16);
    KernArgs cargs(stage_ + kKernargArena, static_cast<uint32_t>(kStageSlot));
    cargs.ptr(dev_args_).ptr(stage_).u64(bytes / 16);
    cargs.hidden(1, kBlock, ks_.copy.kernarg_size);
    // Acquire at system scope: the staged arguments (and, first time, everything) come from the host.
    enqueue(ks_.copy, 1, kBlock, stage_ + kKernargArena, HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_AGENT, hsa_signal_t{0});
    for (auto& d : batch_) {
      // A completion signal per dispatch for its GPU timestamps. Not an interrupt signal (what
      // hsa_signal_create makes): an interrupt at every completion delayed the next barrier
      // packet by ~20 us. The host only spins on the last one, which this signal kind supports.
      HSA_OK(hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &d.sig));
      // Agent scope between kernels, as HIP does on one stream (L2s of the XCDs written back
      // and invalidated; with no fence the next kernel read stale lines and the MD5 tree came
      // out wrong); system-scope release for results the host reads.
      enqueue(*d.k, d.blocks, d.block, dev_args_ + d.slot, d.sys_acquire ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT,
              d.system ? HSA_FENCE_SCOPE_SYSTEM : HSA_FENCE_SCOPE_AGENT, d.sig);
    }
    const hsa_signal_t last = batch_.back().sig;
    // Bounded active wait: the kernels are finite; a wedged GPU must not hang the bring-up
    // (TK8S_GPU_SYNC_TIMEOUT_S, default 30 s). On expiry a fault-injected stall is released and
    // the queue gets a few seconds to drain; the batch is dropped either way, so the next pull
    // starts clean.
    const double bound_ms = (bound_s > 0 ? bound_s : tk8s::gpu_sync_timeout_s()) * 1000.0;
    const auto t0 = std::chrono::steady_clock::now();
    while (hsa_signal_wait_scacquire(last, HSA_SIGNAL_CONDITION_LT, 1, 1000000, HSA_WAIT_STATE_ACTIVE) >= 1) {
      if (ms_since(t0) > bound_ms) {
        stall_release();
        const auto td = std::chrono::steady_clock::now();
        bool drained = false;
        while (!(drained = hsa_signal_load_scacquire(last) < 1) && ms_since(td) < 5000)
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
        for (auto& d : batch_) {
          times_.push_back({0.0, 0.0});
          if (drained) hsa_signal_destroy(d.sig);
        }
        batch_.clear();
        stage_off_ = 0;
        char msg[96];
        std::snprintf(msg, sizeof msg, "GPU dispatch did not complete within %.0f s", bound_ms / 1000.0);
        throw std::runtime_error(msg);
      }
    }
    for (auto& d : batch_) {
      hsa_amd_profiling_dispatch_time_t t{};
      if (hsa_amd_profiling_get_dispatch_time(g_.agent, d.sig, &t) == HSA_STATUS_SUCCESS)
        times_.push_back({t.start * 1e9 / freq_, t.end * 1e9 / freq_});
      else
        times_.push_back({0.0, 0.0});
      hsa_signal_destroy(d.sig);
    }
    batch_.clear();
    stage_off_ = 0;
  }

  // GPU milliseconds from the start of dispatch a to the end of dispatch b (launch() indices;
  // valid after the sync() that completed b).
  double span_ms(size_t a, size_t b) const { return (times_[b].second - times_[a].first) * 1e-6; }

  // ---- the kernels, with the same launch shapes as the HIP wrappers ----
  size_t fill(void* dst, size_t bytes, uint32_t value, bool nt, bool system = false) {
    // stream_kernels.hip hbm_fill: plain = one 128-thread block per CU (the write-front walk),
    // non-temporal = the slab walk over CUs x 16 blocks
    const size_t n16 = bytes / 16;
    const unsigned grid = nt ? grid_for(n16 / 4, 16) : static_cast<unsigned>(std::max(g_.cus, 1u));
    return launch(nt ? ks_.fill_nt : ks_.fill_plain, grid, nt ? kBlock : kFillBlock,
                  [&](KernArgs& a) { a.ptr(dst).u64(n16).u32(value); }, system);
  }
  size_t verify(const void* src, size_t bytes, uint32_t value, void* bad) {
    const size_t n16 = bytes / 16;
    return launch(ks_.verify, grid_for(n16 / 4, 16), kBlock,
                           [&](KernArgs& a) { a.ptr(src).u64(n16).u32(value).ptr(bad); });
  }
  size_t philox(void* dst, size_t bytes, uint64_t seed) {
    const size_t n16 = bytes / 16;
    return launch(ks_.philox, grid_for(n16 / 4, 16), kBlock, [&](KernArgs& a) {
             a.ptr(dst).u64(n16).u32(static_cast<uint32_t>(seed)).u32(static_cast<uint32_t>(seed >> 32));
           });
  }
  // Fault injection: one wave that holds the queue until stall_release() or max_s of the GPU's
  // steady clock -- kernels.h gpu_stall, dispatched on ROCr.
  size_t stall(const uint32_t* flag, double max_s) {
    if (!ks_.stall.found) throw std::runtime_error("stall kernel missing from the code objects");
    uint64_t hz = 0;  // the steady counter the kernel reads (wall_clock64), 1-400 MHz
    if (hsa_agent_get_info(g_.agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_TIMESTAMP_FREQUENCY), &hz) !=
            HSA_STATUS_SUCCESS || hz == 0)
      hz = 100000000;
    const auto ticks = static_cast<uint64_t>(max_s * static_cast<double>(hz));
    return launch(ks_.stall, 1, 64, [&](KernArgs& a) { a.ptr(flag).u64(ticks); });
  }
  size_t copy(void* dst, const void* src, size_t bytes, bool to_host = false, bool from_remote = false) {
    const size_t n16 = bytes / 16;
    return launch(ks_.copy, grid_for(n16 / 8, 16), kBlock,  // stream_kernels.hip: kCopyDepth 8, 16 blocks/CU
                  [&](KernArgs& a) { a.ptr(dst).ptr(src).u64(n16); }, to_host, from_remote);
  }
  // md5_kernels.hip md5_tree: the leaf digests, then fold launches (fan-in 4, a block of 256
  // folding 1024 nodes up to five levels) until one digest; returns (first, last) dispatch.
  std::pair<size_t, size_t> md5_tree(const void* src, size_t nbytes, uint32_t chunk, void* wa, void* wb, void* out) {
    const uint64_t nleaves = nbytes == 0 ? 1 : (nbytes + chunk - 1) / chunk;
    void* leaf_dst = nleaves == 1 ? out : wa;
    size_t first = SIZE_MAX, last = 0;
    const uint64_t ngroups = chunk % 128 == 0 ? (nbytes / chunk) / kWaveChunks : 0;
    if (ngroups) {
      const unsigned grid = static_cast<unsigned>((ngroups + kMd5Block / 64 - 1) / (kMd5Block / 64));
      last = first = launch(ks_.md5c, grid, kMd5Block, [&](KernArgs& a) {
        a.ptr(src).u32(chunk).u64(ngroups).ptr(leaf_dst);
      });
    }
    const uint64_t done = ngroups * kWaveChunks;
    if (!(done >= nleaves && nbytes)) {
      const size_t off = static_cast<size_t>(done) * chunk;
      const uint64_t rest = nleaves - done;
      const unsigned grid = static_cast<unsigned>((rest + kMd5Block - 1) / kMd5Block);
      const auto* s = static_cast<const unsigned char*>(src) + off;
      auto* d = static_cast<unsigned char*>(leaf_dst) + done * 16;
      last = launch(ks_.md5, grid, kMd5Block, [&](KernArgs& a) {
        a.ptr(s).u64(static_cast<uint64_t>(nbytes - off)).u32(chunk).u64(rest).ptr(d);
      });
      first = std::min(first, last);
    }
    auto levels_to_root = [](uint64_t n) {
      int f = 0;
      for (; n > 1; ++f) n = (n + 3) / 4;
      return f;
    };
    const void* in = wa;
    void* bufs[2] = {wb, wa};
    uint64_t n = nleaves;
    for (int k = 0; n > 1; ++k) {
      const int left = levels_to_root(n), levels = std::min(kFoldLevels, left);
      void* dst = levels == left ? out : bufs[k & 1];
      const uint64_t parents = (n + 3) / 4;
      const unsigned grid = static_cast<unsigned>((parents + kFoldBlock - 1) / kFoldBlock);
      last = launch(ks_.md5f, grid, kFoldBlock, [&](KernArgs& a) {
        a.ptr(in).u64(n).u32(static_cast<uint32_t>(levels)).ptr(dst);
      });
      n = grid;
      in = dst;
    }
    return {first, last};
  }
  uint8_t* host() { return host_; }
  const Gpu& gpu() const { return g_; }

  double code_ms = 0, queue_ms = 0, host_alloc_ms = 0;

 private:
  // One AQL kernel dispatch packet (barrier bit set: in queue order, like a stream).
  void enqueue(const Kernel& k, unsigned blocks, uint16_t block, void* kernargs, uint32_t acq, uint32_t rel,
               hsa_signal_t sig) {
    const uint64_t idx = hsa_queue_add_write_index_scacq_screl(q_, 1);
    while (idx - hsa_queue_load_read_index_scacquire(q_) >= q_->size) std::this_thread::yield();
    auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(q_->base_address) + (idx & (q_->size - 1));
    std::memset(reinterpret_cast<uint8_t*>(pkt) + 4, 0, sizeof(*pkt) - 4);
    pkt->workgroup_size_x = block;
    pkt->workgroup_size_y = 1;
    pkt->workgroup_size_z = 1;
    pkt->grid_size_x = blocks * static_cast<uint32_t>(block);
    pkt->grid_size_y = 1;
    pkt->grid_size_z = 1;
    pkt->private_segment_size = k.priv;
    pkt->group_segment_size = k.group;
    pkt->kernel_object = k.object;
    pkt->kernarg_address = kernargs;
    pkt->completion_signal = sig;
    const uint16_t header = static_cast<uint16_t>(
        (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1u << HSA_PACKET_HEADER_BARRIER) |
        (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) | (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    const uint16_t setup = 1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), static_cast<uint32_t>(header) | (static_cast<uint32_t>(setup) << 16),
                     __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q_->doorbell_signal, static_cast<hsa_signal_value_t>(idx));
  }

  static constexpr size_t kKernargArena = 1 << 16;
  static constexpr size_t kStageSlot = 512;  // the argument copy's own arguments, after the arena
  static constexpr size_t kHostBytes = 4096;
  const Gpu& g_;
  const Host& h_;
  double freq_;
  hsa_executable_t exe_{};
  std::vector<hsa_code_object_reader_t> readers_;
  KernelSet ks_;
  hsa_queue_t* q_ = nullptr;
  char* vram_ = nullptr;
  size_t vram_bytes_ = 0;
  uint8_t* stage_ = nullptr;     // host staging arena for the batch's kernel arguments
  uint8_t* dev_args_ = nullptr;  // their VRAM copy, what the packets point at
  size_t stage_off_ = 0;
  uint8_t* host_ = nullptr;
  std::vector<Dispatch> batch_;
  std::vector<std::pair<double, double>> times_;  // GPU start/end (ns) of every completed dispatch
  size_t count_ = 0;
};

// ---- the probes (same semantics and JSON as native/src/probes.cpp) --------------------------
struct DeviceResult {
  std::string hbm, md5, copy, digest, error, host_pull;
  std::vector<std::string> peers;  // pulls INTO this device, one per source GPU
  bool peers_ok = true;
  std::string peer_source_error;  // filling its buffer for the peers failed: a link verdict, not a device one
  double wall_ms = 0, hbm_ms = 0, md5_ms = 0, copy_ms = 0, setup_ms = 0;
  bool ok = true;
  Device* dev = nullptr;  // kept for the peer phase (never freed, see run_device)
  char* base = nullptr;   // start of its VRAM allocation (what peers are granted access to)
};

void run_device(const Gpu& g, const Host& h, const std::vector<std::string>& cos, double freq, const Config& c,
                DeviceResult& r) {
  const auto td = std::chrono::steady_clock::now();
  // Never freed: the process exits right after printing, and tearing down queues and memory
  // first would only delay the result (a GPU process's exit costs tens of ms, benchmarks.md).
  auto* dev = new Device(g, h, cos, freq);
  const size_t ws = c.md5 ? (c.md5 + c.chunk - 1) / c.chunk * 16 : 0;
  // + the MALL flush region (2 x the 256 MB Infinity Cache) written before each timed MD5 pass
  const size_t md5_need = c.md5 ? align_up(std::max<size_t>(c.md5, 16)) + 2 * align_up(ws) + kAlign + kMallFlush : 0;
  const size_t need = std::max({c.hbm ? align_up(c.hbm) + kAlign : 0, md5_need, c.copy ? 2 * align_up(c.copy) + kAlign : 0,
                                (c.peers || c.peers_host) ? 2 * align_up(c.peer) + kAlign : 0, kAlign});
  char* base = dev->vram(need);
  r.dev = dev;
  r.base = base;
  r.setup_ms = ms_since(td);
  uint8_t* host = dev->host();
  const int it = std::max(c.iters, 1);
  const uint32_t value = 0;
  // All three probes go into the queue back to back (barrier packets, stream order); one wait.
  size_t h_cold = 0, h_w0 = 0, h_w1 = 0, h_rd = 0;
  if (c.hbm) {
    char* bad = base + align_up(c.hbm);
    h_cold = dev->fill(base, c.hbm, value ^ 0xFFFFFFFFu, c.nontemporal);
    for (int i = 0; i < it; ++i) {
      const size_t k = dev->fill(base, c.hbm, value, c.nontemporal);
      if (i == 0) h_w0 = k;
      h_w1 = k;
    }
    dev->fill(bad, 16, 0, false);
    h_rd = dev->verify(base, c.hbm, value, bad);
    dev->copy(host + 0, bad, 16, true);
  }
  size_t m_fill = 0;
  std::pair<size_t, size_t> m_cold{0, 0};
  std::vector<std::pair<size_t, size_t>> m_warm;
  if (c.md5) {
    char* data = base;
    char* wa = base + align_up(std::max<size_t>(c.md5, 16));
    char* wb = wa + align_up(ws);
    char* out = wb + align_up(ws);
    char* flush = out + kAlign;
    m_fill = dev->philox(data, c.md5, c.seed);
    m_cold = dev->md5_tree(data, c.md5, c.chunk, wa, wb, out);
    for (int i = 0; i < it; ++i) {
      // each timed pass starts from HBM: 512 MiB written elsewhere first evicts the input from
      // the memory-side Infinity Cache (a 256 MiB input fits the 256 MB MALL)
      dev->fill(flush, kMallFlush, 0x5A5A5A5Au + i, false);
      m_warm.push_back(dev->md5_tree(data, c.md5, c.chunk, wa, wb, out));
    }
    dev->copy(host + 64, out, 16, true);
  }
  size_t c_w0 = 0, c_w1 = 0;
  if (c.copy) {
    char* src = base;
    char* dst = base + align_up(c.copy);
    char* bad = base + 2 * align_up(c.copy);
    dev->fill(src, c.copy, 0xA5A5A5A5u, false);
    dev->copy(dst, src, c.copy);  // warm-up
    for (int i = 0; i < it; ++i) {
      const size_t k = dev->copy(dst, src, c.copy);
      if (i == 0) c_w0 = k;
      c_w1 = k;
    }
    dev->fill(bad, 16, 0, false);
    dev->verify(dst, c.copy, 0xA5A5A5A5u, bad);
    dev->copy(host + 128, bad, 16, true);
  }
  dev->sync();
  auto u64_at = [&](size_t off) {
    uint64_t v = 0;
    std::memcpy(&v, host + off, 8);
    return v;
  };
  if (c.hbm) {
    const uint64_t nbad = u64_at(0);
    const double cold_ms = dev->span_ms(h_cold, h_cold), ms = dev->span_ms(h_w0, h_w1) / it,
                 read_ms = dev->span_ms(h_rd, h_rd);
    // Dispatch timestamps that put a fill or read above the MI355X's 8 TB/s HBM3E peak are not
    // the kernels' (a tool that intercepts the queue, such as rocprofv3, answers them with its
    // own forwarding packets): the data checks still count, the rates are flagged.
    const bool plausible = ms > 0 && read_ms > 0 && c.hbm / (ms * 1e-3) / 1e9 <= kHbmPeakGBps * 1.1 &&
                           c.hbm / (read_ms * 1e-3) / 1e9 <= kHbmPeakGBps * 1.1;
    r.hbm = Json()
                .kv("timing", plausible ? "gpu_timestamps" : "implausible")
                .kv("ok", nbad == 0)
                .kv("probe", "hbm_write")
                .kv("read_ms", read_ms)
                .kv("read_gbps", c.hbm / (read_ms * 1e-3) / 1e9)
                .kv("device", 0)
                .kv("bytes", static_cast<uint64_t>(c.hbm))
                .kv("iters", it)
                .kv("mode", c.nontemporal ? "nontemporal" : "plain")
                .kv("cold_ms", cold_ms)
                .kv("ms", ms)
                .kv("seconds", ms * 1e-3)
                .kv("gbps", c.hbm / (ms * 1e-3) / 1e9)
                .kv("bad_words", nbad)
                .raw("host_ms", Json()
                                    .kv("code_objects", dev->code_ms)
                                    .kv("queue", dev->queue_ms)
                                    .kv("host_alloc", dev->host_alloc_ms)
                                    .kv("setup", r.setup_ms)
                                    .str())
                .str();
    r.ok = r.ok && nbad == 0;
  } else {
    r.hbm = "{\"ok\":true,\"skipped\":true}";
  }
  if (c.md5) {
    r.digest = hex(host + 64, 16);
    double warm = 0;
    for (const auto& w : m_warm) warm += dev->span_ms(w.first, w.second);
    const double fill_ms = dev->span_ms(m_fill, m_fill), cold_ms = dev->span_ms(m_cold.first, m_cold.second),
                 ms = warm / it;
    r.md5 = Json()
                .kv("ok", true)
                .kv("probe", "md5_tree")
                .kv("device", 0)
                .kv("bytes", static_cast<uint64_t>(c.md5))
                .kv("chunk_bytes", c.chunk)
                .kv("seed", static_cast<uint64_t>(c.seed))
                .kv("iters", it)
                .kv("digest", r.digest)
                .kv("fill_ms", fill_ms)
                .kv("fill_gbps", c.md5 / (fill_ms * 1e-3) / 1e9)
                .kv("cold_ms", cold_ms)
                .kv("ms", ms)
                .kv("seconds", ms * 1e-3)
                .kv("mbps", c.md5 / (ms * 1e-3) / 1e6)
                .kv("mall_flushed", true)
                .str();
  }
  if (c.copy) {
    const uint64_t nbad = u64_at(128);
    const double kernel_ms = dev->span_ms(c_w0, c_w1) / it;
    r.copy = Json()
                 .kv("ok", nbad == 0)
                 .kv("probe", "local_copy")
                 .kv("src_device", 0)
                 .kv("dst_device", 0)
                 .kv("bytes", static_cast<uint64_t>(c.copy))
                 .kv("iters", it)
                 .kv("kernel_ms", kernel_ms)
                 .kv("kernel_gbps", c.copy / (kernel_ms * 1e-3) / 1e9)
                 .kv("bad_words", nbad)
                 .str();
    r.ok = r.ok && nbad == 0;
  }
  r.wall_ms = ms_since(td);
}

// ---- N7: xGMI peer pulls --------------------------------------------------------------------
// The source pattern names the GPU it came from, so a pull that read the wrong device (or a
// stale line) fails verification, not just one that read garbage.
uint32_t peer_pattern(int src) { return 0x5EE00000u | static_cast<uint32_t>(src & 0xFFFF); }

std::string pull_json(const char* probe, int src, int dst, const Config& c, const std::string& access, double ms,
                      uint64_t nbad, const std::string& error) {
  Json j;
  j.kv("ok", error.empty() && nbad == 0).kv("probe", probe).kv("src_device", src).kv("dst_device", dst)
      .kv("bytes", static_cast<uint64_t>(c.peer)).kv("iters", std::max(c.peer_iters, 1)).kv("access", access);
  if (error.empty()) j.kv("kernel_ms", ms).kv("kernel_gbps", ms > 0 ? c.peer / (ms * 1e-3) / 1e9 : 0.0).kv("bad_words", nbad);
  else j.kv("error", error);
  return j.str();
}

// One pull of c.peer bytes from `src` (memory of another agent, already granted to this device)
// into this device's scratch: a warm-up, peer_iters timed copies, then a pattern check.
// Returns (GPU ms per copy, bad words).
std::pair<double, uint64_t> pull(DeviceResult& r, const void* src, uint32_t pattern, const Config& c) {
  Device* d = r.dev;
  char* dst = r.base + align_up(c.peer);
  char* bad = dst + align_up(c.peer);
  const int it = std::max(c.peer_iters, 1);
  if (tk8s::fault_armed("probe", "hang", "peers")) {  // TK8S_FAULTS probe.hang@peers: a pull that never ends
    if (uint32_t* f = g_stall_flag.load()) {
      __atomic_store_n(f, 0u, __ATOMIC_SEQ_CST);
      d->stall(f, 2 * tk8s::gpu_sync_timeout_s() + 5);
    }
  }
  d->copy(dst, src, c.peer, false, /*from_remote=*/true);  // warm-up (and the system-scope acquire)
  size_t first = 0, last = 0;
  for (int i = 0; i < it; ++i) {
    const size_t k = d->copy(dst, src, c.peer);
    if (i == 0) first = k;
    last = k;
  }
  d->fill(bad, 16, 0, false);
  d->verify(dst, c.peer, pattern, bad);
  d->copy(d->host() + 192, bad, 16, true);
  d->sync();
  uint64_t nbad = 0;
  std::memcpy(&nbad, d->host() + 192, 8);
  return {d->span_ms(first, last) / it, nbad};
}

void run_peers(const std::vector<int>& devices, const Config& c, std::vector<DeviceResult>& res, const Host& h) {
  const size_t m = devices.size();
  tk8s::fault_point("probe", "peers", /*host_hang=*/false);  // TK8S_FAULTS probe.exit|crash@peers
  if (tk8s::fault_armed("probe", "hang", "peers") && !g_stall_flag.load()) {
    void* f = nullptr;
    HSA_OK(hsa_amd_memory_pool_allocate(h.kernarg, 64, 0, &f));
    std::vector<hsa_agent_t> agents;
    for (size_t k = 0; k < m; ++k)
      if (res[k].dev) agents.push_back(res[k].dev->gpu().agent);
    HSA_OK(hsa_amd_agents_allow_access(static_cast<uint32_t>(agents.size()), agents.data(), nullptr, f));
    g_stall_flag = static_cast<uint32_t*>(f);
  }
  // 1. every source buffer gets its pattern, released at system scope (peers read it next).
  for (size_t k = 0; k < m; ++k) {
    if (!res[k].dev) continue;
    try {
      res[k].dev->fill(res[k].base, c.peer, peer_pattern(devices[k]), false, /*system=*/true);
      res[k].dev->sync();
    } catch (const std::exception& e) {
      // The device itself passed its own checks: this fails the links that read from it (their
      // pulls report "unavailable", peers_ok goes false on both ends), so the machines still get
      // their share of the result and the xGMI verdict keeps the node NotReady.
      res[k].peer_source_error = std::string("peer source fill: ") + e.what();
      res[k].peers_ok = false;
    }
  }
  // 2. grants: who may read whose VRAM. A pool the runtime reports NEVER_ALLOWED for an agent is
  // not granted and not touched (a kernel reading memory it has no mapping for faults the GPU).
  std::vector<std::vector<std::string>> access(m, std::vector<std::string>(m, "self"));
  for (size_t j = 0; j < m; ++j) {
    std::vector<hsa_agent_t> readers;
    std::vector<size_t> idx;
    for (size_t k = 0; k < m; ++k) {
      if (k == j) continue;
      if (!res[j].dev || !res[k].dev || !res[j].error.empty() || !res[k].error.empty() ||
          !res[j].peer_source_error.empty()) {
        access[k][j] = "unavailable";
        continue;
      }
      hsa_amd_memory_pool_access_t a = HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED;
      hsa_amd_agent_memory_pool_get_info(res[k].dev->gpu().agent, res[j].dev->gpu().vram,
                                         HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &a);
      if (a == HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED) {
        access[k][j] = "never_allowed";
        continue;
      }
      readers.push_back(res[k].dev->gpu().agent);
      idx.push_back(k);
    }
    if (readers.empty()) continue;
    const hsa_status_t st = hsa_amd_agents_allow_access(static_cast<uint32_t>(readers.size()), readers.data(), nullptr,
                                                        res[j].base);
    for (size_t k : idx) access[k][j] = st == HSA_STATUS_SUCCESS ? "allowed" : "denied";
  }
  // 3. rounds: in round r every GPU i pulls from GPU (i + r) mod m, all at once -- all of them
  // inside TK8S_PEER_PHASE_TIMEOUT_S (default 20 s): once it has passed, the remaining rounds are
  // reported as not run, so a fabric where every pull times out costs one bound, not m - 1 of
  // them (the host burn-in then re-runs the pulls through the HIP probe: burnin.HostBurnin)
  const auto phase_t0 = std::chrono::steady_clock::now();
  const double phase_ms = tk8s::peer_phase_timeout_s() * 1000.0;
  for (size_t r = 1; r < m; ++r) {
    if (ms_since(phase_t0) > phase_ms) {
      for (size_t k = 0; k < m; ++k) {
        res[k].peers.push_back(pull_json("xgmi_peer_pull", devices[(k + r) % m], devices[k], c, access[k][(k + r) % m], 0,
                                         0, "not run: the peer phase's deadline passed"));
        res[k].peers_ok = false;
      }
      continue;
    }
    std::vector<std::thread> th;
    for (size_t k = 0; k < m; ++k) {
      th.emplace_back([&, k, r] {
        const size_t j = (k + r) % m;
        const std::string& acc = access[k][j];
        DeviceResult& rk = res[k];  // only this thread touches it in this round
        if (acc != "allowed") {
          rk.peers.push_back(pull_json("xgmi_peer_pull", devices[j], devices[k], c, acc, 0, 0, "no access: " + acc));
          rk.peers_ok = false;
          return;
        }
        try {
          const auto p = pull(rk, res[j].base, peer_pattern(devices[j]), c);
          rk.peers.push_back(pull_json("xgmi_peer_pull", devices[j], devices[k], c, acc, p.first, p.second, ""));
          rk.peers_ok = rk.peers_ok && p.second == 0;
        } catch (const std::exception& e) {
          rk.peers.push_back(pull_json("xgmi_peer_pull", devices[j], devices[k], c, acc, 0, 0, e.what()));
          rk.peers_ok = false;
        }
      });
    }
    for (auto& t : th) t.join();
  }
}

// --peers-host: the pull path from a host-memory source (the runtime's fine-grained system pool,
// filled by the CPU, granted to the GPU the way peers are).
void run_host_pull(const Host& h, int device, const Config& c, DeviceResult& r) {
  if (!r.dev) return;
  void* src = nullptr;
  std::string acc = "allowed", err;
  double ms = 0;
  uint64_t nbad = 0;
  try {
    HSA_OK(hsa_amd_memory_pool_allocate(h.kernarg, c.peer, 0, &src));
    const uint32_t pat = peer_pattern(-1);
    auto* w = static_cast<uint32_t*>(src);
    for (size_t i = 0; i < c.peer / 4; ++i) w[i] = pat;
    const hsa_agent_t agent = r.dev->gpu().agent;
    if (hsa_amd_agents_allow_access(1, &agent, nullptr, src) != HSA_STATUS_SUCCESS) acc = "denied";
    if (acc == "allowed") {
      const auto p = pull(r, src, pat, c);
      ms = p.first;
      nbad = p.second;
    } else {
      err = "no access: denied";
    }
  } catch (const std::exception& e) {
    err = e.what();
  }
  r.host_pull = pull_json("host_pull", -1, device, c, acc, ms, nbad, err);
  if (src) hsa_amd_memory_pool_free(src);
}

void emit(const std::string& json, const std::string& out_file) {
  if (!out_file.empty()) {
    const std::string tmp = out_file + ".tmp";
    {
      std::ofstream f(tmp);
      f << json << "\n";
    }
    std::rename(tmp.c_str(), out_file.c_str());
    std::remove((out_file + ".pending").c_str());
  }
  std::printf("%s\n", json.c_str());
  std::fflush(stdout);
}

// The device index in the per-device JSON is the probed position, like tk8s-probe's HIP ordinal.
std::string with_device(const std::string& j, int d) {
  const std::string pat = "\"device\":0";
  const auto p = j.find(pat);
  if (p == std::string::npos || d == 0) return j;
  return j.substr(0, p) + "\"device\":" + std::to_string(d) + j.substr(p + pat.size());
}

}  // namespace

int main(int argc, char** argv) {
  const auto t0 = std::chrono::steady_clock::now();
  // wall clock at main(): against the launcher's spawn time it shows the exec + loader cost
  const double main_unix_ms =
      std::chrono::duration<double, std::milli>(std::chrono::system_clock::now().time_since_epoch()).count();
  std::string out_file;
  try {
    tk8s::Args a(argc, argv);
    out_file = a.str("out", "");
    if (a.has("reuse")) {
      const int rc = tk8s::reuse(a.str("reuse"), static_cast<double>(a.num("reuse-wait", 120)));
      if (rc >= 0) return rc;
    }
    Config c;
    c.hbm = static_cast<size_t>(a.num("hbm-bytes", 1LL << 30));
    c.md5 = a.has("skip-md5") ? 0 : static_cast<size_t>(a.num("md5-bytes", 256LL << 20));
    c.copy = static_cast<size_t>(a.num("copy-bytes", 1LL << 30));
    c.chunk = static_cast<uint32_t>(a.num("chunk", 1024));
    c.seed = static_cast<uint64_t>(a.num("seed", 0));
    c.iters = static_cast<int>(a.num("iters", 5));
    c.nontemporal = a.str("mode", "plain") == "nontemporal";
    c.peers = a.has("peers");
    c.peers_host = a.has("peers-host");
    c.peer = static_cast<size_t>(a.num("peer-bytes", 32LL << 20));
    c.peer_iters = static_cast<int>(a.num("peer-iters", std::min<long long>(c.iters, 2)));
    if (c.hbm % 16 || c.md5 % 16 || c.copy % 16 || c.peer % 16 || c.peer == 0 || c.chunk == 0 || c.chunk % 64)
      throw std::invalid_argument("sizes must be multiples of 16 and --chunk a positive multiple of 64");
    const std::string dir = exe_dir() + "/../lib/";
    const std::vector<std::string> cos = {read_file(dir + "tk8s_stream.co"), read_file(dir + "tk8s_md5.co")};

    tk8s::cachewalk::configure();  // the plan's environment is in place (cachewalk.h)
    HSA_OK(hsa_init());
    const double init_ms = ms_since(t0);
    Topology t;
    HSA_OK(hsa_iterate_agents(collect_agent, &t));
    const int n = static_cast<int>(t.gpus.size());
    if (n == 0 || !t.host.has_kernarg) {
      emit("{\"ok\":false,\"runtime\":\"hsa\",\"error\":\"no GPU agent (or no kernarg pool) visible\"}", out_file);
      return 3;
    }
    for (const Gpu& g : t.gpus)
      if (!g.has_vram) throw std::runtime_error("GPU agent without a VRAM pool");
    std::vector<int> devices;
    if (a.has("all-devices")) {
      for (int d = 0; d < n; ++d) devices.push_back(d);
    } else if (a.has("devices")) {
      // An explicit list; a device may repeat (two queues and arenas on one GPU): on a one-GPU
      // box that runs the multi-device path -- threads, peer grants, rounds of pulls -- end to end.
      const std::string list = a.str("devices");
      size_t pos = 0;
      while (pos <= list.size()) {
        const size_t end = std::min(list.find(',', pos), list.size());
        const std::string item = list.substr(pos, end - pos);
        char* tail = nullptr;
        const long d = std::strtol(item.c_str(), &tail, 10);
        if (item.empty() || *tail != '\0' || d < 0 || d >= n) {
          emit("{\"ok\":false,\"error\":\"bad --devices " + list + "\"}", out_file);
          return 2;
        }
        devices.push_back(static_cast<int>(d));
        pos = end + 1;
      }
    } else {
      const int d = static_cast<int>(a.num("device", 0));
      if (d < 0 || d >= n) {
        emit("{\"ok\":false,\"error\":\"device " + std::to_string(d) + " out of range\"}", out_file);
        return 2;
      }
      devices.push_back(d);
    }
    uint64_t freq = 0;
    HSA_OK(hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &freq));
    std::string info;
    const auto tg = std::chrono::steady_clock::now();
    if (a.has("gpuinfo")) info = gpuinfo_json(t);
    const double gpuinfo_ms = ms_since(tg);

    std::vector<DeviceResult> res(devices.size());
    auto run_one = [&](size_t k) {
      try {
        run_device(t.gpus[devices[k]], t.host, cos, static_cast<double>(freq), c, res[k]);
      } catch (const std::exception& ex) {
        res[k].ok = false;
        res[k].error = ex.what();
      }
    };
    std::vector<std::thread> threads;
    for (size_t k = 1; k < devices.size(); ++k) threads.emplace_back(run_one, k);
    run_one(0);
    for (auto& th : threads) th.join();
    const auto tp = std::chrono::steady_clock::now();
    if (c.peers && devices.size() > 1) run_peers(devices, c, res, t.host);
    if (c.peers_host) run_host_pull(t.host, devices[0], c, res[0]);
    const double peers_ms = ms_since(tp);

    // The known answer is pinned for the default input only. Any other configuration can only be
    // checked for agreement: the digest most devices produced is the reference (a single wrong
    // device is blamed, not the others), and with one device there is nothing to compare, which
    // the result says ("digest_ok": "unpinned", "md5_pinned": false) instead of claiming a pass.
    std::string want;
    const bool pinned = c.md5 == (256u << 20) && c.chunk == 1024 && c.seed == 0;
    if (pinned) {
      want = kKnownDigest256M;
    } else if (c.md5) {
      size_t best = 0;
      for (size_t k = 0; k < res.size(); ++k) {
        size_t votes = 0;
        for (const auto& o : res) votes += (!o.digest.empty() && o.digest == res[k].digest);
        if (votes > best) best = votes, want = res[k].digest;
      }
    }
    const bool unpinned_single = c.md5 && !pinned && res.size() == 1;
    bool ok = true;
    std::vector<std::string> per_dev;
    for (size_t k = 0; k < res.size(); ++k) {
      DeviceResult& r = res[k];
      const bool digest_ok = !c.md5 || (!r.digest.empty() && r.digest == want);
      r.ok = r.ok && digest_ok && r.error.empty();
      ok = ok && r.ok;
      Json d;
      d.kv("device", devices[k]).kv("ok", r.ok).kv("wall_ms", r.wall_ms)
          .raw("phase_ms", Json().kv("setup", r.setup_ms).str());
      if (!r.error.empty()) d.kv("error", r.error);
      if (!r.hbm.empty()) d.raw("hbm", with_device(r.hbm, devices[k]));
      if (c.md5 && !r.md5.empty()) {
        d.raw("md5", with_device(r.md5, devices[k]));
        if (unpinned_single) d.kv("digest_ok", "unpinned");
        else d.kv("digest_ok", digest_ok);
      }
      if (c.copy && !r.copy.empty()) d.raw("copy", r.copy);
      // Data integrity of its incoming pulls; their bandwidth is judged host-wide (xgmi.py).
      if (c.peers) d.raw("peers", Json::array(r.peers)).kv("peers_ok", r.peers_ok);
      if (!r.peer_source_error.empty()) d.kv("peer_source_error", r.peer_source_error);
      if (!r.host_pull.empty()) d.raw("host_pull", r.host_pull);
      per_dev.push_back(d.str());
    }
    Json out;
    out.kv("ok", ok).kv("runtime", "hsa").kv("device", devices[0]).kv("device_count", n)
        .kv("probed", static_cast<int>(devices.size()));
    if (!res[0].hbm.empty()) out.raw("hbm", res[0].hbm);
    if (c.md5 && !res[0].md5.empty()) out.raw("md5", res[0].md5).kv("md5_expected", want).kv("md5_pinned", pinned);
    if (c.copy && !res[0].copy.empty()) out.raw("copy", res[0].copy);
    out.raw("devices", Json::array(per_dev));
    if (!info.empty()) out.raw("gpuinfo", info);
    if (c.peers) out.kv("peer_bytes", static_cast<uint64_t>(c.peer)).kv("peer_rounds", static_cast<int>(devices.size()) - 1);
    out.raw("timings_ms", Json().kv("hip_init", init_ms).kv("runtime_init", init_ms).kv("gpuinfo", gpuinfo_ms)
                              .kv("peers", peers_ms).kv("total", ms_since(t0))
                              .kv("main_unix_ms", main_unix_ms).kv("exec_unix_ms", main_unix_ms)
                              .kv("cpu_cache_walk", tk8s::cachewalk::mode())
                              .kv("cpu_cache_dirs_hidden", tk8s::cachewalk::g_hidden).str());
    emit(out.str(), out_file);
    std::fflush(stdout);
    if (a.has("release-after")) {  // after the result: the reader is not kept waiting for this
      for (auto& r : res) delete r.dev;
      hsa_shut_down();
    }
    // No runtime teardown on the way out (see run_device) -- unless a tool that finalises in
    // exit handlers is attached (rocprofv3: TK8S_PROBE_CLEAN_EXIT=1).
    if (!std::getenv("TK8S_PROBE_CLEAN_EXIT")) _exit(ok ? 0 : 1);
    return ok ? 0 : 1;
  } catch (const std::exception& e) {
    emit(std::string("{\"ok\":false,\"runtime\":\"hsa\",\"error\":") + Json::escape(e.what()) + "}", out_file);
    std::fprintf(stderr, "tk8s-hsaprobe: %s\n", e.what());
    return 2;
  }
}
