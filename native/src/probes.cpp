// Node-validation probes (N1 gpuinfo, N4 HBM write, N5 MD5 tree, N7 copy/xGMI). Host code;
// compiled with hipcc and linked against the kernels in stream_kernels.hip / md5_kernels.hip.
#include "tk8s/probes.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "tk8s/common.h"

namespace tk8s {

namespace {

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
    case 0: return "hypertransport";
    case 1: return "qpi";
    case 2: return "pcie";
    case 3: return "infiniband";
    case 4: return "xgmi";
    default: return "unknown";
  }
}

std::string error_json(const std::string& what) {
  return Json().kv("ok", false).kv("error", what).str();
}

struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int dev) {
    TK8S_HIP_CHECK(hipGetDevice(&prev));
    TK8S_HIP_CHECK(hipSetDevice(dev));
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

// Per-device scratch arena for the local probes. The validation payload runs HBM, MD5 and copy
// probes back to back; giving each its own hipMalloc/hipFree of 0.25-1 GiB cost ~70 ms per
// device on MI355X (more than all the kernels together), so they share one allocation that
// grows on demand and lives until release_probe_scratch() / process exit. Peer copies keep
// their own buffers (another device's thread may be using its arena concurrently).
struct ScratchSlot {
  std::mutex mu;  // per device: growing one GPU's arena never waits on another's
  void* p = nullptr;
  size_t n = 0;
};
std::mutex g_scratch_mu;                 // guards the map only (node-based: slots never move)
std::map<int, ScratchSlot> g_scratch;

char* scratch(int device, size_t bytes) {
  ScratchSlot* slot;
  {
    std::lock_guard<std::mutex> lock(g_scratch_mu);
    slot = &g_scratch[device];
  }
  std::lock_guard<std::mutex> lock(slot->mu);
  if (slot->n < bytes) {
    if (slot->p) TK8S_HIP_CHECK(hipFree(slot->p));
    slot->p = nullptr;
    slot->n = 0;
    TK8S_HIP_CHECK(hipMalloc(&slot->p, bytes));
    slot->n = bytes;
  }
  return static_cast<char*>(slot->p);
}

// One non-blocking stream per device, created on first use and kept: a ROCm stream is backed
// by a hardware queue, and creating one per probe (plus the legacy null stream for the copy's
// source fill) cost milliseconds each on the validation's critical path. Created outside the
// lock: a first queue costs ~20 ms (profiles/r1_init_costs), and the per-device threads of a
// multi-GPU burn-in must not serialise behind each other's creation.
std::mutex g_stream_mu;
std::map<int, hipStream_t> g_streams;

hipStream_t probe_stream(int device) {
  {
    std::lock_guard<std::mutex> lock(g_stream_mu);
    auto it = g_streams.find(device);
    if (it != g_streams.end()) return it->second;
  }
  hipStream_t s{};
  TK8S_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::lock_guard<std::mutex> lock(g_stream_mu);
  const auto ins = g_streams.emplace(device, s);
  if (!ins.second) (void)hipStreamDestroy(s);  // another thread of this device won the race
  return ins.first->second;
}

struct CachedStream {
  hipStream_t s;
  explicit CachedStream(int device) : s(probe_stream(device)) {}
};

constexpr size_t kAlign = 4096;
constexpr size_t kMallFlush = size_t(512) << 20;  // 2 x the MI355X's 256 MB Infinity Cache (MALL)
size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

// The xGMI pulls' buffers, kept per device for the life of the process: a source per GPU, filled
// once with the pull pattern and then only read (by every other GPU), and a destination + error
// counter per pulling GPU (its slot lock is held for the whole pull). Allocating and freeing them
// per pull cost a hipMalloc/hipFree each -- and hipFree synchronises the whole device, so a pull
// from GPU s waited for everything else running on s, its own probes and other GPUs' pulls.
struct PeerSlot {
  std::mutex mu;
  void* p = nullptr;
  size_t n = 0;
  bool filled = false;
};
std::mutex g_peer_mu;  // guards the maps only (node-based: slots never move)
std::map<int, PeerSlot> g_peer_src, g_peer_dst;

PeerSlot& peer_slot(std::map<int, PeerSlot>& m, int device) {
  std::lock_guard<std::mutex> lock(g_peer_mu);
  return m[device];
}

std::vector<std::pair<int, void*>> g_peer_retired;  // outgrown buffers (guarded by g_peer_mu)

// Grow `slot` (held locked by the caller) to at least `bytes` on `device`. An outgrown buffer is
// retired, not freed: another GPU may still be reading an outgrown source.
void* peer_buffer(PeerSlot& slot, int device, size_t bytes) {
  if (slot.n < bytes) {
    DeviceGuard g(device);
    void* p = nullptr;
    TK8S_HIP_CHECK(hipMalloc(&p, bytes));
    if (slot.p) {
      std::lock_guard<std::mutex> lock(g_peer_mu);
      g_peer_retired.emplace_back(device, slot.p);
    }
    slot.p = p;
    slot.n = bytes;
    slot.filled = false;
  }
  return slot.p;
}

constexpr uint32_t kPeerPattern = 0xA5A5A5A5u;

}  // namespace

void release_probe_scratch() {
  {
    std::lock_guard<std::mutex> lock(g_stream_mu);
    for (auto& kv : g_streams) (void)hipStreamDestroy(kv.second);
    g_streams.clear();
  }
  {
    std::lock_guard<std::mutex> lock(g_peer_mu);
    for (auto* m : {&g_peer_src, &g_peer_dst})
      for (auto& kv : *m) {
        std::lock_guard<std::mutex> slot_lock(kv.second.mu);
        if (!kv.second.p) continue;
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second.p);
        (void)hipSetDevice(prev);
        kv.second.p = nullptr;
        kv.second.n = 0;
        kv.second.filled = false;
      }
    g_peer_src.clear();
    g_peer_dst.clear();
    for (const auto& r : g_peer_retired) {
      int prev = 0;
      (void)hipGetDevice(&prev);
      (void)hipSetDevice(r.first);
      (void)hipFree(r.second);
      (void)hipSetDevice(prev);
    }
    g_peer_retired.clear();
  }
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  for (auto& kv : g_scratch) {
    std::lock_guard<std::mutex> slot_lock(kv.second.mu);
    if (!kv.second.p) continue;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(kv.first);
    (void)hipFree(kv.second.p);
    (void)hipSetDevice(prev);
    kv.second.p = nullptr;
    kv.second.n = 0;
  }
  g_scratch.clear();
}

void reserve_probe_scratch(int device, size_t hbm_bytes, size_t md5_bytes, uint32_t chunk_bytes, size_t copy_bytes) {
  size_t need = kAlign;
  if (hbm_bytes) need = std::max(need, align_up(hbm_bytes) + kAlign);
  if (md5_bytes && chunk_bytes) {
    const size_t ws = md5_tree_workspace(md5_bytes, chunk_bytes);
    need = std::max(need, align_up(std::max<size_t>(md5_bytes, 16)) + 2 * align_up(ws) + kAlign + kMallFlush);
  }
  if (copy_bytes) need = std::max(need, 2 * align_up(copy_bytes) + kAlign);
  DeviceGuard g(device);
  (void)scratch(device, need);
}

std::string gpuinfo_json(bool with_links) {
  const auto t0 = std::chrono::steady_clock::now();
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    return Json()
        .kv("ok", false)
        .kv("device_count", 0)
        .kv("error", std::string("hipGetDeviceCount: ") + hipGetErrorString(e))
        .str();
  }
  int rt = 0, drv = 0;
  (void)hipRuntimeGetVersion(&rt);
  (void)hipDriverGetVersion(&drv);
  std::vector<std::string> devs;
  for (int i = 0; i < n; ++i) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, i) != hipSuccess) continue;
    char bdf[64] = {0};
    (void)hipDeviceGetPCIBusId(bdf, sizeof bdf, i);
    hipUUID uuid;
    std::memset(&uuid, 0, sizeof uuid);
    (void)hipDeviceGetUuid(&uuid, i);
    std::string arch = p.gcnArchName;
    const std::string gfx = arch.substr(0, arch.find(':'));
    devs.push_back(Json()
                       .kv("index", i)
                       .kv("name", std::string(p.name))
                       .kv("arch", arch)
                       .kv("gfx", gfx)
                       .kv("total_mem_bytes", static_cast<uint64_t>(p.totalGlobalMem))
                       .kv("cu_count", p.multiProcessorCount)
                       .kv("clock_khz", p.clockRate)
                       .kv("mem_clock_khz", p.memoryClockRate)
                       .kv("mem_bus_width", p.memoryBusWidth)
                       .kv("wavefront_size", p.warpSize)
                       .kv("lds_per_block_bytes", static_cast<uint64_t>(p.sharedMemPerBlock))
                       .kv("pci_bus_id", std::string(bdf))
                       .kv("uuid", hex(reinterpret_cast<const unsigned char*>(uuid.bytes), 16))
                       .str());
  }
  std::vector<std::string> rows;
  if (with_links) {
    for (int i = 0; i < n; ++i) {
      std::vector<std::string> row;
      for (int j = 0; j < n; ++j) {
        if (i == j) {
          row.push_back(Json().kv("type", "self").kv("hops", 0).kv("p2p", true).str());
          continue;
        }
        uint32_t type = 0, hops = 0;
        const bool ok = hipExtGetLinkTypeAndHopCount(i, j, &type, &hops) == hipSuccess;
        int can = 0;
        (void)hipDeviceCanAccessPeer(&can, i, j);
        row.push_back(Json()
                          .kv("type", ok ? link_type_name(type) : std::string("unknown"))
                          .kv("hops", static_cast<int>(ok ? hops : 0))
                          .kv("p2p", can != 0)
                          .str());
      }
      rows.push_back(Json::array(row));
    }
  }
  const double ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  Json j;
  j.kv("ok", true)
      .kv("device_count", n)
      .kv("runtime_version", rt)
      .kv("driver_version", drv)
      .raw("devices", Json::array(devs));
  if (with_links) j.raw("links", Json::array(rows));
  j.kv("discovery_ms", ms);
  return j.str();
}

std::string hbm_write_probe(size_t bytes, int iters, StoreMode mode, int device, uint32_t value) {
  try {
    if (bytes % 16 || bytes == 0) return error_json("bytes must be a positive multiple of 16");
    iters = std::max(iters, 1);
    // Host-side costs of the first probe on a device (stream = a hardware queue, the arena
    // allocation, event creation, the first launch = code-object load): they, not the kernels,
    // dominate a cold validation run, so they are reported separately.
    const auto h0 = std::chrono::steady_clock::now();
    auto lap = [last = h0]() mutable {
      const auto now = std::chrono::steady_clock::now();
      const double ms = std::chrono::duration<double, std::milli>(now - last).count();
      last = now;
      return ms;
    };
    DeviceGuard g(device);
    CachedStream st(device);
    const double stream_ms = lap();
    char* base = scratch(device, align_up(bytes) + kAlign);
    void* buf = base;
    auto* bad = reinterpret_cast<unsigned long long*>(base + align_up(bytes));
    const double alloc_ms = lap();
    EventTimer cold, warm;
    const double events_ms = lap();
    cold.start(st.s);
    hbm_fill(buf, bytes, value ^ 0xFFFFFFFFu, mode, st.s);  // cold write (first touch)
    cold.stop(st.s);
    const double launch_ms = lap();
    const float cold_ms = cold.elapsed_ms();
    const double cold_wait_ms = lap();
    warm.start(st.s);
    for (int i = 0; i < iters; ++i) hbm_fill(buf, bytes, value, mode, st.s);
    warm.stop(st.s);
    const float ms = warm.elapsed_ms() / iters;
    TK8S_HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(unsigned long long), st.s));
    EventTimer rd;  // the verify pass is also the HBM read measurement (every word compared)
    rd.start(st.s);
    verify_fill(buf, bytes, value, bad, st.s);
    rd.stop(st.s);
    const float read_ms = rd.elapsed_ms();
    unsigned long long nbad = 0;
    TK8S_HIP_CHECK(hipMemcpyAsync(&nbad, bad, sizeof nbad, hipMemcpyDeviceToHost, st.s));
    wait_stream(st.s, "hbm probe");
    return Json()
        .kv("ok", nbad == 0)
        .kv("probe", "hbm_write")
        .kv("read_ms", static_cast<double>(read_ms))
        .kv("read_gbps", bytes / (read_ms * 1e-3) / 1e9)
        .kv("device", device)
        .kv("bytes", static_cast<uint64_t>(bytes))
        .kv("iters", iters)
        .kv("mode", mode == StoreMode::kNonTemporal ? "nontemporal" : "plain")
        .kv("cold_ms", static_cast<double>(cold_ms))
        .kv("ms", static_cast<double>(ms))
        .kv("seconds", ms * 1e-3)
        .kv("gbps", bytes / (ms * 1e-3) / 1e9)
        .kv("bad_words", static_cast<uint64_t>(nbad))
        .raw("host_ms", Json()
                            .kv("stream", stream_ms)
                            .kv("alloc", alloc_ms)
                            .kv("events", events_ms)
                            .kv("first_launch", launch_ms)
                            .kv("first_wait", cold_wait_ms)
                            .str())
        .str();
  } catch (const std::exception& ex) {
    return error_json(ex.what());
  }
}

std::string md5_probe(size_t bytes, uint32_t chunk_bytes, uint64_t seed, int iters, int device) {
  try {
    if (bytes % 16) return error_json("bytes must be a multiple of 16");
    if (chunk_bytes == 0 || chunk_bytes % 64) return error_json("chunk must be a multiple of 64");
    iters = std::max(iters, 1);
    DeviceGuard g(device);
    CachedStream st(device);
    const size_t ws = md5_tree_workspace(bytes, chunk_bytes);
    const size_t o_wa = align_up(std::max<size_t>(bytes, 16)), o_wb = o_wa + align_up(ws), o_out = o_wb + align_up(ws),
                 o_flush = o_out + kAlign;
    char* base = scratch(device, o_flush + kMallFlush);
    void *data = base, *wa = base + o_wa, *wb = base + o_wb, *out = base + o_out, *flush = base + o_flush;
    EventTimer fill_t, cold_t;
    fill_t.start(st.s);
    philox_fill(data, bytes, seed, st.s);
    fill_t.stop(st.s);
    const float fill_ms = fill_t.elapsed_ms();
    cold_t.start(st.s);
    md5_tree(data, bytes, chunk_bytes, wa, wb, out, st.s);
    cold_t.stop(st.s);
    const float cold_ms = cold_t.elapsed_ms();
    // each timed pass starts from HBM: 512 MiB written elsewhere first evicts the input from the
    // memory-side Infinity Cache (a 256 MiB input fits the 256 MB MALL)
    std::vector<std::unique_ptr<EventTimer>> warm;
    for (int i = 0; i < iters; ++i) {
      hbm_fill(flush, kMallFlush, 0x5A5A5A5Au + i, StoreMode::kPlain, st.s);
      warm.push_back(std::make_unique<EventTimer>());
      warm.back()->start(st.s);
      md5_tree(data, bytes, chunk_bytes, wa, wb, out, st.s);
      warm.back()->stop(st.s);
    }
    float total = 0.f;
    for (auto& w : warm) total += w->elapsed_ms();
    const float ms = total / iters;
    unsigned char digest[16];
    TK8S_HIP_CHECK(hipMemcpyAsync(digest, out, 16, hipMemcpyDeviceToHost, st.s));
    wait_stream(st.s, "md5 probe");
    return Json()
        .kv("ok", true)
        .kv("probe", "md5_tree")
        .kv("device", device)
        .kv("bytes", static_cast<uint64_t>(bytes))
        .kv("chunk_bytes", chunk_bytes)
        .kv("seed", static_cast<uint64_t>(seed))
        .kv("iters", iters)
        .kv("digest", hex(digest, 16))
        .kv("fill_ms", static_cast<double>(fill_ms))
        .kv("fill_gbps", bytes / (fill_ms * 1e-3) / 1e9)
        .kv("cold_ms", static_cast<double>(cold_ms))
        .kv("ms", static_cast<double>(ms))
        .kv("seconds", ms * 1e-3)
        .kv("mbps", bytes / (ms * 1e-3) / 1e6)
        .kv("mall_flushed", true)
        .str();
  } catch (const std::exception& ex) {
    return error_json(ex.what());
  }
}

std::string copy_probe(int src_device, int dst_device, size_t bytes, int iters, bool dma) {
  // a failed pull still names its link: xgmi.py counts it as a dead link between the two GPUs
  auto link_error = [&](const std::string& what) {
    return Json().kv("ok", false).kv("probe", src_device != dst_device ? "xgmi_peer_copy" : "local_copy")
        .kv("src_device", src_device).kv("dst_device", dst_device).kv("error", what).str();
  };
  try {
    if (bytes % 16 || bytes == 0) return error_json("bytes must be a positive multiple of 16");
    iters = std::max(iters, 1);
    // TK8S_PROBE_PEER_PATH=1: a copy within one GPU takes the peer path (its cached buffers, no
    // peer grant needed) -- how a one-GPU box exercises the code the xGMI pulls run
    const bool forced = std::getenv("TK8S_PROBE_PEER_PATH") != nullptr && src_device == dst_device;
    const bool peer = src_device != dst_device || forced;
    int can = 1;
    if (peer && !forced) {
      TK8S_HIP_CHECK(hipDeviceCanAccessPeer(&can, dst_device, src_device));
      if (!can) return link_error("no peer access from dst to src");
    }
    // Local: src, dst and the error counter are carved from this device's scratch arena.
    // Peer: the cached peer buffers (PeerSlot): the source filled once, the destination held.
    void *src = nullptr, *dst = nullptr;
    unsigned long long* bad = nullptr;
    std::unique_lock<std::mutex> dst_hold;
    if (!peer) {
      DeviceGuard g(src_device);
      char* base = scratch(src_device, 2 * align_up(bytes) + kAlign);
      src = base;
      dst = base + align_up(bytes);
      bad = reinterpret_cast<unsigned long long*>(base + 2 * align_up(bytes));
      const hipStream_t ss = probe_stream(src_device);
      hbm_fill(src, bytes, kPeerPattern, StoreMode::kPlain, ss);
      wait_stream(ss, "copy source fill");
    } else {
      PeerSlot& ps = peer_slot(g_peer_src, src_device);
      std::lock_guard<std::mutex> lock(ps.mu);
      src = peer_buffer(ps, src_device, align_up(bytes));
      if (!ps.filled) {
        DeviceGuard g(src_device);
        const hipStream_t ss = probe_stream(src_device);
        hbm_fill(src, ps.n, kPeerPattern, StoreMode::kPlain, ss);
        wait_stream(ss, "peer source fill");
        ps.filled = true;
      }
      PeerSlot& pd = peer_slot(g_peer_dst, dst_device);
      dst_hold = std::unique_lock<std::mutex>(pd.mu);
      char* base = static_cast<char*>(peer_buffer(pd, dst_device, align_up(bytes) + kAlign));
      dst = base;
      bad = reinterpret_cast<unsigned long long*>(base + align_up(bytes));
    }
    DeviceGuard g(dst_device);
    if (peer && !forced) {
      const hipError_t pe = hipDeviceEnablePeerAccess(src_device, 0);
      if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) TK8S_HIP_CHECK(pe);
      (void)hipGetLastError();
    }
    CachedStream st(dst_device);
    if (peer) {
      // TK8S_FAULTS probe.exit|crash@peers end the process here; probe.hang@peers stalls this
      // pull's queue, so the bounded waits below must give up and name the link (failfast.h)
      fault_point("probe", "peers", /*host_hang=*/false);
      if (fault_armed("probe", "hang", "peers")) gpu_stall(st.s, 2 * gpu_sync_timeout_s() + 5);
    }
    stream_copy(dst, src, bytes, st.s);  // warm-up
    EventTimer kt, dt;
    kt.start(st.s);
    for (int i = 0; i < iters; ++i) stream_copy(dst, src, bytes, st.s);
    kt.stop(st.s);
    const double bound = peer ? peer_sync_timeout_s() : gpu_sync_timeout_s();  // a link is not waited for
    const float kernel_ms = kt.elapsed_ms(bound) / iters;
    TK8S_HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(unsigned long long), st.s));
    verify_fill(dst, bytes, kPeerPattern, bad, st.s);
    unsigned long long nbad = 0;
    TK8S_HIP_CHECK(hipMemcpyAsync(&nbad, bad, sizeof nbad, hipMemcpyDeviceToHost, st.s));
    // The SDMA-engine path only for peers (where it is a separate xGMI data path worth
    // checking); locally it measured nothing the kernel copy does not, and bringing up the
    // copy engine cost ~10 ms of the validation's critical path.
    float dma_ms = 0.f;
    dma = dma && peer;
    if (dma) {
      dt.start(st.s);
      for (int i = 0; i < iters; ++i)
        TK8S_HIP_CHECK(hipMemcpyPeerAsync(dst, dst_device, src, src_device, bytes, st.s));
      dt.stop(st.s);
      dma_ms = dt.elapsed_ms(bound) / iters;
    }
    wait_stream(st.s, "copy probe", bound);
    Json j;
    j.kv("ok", nbad == 0)
        .kv("probe", peer ? "xgmi_peer_copy" : "local_copy")
        .kv("src_device", src_device)
        .kv("dst_device", dst_device)
        .kv("bytes", static_cast<uint64_t>(bytes))
        .kv("iters", iters)
        .kv("kernel_ms", static_cast<double>(kernel_ms))
        .kv("kernel_gbps", bytes / (kernel_ms * 1e-3) / 1e9);
    if (dma) j.kv("dma_ms", static_cast<double>(dma_ms)).kv("dma_gbps", bytes / (dma_ms * 1e-3) / 1e9);
    return j.kv("bad_words", static_cast<uint64_t>(nbad)).str();
  } catch (const std::exception& ex) {
    return link_error(ex.what());
  }
}

}  // namespace tk8s
