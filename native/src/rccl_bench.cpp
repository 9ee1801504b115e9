// N3 RCCL all-reduce sweep: algbw / busbw per message size plus an exact-result check (N6).
//
// busbw = algbw * 2(n-1)/n is the per-GPU link traffic of a ring all-reduce; on MI355X each GPU
// has 7 point-to-point xGMI links (~153 GB/s each), so one ring is bound by one link and RCCL
// reaches higher aggregate busbw only by spreading channels over several links.
#include "tk8s/rccl_bench.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>

#include "tk8s/common.h"

namespace tk8s {

namespace {

struct NcclError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define TK8S_NCCL_CHECK(expr)                                                            \
  do {                                                                                   \
    ncclResult_t _r = (expr);                                                            \
    if (_r != ncclSuccess)                                                               \
      throw NcclError(std::string(#expr) + " failed: " + ncclGetErrorString(_r));        \
  } while (0)

size_t elem_size(DType t) { return t == DType::kF32 ? 4 : 2; }
ncclDataType_t nccl_type(DType t) { return t == DType::kF32 ? ncclFloat32 : ncclBfloat16; }

struct Rank {
  int device = 0;
  int rank = 0;
  hipStream_t stream{};
  ncclComm_t comm{};
  std::unique_ptr<DeviceBuffer> send, recv, scratch;
  std::unique_ptr<EventTimer> timer;
};

std::vector<size_t> sweep_sizes(const AllReduceConfig& cfg, DType dtype) {
  std::vector<size_t> out;
  const size_t es = elem_size(dtype);
  size_t b = std::max(cfg.min_bytes, es);
  const int f = std::max(cfg.factor, 2);
  while (b <= cfg.max_bytes) {
    out.push_back(b / es * es);
    if (b > cfg.max_bytes / f) break;
    b *= f;
  }
  if (out.empty()) out.push_back(es);
  return out;
}

// Runs the sweep on the given ranks (all driven by this process). `all_ranks` = communicator size.
double unix_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::system_clock::now().time_since_epoch()).count();
}

// init_ms: the communicator set-up (ncclCommInitAll / ncclCommInitRank) this process waited for;
// init_done: wall clock when it returned -- across ranks, the spread of init_done is how unevenly
// the ranks' runtimes came up (the fabric check's start-up cost at 8 processes per node).
std::string run_sweep(std::vector<Rank>& ranks, int all_ranks, const AllReduceConfig& cfg,
                      const char* mode, double init_ms, double init_done) {
  const size_t es = elem_size(cfg.dtype);
  const auto sizes = sweep_sizes(cfg, cfg.dtype);
  const size_t maxb = sizes.back();
  const auto t_buf = std::chrono::steady_clock::now();
  for (auto& r : ranks) {
    TK8S_HIP_CHECK(hipSetDevice(r.device));
    r.send = std::make_unique<DeviceBuffer>(maxb);
    r.recv = std::make_unique<DeviceBuffer>(maxb);
    r.scratch = std::make_unique<DeviceBuffer>(64);
    r.timer = std::make_unique<EventTimer>();
    ar_fill(r.send->get(), maxb / es, r.rank, cfg.dtype, r.stream);
  }
  auto launch = [&](size_t count) {
    TK8S_NCCL_CHECK(ncclGroupStart());
    for (auto& r : ranks) {
      TK8S_HIP_CHECK(hipSetDevice(r.device));
      TK8S_NCCL_CHECK(ncclAllReduce(r.send->get(), r.recv->get(), count, nccl_type(cfg.dtype),
                                    ncclSum, r.comm, r.stream));
    }
    TK8S_NCCL_CHECK(ncclGroupEnd());
  };

  for (auto& r : ranks) TK8S_HIP_CHECK(hipStreamSynchronize(r.stream));
  const auto t_sweep = std::chrono::steady_clock::now();
  std::vector<std::string> rows;
  double peak_bus = 0.0;
  bool all_ok = true;
  for (size_t bytes : sizes) {
    const size_t count = bytes / es;
    for (int i = 0; i < cfg.warmup; ++i) launch(count);
    for (auto& r : ranks) {
      TK8S_HIP_CHECK(hipSetDevice(r.device));
      r.timer->start(r.stream);
    }
    for (int i = 0; i < cfg.iters; ++i) launch(count);
    for (auto& r : ranks) {
      TK8S_HIP_CHECK(hipSetDevice(r.device));
      r.timer->stop(r.stream);
    }
    double ms = 0.0;
    for (auto& r : ranks) ms = std::max(ms, static_cast<double>(r.timer->elapsed_ms()));
    const double t_s = ms * 1e-3 / std::max(cfg.iters, 1);
    float max_err = 0.f;
    unsigned long long bad = 0;
    if (cfg.check) {
      for (auto& r : ranks) {
        TK8S_HIP_CHECK(hipSetDevice(r.device));
        TK8S_HIP_CHECK(hipMemsetAsync(r.scratch->get(), 0, 64, r.stream));
        auto* base = static_cast<unsigned char*>(r.scratch->get());
        ar_check(r.recv->get(), count, all_ranks, cfg.dtype, 0.0f,
                 reinterpret_cast<unsigned*>(base), reinterpret_cast<unsigned long long*>(base + 8),
                 r.stream);
        unsigned char host[16];
        TK8S_HIP_CHECK(hipMemcpyAsync(host, base, 16, hipMemcpyDeviceToHost, r.stream));
        TK8S_HIP_CHECK(hipStreamSynchronize(r.stream));
        float e;
        unsigned long long b;
        std::memcpy(&e, host, 4);
        std::memcpy(&b, host + 8, 8);
        max_err = std::max(max_err, e);
        bad += b;
      }
    }
    const double algbw = bytes / t_s / 1e9;
    const double busbw = all_ranks > 1 ? algbw * 2.0 * (all_ranks - 1) / all_ranks : algbw;
    peak_bus = std::max(peak_bus, busbw);
    all_ok = all_ok && bad == 0;
    rows.push_back(Json()
                       .kv("bytes", static_cast<uint64_t>(bytes))
                       .kv("count", static_cast<uint64_t>(count))
                       .kv("time_us", t_s * 1e6)
                       .kv("algbw_gbps", algbw)
                       .kv("busbw_gbps", busbw)
                       .kv("max_err", static_cast<double>(max_err))
                       .kv("bad", static_cast<uint64_t>(bad))
                       .str());
  }
  // What shaped the collective: RCCL's algorithm / protocol / channel overrides (unset = RCCL's
  // own tuning), and the peak against one xGMI link, i.e. how many links' worth of traffic the
  // channels spread the ring over.
  auto env_or = [](const char* k) {
    const char* v = std::getenv(k);
    return std::string(v && *v ? v : "auto");
  };
  constexpr double kXgmiLinkGBps = 153.0;
  const auto t_end = std::chrono::steady_clock::now();
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  return Json()
      .kv("ok", all_ok)
      .kv("mode", mode)
      .kv("nccl_algo", env_or("NCCL_ALGO"))
      .kv("nccl_proto", env_or("NCCL_PROTO"))
      .kv("nccl_min_nchannels", env_or("NCCL_MIN_NCHANNELS"))
      .kv("nccl_max_nchannels", env_or("NCCL_MAX_NCHANNELS"))
      .kv("xgmi_link_gbps", kXgmiLinkGBps)
      .kv("peak_links_equivalent", all_ranks > 1 ? peak_bus / kXgmiLinkGBps : 0.0)
      .kv("nranks", all_ranks)
      .kv("local_ranks", static_cast<int>(ranks.size()))
      .kv("first_rank", ranks.empty() ? 0 : ranks.front().rank)
      .kv("rccl_version", rccl_version())
      .kv("dtype", cfg.dtype == DType::kF32 ? "float32" : "bfloat16")
      .kv("iters", cfg.iters)
      .kv("peak_busbw_gbps", peak_bus)
      .kv("comm_init_ms", init_ms)
      .kv("init_done_unix_ms", init_done)
      .kv("buffers_ms", ms(t_buf, t_sweep))  // allocation + pattern fill of the largest size
      .kv("sweep_ms", ms(t_sweep, t_end))     // every size: warm-up, timed iterations, exact check
      .raw("results", Json::array(rows))
      .str();
}

void release(std::vector<Rank>& ranks) {
  for (auto& r : ranks) {
    (void)hipSetDevice(r.device);
    r.send.reset();
    r.recv.reset();
    r.scratch.reset();
    r.timer.reset();
    if (r.comm) (void)ncclCommDestroy(r.comm);
    if (r.stream) (void)hipStreamDestroy(r.stream);
  }
}

std::string error_json(const std::string& what) {
  return Json().kv("ok", false).kv("error", what).str();
}

}  // namespace

int rccl_version() {
  int v = 0;
  (void)ncclGetVersion(&v);
  return v;
}

std::string nccl_unique_id_hex(const ncclUniqueId& id) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < NCCL_UNIQUE_ID_BYTES; ++i) {
    const auto b = static_cast<unsigned char>(id.internal[i]);
    s += d[b >> 4];
    s += d[b & 15];
  }
  return s;
}

bool nccl_unique_id_from_hex(const std::string& hex, ncclUniqueId* id) {
  if (hex.size() != 2 * NCCL_UNIQUE_ID_BYTES) return false;
  auto nib = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  };
  for (int i = 0; i < NCCL_UNIQUE_ID_BYTES; ++i) {
    const int h = nib(hex[2 * i]), l = nib(hex[2 * i + 1]);
    if (h < 0 || l < 0) return false;
    id->internal[i] = static_cast<char>((h << 4) | l);
  }
  return true;
}

std::string allreduce_single_process(const std::vector<int>& devices, const AllReduceConfig& cfg) {
  std::vector<Rank> ranks(devices.size());
  try {
    if (devices.empty()) return error_json("no devices");
    std::vector<ncclComm_t> comms(devices.size());
    const auto t0 = std::chrono::steady_clock::now();
    TK8S_NCCL_CHECK(ncclCommInitAll(comms.data(), static_cast<int>(devices.size()), devices.data()));
    const double init_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const double init_done = unix_ms();
    for (size_t i = 0; i < devices.size(); ++i) {
      ranks[i].device = devices[i];
      ranks[i].rank = static_cast<int>(i);
      ranks[i].comm = comms[i];
      TK8S_HIP_CHECK(hipSetDevice(devices[i]));
      TK8S_HIP_CHECK(hipStreamCreateWithFlags(&ranks[i].stream, hipStreamNonBlocking));
    }
    std::string out = run_sweep(ranks, static_cast<int>(devices.size()), cfg, "single_process", init_ms, init_done);
    if (cfg.teardown) release(ranks);
    return out;
  } catch (const std::exception& ex) {
    release(ranks);
    return error_json(ex.what());
  }
}

std::string allreduce_rank_group(int first_rank, int nranks, const std::vector<int>& devices,
                                 const ncclUniqueId& id, const AllReduceConfig& cfg) {
  std::vector<Rank> ranks(devices.size());
  try {
    if (devices.empty()) return error_json("no devices");
    if (first_rank < 0 || first_rank + static_cast<int>(devices.size()) > nranks)
      return error_json("ranks " + std::to_string(first_rank) + ".." +
                        std::to_string(first_rank + static_cast<int>(devices.size()) - 1) +
                        " do not fit a communicator of " + std::to_string(nranks));
    for (size_t i = 0; i < devices.size(); ++i) {
      ranks[i].device = devices[i];
      ranks[i].rank = first_rank + static_cast<int>(i);
      TK8S_HIP_CHECK(hipSetDevice(devices[i]));
      TK8S_HIP_CHECK(hipStreamCreateWithFlags(&ranks[i].stream, hipStreamNonBlocking));
    }
    const auto t0 = std::chrono::steady_clock::now();
    // Several ranks of one communicator in one thread: the inits must be one group, or the first
    // would wait forever for its local peers.
    TK8S_NCCL_CHECK(ncclGroupStart());
    for (auto& r : ranks) {
      TK8S_HIP_CHECK(hipSetDevice(r.device));
      TK8S_NCCL_CHECK(ncclCommInitRank(&r.comm, nranks, id, r.rank));
    }
    TK8S_NCCL_CHECK(ncclGroupEnd());
    const double init_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::string out = run_sweep(ranks, nranks, cfg, ranks.size() > 1 ? "rank_group" : "multi_process", init_ms,
                                unix_ms());
    if (cfg.teardown) release(ranks);
    return out;
  } catch (const std::exception& ex) {
    release(ranks);
    return error_json(ex.what());
  }
}

std::string allreduce_rank(int rank, int nranks, int device, const ncclUniqueId& id,
                           const AllReduceConfig& cfg) {
  return allreduce_rank_group(rank, nranks, std::vector<int>{device}, id, cfg);
}

}  // namespace tk8s
