// N3 RCCL all-reduce sweep: algbw / busbw per message size plus an exact-result check (N6),
// with every wait bounded (rccl_bench.h "Fail fast").
//
// busbw = algbw * 2(n-1)/n is the per-GPU link traffic of a ring all-reduce; on MI355X each GPU
// has 7 point-to-point xGMI links (~153 GB/s each), so one ring is bound by one link and RCCL
// reaches higher aggregate busbw only by spreading channels over several links.
#include "tk8s/rccl_bench.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <thread>

#include "tk8s/common.h"

namespace tk8s {

namespace {

// TK8S_TRACE=1: the rank's phases as "TRACE <unix s> rccl <what>" on stderr, in the bring-up's
// merged timeline (tools/tk8s_rccl.cpp traces the steps around them; scripts/trace_bringup.py).
void trace(const char* what) {
  static const bool on = std::getenv("TK8S_TRACE") != nullptr;
  if (!on) return;
  const double t = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
  std::fprintf(stderr, "TRACE %.6f rccl %s\n", t, what);
}

// A failure of one phase of the validator: what ran out or broke, and where.
struct PhaseError : std::runtime_error {
  std::string phase;
  bool timed_out;
  PhaseError(std::string ph, const std::string& what, bool timeout)
      : std::runtime_error(what), phase(std::move(ph)), timed_out(timeout) {}
};

// The phase the validator is in (for errors thrown by the HIP / RCCL checks).
thread_local std::string t_phase = "setup";

#define TK8S_NCCL_CHECK(expr)                                                                      \
  do {                                                                                             \
    ncclResult_t _r = (expr);                                                                      \
    if (_r != ncclSuccess && _r != ncclInProgress)                                                 \
      throw PhaseError(t_phase, std::string(#expr) + " failed: " + ncclGetErrorString(_r), false); \
  } while (0)

size_t elem_size(DType t) { return t == DType::kF32 ? 4 : 2; }
ncclDataType_t nccl_type(DType t) { return t == DType::kF32 ? ncclFloat32 : ncclBfloat16; }
const char* dtype_name(DType t) { return t == DType::kF32 ? "float32" : "bfloat16"; }

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

double unix_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::system_clock::now().time_since_epoch()).count();
}

void enter(const AllReduceConfig& cfg, const std::string& phase) {
  t_phase = phase;
  if (cfg.on_phase) cfg.on_phase(phase, cfg.op_timeout_s);
}

// The first asynchronous RCCL error of the local communicators ("" if none; in-progress is not
// an error).
std::string comm_error(const std::vector<Rank>& ranks, bool* in_progress = nullptr) {
  if (in_progress) *in_progress = false;
  for (const auto& r : ranks) {
    if (!r.comm) continue;
    ncclResult_t st = ncclSuccess;
    const ncclResult_t q = ncclCommGetAsyncError(r.comm, &st);
    if (q != ncclSuccess) return std::string("ncclCommGetAsyncError: ") + ncclGetErrorString(q);
    if (st == ncclInProgress) {
      if (in_progress) *in_progress = true;
    } else if (st != ncclSuccess) {
      return "rank " + std::to_string(r.rank) + ": " + ncclGetErrorString(st);
    }
  }
  return "";
}

// Non-blocking communicators: wait until no local communicator has an operation in progress
// (the init, or an enqueue RCCL finished asynchronously), bounded.
void settle(const std::vector<Rank>& ranks, const AllReduceConfig& cfg) {
  if (cfg.blocking) return;
  std::string err;
  const std::string r = poll_until(
      [&] {
        bool busy = false;
        err = comm_error(ranks, &busy);
        return !err.empty() || !busy;
      },
      cfg.op_timeout_s > 0 ? cfg.op_timeout_s : 1e9);
  if (!err.empty()) throw PhaseError(t_phase, err, false);
  if (!r.empty()) throw PhaseError(t_phase, "communicator " + r, true);
}

// Every local stream drained, bounded, watching the communicators' async errors meanwhile.
void wait_ranks(const std::vector<Rank>& ranks, const AllReduceConfig& cfg) {
  hipError_t bad = hipSuccess;
  const std::string r = poll_until(
      [&] {
        for (const auto& k : ranks) {
          const hipError_t e = hipStreamQuery(k.stream);
          if (e == hipErrorNotReady) return false;
          if (e != hipSuccess) {
            bad = e;
            return true;
          }
        }
        return true;
      },
      cfg.op_timeout_s > 0 ? cfg.op_timeout_s : 1e9, [&] { return comm_error(ranks); });
  if (bad != hipSuccess) throw PhaseError(t_phase, std::string("stream: ") + hipGetErrorString(bad), false);
  if (!r.empty()) throw PhaseError(t_phase, r, r.rfind("timed out", 0) == 0);
}

struct Peaks {
  double alg = 0, bus = 0;
  bool ok = true;
};

// Runs the sweep on the given ranks (all driven by this process). `all_ranks` = communicator size.
// init_ms: the communicator set-up this process waited for; init_done: wall clock when it
// returned -- across ranks, the spread of init_done is how unevenly the ranks' runtimes came up
// (the fabric check's start-up cost at 8 processes per node).
std::string run_sweep(std::vector<Rank>& ranks, int all_ranks, const AllReduceConfig& cfg,
                      const char* mode, double init_ms, double init_done) {
  size_t maxb = 0;
  for (DType dt : cfg.dtypes) maxb = std::max(maxb, sweep_sizes(cfg, dt).back());
  const auto t_buf = std::chrono::steady_clock::now();
  enter(cfg, "sweep");
  for (auto& r : ranks) {
    TK8S_HIP_CHECK(hipSetDevice(r.device));
    r.send = std::make_unique<DeviceBuffer>(maxb);
    r.recv = std::make_unique<DeviceBuffer>(maxb);
    r.scratch = std::make_unique<DeviceBuffer>(64);
    r.timer = std::make_unique<EventTimer>();
  }
  wait_ranks(ranks, cfg);
  trace("buffers ready");
  const auto t_sweep = std::chrono::steady_clock::now();
  if (cfg.stall_phase == "sweep")
    for (auto& r : ranks) {
      TK8S_HIP_CHECK(hipSetDevice(r.device));
      gpu_stall(r.stream, 2 * cfg.op_timeout_s + 10);
    }
  std::vector<std::string> rows, per_dtype;
  Peaks all;
  for (DType dt : cfg.dtypes) {
    const size_t es = elem_size(dt);
    Peaks pk;
    for (auto& r : ranks) {
      TK8S_HIP_CHECK(hipSetDevice(r.device));
      ar_fill(r.send->get(), maxb / es, r.rank, dt, r.stream);
    }
    auto launch = [&](size_t count) {
      TK8S_NCCL_CHECK(ncclGroupStart());
      for (auto& r : ranks) {
        TK8S_HIP_CHECK(hipSetDevice(r.device));
        TK8S_NCCL_CHECK(ncclAllReduce(r.send->get(), r.recv->get(), count, nccl_type(dt), ncclSum, r.comm, r.stream));
      }
      const ncclResult_t g = ncclGroupEnd();
      if (g == ncclInProgress) settle(ranks, cfg);  // an enqueue RCCL completes asynchronously
      else TK8S_NCCL_CHECK(g);
    };
    for (size_t bytes : sweep_sizes(cfg, dt)) {
      const size_t count = bytes / es;
      enter(cfg, "sweep");
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
      wait_ranks(ranks, cfg);  // the collectives of this point, bounded (a dead peer ends here)
      double ms = 0.0;
      for (auto& r : ranks) ms = std::max(ms, static_cast<double>(r.timer->elapsed_ms()));
      const double t_s = ms * 1e-3 / std::max(cfg.iters, 1);
      float max_err = 0.f;
      unsigned long long bad = 0;
      if (cfg.check) {
        enter(cfg, "check");
        for (auto& r : ranks) {
          TK8S_HIP_CHECK(hipSetDevice(r.device));
          if (cfg.stall_phase == "check") gpu_stall(r.stream, 2 * cfg.op_timeout_s + 10);
          TK8S_HIP_CHECK(hipMemsetAsync(r.scratch->get(), 0, 64, r.stream));
          auto* base = static_cast<unsigned char*>(r.scratch->get());
          ar_check(r.recv->get(), count, all_ranks, dt, 0.0f, reinterpret_cast<unsigned*>(base),
                   reinterpret_cast<unsigned long long*>(base + 8), r.stream);
        }
        std::vector<std::array<unsigned char, 16>> host(ranks.size());
        for (size_t k = 0; k < ranks.size(); ++k) {
          TK8S_HIP_CHECK(hipSetDevice(ranks[k].device));
          TK8S_HIP_CHECK(hipMemcpyAsync(host[k].data(), ranks[k].scratch->get(), 16, hipMemcpyDeviceToHost,
                                        ranks[k].stream));
        }
        wait_ranks(ranks, cfg);
        for (const auto& h : host) {
          float e;
          unsigned long long b;
          std::memcpy(&e, h.data(), 4);
          std::memcpy(&b, h.data() + 8, 8);
          max_err = std::max(max_err, e);
          bad += b;
        }
      }
      const double algbw = bytes / t_s / 1e9;
      const double busbw = allreduce_busbw(algbw, all_ranks);
      pk.alg = std::max(pk.alg, algbw);
      pk.bus = std::max(pk.bus, busbw);
      pk.ok = pk.ok && bad == 0;
      rows.push_back(Json()
                         .kv("dtype", dtype_name(dt))
                         .kv("bytes", static_cast<uint64_t>(bytes))
                         .kv("count", static_cast<uint64_t>(count))
                         .kv("time_us", t_s * 1e6)
                         .kv("algbw_gbps", algbw)
                         .kv("busbw_gbps", busbw)
                         .kv("max_err", static_cast<double>(max_err))
                         .kv("bad", static_cast<uint64_t>(bad))
                         .str());
    }
    Json d;
    d.kv("ok", pk.ok).kv("points", static_cast<int>(sweep_sizes(cfg, dt).size())).kv("peak_algbw_gbps", pk.alg);
    if (all_ranks > 1) d.kv("peak_busbw_gbps", pk.bus);
    else d.raw("peak_busbw_gbps", "null");
    per_dtype.push_back(Json().raw(dtype_name(dt), d.str()).str());
    all.alg = std::max(all.alg, pk.alg);
    all.bus = std::max(all.bus, pk.bus);
    all.ok = all.ok && pk.ok;
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
  trace("sweep checked");
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  std::string dtypes;
  std::vector<std::string> dnames;
  for (DType dt : cfg.dtypes) {
    dtypes += (dtypes.empty() ? "" : ",") + std::string(dtype_name(dt));
    dnames.push_back(Json::escape(dtype_name(dt)));
  }
  // per-dtype summaries merged into one object: {"float32": {...}, "bfloat16": {...}}
  std::string merged = "{";
  for (size_t i = 0; i < per_dtype.size(); ++i)
    merged += (i ? "," : "") + per_dtype[i].substr(1, per_dtype[i].size() - 2);
  merged += "}";
  Json j;
  j.kv("ok", all.ok)
      .kv("mode", mode)
      .kv("nccl_algo", env_or("NCCL_ALGO"))
      .kv("nccl_proto", env_or("NCCL_PROTO"))
      .kv("nccl_min_nchannels", env_or("NCCL_MIN_NCHANNELS"))
      .kv("nccl_max_nchannels", env_or("NCCL_MAX_NCHANNELS"))
      .kv("xgmi_link_gbps", kXgmiLinkGBps)
      .kv("nranks", all_ranks)
      .kv("local_ranks", static_cast<int>(ranks.size()))
      .kv("first_rank", ranks.empty() ? 0 : ranks.front().rank)
      .kv("rccl_version", rccl_version())
      .kv("dtype", dtypes)
      .kv("iters", cfg.iters)
      .raw("sweep", Json()
                        .kv("min_bytes", static_cast<uint64_t>(cfg.min_bytes))
                        .kv("max_bytes", static_cast<uint64_t>(cfg.max_bytes))
                        .kv("factor", std::max(cfg.factor, 2))
                        .kv("warmup", cfg.warmup)
                        .kv("iters", cfg.iters)
                        .raw("dtypes", Json::array(dnames))
                        .str())
      .kv("peak_algbw_gbps", all.alg);
  if (all_ranks > 1) {
    j.kv("peak_busbw_gbps", all.bus).kv("peak_links_equivalent", all.bus / kXgmiLinkGBps);
  } else {
    // one rank: the "all-reduce" is a local copy -- no link carried a byte
    j.raw("peak_busbw_gbps", "null").raw("peak_links_equivalent", "null").kv("fabric", "1 GPU: no fabric");
  }
  return j.raw("per_dtype", merged)
      .kv("comm_init_ms", init_ms)
      .kv("init_done_unix_ms", init_done)
      .kv("op_timeout_s", cfg.op_timeout_s)
      .kv("nonblocking", !cfg.blocking)
      .kv("buffers_ms", ms(t_buf, t_sweep))  // allocation of the largest size (fills are in the sweep)
      .kv("sweep_ms", ms(t_sweep, t_end))     // every size: fill, warm-up, timed iterations, exact check
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

// After a failure: let any stalled queue go, abort every local communicator (its kernels give up
// on the peers) and keep the memory -- freeing it would synchronise with whatever still runs;
// the process exits right after. The aborts run on a helper thread given 2 s: aborting an init
// that still waits for an absent peer can block inside RCCL's bootstrap, and a failure report
// must never wait on that (measured on the MI355X: the dead-peer init case). Returns whether
// every abort returned in time.
bool abort_all(std::vector<Rank>& ranks) {
  gpu_stall_release();
  std::vector<ncclComm_t> comms;
  for (auto& r : ranks) {
    if (r.comm) comms.push_back(r.comm);
    r.comm = nullptr;
    (void)r.send.release();
    (void)r.recv.release();
    (void)r.scratch.release();
    (void)r.timer.release();
  }
  if (comms.empty()) return true;
  auto done = std::make_shared<std::atomic<bool>>(false);
  std::thread([comms, done] {
    for (ncclComm_t c : comms) (void)ncclCommAbort(c);
    *done = true;
  }).detach();
  return poll_until([&] { return done->load(); }, 2.0).empty();
}

std::string error_json(const std::string& phase, const std::string& what, bool timed_out, bool aborted,
                       int nranks, int first, int local, bool abort_returned = true) {
  return Json()
      .kv("ok", false)
      .kv("phase", phase)
      .kv("error", what)
      .kv("timed_out", timed_out)
      .kv("aborted", aborted)
      .kv("abort_returned", abort_returned)
      .kv("nranks", nranks)
      .kv("first_rank", first)
      .kv("local_ranks", local)
      .str();
}

std::string run_group(int first_rank, int nranks, const std::vector<int>& devices, const ncclUniqueId& id,
                      const AllReduceConfig& cfg, const char* mode) {
  std::vector<Rank> ranks(devices.size());
  const int local = static_cast<int>(devices.size());
  try {
    t_phase = "init";
    if (devices.empty()) return error_json("init", "no devices", false, false, nranks, first_rank, 0);
    if (first_rank < 0 || first_rank + local > nranks)
      return error_json("init",
                        "ranks " + std::to_string(first_rank) + ".." + std::to_string(first_rank + local - 1) +
                            " do not fit a communicator of " + std::to_string(nranks),
                        false, false, nranks, first_rank, local);
    for (size_t i = 0; i < devices.size(); ++i) {
      ranks[i].device = devices[i];
      ranks[i].rank = first_rank + static_cast<int>(i);
      TK8S_HIP_CHECK(hipSetDevice(devices[i]));
      const auto made = cfg.streams.find(devices[i]);
      if (made != cfg.streams.end() && made->second != nullptr) ranks[i].stream = made->second;
      else TK8S_HIP_CHECK(hipStreamCreateWithFlags(&ranks[i].stream, hipStreamNonBlocking));
    }
    trace("streams created");
    enter(cfg, "init");
    const auto t0 = std::chrono::steady_clock::now();
    // Several ranks of one communicator in one thread: the inits must be one group, or the first
    // would wait forever for its local peers. They run on a helper thread, waited for under the
    // deadline: even with the non-blocking config RCCL's bootstrap blocks the calling thread
    // until every rank has connected (measured on the MI355X: rank 0 of a 2-rank communicator
    // whose peer never came sat in ncclGroupEnd), so the init is bounded from outside; a thread
    // left behind that way holds only its own copy of the inputs, and the process exits next.
    struct Init {
      std::atomic<bool> done{false};
      std::string err;
      std::vector<ncclComm_t> comms;
    };
    auto st = std::make_shared<Init>();
    st->comms.assign(ranks.size(), nullptr);
    std::vector<std::pair<int, int>> who;  // (device, rank)
    for (const auto& r : ranks) who.emplace_back(r.device, r.rank);
    const bool blocking = cfg.blocking;
    std::thread([st, who, nranks, id, blocking] {
      ncclConfig_t conf = NCCL_CONFIG_INITIALIZER;
      conf.blocking = blocking ? 1 : 0;
      ncclResult_t r = ncclGroupStart();
      for (size_t i = 0; i < who.size() && (r == ncclSuccess || r == ncclInProgress); ++i) {
        if (hipSetDevice(who[i].first) != hipSuccess) {
          st->err = "hipSetDevice failed";
          break;
        }
        r = ncclCommInitRankConfig(&st->comms[i], nranks, id, who[i].second, &conf);
      }
      const ncclResult_t g = ncclGroupEnd();
      if (st->err.empty() && r != ncclSuccess && r != ncclInProgress)
        st->err = std::string("ncclCommInitRankConfig failed: ") + ncclGetErrorString(r);
      else if (st->err.empty() && g != ncclSuccess && g != ncclInProgress)
        st->err = std::string("ncclGroupEnd failed: ") + ncclGetErrorString(g);
      st->done = true;
    }).detach();
    const std::string w = poll_until([&] { return st->done.load(); }, cfg.op_timeout_s > 0 ? cfg.op_timeout_s : 1e9);
    if (!w.empty()) throw PhaseError("init", "communicator init " + w + " (a rank never joined)", true);
    if (!st->err.empty()) throw PhaseError("init", st->err, false);
    for (size_t i = 0; i < ranks.size(); ++i) ranks[i].comm = st->comms[i];
    settle(ranks, cfg);  // non-blocking: the inits may still be finishing
    trace("communicator ready");
    const double init_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::string out = run_sweep(ranks, nranks, cfg, mode, init_ms, unix_ms());
    if (cfg.teardown) release(ranks);
    return out;
  } catch (const PhaseError& ex) {
    const bool back = abort_all(ranks);
    return error_json(ex.phase, ex.what(), ex.timed_out, true, nranks, first_rank, local, back);
  } catch (const GpuTimeout& ex) {
    const bool back = abort_all(ranks);
    return error_json(t_phase, ex.what(), true, true, nranks, first_rank, local, back);
  } catch (const std::exception& ex) {
    const bool back = abort_all(ranks);
    return error_json(t_phase, ex.what(), false, true, nranks, first_rank, local, back);
  }
}

}  // namespace

double allreduce_busbw(double algbw_gbps, int nranks) {
  return nranks > 1 ? algbw_gbps * 2.0 * (nranks - 1) / nranks : 0.0;
}

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
  // All n ranks local: one fresh unique id and the n inits in one group -- what ncclCommInitAll
  // does, but with the non-blocking config, so even this init is bounded.
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess)
    return error_json("init", std::string("ncclGetUniqueId failed: ") + ncclGetErrorString(r), false, false,
                      static_cast<int>(devices.size()), 0, static_cast<int>(devices.size()));
  return run_group(0, static_cast<int>(devices.size()), devices, id, cfg, "single_process");
}

std::string allreduce_rank_group(int first_rank, int nranks, const std::vector<int>& devices,
                                 const ncclUniqueId& id, const AllReduceConfig& cfg) {
  return run_group(first_rank, nranks, devices, id, cfg, devices.size() > 1 ? "rank_group" : "multi_process");
}

std::string allreduce_rank(int rank, int nranks, int device, const ncclUniqueId& id,
                           const AllReduceConfig& cfg) {
  return allreduce_rank_group(rank, nranks, std::vector<int>{device}, id, cfg);
}

}  // namespace tk8s
