// tk8s-rccl: N3 RCCL all-reduce validator (RCCL-tests style sweep + exact result check).
//
// Single process, n GPUs:   tk8s-rccl --ngpus N
// One process per GPU:      tk8s-rccl --rank R --nranks N [--device D]
// One process per node:     tk8s-rccl --group-index I --devices D0,D1,.. --nranks N
//                             (ranks I*k .. I*k+k-1 for k devices; or --rank R --devices ..)
//                           ... (--uid-file PATH | --kv-url http://host:port/v1/kv/KEY)
//   The process holding rank 0 creates the RCCL unique id and publishes it (atomic file rename,
//   or HTTP PUT to the control-plane KV); the others wait for it (file poll, or HTTP long-poll).
// Sweep: --min-bytes B (8) --max-bytes B (1 GiB) --factor F (2) --iters K --warmup W
//        --dtype float32|bfloat16|both (default both: the RCCL-tests sweep of SURVEY.md N3)
// [--teardown]: free the communicators before exiting (default: print the result and _Exit)
// Prints one JSON object; exit 0 iff every size reduced exactly.
//
// Fail fast: --op-timeout S (default 20) bounds every wait --
// the unique id fetch, the communicator init, each sweep point, each check; a wait that runs
// out, or an RCCL async error, aborts the communicators and prints {"ok":false,"phase":..,
// "error":..} (exit 1). A watchdog thread ends the process (same JSON, "watchdog":true, exit 4)
// if a phase makes no progress for op-timeout + 10 s at all -- a call blocked inside RCCL.
// Fault points (TK8S_FAULTS): rccl.hang@uid|init (host stops), rccl.hang@sweep|check (the GPU
// queue stalls), rccl.exit@<phase> (exit 3), rccl.crash@<phase> (abort).
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include <atomic>

#include "args.h"
#include "httpkv.h"
#include "tk8s/common.h"
#include "tk8s/failfast.h"
#include "tk8s/rccl_bench.h"
#include "cachewalk.h"

namespace {

bool publish_uid(const tk8s::Args& a, const std::string& hex) {
  if (a.has("uid-file")) {
    const std::string path = a.str("uid-file"), tmp = path + ".tmp";
    {
      std::ofstream f(tmp);
      f << hex;
      if (!f) return false;
    }
    return std::rename(tmp.c_str(), path.c_str()) == 0;
  }
  tk8s::HttpResponse r;
  return tk8s::http_request("PUT", a.str("kv-url"), hex, &r) && r.status / 100 == 2;
}

bool fetch_uid(const tk8s::Args& a, std::string* hex, double timeout_s) {
  const auto deadline = std::chrono::steady_clock::now() +
                        std::chrono::milliseconds(static_cast<long long>(timeout_s * 1000));
  while (std::chrono::steady_clock::now() < deadline) {
    if (a.has("uid-file")) {
      std::ifstream f(a.str("uid-file"));
      if (f) {
        std::stringstream ss;
        ss << f.rdbuf();
        *hex = ss.str();
        if (hex->size() == 2 * NCCL_UNIQUE_ID_BYTES) return true;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    } else {
      tk8s::HttpResponse r;
      // Long-poll: the control plane holds the request until the key exists (or ~wait s), never
      // past the deadline
      const double left = std::chrono::duration<double>(deadline - std::chrono::steady_clock::now()).count();
      const int wait = static_cast<int>(std::max(1.0, std::min(10.0, left)));
      if (tk8s::http_request("GET", a.str("kv-url") + "?wait=" + std::to_string(wait), "", &r, wait + 5) &&
          r.status == 200) {
        *hex = r.body;
        while (!hex->empty() && (hex->back() == '\n' || hex->back() == '\r')) hex->pop_back();
        if (hex->size() == 2 * NCCL_UNIQUE_ID_BYTES) return true;
      } else {
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      }
    }
  }
  return false;
}

// "3,5,7" -> {3,5,7}; empty on any malformed entry.
std::vector<int> parse_devices(const std::string& s) {
  std::vector<int> out;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    char* end = nullptr;
    const long v = std::strtol(tok.c_str(), &end, 10);
    if (tok.empty() || *end != '\0' || v < 0) return {};
    out.push_back(static_cast<int>(v));
  }
  return out;
}

// TK8S_TRACE=1: "TRACE <unix s> rccl <what>" on stderr, merged into the bring-up's timeline by
// scripts/trace_bringup.py (the same format as utils/trace.py)
void trace(const char* what) {
  static const bool on = std::getenv("TK8S_TRACE") != nullptr;
  if (!on) return;
  const double t = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
  std::fprintf(stderr, "TRACE %.6f rccl %s\n", t, what);
}

// TK8S_FAULTS rccl.hang@sweep|check: the GPU-side hang (a stall kernel on the ranks' streams);
// exit / crash at those phases end the process when the validator enters them (on_phase).
std::string stall_phase() {
  for (const char* ph : {"sweep", "check"})
    if (tk8s::fault_armed("rccl", "hang", ph)) return ph;
  return "";
}

// RCCL's device code is one 108 MB code object (the host's unpacked copy, utils/rccl_unpack.py);
// HIP loads it onto a device the first time one of its kernels is referenced there -- inside
// the communicator start, ~160 ms of its ~205 ms on the MI355X (profiles/r5_thp/). Referencing
// a kernel of it right after the runtime's start, on a thread per device, lets that load overlap
// the unique id's creation (~26 ms) or its wait (the other ranks). A second thread per device
// makes the rank's stream meanwhile: the device's first queue, 15-85 ms measured between the
// code load and the communicator start (profiles/r6_rccl_prewarm/). TK8S_RCCL_PREWARM=0: off.
struct Prewarm {
  std::vector<std::thread> threads;
  std::chrono::steady_clock::time_point t0;
  bool started = false;
  std::map<int, hipStream_t> streams;  // each device's rank stream (filled by its own thread)
  std::mutex mu;
};

void prewarm_rccl_code(Prewarm& p, const std::vector<int>& devices) {
  const char* off = std::getenv("TK8S_RCCL_PREWARM");
  if (off != nullptr && std::string(off) == "0") return;
  const void* sym = nullptr;
  for (const char* name : {"_Z23ncclDevKernel_Generic_124ncclDevKernelArgsStorageILm4096EE",
                           "_Z23ncclDevKernel_Generic_224ncclDevKernelArgsStorageILm4096EE"}) {
    if ((sym = dlsym(RTLD_DEFAULT, name)) != nullptr) break;
  }
  if (sym == nullptr) return;  // another RCCL's names: its start loads the code as before
  p.t0 = std::chrono::steady_clock::now();
  p.started = true;
  for (int d : devices) {
    p.threads.emplace_back([d, sym] {  // the code load
      if (hipSetDevice(d) != hipSuccess) return;
      hipFuncAttributes attr;
      (void)hipFuncGetAttributes(&attr, sym);
    });
    p.threads.emplace_back([d, &p] {  // the rank's stream: the device's first queue (15-85 ms)
      hipStream_t s = nullptr;
      if (hipSetDevice(d) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return;
      std::lock_guard<std::mutex> g(p.mu);
      p.streams[d] = s;
    });
  }
}

// What the process is doing, for the watchdog's error line.
std::atomic<int> g_nranks{1}, g_first{0}, g_local{1};

}  // namespace

int main(int argc, char** argv) {
  trace("main");
  tk8s::cachewalk::configure();  // before the HIP runtime starts (cachewalk.h)
  try {
    tk8s::Args a(argc, argv);
    tk8s::AllReduceConfig cfg;
    cfg.min_bytes = static_cast<size_t>(a.num("min-bytes", 8));
    cfg.max_bytes = static_cast<size_t>(a.num("max-bytes", 1LL << 30));
    cfg.factor = static_cast<int>(a.num("factor", 2));
    cfg.iters = static_cast<int>(a.num("iters", 20));
    cfg.warmup = static_cast<int>(a.num("warmup", 5));
    const std::string dt = a.str("dtype", "both");
    if (dt == "float32") cfg.dtypes = {tk8s::DType::kF32};
    else if (dt == "bfloat16") cfg.dtypes = {tk8s::DType::kBF16};
    else if (dt == "both") cfg.dtypes = {tk8s::DType::kF32, tk8s::DType::kBF16};
    else {
      std::fprintf(stderr, "tk8s-rccl: --dtype must be float32, bfloat16 or both\n");
      return 2;
    }
    cfg.check = !a.has("no-check");
    cfg.op_timeout_s = std::strtod(a.str("op-timeout", "20").c_str(), nullptr);
    cfg.blocking = std::getenv("TK8S_RCCL_BLOCKING") && std::string(std::getenv("TK8S_RCCL_BLOCKING")) == "1";
    // the process exits right after its JSON line (see below) -- unless a profiler's library is
    // preloaded: its exit handlers write the trace, and _Exit would skip them
    const char* preload = std::getenv("LD_PRELOAD");
    cfg.teardown = a.has("teardown") || (preload && std::strstr(preload, "rocprof"));
    // The backstop: no progress in a phase for op-timeout + 10 s (a call blocked inside a library)
    // ends the process with the phase named.
    const double grace = 10.0;
    tk8s::Watchdog dog([](const std::string& phase, double waited) {
      std::printf("%s\n", tk8s::Json()
                              .kv("ok", false)
                              .kv("phase", phase)
                              .kv("error", "watchdog: no progress in phase " + phase + " for " +
                                               std::to_string(static_cast<int>(waited)) + " s")
                              .kv("timed_out", true)
                              .kv("watchdog", true)
                              .kv("nranks", g_nranks.load())
                              .kv("first_rank", g_first.load())
                              .kv("local_ranks", g_local.load())
                              .str()
                              .c_str());
      trace("watchdog");
    });
    const bool bounded = cfg.op_timeout_s > 0;
    cfg.on_phase = [&dog, bounded, grace](const std::string& phase, double s) {
      if (bounded) dog.arm(phase, s + grace);
      tk8s::fault_point("rccl", phase, /*host_hang=*/false);  // rccl.exit|crash@sweep|check
    };
    std::string out;
    if (a.has("rank") || a.has("group-index")) {
      const int nranks = static_cast<int>(a.num("nranks", 1));
      std::vector<int> devices = a.has("devices") ? parse_devices(a.str("devices"))
                                                  : std::vector<int>{static_cast<int>(a.num("device", 0))};
      if (devices.empty()) {
        std::fprintf(stderr, "tk8s-rccl: bad --devices '%s'\n", a.str("devices").c_str());
        return 2;
      }
      const int first = a.has("rank") ? static_cast<int>(a.num("rank", 0))
                                      : static_cast<int>(a.num("group-index", 0)) * static_cast<int>(devices.size());
      g_nranks = nranks;
      g_first = first;
      g_local = static_cast<int>(devices.size());
      tk8s::set_fault_ranks(first, static_cast<long>(devices.size()));  // ":<rank>"-targeted fault points
      if (!a.has("uid-file") && !a.has("kv-url")) {
        std::fprintf(stderr, "tk8s-rccl: --rank/--group-index needs --uid-file or --kv-url\n");
        return 2;
      }
      ncclUniqueId id;
      std::string hex;
      {
        int n = 0;  // the runtime's start, on its own (RCCL would start it inside ncclGetUniqueId)
        (void)hipGetDeviceCount(&n);
        trace("hip runtime up");
      }
      Prewarm warm;
      prewarm_rccl_code(warm, devices);
      // the uid exchange is bounded by the same budget as every other wait
      const double uid_timeout = std::strtod(a.str("uid-timeout", a.str("op-timeout", "20")).c_str(), nullptr);
      if (bounded) dog.arm("uid", uid_timeout + grace);
      tk8s::fault_point("rccl", "uid");
      if (first == 0) {
        trace("ncclGetUniqueId");
        if (ncclGetUniqueId(&id) != ncclSuccess) {
          std::printf("{\"ok\":false,\"phase\":\"uid\",\"error\":\"ncclGetUniqueId failed\"}\n");
          return 2;
        }
        hex = tk8s::nccl_unique_id_hex(id);
        if (!publish_uid(a, hex)) {
          std::printf("{\"ok\":false,\"phase\":\"uid\",\"error\":\"could not publish the unique id\"}\n");
          return 2;
        }
      } else {
        if (!fetch_uid(a, &hex, uid_timeout > 0 ? uid_timeout : 1e9) || !tk8s::nccl_unique_id_from_hex(hex, &id)) {
          std::printf("%s\n", tk8s::Json()
                                  .kv("ok", false)
                                  .kv("phase", "uid")
                                  .kv("error", "no unique id from rank 0 within " + a.str("uid-timeout", a.str("op-timeout", "20")) + " s")
                                  .kv("timed_out", true)
                                  .kv("nranks", nranks)
                                  .kv("first_rank", first)
                                  .str()
                                  .c_str());
          std::fflush(stdout);
          std::_Exit(1);
        }
      }
      trace(first == 0 ? "unique id published" : "unique id fetched");
      if (bounded) dog.arm("init", cfg.op_timeout_s + grace);  // (the code load below included)
      for (auto& th : warm.threads) th.join();
      const double prewarm_ms =
          warm.started ? std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - warm.t0).count() : -1;
      if (warm.started) trace("rccl code loaded");
      cfg.streams = warm.streams;
      tk8s::fault_point("rccl", "init");
      cfg.stall_phase = stall_phase();
      out = tk8s::allreduce_rank_group(first, nranks, devices, id, cfg);
      if (warm.started && !out.empty() && out.back() == '}') {  // how long the code load still took past the uid
        char buf[64];
        std::snprintf(buf, sizeof(buf), ",\"rccl_code_prewarm_ms\":%.3f}", prewarm_ms);
        out.pop_back();
        out += buf;
      }
      trace("sweep done");
    } else {
      int n = 0;
      if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        std::printf("{\"ok\":false,\"error\":\"no HIP device visible\"}\n");
        return 3;
      }
      const int want = static_cast<int>(a.num("ngpus", n));
      std::vector<int> devs;
      for (int i = 0; i < want && i < n; ++i) devs.push_back(i);
      g_nranks = static_cast<int>(devs.size());
      g_local = static_cast<int>(devs.size());
      tk8s::set_fault_ranks(0, static_cast<long>(devs.size()));
      if (bounded) dog.arm("init", cfg.op_timeout_s + grace);
      tk8s::fault_point("rccl", "init");
      cfg.stall_phase = stall_phase();
      out = tk8s::allreduce_single_process(devs, cfg);
    }
    dog.disarm();
    std::printf("%s\n", out.c_str());
    const bool ok = out.find("\"ok\":true") != std::string::npos;
    const int rc = ok ? 0 : 1;
    // the result is out: leave without the communicators' and runtime's teardown (always after a
    // failure: an aborted communicator has nothing left worth a clean exit)
    if (!cfg.teardown || !ok) {
      std::fflush(stdout);
      std::fflush(stderr);
      trace("exit");
      std::_Exit(rc);
    }
    return rc;
  } catch (const std::exception& e) {
    std::printf("%s\n", tk8s::Json().kv("ok", false).kv("phase", "setup").kv("error", e.what()).str().c_str());
    std::fprintf(stderr, "tk8s-rccl: %s\n", e.what());
    return 2;
  }
}
