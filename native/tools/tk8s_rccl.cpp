// tk8s-rccl: N3 RCCL all-reduce validator (RCCL-tests style sweep + exact result check).
//
// Single process, n GPUs:   tk8s-rccl --ngpus N
// One process per GPU:      tk8s-rccl --rank R --nranks N [--device D]
// One process per node:     tk8s-rccl --group-index I --devices D0,D1,.. --nranks N
//                             (ranks I*k .. I*k+k-1 for k devices; or --rank R --devices ..)
//                           ... (--uid-file PATH | --kv-url http://host:port/v1/kv/KEY)
//   The process holding rank 0 creates the RCCL unique id and publishes it (atomic file rename,
//   or HTTP PUT to the control-plane KV); the others wait for it (file poll, or HTTP long-poll).
// Sweep: --min-bytes B --max-bytes B --factor F --iters K --warmup W --dtype float32|bfloat16
// [--teardown]: free the communicators before exiting (default: print the result and _Exit)
// Prints one JSON object; exit 0 iff every size reduced exactly.
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "args.h"
#include "httpkv.h"
#include "tk8s/common.h"
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

bool fetch_uid(const tk8s::Args& a, std::string* hex, int timeout_s) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
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
      // Long-poll: the control plane holds the request until the key exists (or ~wait s).
      if (tk8s::http_request("GET", a.str("kv-url") + "?wait=10", "", &r, 15) && r.status == 200) {
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

}  // namespace

int main(int argc, char** argv) {
  trace("main");
  tk8s::cachewalk::configure();  // before the HIP runtime starts (cachewalk.h)
  try {
    tk8s::Args a(argc, argv);
    tk8s::AllReduceConfig cfg;
    cfg.min_bytes = static_cast<size_t>(a.num("min-bytes", 8));
    cfg.max_bytes = static_cast<size_t>(a.num("max-bytes", 1LL << 28));
    cfg.factor = static_cast<int>(a.num("factor", 2));
    cfg.iters = static_cast<int>(a.num("iters", 20));
    cfg.warmup = static_cast<int>(a.num("warmup", 5));
    cfg.dtype = a.str("dtype", "float32") == "bfloat16" ? tk8s::DType::kBF16 : tk8s::DType::kF32;
    cfg.check = !a.has("no-check");
    // the process exits right after its JSON line (see below) -- unless a profiler's library is
    // preloaded: its exit handlers write the trace, and _Exit would skip them
    const char* preload = std::getenv("LD_PRELOAD");
    cfg.teardown = a.has("teardown") || (preload && std::strstr(preload, "rocprof"));
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
      if (first == 0) {
        trace("ncclGetUniqueId");
        if (ncclGetUniqueId(&id) != ncclSuccess) {
          std::fprintf(stderr, "tk8s-rccl: ncclGetUniqueId failed\n");
          return 2;
        }
        hex = tk8s::nccl_unique_id_hex(id);
        if (!publish_uid(a, hex)) {
          std::fprintf(stderr, "tk8s-rccl: could not publish unique id\n");
          return 2;
        }
      } else {
        if (!fetch_uid(a, &hex, static_cast<int>(a.num("uid-timeout", 120))) ||
            !tk8s::nccl_unique_id_from_hex(hex, &id)) {
          std::fprintf(stderr, "tk8s-rccl: timed out waiting for the unique id\n");
          return 2;
        }
      }
      trace(first == 0 ? "unique id published" : "unique id fetched");
      out = tk8s::allreduce_rank_group(first, nranks, devices, id, cfg);
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
      out = tk8s::allreduce_single_process(devs, cfg);
    }
    std::printf("%s\n", out.c_str());
    const int rc = out.find("\"ok\":true") != std::string::npos ? 0 : 1;
    if (!cfg.teardown) {  // the result is out: leave without the communicators' and runtime's teardown
      std::fflush(stdout);
      std::fflush(stderr);
      trace("exit");
      std::_Exit(rc);
    }
    return rc;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "tk8s-rccl: %s\n", e.what());
    return 2;
  }
}
