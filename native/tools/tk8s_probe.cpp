// tk8s-probe: per-node GPU validation payload (the validation DaemonSet pod).
// Runs N4 (HBM write + verify), N5 (Philox + MD5 tree, checked against a known answer), N7
// (local copy, and xGMI peer pulls with --peers) and prints ONE JSON object.
//
//   tk8s-probe [--device D | --all-devices] [--gpuinfo] [--peers] [--hbm-bytes B]
//              [--md5-bytes B] [--chunk C] [--seed S] [--copy-bytes B] [--peer-bytes B] [--no-peer-dma]
//              [--iters K] [--mode plain|nontemporal] [--skip-md5]
//              [--out FILE] [--reuse FILE [--reuse-wait S]]
//
// --all-devices probes every visible GPU concurrently, one host thread per device (a node with
// k GPUs validates in the time of one). --peers then pulls --peer-bytes from every other GPU
// into each GPU over xGMI (each destination thread walks its sources in turn, so at most one
// transfer per destination is in flight). Exit 0 iff every probe passed.
//
// Pipelined validation (node bring-up): `--out FILE` is the early burn-in started while the
// control plane comes up; it writes the JSON atomically (FILE.tmp -> FILE) and removes the
// FILE.pending marker its launcher created. The validation pod then runs `--reuse FILE`: if FILE
// exists, or FILE.pending says a burn-in is still running (waited for up to --reuse-wait s,
// default 120), it prints that result instead of probing again; otherwise it probes itself.
//
// Known answer: with the default seed 0 and 1 KiB chunks, the MD5 tree of the first 256 MiB of
// the Philox stream is 6a21931a145024b03ee4405e01204ce2 (host oracle:
// tritonk8ssupervisor_amd/ops/reference.py md5_tree(philox_bytes(256 MiB, 0), 1024)); every
// device must reproduce it, and for other sizes every device must agree with device 0.
#include <signal.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "args.h"
#include "reuse.h"
#include "tk8s/common.h"
#include "tk8s/probes.h"
#include "cachewalk.h"

using tk8s::exists;
using tk8s::ok_of;
using tk8s::reuse;

namespace {

constexpr const char* kKnownDigest256M = "6a21931a145024b03ee4405e01204ce2";

std::string field(const std::string& j, const std::string& key) {
  const std::string pat = "\"" + key + "\":\"";
  const auto p = j.find(pat);
  if (p == std::string::npos) return "";
  const auto e = j.find('"', p + pat.size());
  return j.substr(p + pat.size(), e - p - pat.size());
}

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

struct DeviceResult {
  std::string hbm, md5, copy, digest;
  std::vector<std::string> peers;
  double wall_ms = 0, hbm_ms = 0, md5_ms = 0, copy_ms = 0, peers_ms = 0;  // host wall clock per phase
  bool ok = true;
  bool peers_ok = true;  // the links into this device: judged by xgmi.py, not part of `ok`
};

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
}

}  // namespace

int main(int argc, char** argv) {
  tk8s::cachewalk::configure();  // before the HIP runtime starts (cachewalk.h)
  const auto t0 = std::chrono::steady_clock::now();
  std::string out_file;
  try {
    tk8s::Args a(argc, argv);
    out_file = a.str("out", "");
    if (a.has("reuse")) {
      const int rc = reuse(a.str("reuse"), static_cast<double>(a.num("reuse-wait", 120)));
      if (rc >= 0) return rc;
    }
    const size_t hbm = static_cast<size_t>(a.num("hbm-bytes", 1LL << 30));
    const size_t md5 = a.has("skip-md5") ? 0 : static_cast<size_t>(a.num("md5-bytes", 256LL << 20));
    // 1 GiB each way: 8 x the 256 MB Infinity Cache, so the copy rate is an HBM rate
    const size_t copy = static_cast<size_t>(a.num("copy-bytes", 1LL << 30));
    const size_t peer_bytes = static_cast<size_t>(a.num("peer-bytes", 64LL << 20));
    const auto chunk = static_cast<uint32_t>(a.num("chunk", 1024));
    const auto seed = static_cast<uint64_t>(a.num("seed", 0));
    const int iters = static_cast<int>(a.num("iters", 5));
    const auto mode = a.str("mode", "plain") == "nontemporal" ? tk8s::StoreMode::kNonTemporal
                                                              : tk8s::StoreMode::kPlain;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
      emit("{\"ok\":false,\"error\":\"no HIP device visible\"}", out_file);
      return 3;
    }
    const double init_ms = ms_since(t0);
    std::vector<int> devices;
    if (a.has("all-devices")) {
      for (int d = 0; d < n; ++d) devices.push_back(d);
    } else {
      const int d = static_cast<int>(a.num("device", 0));
      if (d < 0 || d >= n) {
        emit("{\"ok\":false,\"error\":\"device " + std::to_string(d) + " out of range\"}", out_file);
        return 2;
      }
      devices.push_back(d);
    }
    std::string info;
    const auto tg = std::chrono::steady_clock::now();
    if (a.has("gpuinfo")) info = tk8s::gpuinfo_json(true);
    const double gpuinfo_ms = ms_since(tg);

    std::vector<DeviceResult> res(devices.size());
    auto run_one = [&](size_t k) {
      const auto td = std::chrono::steady_clock::now();
      DeviceResult& r = res[k];
      const int dev = devices[k];
      try {  // one allocation for every local probe (a regrow between them synchronises the device)
        tk8s::reserve_probe_scratch(dev, hbm, md5, chunk, copy);
      } catch (const std::exception&) {  // the probes grow it themselves, and report what fails
      }
      auto t = std::chrono::steady_clock::now();
      r.hbm = hbm ? tk8s::hbm_write_probe(hbm, iters, mode, dev) : std::string("{\"ok\":true,\"skipped\":true}");
      r.hbm_ms = ms_since(t);
      t = std::chrono::steady_clock::now();
      if (md5) {
        r.md5 = tk8s::md5_probe(md5, chunk, seed, iters, dev);
        r.digest = field(r.md5, "digest");
      }
      r.md5_ms = ms_since(t);
      t = std::chrono::steady_clock::now();
      if (copy) r.copy = tk8s::copy_probe(dev, dev, copy, iters);
      r.copy_ms = ms_since(t);
      r.ok = ok_of(r.hbm) && (r.md5.empty() || ok_of(r.md5)) && (r.copy.empty() || ok_of(r.copy));
      t = std::chrono::steady_clock::now();
      if (a.has("peers"))
        // Offset order: device k pulls from k+1, k+2, ... (mod m), so at any moment the devices
        // read from different sources over different links instead of all from device 0 first.
        // All of it inside the peer phase's bound (failfast.h peer_phase_timeout_s).
        for (size_t off = 1; off < devices.size(); ++off) {
          const int s = devices[(k + off) % devices.size()];
          if (ms_since(t) > tk8s::peer_phase_timeout_s() * 1000.0) {
            r.peers.push_back(tk8s::Json().kv("ok", false).kv("probe", "xgmi_peer_copy").kv("src_device", s)
                                  .kv("dst_device", dev).kv("error", "not run: the peer phase's deadline passed").str());
            r.peers_ok = false;
            continue;
          }
          // A failed pull is a link verdict (xgmi.link_report: dead link -> the nodes at both
          // ends NotReady), not a device one: the device keeps its own result, so every machine
          // still gets its share of the burn-in.
          r.peers.push_back(tk8s::copy_probe(s, dev, peer_bytes, iters, !a.has("no-peer-dma")));
          r.peers_ok = r.peers_ok && ok_of(r.peers.back());
        }
      r.peers_ms = ms_since(t);
      r.wall_ms = ms_since(td);
    };
    std::vector<std::thread> threads;
    for (size_t k = 1; k < devices.size(); ++k) threads.emplace_back(run_one, k);
    run_one(0);
    for (auto& t : threads) t.join();

    // MD5 known answer / cross-device agreement (a device that computes wrong bits fails).
    // Unpinned inputs: the majority digest is the reference, one device alone is "unpinned".
    std::string want;
    const bool pinned = md5 == (256u << 20) && chunk == 1024 && seed == 0;
    if (pinned) {
      want = kKnownDigest256M;
    } else if (md5) {
      size_t best = 0;
      for (size_t k = 0; k < res.size(); ++k) {
        size_t votes = 0;
        for (const auto& o : res) votes += (!o.digest.empty() && o.digest == res[k].digest);
        if (votes > best) best = votes, want = res[k].digest;
      }
    }
    const bool unpinned_single = md5 && !pinned && res.size() == 1;
    bool ok = true;
    std::vector<std::string> per_dev;
    for (size_t k = 0; k < res.size(); ++k) {
      DeviceResult& r = res[k];
      const bool digest_ok = !md5 || (!r.digest.empty() && r.digest == want);
      r.ok = r.ok && digest_ok;
      ok = ok && r.ok;
      tk8s::Json d;
      d.kv("device", devices[k]).kv("ok", r.ok).kv("wall_ms", r.wall_ms)
          .raw("phase_ms", tk8s::Json().kv("hbm", r.hbm_ms).kv("md5", r.md5_ms).kv("copy", r.copy_ms)
                               .kv("peers", r.peers_ms).str())
          .raw("hbm", r.hbm);
      if (md5) {
        d.raw("md5", r.md5);
        if (unpinned_single) d.kv("digest_ok", "unpinned");
        else d.kv("digest_ok", digest_ok);
      }
      if (copy) d.raw("copy", r.copy);
      if (!r.peers.empty()) d.raw("peers", tk8s::Json::array(r.peers)).kv("peers_ok", r.peers_ok);
      per_dev.push_back(d.str());
    }
    tk8s::Json out;
    out.kv("ok", ok).kv("runtime", "hip").kv("device", devices[0]).kv("device_count", n)
        .kv("probed", static_cast<int>(devices.size()));
    // Top-level copies of the first device's results (what the control plane annotates).
    out.raw("hbm", res[0].hbm);
    if (md5) out.raw("md5", res[0].md5).kv("md5_expected", want).kv("md5_pinned", pinned);
    if (copy) out.raw("copy", res[0].copy);
    out.raw("devices", tk8s::Json::array(per_dev));
    if (!info.empty()) out.raw("gpuinfo", info);
    out.raw("timings_ms", tk8s::Json().kv("hip_init", init_ms).kv("gpuinfo", gpuinfo_ms).kv("total", ms_since(t0))
                              .kv("cpu_cache_walk", tk8s::cachewalk::mode()).str());
    emit(out.str(), out_file);
    if (a.has("release-after")) {  // free the arena + streams before exit (experiment knob)
      const auto tr = std::chrono::steady_clock::now();
      tk8s::release_probe_scratch();
      std::fprintf(stderr, "{\"release_ms\": %.3f}\n", ms_since(tr));
    }
    return ok ? 0 : 1;
  } catch (const std::exception& e) {
    emit(std::string("{\"ok\":false,\"error\":\"") + e.what() + "\"}", out_file);
    std::fprintf(stderr, "tk8s-probe: %s\n", e.what());
    return 2;
  }
}
