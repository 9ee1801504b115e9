// tk8s-probe: per-node GPU validation payload (the validation DaemonSet pod).
// Runs N4 (HBM write), N5 (Philox + MD5 tree), N7 (local copy, and xGMI peer pulls with
// --peers) on the visible device(s) and prints one JSON object.
//   tk8s-probe [--device D] [--hbm-bytes B] [--md5-bytes B] [--chunk C] [--seed S]
//              [--iters K] [--mode nontemporal|plain] [--copy-bytes B] [--peers] [--skip-md5]
#include <cstdio>
#include <string>
#include <vector>

#include "args.h"
#include "tk8s/common.h"
#include "tk8s/probes.h"

int main(int argc, char** argv) {
  try {
    tk8s::Args a(argc, argv);
    const int device = static_cast<int>(a.num("device", 0));
    const size_t hbm = static_cast<size_t>(a.num("hbm-bytes", 1LL << 30));
    const size_t md5 = static_cast<size_t>(a.num("md5-bytes", 256LL << 20));
    const size_t copy = static_cast<size_t>(a.num("copy-bytes", 256LL << 20));
    const auto chunk = static_cast<uint32_t>(a.num("chunk", 1024));
    const auto seed = static_cast<uint64_t>(a.num("seed", 0));
    const int iters = static_cast<int>(a.num("iters", 5));
    const auto mode = a.str("mode", "nontemporal") == "plain" ? tk8s::StoreMode::kPlain
                                                             : tk8s::StoreMode::kNonTemporal;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
      std::printf("{\"ok\":false,\"error\":\"no HIP device visible\"}\n");
      return 3;
    }
    tk8s::Json out;
    bool ok = true;
    auto add = [&](const char* key, const std::string& j) {
      ok = ok && j.find("\"ok\":true") != std::string::npos;
      out.raw(key, j);
    };
    add("hbm", hbm ? tk8s::hbm_write_probe(hbm, iters, mode, device)
                   : std::string("{\"ok\":true,\"skipped\":true}"));
    if (!a.has("skip-md5") && md5)
      add("md5", tk8s::md5_probe(md5, chunk, seed, iters, device));
    if (copy) add("copy", tk8s::copy_probe(device, device, copy, iters));
    if (a.has("peers")) {
      std::vector<std::string> peers;
      for (int s = 0; s < n; ++s) {
        if (s == device) continue;
        const std::string j = tk8s::copy_probe(s, device, copy ? copy : (64 << 20), iters);
        ok = ok && j.find("\"ok\":true") != std::string::npos;
        peers.push_back(j);
      }
      out.raw("peers", tk8s::Json::array(peers));
    }
    out.kv("ok", ok).kv("device", device).kv("device_count", n);
    std::printf("%s\n", out.str().c_str());
    return ok ? 0 : 1;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "tk8s-probe: %s\n", e.what());
    return 2;
  }
}
