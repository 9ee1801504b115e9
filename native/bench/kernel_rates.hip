// Development driver (not part of the product build) for per-size kernel profiles: runs ONE of
// the production launchers of libtk8s (or a runtime control) at ONE size, `reps` times, so a
// rocprofv3 --kernel-trace --stats run over it yields that kernel's rate at that size alone --
// no warm-up or other sizes averaged in.
//
//   hipcc -O3 --offload-arch=gfx950 -Inative/include -o build/kernel_rates native/bench/kernel_rates.hip \
//         -Ltritonk8ssupervisor_amd/lib -ltk8s -Wl,-rpath,$PWD/tritonk8ssupervisor_amd/lib
//   kernel_rates <fill|fill_nt|verify|copy|md5|philox|memcpy|memset> <bytes> [reps=20]
//
// Kinds: fill / fill_nt = hbm_fill plain / non-temporal; verify = verify_fill over a filled
// buffer; copy = stream_copy (src and dst of <bytes> each); md5 = md5_tree over <bytes> of Philox
// data with a 512 MiB MALL flush before each pass; philox = philox_fill; memcpy = hipMemcpyAsync
// device-to-device (the runtime's copy kernel: the FETCH_SIZE control); memset = hipMemsetD32Async.
// The untimed first launch of each kind is a smaller (1 MiB) one, so a profile's per-size rows
// can be told apart by grid or by count. Prints one JSON line with the event-timed median.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "tk8s/kernels.h"

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                         \
    }                                                                                       \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: kernel_rates <kind> <bytes> [reps]\n");
    return 2;
  }
  const std::string kind = argv[1];
  const size_t bytes = std::strtoull(argv[2], nullptr, 10);
  const int reps = argc > 3 ? std::atoi(argv[3]) : 20;
  if (bytes == 0 || bytes % 16 || reps < 1 || reps > 200) {
    std::fprintf(stderr, "bytes must be a positive multiple of 16, reps 1..200\n");
    return 2;
  }
  constexpr size_t kFlush = size_t(512) << 20;
  const size_t ws = tk8s::md5_tree_workspace(bytes, 1024);
  const size_t need = kind == "copy" || kind == "memcpy" ? 2 * bytes
                      : kind == "md5"                     ? bytes + 2 * ws + 4096 + kFlush
                                                          : bytes;
  char* base = nullptr;
  unsigned long long* bad = nullptr;
  CK(hipMalloc(&base, need));
  CK(hipMalloc(&bad, 64));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  char* src = base;
  char* dst = base + bytes;
  char* wa = base + bytes;
  char* wb = wa + ws;
  char* out = wb + ws;
  char* flush = out + 4096;
  auto run = [&](size_t n, int i) {
    if (kind == "fill") tk8s::hbm_fill(src, n, 7u + i, tk8s::StoreMode::kPlain, s);
    else if (kind == "fill_nt") tk8s::hbm_fill(src, n, 7u + i, tk8s::StoreMode::kNonTemporal, s);
    else if (kind == "verify") tk8s::verify_fill(src, n, 7u, bad, s);
    else if (kind == "copy") tk8s::stream_copy(dst, src, n, s);
    else if (kind == "philox") tk8s::philox_fill(src, n, 11 + i, s);
    else if (kind == "memcpy") CK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, s));
    else if (kind == "memset") CK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(src), 7u + i, n / 4, s));
    else if (kind == "md5") tk8s::md5_tree(src, n, 1024, wa, wb, out, s);
    else {
      std::fprintf(stderr, "unknown kind %s\n", kind.c_str());
      std::exit(2);
    }
  };
  // inputs
  if (kind == "verify" || kind == "copy" || kind == "memcpy") tk8s::hbm_fill(src, bytes, 7u, tk8s::StoreMode::kPlain, s);
  if (kind == "md5") tk8s::philox_fill(src, bytes, 0, s);
  CK(hipMemsetAsync(bad, 0, 64, s));
  run(std::min<size_t>(bytes, 1 << 20), 0);  // warm-up, a different size
  CK(hipStreamSynchronize(s));
  std::vector<hipEvent_t> ev(2 * reps);
  for (auto& e : ev) CK(hipEventCreate(&e));
  for (int i = 0; i < reps; ++i) {
    if (kind == "md5") tk8s::hbm_fill(flush, kFlush, 0x5A5A5A5Au + i, tk8s::StoreMode::kPlain, s);
    CK(hipEventRecord(ev[2 * i], s));
    run(bytes, i);
    CK(hipEventRecord(ev[2 * i + 1], s));
  }
  CK(hipStreamSynchronize(s));
  std::vector<float> ms(reps);
  for (int i = 0; i < reps; ++i) CK(hipEventElapsedTime(&ms[i], ev[2 * i], ev[2 * i + 1]));
  std::sort(ms.begin(), ms.end());
  unsigned long long nbad = 0;
  CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
  const double moved = (kind == "copy" || kind == "memcpy") ? 2.0 * bytes : static_cast<double>(bytes);
  std::printf("{\"kind\":\"%s\",\"bytes\":%zu,\"reps\":%d,\"median_us\":%.2f,\"best_us\":%.2f,\"worst_us\":%.2f,"
              "\"median_gbps\":%.1f,\"bytes_moved_per_rep\":%.0f,\"verify_bad\":%llu}\n",
              kind.c_str(), bytes, reps, ms[reps / 2] * 1e3, ms[0] * 1e3, ms[reps - 1] * 1e3,
              moved / (ms[reps / 2] * 1e-3) / 1e9, moved, nbad);
  return 0;
}
