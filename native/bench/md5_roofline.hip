// Development microbenchmark (not part of the product build): the fan-in-4 MD5 tree's pieces on
// gfx950, each event-timed on its own, back to back in ONE process.
//
//   hipcc -O3 --offload-arch=gfx950 -Inative/include -o build/md5_roofline native/bench/md5_roofline.hip
//   md5_roofline [MiB=256] [reps=20] [cold]   (cold: a 512 MiB fill before every timed launch)
//
// Includes md5_kernels.hip itself, so the kernels timed are the production ones (both fold block
// sizes are instantiated there). One JSON line per variant: median / best of `reps` launches,
// each bracketed by its own event pair; "empty" is a launch that does nothing (the floor).
#include "../src/md5_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                         \
    }                                                                                       \
  } while (0)

namespace tk8s {
// The r1-r6 leaf kernel: the same code without the empty asm that keeps the staging (and its
// wait for the next step's loads) after the compressions.
__global__ __launch_bounds__(kMd5Block) void md5_chunks_coalesced_unpinned(const unsigned char* __restrict__ src,
                                                                        unsigned chunk_bytes,
                                                                        unsigned long long ngroups,
                                                                        u32x4* __restrict__ digests) {
  __shared__ u32x4 tile[kMd5Block / 64][kWaveChunks * kRowVec];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long group = static_cast<unsigned long long>(blockIdx.x) * (kMd5Block / 64) + w;
  if (group >= ngroups) return;  // wave-uniform
  u32x4* my = tile[w];
  const unsigned char* gbase = src + group * kWaveChunks * chunk_bytes;
  const int sub = lane >> 3, piece = lane & 7;
  const unsigned steps = chunk_bytes / 128;
  u32x4 r[8];
  auto load = [&](unsigned step) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      r[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
          gbase + static_cast<size_t>(8 * i + sub) * chunk_bytes + step * 128u + piece * 16u));
  };
  auto stage = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) my[(8 * i + sub) * kRowVec + piece] = r[i];
  };
  unsigned st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  load(0);
  stage();
  for (unsigned step = 0; step < steps; ++step) {
    if (step + 1 < steps) load(step + 1);
    wave_sync_lds();
    u32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = my[lane * kRowVec + k];
    unsigned m[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      m[4 * q + 0] = v[q].x;
      m[4 * q + 1] = v[q].y;
      m[4 * q + 2] = v[q].z;
      m[4 * q + 3] = v[q].w;
    }
    md5_compress(st, m);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      m[4 * q + 0] = v[4 + q].x;
      m[4 * q + 1] = v[4 + q].y;
      m[4 * q + 2] = v[4 + q].z;
      m[4 * q + 3] = v[4 + q].w;
    }
    md5_compress(st, m);
    wave_sync_lds();
    if (step + 1 < steps) stage();
  }
  // RFC 1321 padding of a full chunk: 0x80, zeros, 64-bit bit length.
  unsigned m[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) m[q] = 0;
  m[0] = 0x80u;
  const unsigned long long bits = static_cast<unsigned long long>(chunk_bytes) * 8ull;
  m[14] = static_cast<unsigned>(bits);
  m[15] = static_cast<unsigned>(bits >> 32);
  md5_compress(st, m);
  digests[group * kWaveChunks + lane] = u32x4{st[0], st[1], st[2], st[3]};
}

}  // namespace tk8s

namespace tk8s {
// Leaf-kernel variants for the leaf-size question: kStep bytes of each of a wave's 64 chunks per
// step (128: the production kernel's shape; 64: a 5 KiB LDS tile per wave, so 8 waves per SIMD
// fit -- the grid has that many only with 512-byte leaves).
template <int kStep>
__global__ __launch_bounds__(256, kStep == 64 ? 8 : 4) void md5_leaves_step(const unsigned char* __restrict__ src,
                                                                           unsigned chunk_bytes,
                                                                           unsigned long long ngroups,
                                                                           u32x4* __restrict__ digests) {
  constexpr int kVec = kStep / 16, kRowV = kVec + 1, kPerInst = 64 / kVec;
  __shared__ u32x4 tile[4][64 * kRowV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long group = static_cast<unsigned long long>(blockIdx.x) * 4 + w;
  if (group >= ngroups) return;
  u32x4* my = tile[w];
  const unsigned char* gbase = src + group * 64ull * chunk_bytes;
  const int sub = lane / kVec, piece = lane % kVec;
  const unsigned steps = chunk_bytes / kStep;
  u32x4 r[kVec];
  auto load = [&](unsigned step) {
#pragma unroll
    for (int i = 0; i < kVec; ++i)
      r[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
          gbase + static_cast<size_t>(kPerInst * i + sub) * chunk_bytes + step * kStep + piece * 16u));
  };
  auto stage = [&]() {
#pragma unroll
    for (int i = 0; i < kVec; ++i) my[(kPerInst * i + sub) * kRowV + piece] = r[i];
  };
  unsigned st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  load(0);
  stage();
  for (unsigned step = 0; step < steps; ++step) {
    if (step + 1 < steps) load(step + 1);
    wave_sync_lds();
    u32x4 v[kVec];
#pragma unroll
    for (int k = 0; k < kVec; ++k) v[k] = my[lane * kRowV + k];
#pragma unroll
    for (int b = 0; b < kVec / 4; ++b) {
      unsigned m[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        m[4 * q + 0] = v[4 * b + q].x;
        m[4 * q + 1] = v[4 * b + q].y;
        m[4 * q + 2] = v[4 * b + q].z;
        m[4 * q + 3] = v[4 * b + q].w;
      }
      md5_compress(st, m);
    }
    asm volatile("" ::"v"(st[0]), "v"(st[1]), "v"(st[2]), "v"(st[3]) : "memory");
    wave_sync_lds();
    if (step + 1 < steps) stage();
  }
  unsigned m[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) m[q] = 0;
  m[0] = 0x80u;
  const unsigned long long bits = static_cast<unsigned long long>(chunk_bytes) * 8ull;
  m[14] = static_cast<unsigned>(bits);
  m[15] = static_cast<unsigned>(bits >> 32);
  md5_compress(st, m);
  digests[group * 64 + lane] = u32x4{st[0], st[1], st[2], st[3]};
}
}  // namespace tk8s

int main(int argc, char** argv) {
  using namespace tk8s;
  const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 256;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
  const bool cold = argc > 3 && std::string(argv[3]) == "cold";
  if (mib < 1 || mib > 4096 || reps < 1 || reps > 200) {
    std::fprintf(stderr, "MiB 1..4096, reps 1..200\n");
    return 2;
  }
  const size_t bytes = mib << 20;
  const unsigned chunk = 1024;
  const unsigned long long nleaves = bytes / chunk;
  unsigned char* src = nullptr;
  u32x4 *wa = nullptr, *wb = nullptr, *out = nullptr;
  CK(hipMalloc(&src, bytes));
  const size_t ws = (bytes / 512) * 16;  // the digests of the smallest leaves timed below (512 B)
  CK(hipMalloc(&wa, ws));
  CK(hipMalloc(&wb, ws));
  CK(hipMalloc(&out, 16));
  constexpr size_t kFlush = 512ull << 20;
  void* flush = nullptr;
  CK(hipMalloc(&flush, kFlush));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  philox_fill(src, bytes, 0, s);
  CK(hipStreamSynchronize(s));

  struct V {
    std::string name;
    std::function<void()> go;
  };
  std::vector<V> vs;
  vs.push_back({"leaves", [&] { md5_chunks(src, bytes, chunk, wa, s); }});
  const unsigned long long ngroups = nleaves / 64;
  vs.push_back({"leaves_unpinned", [&] {
                  hipLaunchKernelGGL(md5_chunks_coalesced_unpinned, dim3((ngroups + 3) / 4), dim3(256), 0, s, src, chunk,
                                     ngroups, wa);
                }});
  vs.push_back({"leaves_again", [&] { md5_chunks(src, bytes, chunk, wa, s); }});  // order control
  // the leaf-size question: 1 KiB vs 512-byte leaves, 128- vs 64-byte steps, and one lane per
  // chunk without LDS (the tail kernel), each over the same 256 MiB
  for (unsigned cb : {1024u, 512u}) {
    const unsigned long long ng = bytes / cb / 64;
    const std::string tag = std::to_string(cb);
    vs.push_back({"step128_c" + tag, [&, cb, ng] {
                    hipLaunchKernelGGL(md5_leaves_step<128>, dim3((ng + 3) / 4), dim3(256), 0, s, src, cb, ng, wa);
                  }});
    vs.push_back({"step64_c" + tag, [&, cb, ng] {
                    hipLaunchKernelGGL(md5_leaves_step<64>, dim3((ng + 3) / 4), dim3(256), 0, s, src, cb, ng, wa);
                  }});
    vs.push_back({"lane_c" + tag, [&, cb] {
                    const unsigned long long n = bytes / cb;
                    hipLaunchKernelGGL(md5_chunks_kernel, dim3((n + 255) / 256), dim3(256), 0, s, src,
                                       static_cast<unsigned long long>(bytes), cb, n, wa);
                  }});
  }
  for (unsigned long long n : {nleaves, nleaves / 1024, 4096ull, 256ull, 64ull, 4ull}) {
    if (n > nleaves) continue;
    const std::string tag = std::to_string(n);
    for (int levels = 1; levels <= 5; levels += 4) {
      vs.push_back({"fold256_L" + std::to_string(levels) + "_n" + tag, [&, n, levels] {
                      const unsigned g = static_cast<unsigned>(((n + 3) / 4 + 255) / 256);
                      hipLaunchKernelGGL(md5_fold_kernel<256>, dim3(g), dim3(256), 0, s, wa, n, levels, wb);
                    }});
    }
    vs.push_back({"fold64_L4_n" + tag, [&, n] {
                    const unsigned g = static_cast<unsigned>(((n + 3) / 4 + 63) / 64);
                    hipLaunchKernelGGL(md5_fold_kernel<64>, dim3(g), dim3(64), 0, s, wa, n, 4, wb);
                  }});
  }
  vs.push_back({"folds256_all", [&] { fold<256>(wa, nleaves, wa, wb, out, s); }});
  vs.push_back({"folds64_all", [&] { fold<64>(wa, nleaves, wa, wb, out, s); }});
  vs.push_back({"tree", [&] { md5_tree(src, bytes, chunk, wa, wb, out, s); }});
  vs.push_back({"empty", [&] { hipLaunchKernelGGL(md5_fold_kernel<64>, dim3(1), dim3(64), 0, s, wa, 1ull, 0, wb); }});

  std::vector<hipEvent_t> ev(2 * reps);
  for (auto& e : ev) CK(hipEventCreate(&e));
  for (const auto& v : vs) {
    v.go();  // warm-up
    CK(hipGetLastError());
    for (int i = 0; i < reps; ++i) {
      if (cold) hbm_fill(flush, kFlush, 0u, StoreMode::kPlain, s);  // evict the 256 MB MALL: the source comes from HBM
      CK(hipEventRecord(ev[2 * i], s));
      v.go();
      CK(hipEventRecord(ev[2 * i + 1], s));
    }
    CK(hipStreamSynchronize(s));
    std::vector<float> ms(reps);
    for (int i = 0; i < reps; ++i) CK(hipEventElapsedTime(&ms[i], ev[2 * i], ev[2 * i + 1]));
    std::sort(ms.begin(), ms.end());
    std::printf("{\"variant\": \"%s\", \"MiB\": %zu, \"cold\": %s, \"launches\": %d, \"median_us\": %.2f, \"best_us\": %.2f}\n",
                v.name.c_str(), mib, cold ? "true" : "false", reps, ms[reps / 2] * 1e3, ms[0] * 1e3);
    std::fflush(stdout);
  }
  unsigned char dig[16];
  CK(hipMemcpy(dig, out, 16, hipMemcpyDeviceToHost));
  std::printf("{\"digest\": \"");
  for (unsigned char b : dig) std::printf("%02x", b);
  std::printf("\"}\n");
  return 0;
}
