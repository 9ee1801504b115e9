// Development microbenchmark (not part of the product build): the N5 Philox fill's launch shape
// on gfx950, A/B in ONE process against the production shape and the plain fill.
//
//   hipcc -O3 --offload-arch=gfx950 -o build/philox_roofline native/bench/philox_roofline.hip
//   philox_roofline [MiB=256] [reps=15] [rounds=3]
//
// Philox4x32-10 per 16 B is ~10 rounds of 2 mul_lo + 2 mul_hi + xors: ~23 us of VALU for 256 MiB
// on 256 CUs, against ~39 us of HBM writes at the fill's 6.9 TB/s -- it hides only with enough
// waves per SIMD. Every variant's output is compared word for word with the production shape's.
// One JSON line per (round, variant): median / best of `reps` event-timed launches.
//
// Variants: slab<U>xP (block-contiguous slabs, U stores in flight per lane, P blocks of 256 per
// CU; production: <4>x16) and gs<V>bBxK (grid-stride write front, K blocks of B per CU, V
// contiguous 16-B elements per lane per step).
#include <hip/hip_runtime.h>

#include <algorithm>
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

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 philox(unsigned long long idx, unsigned k0, unsigned k1) {
  unsigned c0 = static_cast<unsigned>(idx), c1 = static_cast<unsigned>(idx >> 32), c2 = 0, c3 = 0;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const unsigned lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const unsigned lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const unsigned n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  return u32x4{c0, c1, c2, c3};
}

template <int U>
__global__ __launch_bounds__(256) void px_slab(u32x4* __restrict__ dst, size_t n16, unsigned k0, unsigned k1) {
  constexpr int B = 256;
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const size_t lo = per * blockIdx.x;
  const size_t hi = lo + per < n16 ? lo + per : n16;
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * B < hi; i += U * B) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = philox(i + u * B, k0, k1);
#pragma unroll
    for (int u = 0; u < U; ++u) dst[i + u * B] = v[u];
  }
  for (; i < hi; i += B) dst[i] = philox(i, k0, k1);
}

template <int V>
__global__ void px_gs(u32x4* __restrict__ dst, size_t n16, unsigned k0, unsigned k1) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x * V;
  size_t i = (static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x) * V;
  for (; i + V <= n16; i += stride) {
    u32x4 v[V];
#pragma unroll
    for (int u = 0; u < V; ++u) v[u] = philox(i + u, k0, k1);
#pragma unroll
    for (int u = 0; u < V; ++u) dst[i + u] = v[u];
  }
  for (; i < n16; ++i) dst[i] = philox(i, k0, k1);
}

__global__ void diff(const u32x4* __restrict__ a, const u32x4* __restrict__ b, size_t n16, unsigned long long* bad) {
  unsigned long long mine = 0;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n16;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const u32x4 x = a[i], y = b[i];
    mine += (x.x != y.x) + (x.y != y.y) + (x.z != y.z) + (x.w != y.w);
  }
  if (mine) atomicAdd(bad, mine);
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 256;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 15;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 3;
  if (mib == 0 || mib > 8192 || reps < 1 || reps > 100 || rounds < 1 || rounds > 10) {
    std::fprintf(stderr, "MiB 1..8192, reps 1..100, rounds 1..10\n");
    return 2;
  }
  const size_t bytes = mib << 20, n16 = bytes / 16;
  const unsigned k0 = 11u, k1 = 0u;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  u32x4 *ref = nullptr, *dst = nullptr;
  unsigned long long* bad = nullptr;
  CK(hipMalloc(&ref, bytes));
  CK(hipMalloc(&dst, bytes));
  CK(hipMalloc(&bad, 8));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(px_slab<4>, dim3(cus * 16), dim3(256), 0, s, ref, n16, k0, k1);  // the production shape
  CK(hipGetLastError());

  struct Variant {
    std::string name;
    unsigned grid, block;
    std::function<void()> launch;
  };
  std::vector<Variant> vs;
#define SLAB(U, P)                                                                                      \
  vs.push_back({"slab<" #U ">x" #P, static_cast<unsigned>(cus * P), 256u, [&, g = cus * P] {            \
                  hipLaunchKernelGGL((px_slab<U>), dim3(g), dim3(256), 0, s, dst, n16, k0, k1);          \
                }});
  SLAB(4, 16)  // production
  SLAB(2, 16)
  SLAB(8, 16)
  SLAB(4, 8)
  SLAB(4, 32)
  SLAB(2, 32)
  SLAB(1, 32)
#define GS(V, B, K)                                                                                             \
  vs.push_back({"gs<" #V ">b" #B "x" #K, static_cast<unsigned>(cus * K), static_cast<unsigned>(B),             \
                [&, g = cus * K] { hipLaunchKernelGGL((px_gs<V>), dim3(g), dim3(B), 0, s, dst, n16, k0, k1); }});
  GS(1, 256, 4)
  GS(1, 256, 8)
  GS(2, 256, 4)
  GS(2, 256, 8)
  GS(1, 512, 4)
  GS(2, 128, 1)  // the fill's own shape

  std::vector<hipEvent_t> ev(2 * reps);
  for (auto& e : ev) CK(hipEventCreate(&e));
  for (int r = 0; r < rounds; ++r) {
    for (const auto& v : vs) {
      CK(hipMemsetAsync(dst, 0, bytes, s));
      v.launch();  // warm-up (untimed)
      CK(hipGetLastError());
      for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(ev[2 * i], s));
        v.launch();
        CK(hipEventRecord(ev[2 * i + 1], s));
      }
      CK(hipGetLastError());
      CK(hipMemsetAsync(bad, 0, 8, s));
      hipLaunchKernelGGL(diff, dim3(cus * 8), dim3(256), 0, s, dst, ref, n16, bad);
      CK(hipStreamSynchronize(s));
      std::vector<float> ms(reps);
      for (int i = 0; i < reps; ++i) CK(hipEventElapsedTime(&ms[i], ev[2 * i], ev[2 * i + 1]));
      std::sort(ms.begin(), ms.end());
      unsigned long long nbad = 0;
      CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
      const double med = ms[reps / 2] * 1e-3, best = ms[0] * 1e-3;
      std::printf("{\"round\": %d, \"variant\": \"%s\", \"grid\": %u, \"block\": %u, \"launches\": %d, "
                  "\"median_us\": %.2f, \"best_us\": %.2f, \"median_tbps\": %.4f, \"bad_words\": %llu}\n",
                  r, v.name.c_str(), v.grid, v.block, reps, med * 1e6, best * 1e6, bytes / med / 1e12, nbad);
      std::fflush(stdout);
    }
  }
  return 0;
}
