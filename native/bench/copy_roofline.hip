// Development microbenchmark (not part of the product build): the N7 copy against the HBM3E
// roofline on gfx950, A/B against the runtime's own device-to-device copy in ONE process.
//
//   hipcc -O3 --offload-arch=gfx950 -o build/copy_roofline native/bench/copy_roofline.hip
//   copy_roofline [MiB=1024] [reps=15] [rounds=3]
//
// Source and destination are MiB each (2x MiB working set: 8x the 256 MB MALL at the default).
// The source holds a position-dependent pattern; after each variant the destination is checked
// word by word (`bad_words`) and cleared (outside the timed launches). Each launch is timed by its
// own pair of events; one JSON line per (round, variant) with the median and best launch; every
// round re-runs every variant in the same order. Rates count read + write bytes.
//
// Variants:
//  * memcpy: hipMemcpyAsync D2D (the runtime's copy kernel) -- the control.
//  * slab<U,L,S>xP: block b owns a contiguous slab, U 16-B loads in flight per lane then U stores,
//    P blocks of 256 per CU; L/S = 1: non-temporal loads / stores (production: <4,1,1>x32).
//  * gs<V,L,S>bBxK: grid-stride write front (the r6 fill's shape): K blocks of B per CU, each
//    lane V contiguous 16-B elements per step, the whole grid covering one contiguous span.
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

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int U, bool L, bool S>
__global__ __launch_bounds__(256) void copy_slab(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n16) {
  constexpr int B = 256;
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const size_t lo = per * blockIdx.x;
  const size_t hi = lo + per < n16 ? lo + per : n16;
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * B < hi; i += U * B) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<L>(src + i + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u) st<S>(dst + i + u * B, v[u]);
  }
  for (; i < hi; i += B) st<S>(dst + i, ld<L>(src + i));
}

template <int V, bool L, bool S>
__global__ void copy_gs(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n16) {
  const size_t lanes = static_cast<size_t>(gridDim.x) * blockDim.x;
  const size_t stride = lanes * V;
  size_t i = (static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x) * V;
  for (; i + V <= n16; i += stride) {
    u32x4 v[V];
#pragma unroll
    for (int u = 0; u < V; ++u) v[u] = ld<L>(src + i + u);
#pragma unroll
    for (int u = 0; u < V; ++u) st<S>(dst + i + u, v[u]);
  }
  for (; i < n16; ++i) st<S>(dst + i, ld<L>(src + i));
}

__global__ void pattern(u32x4* __restrict__ p, size_t n16) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n16;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const unsigned x = static_cast<unsigned>(i) * 2654435761u;
    p[i] = u32x4{x, x ^ 0x9E3779B9u, x + 7u, ~x};
  }
}

__global__ void check(const u32x4* __restrict__ p, size_t n16, unsigned long long* bad) {
  unsigned long long mine = 0;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n16;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const unsigned x = static_cast<unsigned>(i) * 2654435761u;
    const u32x4 v = p[i];
    mine += (v.x != x) + (v.y != (x ^ 0x9E3779B9u)) + (v.z != x + 7u) + (v.w != ~x);
  }
  if (mine) atomicAdd(bad, mine);
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 15;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 3;
  if (mib == 0 || mib > 16384 || reps < 1 || reps > 100 || rounds < 1 || rounds > 10) {
    std::fprintf(stderr, "MiB 1..16384, reps 1..100, rounds 1..10\n");
    return 2;
  }
  const size_t bytes = mib << 20, n16 = bytes / 16;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  u32x4 *src = nullptr, *dst = nullptr;
  unsigned long long* bad = nullptr;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&dst, bytes));
  CK(hipMalloc(&bad, 8));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(pattern, dim3(cus * 8), dim3(256), 0, s, src, n16);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(s));

  struct Variant {
    std::string name;
    unsigned grid, block;
    std::function<void()> launch;
  };
  std::vector<Variant> vs;
  vs.push_back({"memcpy", 0, 0, [&] { CK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s)); }});
#define SLAB(U, L, S, P)                                                                                 \
  vs.push_back({"slab<" #U "," #L "," #S ">x" #P, static_cast<unsigned>(cus * P), 256u, [&, g = cus * P] { \
                  hipLaunchKernelGGL((copy_slab<U, L, S>), dim3(g), dim3(256), 0, s, dst, src, n16);     \
                }});
  SLAB(4, 1, 1, 32)  // production
  SLAB(4, 0, 0, 32)
  SLAB(4, 1, 0, 32)
  SLAB(4, 0, 1, 32)
  SLAB(2, 1, 1, 32)
  SLAB(8, 1, 1, 16)
  SLAB(4, 1, 1, 16)
  SLAB(4, 1, 1, 64)
#define GS(V, L, S, B, K)                                                                                      \
  vs.push_back({"gs<" #V "," #L "," #S ">b" #B "x" #K, static_cast<unsigned>(cus * K), static_cast<unsigned>(B), \
                [&, g = cus * K] { hipLaunchKernelGGL((copy_gs<V, L, S>), dim3(g), dim3(B), 0, s, dst, src, n16); }});
  GS(2, 0, 0, 128, 1)
  GS(2, 1, 1, 128, 1)
  GS(4, 0, 0, 128, 1)
  GS(4, 1, 1, 128, 1)
  GS(2, 0, 0, 256, 1)
  GS(2, 1, 1, 256, 1)
  GS(2, 0, 0, 128, 2)
  GS(2, 1, 1, 128, 2)
  GS(2, 1, 1, 256, 2)
  GS(2, 1, 1, 256, 4)
  GS(1, 1, 1, 256, 8)
  GS(4, 1, 1, 256, 4)

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
      hipLaunchKernelGGL(check, dim3(cus * 8), dim3(256), 0, s, dst, n16, bad);
      CK(hipStreamSynchronize(s));
      std::vector<float> ms(reps);
      for (int i = 0; i < reps; ++i) CK(hipEventElapsedTime(&ms[i], ev[2 * i], ev[2 * i + 1]));
      std::sort(ms.begin(), ms.end());
      unsigned long long nbad = 0;
      CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
      const double med = ms[reps / 2] * 1e-3, best = ms[0] * 1e-3;
      std::printf("{\"round\": %d, \"variant\": \"%s\", \"grid\": %u, \"block\": %u, \"launches\": %d, "
                  "\"median_us\": %.2f, \"best_us\": %.2f, \"worst_us\": %.2f, \"median_tbps\": %.4f, "
                  "\"best_tbps\": %.4f, \"bad_words\": %llu}\n",
                  r, v.name.c_str(), v.grid, v.block, reps, med * 1e6, best * 1e6, ms[reps - 1] * 1e3,
                  2.0 * bytes / med / 1e12, 2.0 * bytes / best / 1e12, nbad);
      std::fflush(stdout);
    }
  }
  return 0;
}
