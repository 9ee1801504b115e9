// Development microbenchmark (not part of the product build): how close the N4 fill gets to the
// HBM3E write roofline on gfx950, A/B against the runtime's own fills in ONE process.
//
//   hipcc -O3 --offload-arch=gfx950 -o build/fill_roofline native/bench/fill_roofline.hip
//   fill_roofline [fill_MiB=1024] [reps=15] [rounds=3]
//
// Every variant writes every byte of the buffer exactly once per launch (16 B per lane per
// store) and is checked afterwards (a verify pass counts words != the variant's value). Each
// launch is timed on its own by a pair of events; the line reports the median and best launch,
// and each round re-runs every variant in the same order so drift shows up as round-to-round
// spread rather than as one variant's advantage. One JSON line per (round, variant).
//
// Variants:
//  * memsetD32 / memsetD8: hipMemsetD32Async / hipMemsetAsync (the runtime's fill kernels).
//  * slab<B,U>xP: the production shape (stream_kernels.hip hbm_fill_kernel): block b owns a
//    contiguous slab, U 16-B stores in flight per lane, P blocks per CU.
//  * bslab<U,aux>xP: the same walk through buffer stores with explicit cache-policy bits
//    (aux 0 plain, 1 sc0, 2 nt, 16 sc1, 17 sc0|sc1, 18 nt|sc1).
//  * chunk<C,U>xP: persistent blocks over C-KiB chunks handed out grid-stride (chunk c to block
//    c % grid): the chip's write front stays one contiguous region of grid x C KiB.
//  * xslab<U>xP: slabs renumbered so each XCD (blocks are dealt to the 8 XCDs round-robin) owns
//    one contiguous eighth of the buffer.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

template <int B, int U>
__global__ __launch_bounds__(B) void fill_slab(u32x4* __restrict__ dst, size_t n16, unsigned v) {
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const size_t lo = per * blockIdx.x;
  const size_t hi = lo + per < n16 ? lo + per : n16;
  const u32x4 x = {v, v, v, v};
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * B < hi; i += U * B) {
#pragma unroll
    for (int u = 0; u < U; ++u) dst[i + u * B] = x;
  }
  for (; i < hi; i += B) dst[i] = x;
}

// Buffer-store slab walk: the descriptor covers this block's slab only (wave-uniform base and
// size), so the 32-bit offsets stay small and any lane past the end is dropped by the range check.
template <int U, int AUX>
__global__ __launch_bounds__(256) void fill_bslab(u32x4* __restrict__ dst, size_t n16, unsigned v) {
  constexpr int B = 256;
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const size_t lo = per * blockIdx.x;
  if (lo >= n16) return;
  const size_t hi = lo + per < n16 ? lo + per : n16;
  const unsigned cnt = static_cast<unsigned>(hi - lo);
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(dst + lo, 0, static_cast<int>(cnt * 16u), 0x00020000);
  const u32x4 x = {v, v, v, v};
  unsigned i = threadIdx.x;
  for (; i + (U - 1) * B < cnt; i += U * B) {
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(x, r, static_cast<int>((i + u * B) * 16u), 0, AUX);
  }
  for (; i < cnt; i += B) __builtin_amdgcn_raw_buffer_store_b128(x, r, static_cast<int>(i * 16u), 0, AUX);
}

// Persistent chunks: chunk c (C KiB) goes to block c % grid; inside a chunk the block walks 4 KiB
// per block-instruction, U in flight per lane.
template <int CKIB, int U>
__global__ __launch_bounds__(256) void fill_chunk(u32x4* __restrict__ dst, size_t n16, unsigned v) {
  constexpr int B = 256;
  constexpr size_t C16 = static_cast<size_t>(CKIB) * 1024 / 16;
  const size_t nchunks = (n16 + C16 - 1) / C16;
  const u32x4 x = {v, v, v, v};
  for (size_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const size_t lo = c * C16;
    const size_t hi = lo + C16 < n16 ? lo + C16 : n16;
    size_t i = lo + threadIdx.x;
    for (; i + (U - 1) * B < hi; i += U * B) {
#pragma unroll
      for (int u = 0; u < U; ++u) dst[i + u * B] = x;
    }
    for (; i < hi; i += B) dst[i] = x;
  }
}

// XCD-contiguous slabs: block b runs on XCD b % 8 (round-robin dispatch); its slab index is
// renumbered so XCD x owns slabs [x*G/8, (x+1)*G/8). Needs gridDim.x % 8 == 0 (host checks).
template <int U>
__global__ __launch_bounds__(256) void fill_xslab(u32x4* __restrict__ dst, size_t n16, unsigned v) {
  constexpr int B = 256;
  const unsigned g = gridDim.x, per_xcd = g / 8;
  const unsigned slab = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  const size_t per = (n16 + g - 1) / g;
  const size_t lo = per * slab;
  const size_t hi = lo + per < n16 ? lo + per : n16;
  const u32x4 x = {v, v, v, v};
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * B < hi; i += U * B) {
#pragma unroll
    for (int u = 0; u < U; ++u) dst[i + u * B] = x;
  }
  for (; i < hi; i += B) dst[i] = x;
}

// Grid-stride: thread t of the grid writes 16*W contiguous bytes at (t + k*T)*W (T = grid
// threads), U of those iterations unrolled. The runtime's fillBufferAligned is this shape with
// one 256-thread block per CU (the chip's write front is one contiguous T*16*W-byte window).
template <int U, int W, bool NT, int B = 256>
__global__ __launch_bounds__(B) void fill_gs(u32x4* __restrict__ dst, size_t n16, unsigned v) {
  const size_t T = static_cast<size_t>(gridDim.x) * B;
  const size_t nw = n16 / W;  // whole W-vectors; n16 % W == 0 (host checks)
  const u32x4 x = {v, v, v, v};
  size_t i = static_cast<size_t>(blockIdx.x) * B + threadIdx.x;
  for (; i + (U - 1) * T < nw; i += U * T) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int w = 0; w < W; ++w) {
        if constexpr (NT) __builtin_nontemporal_store(x, dst + (i + u * T) * W + w);
        else dst[(i + u * T) * W + w] = x;
      }
  }
  for (; i < nw; i += T)
#pragma unroll
    for (int w = 0; w < W; ++w) dst[i * W + w] = x;
}

// fill_gs with the blocks' pieces of each window renumbered XCD-contiguous (block b runs on XCD
// b % 8): XCD x writes one contiguous eighth of every T*16-byte window. grid % 8 == 0.
template <int B>
__global__ __launch_bounds__(B) void fill_gsx(u32x4* __restrict__ dst, size_t n16, unsigned v) {
  const size_t T = static_cast<size_t>(gridDim.x) * B;
  const unsigned piece = (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
  const u32x4 x = {v, v, v, v};
  for (size_t i = static_cast<size_t>(piece) * B + threadIdx.x; i < n16; i += T) dst[i] = x;
}

// Read side (the verify pass): count words != v, U 16-B loads in flight per lane.
template <int B, int U>
__global__ __launch_bounds__(B) void read_gs(const u32x4* __restrict__ src, size_t n16, unsigned v,
                                             unsigned long long* bad) {
  const size_t T = static_cast<size_t>(gridDim.x) * B;
  unsigned long long b = 0;
  size_t i = static_cast<size_t>(blockIdx.x) * B + threadIdx.x;
  for (; i + (U - 1) * T < n16; i += U * T) {
    u32x4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = __builtin_nontemporal_load(src + i + u * T);
#pragma unroll
    for (int u = 0; u < U; ++u) b += (w[u].x != v) + (w[u].y != v) + (w[u].z != v) + (w[u].w != v);
  }
  for (; i < n16; i += T) {
    const u32x4 w = src[i];
    b += (w.x != v) + (w.y != v) + (w.z != v) + (w.w != v);
  }
  for (int off = 32; off > 0; off >>= 1) b += __shfl_xor(b, off, 64);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(bad, b);
}

template <int B, int U>
__global__ __launch_bounds__(B) void read_slab(const u32x4* __restrict__ src, size_t n16, unsigned v,
                                               unsigned long long* bad) {
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const size_t lo = per * blockIdx.x;
  const size_t hi = lo + per < n16 ? lo + per : n16;
  unsigned long long b = 0;
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * B < hi; i += U * B) {
    u32x4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = __builtin_nontemporal_load(src + i + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u) b += (w[u].x != v) + (w[u].y != v) + (w[u].z != v) + (w[u].w != v);
  }
  for (; i < hi; i += B) {
    const u32x4 w = src[i];
    b += (w.x != v) + (w.y != v) + (w.z != v) + (w.w != v);
  }
  for (int off = 32; off > 0; off >>= 1) b += __shfl_xor(b, off, 64);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(bad, b);
}

__global__ __launch_bounds__(256) void count_bad(const u32x4* __restrict__ src, size_t n16, unsigned v,
                                                 unsigned long long* bad) {
  unsigned long long b = 0;
  for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n16; i += static_cast<size_t>(gridDim.x) * 256) {
    const u32x4 w = src[i];
    b += (w.x != v) + (w.y != v) + (w.z != v) + (w.w != v);
  }
  for (int off = 32; off > 0; off >>= 1) b += __shfl_xor(b, off, 64);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(bad, b);
}

struct Variant {
  std::string name;
  unsigned grid;
  int block;
  void (*launch)(u32x4*, size_t, unsigned, unsigned);  // (dst, n16, value, grid)
  bool read = false;  // a read variant: counts mismatches of the buffer against `value`
};

template <int B, int U>
void L_slab(u32x4* d, size_t n, unsigned v, unsigned g) { hipLaunchKernelGGL((fill_slab<B, U>), dim3(g), dim3(B), 0, 0, d, n, v); }
template <int U, int AUX>
void L_bslab(u32x4* d, size_t n, unsigned v, unsigned g) { hipLaunchKernelGGL((fill_bslab<U, AUX>), dim3(g), dim3(256), 0, 0, d, n, v); }
template <int C, int U>
void L_chunk(u32x4* d, size_t n, unsigned v, unsigned g) { hipLaunchKernelGGL((fill_chunk<C, U>), dim3(g), dim3(256), 0, 0, d, n, v); }
template <int U>
void L_xslab(u32x4* d, size_t n, unsigned v, unsigned g) { hipLaunchKernelGGL((fill_xslab<U>), dim3(g), dim3(256), 0, 0, d, n, v); }
template <int U, int W, bool NT, int B = 256>
void L_gs(u32x4* d, size_t n, unsigned v, unsigned g) { hipLaunchKernelGGL((fill_gs<U, W, NT, B>), dim3(g), dim3(B), 0, 0, d, n, v); }
template <int B>
void L_gsx(u32x4* d, size_t n, unsigned v, unsigned g) { hipLaunchKernelGGL((fill_gsx<B>), dim3(g), dim3(B), 0, 0, d, n, v); }
// Read variants: the buffer holds `v` (a fill ran first); the launch counts mismatches into g_bad.
unsigned long long* g_bad = nullptr;
template <int B, int U>
void L_rgs(u32x4* d, size_t n, unsigned v, unsigned g) { hipLaunchKernelGGL((read_gs<B, U>), dim3(g), dim3(B), 0, 0, d, n, v, g_bad); }
template <int B, int U>
void L_rslab(u32x4* d, size_t n, unsigned v, unsigned g) { hipLaunchKernelGGL((read_slab<B, U>), dim3(g), dim3(B), 0, 0, d, n, v, g_bad); }
void L_memset32(u32x4* d, size_t n, unsigned v, unsigned) { CK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d), v, n * 4, 0)); }
void L_memset8(u32x4* d, size_t n, unsigned v, unsigned) { CK(hipMemsetAsync(d, static_cast<int>(v & 0xFF), n * 16, 0)); }

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024) << 20;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 15;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 3;
  if (bytes == 0 || bytes % (1 << 20) || reps < 1 || rounds < 1) {
    std::fprintf(stderr, "usage: fill_roofline [MiB>0] [reps>0] [rounds>0]\n");
    return 2;
  }
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  u32x4* a = nullptr;
  unsigned long long* bad = nullptr;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&bad, sizeof *bad));
  CK(hipMalloc(&g_bad, sizeof *g_bad));
  const size_t n16 = bytes / 16;
  const unsigned C = static_cast<unsigned>(cus);
  std::vector<Variant> vs = {
      {"memsetD32", 0, 0, L_memset32},
      {"slab<256,4>x16 (production)", C * 16, 256, L_slab<256, 4>},
      {"gs<1,2>b128x1", C * 1, 128, L_gs<1, 2, false, 128>},
      {"gs<1,2>b64x1", C * 1, 64, L_gs<1, 2, false, 64>},
      {"gs<1,2>b64x2", C * 2, 64, L_gs<1, 2, false, 64>},
      {"gs<1,4>b64x1", C * 1, 64, L_gs<1, 4, false, 64>},
      {"gs<1,4>b32x1", C * 1, 32, L_gs<1, 4, false, 32>},
      {"gs<1,2>b128x2", C * 2, 128, L_gs<1, 2, false, 128>},
      {"gs<2,2>b128x1", C * 1, 128, L_gs<2, 2, false, 128>},
      {"gs<4,2>b128x1", C * 1, 128, L_gs<4, 2, false, 128>},
      {"gs<1,2>b128x1 nt", C * 1, 128, L_gs<1, 2, true, 128>},
      {"gs<1,2>b128x3/4", C * 3 / 4, 128, L_gs<1, 2, false, 128>},
      {"gs<1,2>b128x5/4", C * 5 / 4, 128, L_gs<1, 2, false, 128>},
      {"gs<1,2>b256x1/2", C / 2, 256, L_gs<1, 2, false, 256>},
      {"gs<1,1>b256x1", C * 1, 256, L_gs<1, 1, false>},
      {"gs<1,2>b128x1 again", C * 1, 128, L_gs<1, 2, false, 128>},
      {"memsetD32 again", 0, 0, L_memset32},
  };
  hipEvent_t ev[64];
  const int nev = 2 * std::min(reps, 32);
  for (int i = 0; i < nev; ++i) CK(hipEventCreate(&ev[i]));
  int failures = 0;
  for (int round = 0; round < rounds; ++round) {
    unsigned value = 0x1000u * (round + 1);
    for (const auto& var : vs) {
      ++value;
      if (var.grid % 8 && (var.name.rfind("xslab", 0) == 0 || var.name.rfind("gsx", 0) == 0)) continue;
      if (var.grid == 0 && !var.name.empty() && var.name[0] != 'm') continue;  // grid rounded to 0
      if (var.read) {  // the buffer holds `value`; every read launch must count 0 mismatches
        L_memset32(a, n16, value, 0);
        CK(hipMemset(g_bad, 0, sizeof *g_bad));
        var.launch(a, n16, value, var.grid);  // warm
      } else {
        var.launch(a, n16, value ^ 0xFFFFFFFFu, var.grid);  // warm (and a different value first)
      }
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      const int n = nev / 2;
      for (int r = 0; r < n; ++r) {
        CK(hipEventRecord(ev[2 * r], 0));
        var.launch(a, n16, value, var.grid);
        CK(hipEventRecord(ev[2 * r + 1], 0));
      }
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      std::vector<float> ms(n);
      for (int r = 0; r < n; ++r) CK(hipEventElapsedTime(&ms[r], ev[2 * r], ev[2 * r + 1]));
      std::sort(ms.begin(), ms.end());
      CK(hipMemset(bad, 0, sizeof *bad));
      // memsetD8 writes a byte pattern: check against the replicated byte
      const unsigned want = var.name == "memsetD8" ? (value & 0xFFu) * 0x01010101u : value;
      hipLaunchKernelGGL(count_bad, dim3(C * 8), dim3(256), 0, 0, a, n16, want, bad);
      unsigned long long nbad = 0, rbad = 0;
      CK(hipMemcpy(&nbad, bad, sizeof nbad, hipMemcpyDeviceToHost));
      if (var.read) {
        CK(hipMemcpy(&rbad, g_bad, sizeof rbad, hipMemcpyDeviceToHost));
        nbad += rbad;  // a read variant that miscounts fails too
      }
      failures += nbad != 0;
      const double med = ms[n / 2], best = ms[0];
      std::printf("{\"round\": %d, \"variant\": \"%s\", \"grid\": %u, \"block\": %d, \"launches\": %d, "
                  "\"median_us\": %.2f, \"best_us\": %.2f, \"worst_us\": %.2f, \"median_tbps\": %.4f, "
                  "\"best_tbps\": %.4f, \"bad_words\": %llu}\n",
                  round, var.name.c_str(), var.grid, var.block, n, med * 1e3, best * 1e3, ms[n - 1] * 1e3,
                  bytes / (med * 1e-3) / 1e12, bytes / (best * 1e-3) / 1e12, nbad);
      std::fflush(stdout);
    }
  }
  for (int i = 0; i < nev; ++i) CK(hipEventDestroy(ev[i]));
  CK(hipFree(bad));
  CK(hipFree(a));
  return failures ? 1 : 0;
}
