// Streaming validation kernels for gfx950 (CDNA4): HBM fill/verify (N4), Philox fill (N5 input),
// copy (N7 local + xGMI peer pull), all-reduce fill/check (N6).
//
// Design notes (MI355X-first, see /opt/skills/guides; shapes picked by measurement with
// native/bench/stream_variants.hip on one MI355X, profiles/r1_bd2/stream_variants.jsonl):
//  * 16 B per lane per access (global_{load,store}_dwordx4): 1 KiB per wave-instruction.
//  * Block-contiguous SLABS, not a grid-stride interleave: block b owns bytes
//    [b*per, (b+1)*per) and walks them 4 KiB (one block-instruction) at a time, 4 instructions
//    in flight per lane. Each block then streams through whole DRAM pages instead of touching
//    a new page per instruction. Measured on 1 GiB fill: grid-stride 4.3 TB/s -> slab 6.2 TB/s
//    (hipMemsetD32 6.66); 256 MiB copy (read + write counted): 4.96 -> 6.42 TB/s (hipMemcpy
//    D2D 4.96-5.43). HBM3E spec peak is 8 TB/s.
//  * The plain HBM fill is the exception (round 6, native/bench/fill_roofline.hip, four sweeps,
//    profiles/r6_fill/): ONE block of 128 threads per CU, grid-stride, each lane storing 32
//    contiguous bytes (two dwordx4) per step. The whole chip's write front is then one
//    contiguous 1 MiB window moving through memory: 1 GiB in 153-156 us (6.9 TB/s, ~86 % of the
//    8 TB/s HBM3E peak) against 162-166 us for the runtime's own hipMemsetD32 (one 256-thread
//    block per CU, grid-stride, 16 B per lane) and 171-176 us for the old slab form. More waves
//    per CU, wider or narrower windows, non-temporal and sc1 stores were all slower.
//  * Grid = CUs x 16 blocks of 256 threads for the other streams, CUs x 32 for the copy (best
//    of the 4/8/16/32 per-CU sweep); non-temporal loads+stores for the once-touched copy.
//  * Reductions: wave64 __shfl_xor butterfly -> LDS across the 4 waves -> ONE atomic per block
//    (cdna_hip_programming.md Guideline 12).
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>
#include <vector>

#include "tk8s/common.h"
#include "tk8s/kernels.h"

namespace tk8s {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;  // 4 wave64s
constexpr int kWaves = kBlock / 64;

int streaming_grid(int blocks_per_cu) {
  static std::mutex mu;
  static std::vector<int> cu_count;
  int dev = 0;
  TK8S_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(mu);
  if (static_cast<int>(cu_count.size()) <= dev) cu_count.resize(dev + 1, 0);
  if (cu_count[dev] == 0) {
    int cus = 0;
    TK8S_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    cu_count[dev] = cus > 0 ? cus : 1;
  }
  return cu_count[dev] * blocks_per_cu;
}

static unsigned grid_for(size_t items, int blocks_per_cu = 8) {
  size_t need = (items + kBlock - 1) / kBlock;
  size_t cap = static_cast<size_t>(streaming_grid(blocks_per_cu));
  size_t g = need < cap ? need : cap;
  return static_cast<unsigned>(g ? g : 1);
}

// ------------------------------------------------------------------------------------------
// N4: HBM fill
// ------------------------------------------------------------------------------------------
// Slab bounds of block b over n items: [lo, hi).
__device__ __forceinline__ void slab_bounds(size_t n, size_t* lo, size_t* hi) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  *lo = per * blockIdx.x;
  const size_t end = *lo + per;
  *hi = end < n ? end : n;
}

// kNT = false (the probe's default, StoreMode::kPlain): the write-front walk above, launched as
// CUs x kFillBlock; kNT = true: non-temporal stores in the slab walk, launched as CUs x 16 x
// kBlock (the write-front walk with nt stores measured 2.4 TB/s).
constexpr int kFillBlock = 128;

template <bool kNT>
__global__ __launch_bounds__(kBlock) void hbm_fill_kernel(u32x4* __restrict__ dst, size_t n16,
                                                          unsigned value) {
  const u32x4 v = {value, value, value, value};
  if constexpr (!kNT) {
    const size_t threads = static_cast<size_t>(gridDim.x) * blockDim.x;
    const size_t tid = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const size_t pairs = n16 / 2;
    for (size_t i = tid; i < pairs; i += threads) {
      dst[2 * i] = v;
      dst[2 * i + 1] = v;
    }
    if ((n16 & 1) && tid == 0) dst[n16 - 1] = v;  // an odd count: the last 16 B
  } else {
    size_t lo, hi;
    slab_bounds(n16, &lo, &hi);
    size_t i = lo + threadIdx.x;
    for (; i + 3 * kBlock < hi; i += 4 * kBlock) {
#pragma unroll
      for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v, dst + i + u * kBlock);
    }
    for (; i < hi; i += kBlock) __builtin_nontemporal_store(v, dst + i);
  }
}

void hbm_fill(void* dst, size_t nbytes, uint32_t value, StoreMode mode, hipStream_t stream) {
  if (nbytes % 16) throw std::invalid_argument("hbm_fill: nbytes must be a multiple of 16");
  const size_t n16 = nbytes / 16;
  if (!n16) return;
  if (mode == StoreMode::kNonTemporal)
    hipLaunchKernelGGL(hbm_fill_kernel<true>, dim3(grid_for(n16 / 4, 16)), dim3(kBlock), 0, stream,
                       static_cast<u32x4*>(dst), n16, value);
  else
    hipLaunchKernelGGL(hbm_fill_kernel<false>, dim3(streaming_grid(1)), dim3(kFillBlock), 0, stream,
                       static_cast<u32x4*>(dst), n16, value);
  TK8S_HIP_CHECK(hipGetLastError());
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ float wave_max_f32(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

__global__ __launch_bounds__(kBlock) void verify_fill_kernel(const u32x4* __restrict__ src,
                                                             size_t n16, unsigned value,
                                                             unsigned long long* bad_words) {
  size_t lo, hi;
  slab_bounds(n16, &lo, &hi);
  unsigned long long bad = 0;
  size_t i = lo + threadIdx.x;
  for (; i + 3 * kBlock < hi; i += 4 * kBlock) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + i + u * kBlock);
#pragma unroll
    for (int u = 0; u < 4; ++u) bad += (v[u].x != value) + (v[u].y != value) + (v[u].z != value) + (v[u].w != value);
  }
  for (; i < hi; i += kBlock) {
    const u32x4 v = src[i];
    bad += (v.x != value) + (v.y != value) + (v.z != value) + (v.w != value);
  }
  __shared__ unsigned long long part[kWaves];
  bad = wave_sum_u64(bad);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) part[wid] = bad;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += part[w];
    if (s) atomicAdd(bad_words, s);
  }
}

void verify_fill(const void* src, size_t nbytes, uint32_t value, unsigned long long* bad_words,
                 hipStream_t stream) {
  if (nbytes % 16) throw std::invalid_argument("verify_fill: nbytes must be a multiple of 16");
  const size_t n16 = nbytes / 16;
  if (!n16) return;
  hipLaunchKernelGGL(verify_fill_kernel, dim3(grid_for(n16 / 4, 16)), dim3(kBlock), 0, stream,
                     static_cast<const u32x4*>(src), n16, value, bad_words);
  TK8S_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------
// N5 input: Philox4x32-10 (Salmon et al., Random123). Counter = (block index lo, hi, 0, 0),
// key = (seed lo, seed hi). Bit-identical host reference: tritonk8ssupervisor_amd/ops/reference.py
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ u32x4 philox4x32_10(unsigned long long idx, unsigned k0, unsigned k1) {
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

__global__ __launch_bounds__(kBlock) void philox_fill_kernel(u32x4* __restrict__ dst, size_t n16,
                                                             unsigned k0, unsigned k1) {
  // Same slab walk as the HBM fill (block-contiguous, 4 stores in flight per lane); the 10
  // Philox rounds per 16 B (~40 VALU ops) hide under the store stream.
  size_t lo, hi;
  slab_bounds(n16, &lo, &hi);
  size_t i = lo + threadIdx.x;
  for (; i + 3 * kBlock < hi; i += 4 * kBlock) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = philox4x32_10(i + u * kBlock, k0, k1);
#pragma unroll
    for (int u = 0; u < 4; ++u) dst[i + u * kBlock] = v[u];
  }
  for (; i < hi; i += kBlock) dst[i] = philox4x32_10(i, k0, k1);
}

void philox_fill(void* dst, size_t nbytes, uint64_t seed, hipStream_t stream) {
  if (nbytes % 16) throw std::invalid_argument("philox_fill: nbytes must be a multiple of 16");
  const size_t n16 = nbytes / 16;
  if (!n16) return;
  hipLaunchKernelGGL(philox_fill_kernel, dim3(grid_for(n16 / 4, 16)), dim3(kBlock), 0, stream,
                     static_cast<u32x4*>(dst), n16, static_cast<unsigned>(seed),
                     static_cast<unsigned>(seed >> 32));
  TK8S_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------
// N7: copy (local D2D, or peer pull when src is another GPU's memory with peer access enabled)
// ------------------------------------------------------------------------------------------
// 8 loads in flight per lane, then 8 stores, non-temporal both ways, 16 blocks per CU: the best
// of a 20-shape sweep on the MI355X (profiles/r6_copy/: 381.5 us for 1 GiB -> 1 GiB, 5.63 TB/s
// read + write, against 387.5 us for the former 4-deep x 32 and 456.5 us for hipMemcpyAsync's
// copy kernel in the same process; the fill's single-write-front shape loses here, 5.3 TB/s).
constexpr int kCopyDepth = 8;
__global__ __launch_bounds__(kBlock) void stream_copy_kernel(u32x4* __restrict__ dst,
                                                             const u32x4* __restrict__ src,
                                                             size_t n16) {
  size_t lo, hi;
  slab_bounds(n16, &lo, &hi);
  size_t i = lo + threadIdx.x;
  for (; i + (kCopyDepth - 1) * kBlock < hi; i += kCopyDepth * kBlock) {
    u32x4 v[kCopyDepth];
#pragma unroll
    for (int u = 0; u < kCopyDepth; ++u) v[u] = __builtin_nontemporal_load(src + i + u * kBlock);
#pragma unroll
    for (int u = 0; u < kCopyDepth; ++u) __builtin_nontemporal_store(v[u], dst + i + u * kBlock);
  }
  for (; i < hi; i += kBlock) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

void stream_copy(void* dst, const void* src, size_t nbytes, hipStream_t stream) {
  if (nbytes % 16) throw std::invalid_argument("stream_copy: nbytes must be a multiple of 16");
  const size_t n16 = nbytes / 16;
  if (!n16) return;
  hipLaunchKernelGGL(stream_copy_kernel, dim3(grid_for(n16 / kCopyDepth, 16)), dim3(kBlock), 0, stream,
                     static_cast<u32x4*>(dst), static_cast<const u32x4*>(src), n16);
  TK8S_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------
// N6: all-reduce pattern + checker. Values are small integers, exact in f32 and bf16 for
// nranks <= 16, so any |err| > 0 is a real transport/reduction error.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float bf16_bits_to_f32(unsigned short h) {
  return __uint_as_float(static_cast<unsigned>(h) << 16);
}
__device__ __forceinline__ unsigned short f32_to_bf16_bits(float f) {
  const unsigned u = __float_as_uint(f);
  return static_cast<unsigned short>((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

template <class T>
__global__ __launch_bounds__(kBlock) void ar_fill_kernel(T* __restrict__ buf, size_t count,
                                                         float base) {
  size_t lo, hi;
  slab_bounds(count, &lo, &hi);
  for (size_t i = lo + threadIdx.x; i < hi; i += kBlock) {
    const float v = base + static_cast<float>(i % 7);
    if constexpr (sizeof(T) == 4) buf[i] = v;
    else buf[i] = f32_to_bf16_bits(v);
  }
}

void ar_fill(void* buf, size_t count, int rank, DType dtype, hipStream_t stream) {
  if (!count) return;
  const unsigned grid = grid_for(count);
  const float base = static_cast<float>(rank + 1);
  if (dtype == DType::kF32)
    hipLaunchKernelGGL(ar_fill_kernel<float>, dim3(grid), dim3(kBlock), 0, stream,
                       static_cast<float*>(buf), count, base);
  else
    hipLaunchKernelGGL(ar_fill_kernel<unsigned short>, dim3(grid), dim3(kBlock), 0, stream,
                       static_cast<unsigned short*>(buf), count, base);
  TK8S_HIP_CHECK(hipGetLastError());
}

template <class T>
__global__ __launch_bounds__(kBlock) void ar_check_kernel(const T* __restrict__ buf, size_t count,
                                                          float base, float per_mod, float tol,
                                                          unsigned* max_err_bits,
                                                          unsigned long long* bad_count) {
  size_t lo, hi;
  slab_bounds(count, &lo, &hi);
  float emax = 0.f;
  unsigned long long bad = 0;
  for (size_t i = lo + threadIdx.x; i < hi; i += kBlock) {
    float v;
    if constexpr (sizeof(T) == 4) v = buf[i];
    else v = bf16_bits_to_f32(buf[i]);
    const float expect = base + per_mod * static_cast<float>(i % 7);
    float e = fabsf(v - expect);
    if (!(e == e)) e = __int_as_float(0x7f800000);  // NaN -> +inf so it wins the max
    emax = fmaxf(emax, e);
    bad += e > tol;
  }
  __shared__ float pmax[kWaves];
  __shared__ unsigned long long pbad[kWaves];
  emax = wave_max_f32(emax);
  bad = wave_sum_u64(bad);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    pmax[wid] = emax;
    pbad[wid] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = 0.f;
    unsigned long long b = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      m = fmaxf(m, pmax[w]);
      b += pbad[w];
    }
    // Non-negative floats order like their bit patterns.
    atomicMax(max_err_bits, __float_as_uint(m));
    if (b) atomicAdd(bad_count, b);
  }
}

void ar_check(const void* buf, size_t count, int nranks, DType dtype, float tol,
              unsigned int* max_err_bits, unsigned long long* bad, hipStream_t stream) {
  if (!count) return;
  const unsigned grid = grid_for(count);
  const float base = 0.5f * static_cast<float>(nranks) * static_cast<float>(nranks + 1);
  const float per_mod = static_cast<float>(nranks);
  if (dtype == DType::kF32)
    hipLaunchKernelGGL(ar_check_kernel<float>, dim3(grid), dim3(kBlock), 0, stream,
                       static_cast<const float*>(buf), count, base, per_mod, tol, max_err_bits, bad);
  else
    hipLaunchKernelGGL(ar_check_kernel<unsigned short>, dim3(grid), dim3(kBlock), 0, stream,
                       static_cast<const unsigned short*>(buf), count, base, per_mod, tol,
                       max_err_bits, bad);
  TK8S_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------
// Fault injection: a queue stall that always ends (kernels.h gpu_stall). One wave; lane 0 polls
// a flag in fine-grained host memory at system scope, sleeping between polls, and gives up after
// max_ticks of the GPU's constant-rate wall clock: the grid drains whether or not the host ever
// releases it. The flag is only read here; the host writes it.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void stall_kernel(const unsigned* flag, unsigned long long max_ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = wall_clock64();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u &&
         wall_clock64() - t0 < max_ticks)
    __builtin_amdgcn_s_sleep(127);
}

namespace {
std::mutex g_stall_mu;
unsigned* g_stall_flag = nullptr;  // fine-grained host memory; never freed (a kernel may read it)
std::atomic<bool> g_stall_armed{false};
}  // namespace

void gpu_stall(hipStream_t stream, double max_s) {
  int dev = 0, khz = 0;
  TK8S_HIP_CHECK(hipGetDevice(&dev));
  TK8S_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  if (khz <= 0) khz = 100000;  // gfx9: 100 MHz
  {
    std::lock_guard<std::mutex> lock(g_stall_mu);
    if (!g_stall_flag) {
      void* p = nullptr;
      TK8S_HIP_CHECK(hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped));
      g_stall_flag = static_cast<unsigned*>(p);
    }
    __atomic_store_n(g_stall_flag, 0u, __ATOMIC_SEQ_CST);
    g_stall_armed = true;
  }
  const double s = max_s > 0 ? (max_s < 600 ? max_s : 600) : 1;
  const auto ticks = static_cast<unsigned long long>(s * khz * 1000.0);
  hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, stream, g_stall_flag, ticks);
  TK8S_HIP_CHECK(hipGetLastError());
}

void gpu_stall_release() {
  if (!g_stall_armed.exchange(false)) return;
  std::lock_guard<std::mutex> lock(g_stall_mu);
  if (g_stall_flag) __atomic_store_n(g_stall_flag, 1u, __ATOMIC_SEQ_CST);
}

}  // namespace tk8s
