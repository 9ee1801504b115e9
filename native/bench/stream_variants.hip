// Development microbenchmark (not part of the product build): HBM fill / copy kernel shapes on
// gfx950, to pick the production form of hbm_fill / stream_copy (native/src/stream_kernels.hip).
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/stream_variants native/bench/stream_variants.hip
//   stream_variants [fill_MiB=1024] [copy_MiB=256] [iters=20]
//
// Prints one JSON line per variant: {"kernel", "variant", "grid", "block", "ms", "tbps"} where
// tbps counts bytes moved (fill: written; copy: read + written).
#include <hip/hip_runtime.h>

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

// A: grid-stride, U stores in flight per lane, spaced by the grid stride
template <int B, int U, bool NT>
__global__ __launch_bounds__(B) void fill_gridstride(u32x4* __restrict__ dst, size_t n16, unsigned v) {
  const size_t stride = static_cast<size_t>(gridDim.x) * B;
  size_t i = static_cast<size_t>(blockIdx.x) * B + threadIdx.x;
  const u32x4 x = {v, v, v, v};
  for (; i + (U - 1) * stride < n16; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (NT) __builtin_nontemporal_store(x, dst + i + u * stride);
      else dst[i + u * stride] = x;
    }
  }
  for (; i < n16; i += stride) dst[i] = x;
}

// B: block-contiguous slabs; per iteration the block writes U * B * 16 contiguous bytes
template <int B, int U, bool NT>
__global__ __launch_bounds__(B) void fill_slab(u32x4* __restrict__ dst, size_t n16, unsigned v) {
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const size_t lo = per * blockIdx.x;
  const size_t hi = lo + per < n16 ? lo + per : n16;
  const u32x4 x = {v, v, v, v};
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * B < hi; i += U * B) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (NT) __builtin_nontemporal_store(x, dst + i + u * B);
      else dst[i + u * B] = x;
    }
  }
  for (; i < hi; i += B) dst[i] = x;
}

template <int B, int U, bool NT>
__global__ __launch_bounds__(B) void copy_gridstride(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                     size_t n16) {
  const size_t stride = static_cast<size_t>(gridDim.x) * B;
  size_t i = static_cast<size_t>(blockIdx.x) * B + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (NT) __builtin_nontemporal_store(r[u], dst + i + u * stride);
      else dst[i + u * stride] = r[u];
    }
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

template <int B, int U, bool NT>
__global__ __launch_bounds__(B) void copy_slab(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n16) {
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const size_t lo = per * blockIdx.x;
  const size_t hi = lo + per < n16 ? lo + per : n16;
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * B < hi; i += U * B) {
    u32x4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = NT ? __builtin_nontemporal_load(src + i + u * B) : src[i + u * B];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (NT) __builtin_nontemporal_store(r[u], dst + i + u * B);
      else dst[i + u * B] = r[u];
    }
  }
  for (; i < hi; i += B) dst[i] = src[i];
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  ~Timer() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); }
};

template <class F>
double time_ms(F&& launch, int iters) {
  Timer t;
  launch();  // warm
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(t.a, 0));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(t.b, 0));
  CK(hipEventSynchronize(t.b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, t.a, t.b));
  return ms / iters;
}

void report(const char* kernel, const std::string& variant, unsigned grid, int block, double ms, double bytes) {
  std::printf("{\"kernel\": \"%s\", \"variant\": \"%s\", \"grid\": %u, \"block\": %d, \"ms\": %.5f, \"tbps\": %.4f}\n",
              kernel, variant.c_str(), grid, block, ms, bytes / (ms * 1e-3) / 1e12);
  std::fflush(stdout);
}

int main(int argc, char** argv) {
  const size_t fill_bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024) << 20;
  const size_t copy_bytes = (argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 256) << 20;
  const int iters = argc > 3 ? std::atoi(argv[3]) : 20;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  u32x4 *a = nullptr, *b = nullptr;
  CK(hipMalloc(&a, fill_bytes));
  CK(hipMalloc(&b, copy_bytes));
  const size_t nf = fill_bytes / 16, nc = copy_bytes / 16;

#define FILL(KERNEL, B, U, NT, PERCU)                                                              \
  {                                                                                                \
    const unsigned g = cus * (PERCU);                                                              \
    double ms = time_ms([&] { hipLaunchKernelGGL((KERNEL<B, U, NT>), dim3(g), dim3(B), 0, 0, a, nf, 7u); }, iters); \
    report("fill", std::string(#KERNEL) + "<" #B "," #U "," #NT ">x" #PERCU, g, B, ms, fill_bytes);  \
  }
  FILL(fill_gridstride, 256, 4, true, 8)
  FILL(fill_slab, 256, 4, false, 8)
  FILL(fill_slab, 256, 4, false, 16)
  FILL(fill_slab, 256, 4, false, 32)
  FILL(fill_slab, 256, 2, false, 16)
  FILL(fill_slab, 256, 1, false, 16)
  FILL(fill_slab, 256, 8, false, 16)
  FILL(fill_slab, 512, 2, false, 8)
  FILL(fill_slab, 512, 4, false, 8)
  FILL(fill_slab, 1024, 1, false, 2)
  FILL(fill_slab, 1024, 2, false, 4)
  FILL(fill_slab, 1024, 4, false, 4)
  FILL(fill_slab, 1024, 2, true, 4)
  FILL(fill_slab, 256, 4, true, 32)
  {
    double ms = time_ms([&] { CK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(a), 7u, fill_bytes / 4, 0)); }, iters);
    report("fill", "hipMemsetD32Async", 0, 0, ms, fill_bytes);
  }
  u32x4* src = a;  // copy source: the first copy_bytes of the fill buffer
#define COPY(KERNEL, B, U, NT, PERCU)                                                              \
  {                                                                                                \
    const unsigned g = cus * (PERCU);                                                              \
    double ms = time_ms([&] { hipLaunchKernelGGL((KERNEL<B, U, NT>), dim3(g), dim3(B), 0, 0, b, src, nc); }, iters); \
    report("copy", std::string(#KERNEL) + "<" #B "," #U "," #NT ">x" #PERCU, g, B, ms, 2.0 * copy_bytes); \
  }
  COPY(copy_gridstride, 256, 4, true, 8)
  COPY(copy_slab, 256, 4, true, 8)
  COPY(copy_slab, 256, 4, true, 16)
  COPY(copy_slab, 256, 2, true, 16)
  COPY(copy_slab, 256, 8, true, 16)
  COPY(copy_slab, 256, 4, true, 32)
  COPY(copy_slab, 512, 4, true, 8)
  COPY(copy_slab, 512, 2, true, 8)
  COPY(copy_slab, 1024, 2, true, 4)
  COPY(copy_slab, 1024, 4, true, 2)
  COPY(copy_slab, 1024, 1, true, 4)
  {
    double ms = time_ms([&] { CK(hipMemcpyAsync(b, src, copy_bytes, hipMemcpyDeviceToDevice, 0)); }, iters);
    report("copy", "hipMemcpyAsync", 0, 0, ms, 2.0 * copy_bytes);
  }
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
