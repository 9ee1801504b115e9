// N5: chunked MD5 tree hash on gfx950 — the GPU analogue of the reference's "/cpu" benchmark
// (docs/benchmarks.md:11-12: md5 of 268435456 random bytes, 16.86 s on a Triton KVM).
//
// MD5 is a Merkle-Damgard chain, so one digest over 256 MiB is a serial dependency chain.
// The GPU form splits the input into fixed chunks (default 1 KiB), one chunk per lane, hashes
// every chunk with standard RFC 1321 MD5 (padding + length included), then folds the digests
// FOUR at a time -- a parent is the MD5 of its (up to) four children's 16-byte digests, 64 B --
// level after level until one digest remains. An input of one chunk is its plain MD5.
// The exact host oracle is hashlib-based: tritonk8ssupervisor_amd/ops/reference.py:md5_tree.
//
// Why fan-in 4 above the leaves: every level is a serial chain of (bytes per node / 64 + 1)
// dependent compressions that no amount of parallelism shortens. Folding 1 KiB of digests per
// node (the r1-r6 tree) cost 17 compressions per level and three nearly empty launches after
// the leaves -- 47 us of a 108 us tree at 256 MiB (profiles/r6_kernels). A 64-byte node costs 2,
// and a block of 256 threads folds 1024 nodes five levels up in one launch (md5_fold_kernel):
// 256 MiB is the leaf launch plus two fold launches. The fold stays out of the leaf kernel: each
// leaf wave's own serial chain sets the leaves' time (4 chains per SIMD at the grid's 16 waves
// per CU), and a fold there adds 6 compressions to it, on a quarter of the lanes (+27 us
// measured, profiles/r6_md5).
//
// Per lane: 16 message words per 64-byte block via four 16-byte loads (the next block is
// loaded before the current one is compressed, so its latency hides under 64 ALU steps);
// the 64 steps are fully unrolled with constant K/s (VALU: v_bitop3 / v_alignbit / v_add3).
// With 1 KiB chunks a 256 MiB input is 262144 lanes = 4096 wave64s = 16 waves per CU on
// 256 CUs, enough to keep the HBM stream and the integer pipes busy together.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "tk8s/common.h"
#include "tk8s/kernels.h"

namespace tk8s {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kMd5Block = 256;

#define TK8S_F(x, y, z) ((z) ^ ((x) & ((y) ^ (z))))
#define TK8S_G(x, y, z) ((y) ^ ((z) & ((x) ^ (y))))
#define TK8S_H(x, y, z) __builtin_amdgcn_bitop3_b32((x), (y), (z), 0x96)  // x ^ y ^ z in one VALU op
#define TK8S_I(x, y, z) ((y) ^ ((x) | ~(z)))
#define TK8S_STEP(f, a, b, c, d, x, k, s)               \
  do {                                                  \
    (a) += f((b), (c), (d)) + (x) + (k);                \
    (a) = __builtin_rotateleft32((a), (s)) + (b);       \
  } while (0)

__device__ __forceinline__ void md5_compress(unsigned st[4], const unsigned m[16]) {
  unsigned a = st[0], b = st[1], c = st[2], d = st[3];
  TK8S_STEP(TK8S_F, a, b, c, d, m[0], 0xd76aa478u, 7);
  TK8S_STEP(TK8S_F, d, a, b, c, m[1], 0xe8c7b756u, 12);
  TK8S_STEP(TK8S_F, c, d, a, b, m[2], 0x242070dbu, 17);
  TK8S_STEP(TK8S_F, b, c, d, a, m[3], 0xc1bdceeeu, 22);
  TK8S_STEP(TK8S_F, a, b, c, d, m[4], 0xf57c0fafu, 7);
  TK8S_STEP(TK8S_F, d, a, b, c, m[5], 0x4787c62au, 12);
  TK8S_STEP(TK8S_F, c, d, a, b, m[6], 0xa8304613u, 17);
  TK8S_STEP(TK8S_F, b, c, d, a, m[7], 0xfd469501u, 22);
  TK8S_STEP(TK8S_F, a, b, c, d, m[8], 0x698098d8u, 7);
  TK8S_STEP(TK8S_F, d, a, b, c, m[9], 0x8b44f7afu, 12);
  TK8S_STEP(TK8S_F, c, d, a, b, m[10], 0xffff5bb1u, 17);
  TK8S_STEP(TK8S_F, b, c, d, a, m[11], 0x895cd7beu, 22);
  TK8S_STEP(TK8S_F, a, b, c, d, m[12], 0x6b901122u, 7);
  TK8S_STEP(TK8S_F, d, a, b, c, m[13], 0xfd987193u, 12);
  TK8S_STEP(TK8S_F, c, d, a, b, m[14], 0xa679438eu, 17);
  TK8S_STEP(TK8S_F, b, c, d, a, m[15], 0x49b40821u, 22);

  TK8S_STEP(TK8S_G, a, b, c, d, m[1], 0xf61e2562u, 5);
  TK8S_STEP(TK8S_G, d, a, b, c, m[6], 0xc040b340u, 9);
  TK8S_STEP(TK8S_G, c, d, a, b, m[11], 0x265e5a51u, 14);
  TK8S_STEP(TK8S_G, b, c, d, a, m[0], 0xe9b6c7aau, 20);
  TK8S_STEP(TK8S_G, a, b, c, d, m[5], 0xd62f105du, 5);
  TK8S_STEP(TK8S_G, d, a, b, c, m[10], 0x02441453u, 9);
  TK8S_STEP(TK8S_G, c, d, a, b, m[15], 0xd8a1e681u, 14);
  TK8S_STEP(TK8S_G, b, c, d, a, m[4], 0xe7d3fbc8u, 20);
  TK8S_STEP(TK8S_G, a, b, c, d, m[9], 0x21e1cde6u, 5);
  TK8S_STEP(TK8S_G, d, a, b, c, m[14], 0xc33707d6u, 9);
  TK8S_STEP(TK8S_G, c, d, a, b, m[3], 0xf4d50d87u, 14);
  TK8S_STEP(TK8S_G, b, c, d, a, m[8], 0x455a14edu, 20);
  TK8S_STEP(TK8S_G, a, b, c, d, m[13], 0xa9e3e905u, 5);
  TK8S_STEP(TK8S_G, d, a, b, c, m[2], 0xfcefa3f8u, 9);
  TK8S_STEP(TK8S_G, c, d, a, b, m[7], 0x676f02d9u, 14);
  TK8S_STEP(TK8S_G, b, c, d, a, m[12], 0x8d2a4c8au, 20);

  TK8S_STEP(TK8S_H, a, b, c, d, m[5], 0xfffa3942u, 4);
  TK8S_STEP(TK8S_H, d, a, b, c, m[8], 0x8771f681u, 11);
  TK8S_STEP(TK8S_H, c, d, a, b, m[11], 0x6d9d6122u, 16);
  TK8S_STEP(TK8S_H, b, c, d, a, m[14], 0xfde5380cu, 23);
  TK8S_STEP(TK8S_H, a, b, c, d, m[1], 0xa4beea44u, 4);
  TK8S_STEP(TK8S_H, d, a, b, c, m[4], 0x4bdecfa9u, 11);
  TK8S_STEP(TK8S_H, c, d, a, b, m[7], 0xf6bb4b60u, 16);
  TK8S_STEP(TK8S_H, b, c, d, a, m[10], 0xbebfbc70u, 23);
  TK8S_STEP(TK8S_H, a, b, c, d, m[13], 0x289b7ec6u, 4);
  TK8S_STEP(TK8S_H, d, a, b, c, m[0], 0xeaa127fau, 11);
  TK8S_STEP(TK8S_H, c, d, a, b, m[3], 0xd4ef3085u, 16);
  TK8S_STEP(TK8S_H, b, c, d, a, m[6], 0x04881d05u, 23);
  TK8S_STEP(TK8S_H, a, b, c, d, m[9], 0xd9d4d039u, 4);
  TK8S_STEP(TK8S_H, d, a, b, c, m[12], 0xe6db99e5u, 11);
  TK8S_STEP(TK8S_H, c, d, a, b, m[15], 0x1fa27cf8u, 16);
  TK8S_STEP(TK8S_H, b, c, d, a, m[2], 0xc4ac5665u, 23);

  TK8S_STEP(TK8S_I, a, b, c, d, m[0], 0xf4292244u, 6);
  TK8S_STEP(TK8S_I, d, a, b, c, m[7], 0x432aff97u, 10);
  TK8S_STEP(TK8S_I, c, d, a, b, m[14], 0xab9423a7u, 15);
  TK8S_STEP(TK8S_I, b, c, d, a, m[5], 0xfc93a039u, 21);
  TK8S_STEP(TK8S_I, a, b, c, d, m[12], 0x655b59c3u, 6);
  TK8S_STEP(TK8S_I, d, a, b, c, m[3], 0x8f0ccc92u, 10);
  TK8S_STEP(TK8S_I, c, d, a, b, m[10], 0xffeff47du, 15);
  TK8S_STEP(TK8S_I, b, c, d, a, m[1], 0x85845dd1u, 21);
  TK8S_STEP(TK8S_I, a, b, c, d, m[8], 0x6fa87e4fu, 6);
  TK8S_STEP(TK8S_I, d, a, b, c, m[15], 0xfe2ce6e0u, 10);
  TK8S_STEP(TK8S_I, c, d, a, b, m[6], 0xa3014314u, 15);
  TK8S_STEP(TK8S_I, b, c, d, a, m[13], 0x4e0811a1u, 21);
  TK8S_STEP(TK8S_I, a, b, c, d, m[4], 0xf7537e82u, 6);
  TK8S_STEP(TK8S_I, d, a, b, c, m[11], 0xbd3af235u, 10);
  TK8S_STEP(TK8S_I, c, d, a, b, m[2], 0x2ad7d2bbu, 15);
  TK8S_STEP(TK8S_I, b, c, d, a, m[9], 0xeb86d391u, 21);
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
}

#undef TK8S_F
#undef TK8S_G
#undef TK8S_H
#undef TK8S_I
#undef TK8S_STEP

__device__ __forceinline__ void load_block(const u32x4* __restrict__ p, u32x4 (&v)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = p[q];
}

__device__ __forceinline__ void unpack(const u32x4 (&v)[4], unsigned (&m)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    m[4 * q + 0] = v[q].x;
    m[4 * q + 1] = v[q].y;
    m[4 * q + 2] = v[q].z;
    m[4 * q + 3] = v[q].w;
  }
}

// Tail of a message: `rem` (< 64) bytes at p, total message length `len` bytes.
// Byte loads only here (at most once per chunk, for the final partial chunk).
__device__ void md5_finish(unsigned st[4], const unsigned char* __restrict__ p, unsigned rem,
                           unsigned long long len) {
  unsigned m[16];
#pragma unroll
  for (int w = 0; w < 16; ++w) m[w] = 0;
  for (unsigned i = 0; i < rem; ++i) m[i >> 2] |= static_cast<unsigned>(p[i]) << (8 * (i & 3));
  m[rem >> 2] |= 0x80u << (8 * (rem & 3));
  const unsigned long long bits = len * 8ull;
  if (rem >= 56) {
    md5_compress(st, m);
#pragma unroll
    for (int w = 0; w < 16; ++w) m[w] = 0;
  }
  m[14] = static_cast<unsigned>(bits);
  m[15] = static_cast<unsigned>(bits >> 32);
  md5_compress(st, m);
}

// ------------------------------------------------------------------------------------------
// Leaves, one lane per chunk: chunk sizes the coalesced kernel does not take, and the chunks
// after its whole groups.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kMd5Block) void md5_chunks_kernel(const unsigned char* __restrict__ src,
                                                              unsigned long long nbytes,
                                                              unsigned chunk_bytes,
                                                              unsigned long long nchunks,
                                                              u32x4* __restrict__ digests) {
  const unsigned long long c = static_cast<unsigned long long>(blockIdx.x) * kMd5Block + threadIdx.x;
  if (c >= nchunks) return;
  const unsigned long long start = c * chunk_bytes;
  const unsigned long long left = nbytes > start ? nbytes - start : 0;
  const unsigned long long len = left < chunk_bytes ? left : chunk_bytes;
  unsigned st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};

  const unsigned nfull = static_cast<unsigned>(len >> 6);
  const u32x4* blk = reinterpret_cast<const u32x4*>(src + start);
  if (nfull) {
    u32x4 cur[4], nxt[4];
    load_block(blk, cur);
    for (unsigned b = 0; b < nfull; ++b) {
      if (b + 1 < nfull) load_block(blk + 4 * (b + 1), nxt);
      unsigned m[16];
      unpack(cur, m);
      md5_compress(st, m);
#pragma unroll
      for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
    }
  }
  md5_finish(st, src + start + (static_cast<unsigned long long>(nfull) << 6),
             static_cast<unsigned>(len & 63), len);
  digests[c] = u32x4{st[0], st[1], st[2], st[3]};
}

// ------------------------------------------------------------------------------------------
// Coalesced leaves for full chunks whose size is a multiple of 128 B (the default 1 KiB):
// one wave owns 64 consecutive chunks. Per step it pulls the next 128 B of all 64 chunks with
// 8 wave-instructions (lane l of instruction i loads 16 B of chunk 8i + l/8), i.e. every
// instruction reads 8 whole 128-B lines instead of 64 scattered 16-B pieces (the one-lane-
// per-chunk loads above), stages them in a wave-private LDS tile and each lane reads its own
// chunk's 32 words back. Rows are padded to 144 B (36 dwords): the 16 lanes of a ds_read_b128
// phase then start on banks 36*l mod 64, all distinct, so the read-back is conflict-free.
// The next step's global loads are issued before the current step's two compressions and
// staged only after them, so HBM latency hides under 128 MD5 steps. (Left to itself the
// compiler hoists the staging -- and its wait for those loads -- above the compressions, which
// are pure register work: the empty asm below pins the order. profiles/r6_md5.) LDS: 4 waves x
// 9 KiB per block -> 4 blocks (16 waves) per CU.
// ------------------------------------------------------------------------------------------
constexpr int kWaveChunks = 64;
constexpr int kRowVec = 9;  // u32x4 per LDS row: 8 of data + 1 of padding

__device__ __forceinline__ void wave_sync_lds() {
  // LDS ops of one wave complete in issue order; this only stops the compiler from moving the
  // staging stores across the read-back (and vice versa).
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(kMd5Block) void md5_chunks_coalesced_kernel(const unsigned char* __restrict__ src,
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
    // The compressions first, then the staging that waits for the next step's loads.
    asm volatile("" ::"v"(st[0]), "v"(st[1]), "v"(st[2]), "v"(st[3]) : "memory");
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

// ------------------------------------------------------------------------------------------
// The levels above the leaves, fan-in 4. Block b of B threads folds the 4B nodes
// [4Bb, 4Bb + 4B) of a level of n nodes up `levels` (<= 1 + log4 B) levels: every thread makes
// one parent from four children read from global memory (all lanes busy), then the block's
// parents fold in LDS -- B/4 threads, B/16, ... -- until one node, node b of that level. Each
// level is 2 dependent compressions (one if a parent has fewer than 4 children) and nothing
// else: the fold is latency-bound, so a launch takes as many levels as a block can hold.
// ------------------------------------------------------------------------------------------
constexpr int kFanIn = 4;
constexpr int kFoldBlock = 256;  // 5 levels (1024 -> 1) per launch

// MD5 of a node: `count` (1..4) child digests, 16 * count bytes. Four children fill one block
// and the padding takes a second; fewer leave room for the padding in the first.
__device__ __forceinline__ u32x4 md5_node(const u32x4 (&c)[kFanIn], unsigned count) {
  unsigned st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  unsigned m[16];
#pragma unroll
  for (int q = 0; q < kFanIn; ++q) {
    const bool have = static_cast<unsigned>(q) < count;
    m[4 * q + 0] = have ? c[q].x : (static_cast<unsigned>(q) == count ? 0x80u : 0u);
    m[4 * q + 1] = have ? c[q].y : 0u;
    m[4 * q + 2] = have ? c[q].z : 0u;
    m[4 * q + 3] = have ? c[q].w : 0u;
  }
  if (count < kFanIn) m[14] = 128u * count;  // bit length; m[15] stays 0
  md5_compress(st, m);
  if (count == kFanIn) {
#pragma unroll
    for (int w = 0; w < 16; ++w) m[w] = 0;
    m[0] = 0x80u;
    m[14] = 512u;
    md5_compress(st, m);
  }
  return u32x4{st[0], st[1], st[2], st[3]};
}

__device__ __forceinline__ unsigned children(unsigned long long first, unsigned long long n) {
  return first >= n ? 0u : (n - first >= kFanIn ? kFanIn : static_cast<unsigned>(n - first));
}

template <int B>
__global__ __launch_bounds__(B) void md5_fold_kernel(const u32x4* __restrict__ in, unsigned long long n, int levels,
                                                    u32x4* __restrict__ out) {
  __shared__ u32x4 nodes[B];
  const int t = threadIdx.x;
  unsigned long long base = static_cast<unsigned long long>(blockIdx.x) * B;  // first parent of this block
  u32x4 d = u32x4{0u, 0u, 0u, 0u};
  {
    const unsigned long long p = base + t;
    const unsigned count = children(kFanIn * p, n);
    if (count) {
      u32x4 c[kFanIn];
#pragma unroll
      for (int i = 0; i < kFanIn; ++i) c[i] = static_cast<unsigned>(i) < count ? in[kFanIn * p + i] : u32x4{0u, 0u, 0u, 0u};
      d = md5_node(c, count);
    }
  }
  unsigned long long nl = (n + kFanIn - 1) / kFanIn;  // nodes of the level just made
  for (int l = 1; l < levels; ++l) {
    nodes[t] = d;
    __syncthreads();
    const unsigned long long p = base / kFanIn + t;  // parent (global index) this thread makes
    const unsigned count = t < (B >> (2 * l)) ? children(kFanIn * p, nl) : 0u;
    if (count) {
      u32x4 c[kFanIn];
#pragma unroll
      for (int i = 0; i < kFanIn; ++i) c[i] = nodes[kFanIn * t + i];
      d = md5_node(c, count);
    }
    __syncthreads();
    base /= kFanIn;
    nl = (nl + kFanIn - 1) / kFanIn;
  }
  if (t == 0) out[blockIdx.x] = d;
}

template __global__ void md5_fold_kernel<64>(const u32x4*, unsigned long long, int, u32x4*);
template __global__ void md5_fold_kernel<256>(const u32x4*, unsigned long long, int, u32x4*);

static unsigned long long n_chunks(size_t nbytes, uint32_t chunk_bytes) {
  return nbytes == 0 ? 1ull : (nbytes + chunk_bytes - 1) / chunk_bytes;
}

// Levels left until one node, above a level of n.
static int levels_to_root(unsigned long long n) {
  int f = 0;
  for (; n > 1; ++f) n = (n + kFanIn - 1) / kFanIn;
  return f;
}

void md5_chunks(const void* src, size_t nbytes, uint32_t chunk_bytes, void* digests,
                hipStream_t stream) {
  if (chunk_bytes == 0 || chunk_bytes % 64)
    throw std::invalid_argument("md5_chunks: chunk_bytes must be a positive multiple of 64");
  if (reinterpret_cast<uintptr_t>(src) % 16)
    throw std::invalid_argument("md5_chunks: src must be 16-byte aligned");
  const unsigned long long nchunks = n_chunks(nbytes, chunk_bytes);
  // Whole groups of 64 full chunks take the coalesced kernel; the rest (and other chunk sizes)
  // the one-lane-per-chunk kernel on the remaining bytes.
  unsigned long long ngroups = 0;
  if (chunk_bytes % 128 == 0) ngroups = (nbytes / chunk_bytes) / kWaveChunks;
  if (ngroups) {
    const unsigned waves_per_block = kMd5Block / 64;
    const unsigned grid = static_cast<unsigned>((ngroups + waves_per_block - 1) / waves_per_block);
    hipLaunchKernelGGL(md5_chunks_coalesced_kernel, dim3(grid), dim3(kMd5Block), 0, stream,
                       static_cast<const unsigned char*>(src), chunk_bytes, ngroups, static_cast<u32x4*>(digests));
    TK8S_HIP_CHECK(hipGetLastError());
  }
  const unsigned long long done = ngroups * kWaveChunks;
  if (done >= nchunks && nbytes) return;
  const size_t off = static_cast<size_t>(done) * chunk_bytes;
  const unsigned long long rest = nchunks - done;
  const unsigned grid = static_cast<unsigned>((rest + kMd5Block - 1) / kMd5Block);
  hipLaunchKernelGGL(md5_chunks_kernel, dim3(grid), dim3(kMd5Block), 0, stream,
                     static_cast<const unsigned char*>(src) + off, static_cast<unsigned long long>(nbytes - off),
                     chunk_bytes, rest, static_cast<u32x4*>(digests) + done);
  TK8S_HIP_CHECK(hipGetLastError());
}

size_t md5_tree_workspace(size_t nbytes, uint32_t chunk_bytes) {
  if (chunk_bytes == 0 || chunk_bytes % 64)
    throw std::invalid_argument("md5_tree_workspace: chunk_bytes must be a positive multiple of 64");
  return static_cast<size_t>(n_chunks(nbytes, chunk_bytes)) * 16;
}

// The fold launches over a level of n nodes at `in`, ending with the root in out16.
template <int B>
static void fold(const void* in, unsigned long long n, void* ws_a, void* ws_b, void* out16, hipStream_t stream) {
  constexpr int kMax = B == 64 ? 4 : B == 256 ? 5 : 0;
  static_assert(kMax, "fold block: 64 or 256 threads");
  void* bufs[2] = {ws_b, ws_a};
  for (int launch = 0; n > 1; ++launch) {
    const int left = levels_to_root(n), levels = left < kMax ? left : kMax;
    void* dst = levels == left ? out16 : bufs[launch & 1];
    const unsigned long long parents = (n + kFanIn - 1) / kFanIn;
    const unsigned grid = static_cast<unsigned>((parents + B - 1) / B);
    hipLaunchKernelGGL(md5_fold_kernel<B>, dim3(grid), dim3(B), 0, stream, static_cast<const u32x4*>(in), n, levels,
                       static_cast<u32x4*>(dst));
    TK8S_HIP_CHECK(hipGetLastError());
    n = grid;  // one node per block
    in = dst;
  }
}

void md5_tree(const void* src, size_t nbytes, uint32_t chunk_bytes, void* ws_a, void* ws_b,
              void* out16, hipStream_t stream) {
  const unsigned long long n = n_chunks(nbytes, chunk_bytes);
  if (n == 1) {  // one chunk: its plain MD5
    md5_chunks(src, nbytes, chunk_bytes, out16, stream);
    return;
  }
  md5_chunks(src, nbytes, chunk_bytes, ws_a, stream);
  fold<kFoldBlock>(ws_a, n, ws_a, ws_b, out16, stream);
}

}  // namespace tk8s
