// Host-side launch API for the tk8s validation kernels (gfx950 / CDNA4).
//
// Kernel inventory:
//   N4  hbm_fill          — HBM write-bandwidth probe (GPU analogue of docs/benchmarks.md:8-9,
//                           "pipes a gigabyte of zeros").
//   N5  philox_fill +     — on-device random data + chunked MD5 tree hash (GPU analogue of
//       md5_tree            docs/benchmarks.md:11-12, "fetches random numbers and md5 hashes them").
//   N6  ar_fill/ar_check  — all-reduce pattern generator + max-abs-error checker.
//   N7  stream_copy       — device copy kernel used for local and xGMI peer-pull bandwidth probes.
//
// All launchers are asynchronous on `stream` and never allocate, synchronise or free, so a
// caller may capture them into a hipGraph.
#pragma once

#include <cstddef>
#include <cstdint>

#include <hip/hip_runtime.h>

namespace tk8s {

enum class StoreMode : int { kNonTemporal = 0, kPlain = 1 };
enum class DType : int { kF32 = 0, kBF16 = 1 };

// Number of workgroups for a grid-stride streaming kernel on the current device
// (CU count x blocks_per_cu, cached per device).
int streaming_grid(int blocks_per_cu = 8);

// N4: write `nbytes` (multiple of 16) of the 32-bit pattern `value` to dst.
void hbm_fill(void* dst, size_t nbytes, uint32_t value, StoreMode mode, hipStream_t stream);

// Counts 32-bit words in src (nbytes multiple of 16) that differ from `value`; *bad_words must
// point to device memory that the caller zeroed.
void verify_fill(const void* src, size_t nbytes, uint32_t value, unsigned long long* bad_words,
                 hipStream_t stream);

// N5: fill dst with Philox4x32-10 output (counter = 16-byte block index, key = seed).
// nbytes must be a multiple of 16.
void philox_fill(void* dst, size_t nbytes, uint64_t seed, hipStream_t stream);

// N5: one level of the MD5 tree: digest of every `chunk_bytes` chunk of src (last chunk may be
// partial) into `digests` (16 bytes each). chunk_bytes must be a multiple of 64.
void md5_chunks(const void* src, size_t nbytes, uint32_t chunk_bytes, void* digests,
                hipStream_t stream);

// Number of digest bytes needed as workspace by md5_tree for `nbytes` input (two ping-pong
// buffers of this size).
size_t md5_tree_workspace(size_t nbytes, uint32_t chunk_bytes);

// N5: MD5 tree hash. Level 0 hashes chunks of src; each next level hashes the concatenated
// digests of the previous one, until one digest remains. Writes 16 bytes to out16 (device).
// ws_a/ws_b: device workspaces of md5_tree_workspace() bytes each.
void md5_tree(const void* src, size_t nbytes, uint32_t chunk_bytes, void* ws_a, void* ws_b,
              void* out16, hipStream_t stream);

// N6: buf[i] = (rank + 1) + (i % 7) in dtype.
void ar_fill(void* buf, size_t count, int rank, DType dtype, hipStream_t stream);

// N6: compares buf (after a sum all-reduce over nranks ranks filled by ar_fill) with the exact
// expected value nranks*(nranks+1)/2 + nranks*(i % 7). Writes max |err| as float bits into
// *max_err_bits (device, caller-zeroed) and the number of elements with |err| > tol into
// *bad (device, caller-zeroed).
void ar_check(const void* buf, size_t count, int nranks, DType dtype, float tol,
              unsigned int* max_err_bits, unsigned long long* bad, hipStream_t stream);

// N7: dst[i] = src[i] for nbytes (multiple of 16). src may live on a peer GPU (xGMI pull).
void stream_copy(void* dst, const void* src, size_t nbytes, hipStream_t stream);

// Fault injection (TK8S_FAULTS "...hang@<phase>" on a GPU phase, failfast.h): enqueue on `stream`
// a one-wave kernel that spins until gpu_stall_release() (common.h) is called or `max_s` seconds
// of GPU wall clock pass -- so a stalled queue always drains, whoever forgets to release it.
// Everything queued behind it on `stream` waits: a hung collective or pull, made on purpose.
void gpu_stall(hipStream_t stream, double max_s);

}  // namespace tk8s
