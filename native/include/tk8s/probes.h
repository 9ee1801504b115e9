// Node-validation probes built on the tk8s kernels. Every entry point returns one JSON object
// (std::string) so the CLI tools, the pybind11 module and the node agent share one format.
//
// Reference anchors: N1 gpuinfo replaces the docker version probe of
// ansible/roles/dockersetup/tasks/main.yml:2-4; N4/N5 are the GPU analogues of
// docs/benchmarks.md:8-12; N7 extends the per-node health checks of setup.sh:71-73.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

#include "tk8s/kernels.h"

namespace tk8s {

// N1: device discovery. {"ok":..,"device_count":n,"runtime_version":..,"devices":[..],"links":[[..]]}
// Never throws: a host without a usable GPU yields ok=false and an "error" string.
std::string gpuinfo_json(bool with_links = true);

// N4: write `bytes` of `value` `iters` times (after one untimed warm-up), verify the result.
std::string hbm_write_probe(size_t bytes, int iters, StoreMode mode, int device, uint32_t value = 0);

// N5: Philox-fill `bytes` then MD5-tree them `iters` times; reports the digest (hex) so a host
// oracle can check it, plus fill and hash throughput.
std::string md5_probe(size_t bytes, uint32_t chunk_bytes, uint64_t seed, int iters, int device);

// N7: copy bandwidth from device src to device dst (src == dst: local D2D copy). Kernel pull
// over xGMI (peer access enabled) and the SDMA engine path (hipMemcpyPeerAsync).
// dma: also time the SDMA-engine path (hipMemcpyPeerAsync) for a peer copy.
std::string copy_probe(int src_device, int dst_device, size_t bytes, int iters, bool dma = true);

// The local probes share one grow-on-demand device allocation per device (see probes.cpp);
// free them (e.g. from a long-lived process once validation is done).
void release_probe_scratch();

// Size that allocation once, up front, for a run of the local probes with these sizes (0 = the
// probe is skipped): growing it between probes costs a hipFree, which synchronises the device.
void reserve_probe_scratch(int device, size_t hbm_bytes, size_t md5_bytes, uint32_t chunk_bytes, size_t copy_bytes);

}  // namespace tk8s
