// N2 core: xGMI-aware GPU set selection for the amd.com/gpu device plugin.
//
// Pure C++ (no HIP dependency) so the node agent can load it without touching the GPU. The
// reference joins hosts to Rancher without any device awareness (ansible/roles/rancherhost/
// tasks/main.yml:26-34); here a pod asking for k of a node's GPUs gets the k-set with the best
// pairwise connectivity: maximise the weakest link first (a fully connected xGMI set), then the
// total link score, then prefer the lowest indices for determinism.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace tk8s {

// Link score for one directed GPU pair. type: "self","xgmi","pcie",... hops >= 0.
int link_weight(const std::string& type, int hops);

struct AllocationResult {
  std::vector<int> devices;  // sorted ascending
  int min_link = 0;          // weakest pairwise weight inside the set (0 for singletons)
  int64_t total_link = 0;    // sum of pairwise weights inside the set
  bool exhaustive = true;    // false when the greedy fallback was used
};

// weights: n*n row-major matrix (weights[i*n+j]). available/must_include: device indices.
// Throws std::invalid_argument on inconsistent inputs.
AllocationResult preferred_allocation(int n, const std::vector<int>& weights,
                                      const std::vector<int>& available,
                                      const std::vector<int>& must_include, int size);

}  // namespace tk8s
