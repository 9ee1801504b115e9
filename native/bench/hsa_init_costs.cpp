// Development microbenchmark: where does a HIP process's ~200 ms start go on gfx950? Times the
// ROCr (HSA) layer underneath HIP directly: hsa_init, agent discovery, and hardware-queue
// creation at several ring sizes (a HIP stream is one such queue). Prints one JSON object.
//   g++ -O2 -std=c++17 -I/opt/rocm/include hsa_init_costs.cpp -L/opt/rocm/lib -lhsa-runtime64 \
//       -Wl,-rpath,/opt/rocm/lib -o /tmp/hsa_init_costs
#include <hsa/hsa.h>

#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double, std::milli>(b - a).count();
}

static hsa_status_t collect_gpu(hsa_agent_t agent, void* data) {
  hsa_device_type_t type;
  if (hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (type == HSA_DEVICE_TYPE_GPU) static_cast<std::vector<hsa_agent_t>*>(data)->push_back(agent);
  return HSA_STATUS_SUCCESS;
}

int main(int argc, char** argv) {
  const auto t0 = clk::now();
  if (argc > 2 && std::string(argv[1]) == "hold") {  // keep a live GPU process for N seconds
    if (hsa_init() != HSA_STATUS_SUCCESS) return 1;
    std::printf("{\"hold_init_ms\": %.3f}\n", ms(t0, clk::now()));
    std::fflush(stdout);
    usleep(static_cast<useconds_t>(std::atof(argv[2]) * 1e6));
    hsa_shut_down();
    return 0;
  }
  if (hsa_init() != HSA_STATUS_SUCCESS) {
    std::printf("{\"ok\": false, \"error\": \"hsa_init\"}\n");
    return 1;
  }
  const auto t1 = clk::now();
  std::vector<hsa_agent_t> gpus;
  hsa_iterate_agents(collect_gpu, &gpus);
  const auto t2 = clk::now();
  std::string queues;
  if (!gpus.empty()) {
    uint32_t max_size = 0;
    hsa_agent_get_info(gpus[0], HSA_AGENT_INFO_QUEUE_MAX_SIZE, &max_size);
    for (uint32_t size : {64u, 1024u, 16384u, 64u}) {
      if (size > max_size) continue;
      hsa_queue_t* q = nullptr;
      const auto a = clk::now();
      const hsa_status_t st = hsa_queue_create(gpus[0], size, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr,
                                               UINT32_MAX, UINT32_MAX, &q);
      const auto b = clk::now();
      if (st == HSA_STATUS_SUCCESS) hsa_queue_destroy(q);
      const auto c = clk::now();
      char buf[160];
      std::snprintf(buf, sizeof buf, "%s{\"size\": %u, \"create_ms\": %.3f, \"destroy_ms\": %.3f, \"ok\": %s}",
                    queues.empty() ? "" : ", ", size, ms(a, b), ms(b, c), st == HSA_STATUS_SUCCESS ? "true" : "false");
      queues += buf;
    }
  }
  const auto t3 = clk::now();
  hsa_shut_down();
  const auto t4 = clk::now();
  std::printf("{\"ok\": true, \"gpus\": %zu, \"hsa_init_ms\": %.3f, \"iterate_agents_ms\": %.3f, \"queues\": [%s], "
              "\"shut_down_ms\": %.3f, \"total_ms\": %.3f}\n",
              gpus.size(), ms(t0, t1), ms(t1, t2), queues.c_str(), ms(t3, t4), ms(t0, t4));
  return 0;
}
