// tk8s-smi: N1 GPU health and telemetry through AMD SMI (no HIP runtime, no KFD process).
//   tk8s-smi [--no-links]
// Exit status: 0 every GPU healthy, 1 a GPU reports uncorrectable/deferred ECC errors,
// 3 no GPU (or no amdgpu driver). The node agent runs it periodically for device health.
#include <cstdio>

#include "args.h"
#include "tk8s/smi.h"

int main(int argc, char** argv) {
  try {
    tk8s::Args a(argc, argv);
    const std::string j = tk8s::smi_health_json(!a.has("no-links"));
    std::printf("%s\n", j.c_str());
    if (j.find("\"ok\":true") == std::string::npos) return 3;
    return j.find("\"healthy\":true") != std::string::npos ? 0 : 1;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "tk8s-smi: %s\n", e.what());
    return 2;
  }
}
