// tk8s-gpuinfo: N1 device discovery for the amd.com/gpu device plugin. Prints one JSON object.
//   tk8s-gpuinfo [--no-links]
#include <cstdio>

#include "args.h"
#include "cachewalk.h"
#include "tk8s/probes.h"

int main(int argc, char** argv) {
  tk8s::cachewalk::configure();  // before the HIP runtime starts (cachewalk.h)
  try {
    tk8s::Args a(argc, argv);
    const std::string j = tk8s::gpuinfo_json(!a.has("no-links"));
    std::printf("%s\n", j.c_str());
    return j.find("\"ok\":true") != std::string::npos ? 0 : 3;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "tk8s-gpuinfo: %s\n", e.what());
    return 2;
  }
}
