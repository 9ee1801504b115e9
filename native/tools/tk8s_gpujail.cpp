// tk8s-gpujail: run a pod's command so that it can open only the GPUs it was allocated, and none
// of the node's credentials.
//
//   tk8s-gpujail [--allow-render M]... [--dri-root DIR] [--hide-topology [--allow-node N]...
//                [--kfd-root DIR]] [--deny PATH]... [--read-only PATH]... [--allow PATH]...
//                [--scope-signals] [--cgroup-procs FILE]... [--cpus LIST] [--rlimit-data BYTES] [--best-effort] -- CMD ARGS...
//   tk8s-gpujail --probe            (prints {"landlock_abi": N, ...}; exit 0 when usable)
//   tk8s-gpujail [policy options] --plan   (prints the rules it would add, one JSON line each)
//
// The reference ran every workload in a Docker container (ansible/roles/rancherhost/tasks/
// main.yml:26-34, dockersetup), whose device cgroup decides which /dev nodes a container may
// open. tk8s process pods are children of the node agent, and HIP_VISIBLE_DEVICES alone is
// advice a pod can clear. This jail makes it a kernel rule with no privilege (the node agent and
// the GPU tier run as an ordinary user; user namespaces are off on the GPU hosts): Landlock
// denies opening the render nodes of every GPU the pod does not hold, and the --deny paths (the
// node's state: kubeconfig, keys, other pods' tokens) but the --allow paths beneath them
// (gpujail.h has the policy). Image pods get the same jail inside tk8s-container. First of all
// it joins the pod's cgroups and CPUs (--cgroup-procs, --cpus: agent/resources.py), so every
// process of the pod starts inside its limits.
//
// The child's environment gets TK8S_GPU_ISOLATION=landlock:abi<N>:denied=<k> (or none:<why>
// under --best-effort when Landlock is unavailable; without --best-effort that is exit 125).
#include <cstdio>

#include "gpujail.h"

namespace {

int usage() {
  std::fprintf(stderr,
               "usage: tk8s-gpujail [--allow-render M]... [--dri-root DIR] [--hide-topology [--allow-node N]...\n"
               "                    [--kfd-root DIR]] [--deny PATH]... [--read-only PATH]... [--allow PATH]...\n"
               "                    [--scope-signals] [--cgroup-procs FILE]... [--cpus LIST] [--rlimit-data BYTES] [--best-effort]\n"
               "                    -- CMD ARGS...\n       tk8s-gpujail --probe\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  tk8s::jail::Policy policy;
  bool best_effort = false, probe = false, show_plan = false;
  int i = 1;
  for (; i < argc; ++i) {
    const std::string a = argv[i];
    try {
      if (a == "--") {
        ++i;
        break;
      }
      if (tk8s::jail::parse_option(policy, argc, argv, i)) continue;
      if (a == "--best-effort") best_effort = true;
      else if (a == "--probe") probe = true;
      else if (a == "--plan") show_plan = true;
      else return usage();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "tk8s-gpujail: %s\n", e.what());
      return usage();
    }
  }
  if (probe) {
    const int abi = tk8s::jail::abi();
    const std::string err = abi > 0 ? "" : std::string(", \"error\": \"") + std::strerror(-abi) + "\"";
    std::printf("{\"landlock_abi\": %d, \"usable\": %s, \"signal_scoping\": %s%s}\n", abi > 0 ? abi : 0,
                abi > 0 ? "true" : "false", abi >= 6 ? "true" : "false", err.c_str());
    return abi > 0 ? 0 : 1;
  }
  if (show_plan) {  // the rules, as JSON lines {"path": ..., "access": "r"|"rw"}; nothing applied
    for (const auto& [path, acc] : tk8s::jail::plan(policy)) {
      std::string esc;
      for (char c : path) {
        if (c == '"' || c == '\\') esc += '\\';
        esc += c;
      }
      std::printf("{\"path\": \"%s\", \"access\": \"%s\"}\n", esc.c_str(),
                  acc == tk8s::jail::Access::kRead ? "r" : "rw");
    }
    return 0;
  }
  if (i >= argc) return usage();
  if (const std::string why = tk8s::jail::join_limits(policy); !why.empty()) {
    std::fprintf(stderr, "tk8s-gpujail: %s\n", why.c_str());
    return 125;
  }
  const std::string mode = tk8s::jail::apply(policy);
  if (mode.rfind("none:", 0) == 0 && !best_effort) {
    std::fprintf(stderr, "tk8s-gpujail: %s\n", mode.c_str());
    return 125;
  }
  setenv("TK8S_GPU_ISOLATION", mode.c_str(), 1);
  execvp(argv[i], argv + i);
  std::fprintf(stderr, "tk8s-gpujail: exec %s: %s\n", argv[i], std::strerror(errno));
  return 127;
}
