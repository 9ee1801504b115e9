// tk8s-gpujail: run a pod's command so that it can open only the GPUs it was allocated.
//
//   tk8s-gpujail [--allow-render M]... [--dri-root DIR] [--hide-topology [--allow-node N]...
//                [--kfd-root DIR]] [--best-effort] -- CMD ARGS...
//   tk8s-gpujail --probe            (prints {"landlock_abi": N, ...}; exit 0 when usable)
//
// The reference ran every workload in a Docker container (ansible/roles/rancherhost/tasks/
// main.yml:26-34, dockersetup), whose device cgroup decides which /dev nodes a container may
// open. tk8s pods are processes of the node agent, and HIP_VISIBLE_DEVICES alone is advice a pod
// can clear. This jail makes it a kernel rule, with no privileges needed (the node agent and the
// GPU tier run as an ordinary user; user namespaces are off on the GPU hosts):
//
//   Landlock (kernel >= 5.13) restricts READ_FILE / WRITE_FILE for this process and everything it
//   starts, permanently. Granted: every path of the file system EXCEPT the DRM device nodes of the
//   GPUs that are not the pod's (/dev/dri/renderD<m>, card*). Landlock rules can only grant, so
//   the exceptions are carved out by granting each sibling along the way from / to them.
//
// ROCr's thunk skips a GPU whose render node it cannot open (as in a container given a subset of
// /dev/dri), so the pod's runtime sees exactly its GPUs whatever its *_VISIBLE_DEVICES say; and
// without the render node no process can acquire a GPU VM for that device through /dev/kfd, i.e.
// map its memory or create queues on it. The KFD topology in sysfs stays readable, as in a
// container: measured on the MI355X box with ROCm 7.2 (profiles/r3_gpujail/), denying a GPU's
// topology node makes the thunk fail its whole start (HSA_STATUS_ERROR_OUT_OF_RESOURCES) even for
// the allowed GPUs, while a denied render node is skipped cleanly. --hide-topology adds the
// topology nodes anyway (for runtimes that skip them).
//
// The child's environment gets TK8S_GPU_ISOLATION=landlock:abi<N> (or none:<why> under
// --best-effort when Landlock is unavailable; without --best-effort that is exit 125).
#include <dirent.h>
#include <fcntl.h>
#include <linux/landlock.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <set>
#include <string>
#include <vector>

namespace {

long ll_create(const landlock_ruleset_attr* attr, size_t size, unsigned flags) {
  return syscall(SYS_landlock_create_ruleset, attr, size, flags);
}
long ll_add(int fd, landlock_rule_type type, const void* attr, unsigned flags) {
  return syscall(SYS_landlock_add_rule, fd, type, attr, flags);
}
long ll_restrict(int fd, unsigned flags) { return syscall(SYS_landlock_restrict_self, fd, flags); }

int landlock_abi() {
  const long v = ll_create(nullptr, 0, LANDLOCK_CREATE_RULESET_VERSION);
  return v < 0 ? -errno : static_cast<int>(v);
}

std::string real(const std::string& p) {
  char buf[PATH_MAX];
  return realpath(p.c_str(), buf) ? std::string(buf) : std::string();
}

bool is_cpu_node(const std::string& node_dir) {
  std::ifstream f(node_dir + "/properties");
  if (!f) return false;  // unreadable: not ours to open either
  std::string k;
  long long v;
  while (f >> k >> v)
    if (k == "simd_count") return v == 0;
  return false;
}

std::vector<std::string> list_dir(const std::string& d) {
  std::vector<std::string> out;
  if (DIR* dir = opendir(d.c_str())) {
    while (dirent* e = readdir(dir)) {
      if (std::strcmp(e->d_name, ".") && std::strcmp(e->d_name, "..")) out.emplace_back(e->d_name);
    }
    closedir(dir);
  }
  return out;
}

// True if `a` is `b` or one of b's ancestors.
bool covers(const std::string& a, const std::string& b) {
  if (a == "/") return true;
  return b == a || (b.size() > a.size() && b.compare(0, a.size(), a) == 0 && b[a.size()] == '/');
}

struct Jail {
  int fd = -1;
  int rules = 0;
  const __u64 rights = LANDLOCK_ACCESS_FS_READ_FILE | LANDLOCK_ACCESS_FS_WRITE_FILE;

  void grant(const std::string& path) {
    const int pfd = open(path.c_str(), O_PATH | O_CLOEXEC | O_NOFOLLOW);
    if (pfd < 0) return;  // vanished meanwhile: nothing to grant
    landlock_path_beneath_attr pb{};
    pb.allowed_access = rights;
    pb.parent_fd = pfd;
    struct stat st {};
    if (fstat(pfd, &st) == 0 && S_ISLNK(st.st_mode)) {  // a link itself: opening through it checks the target
      close(pfd);
      return;
    }
    if (ll_add(fd, LANDLOCK_RULE_PATH_BENEATH, &pb, 0) == 0) ++rules;
    close(pfd);
  }

  // Grant everything under `dir` except the `deny` paths (all beneath `dir`).
  void grant_except(const std::string& dir, const std::set<std::string>& deny) {
    for (const auto& name : list_dir(dir)) {
      const std::string p = (dir == "/" ? "" : dir) + "/" + name;
      bool denied = false, ancestor = false;
      for (const auto& d : deny) {
        if (d == p) denied = true;
        else if (covers(p, d)) ancestor = true;
      }
      if (denied) continue;
      if (ancestor) {
        grant_except(p, deny);
      } else {
        grant(p);
      }
    }
  }
};

int usage() {
  std::fprintf(stderr,
               "usage: tk8s-gpujail [--allow-render M]... [--dri-root DIR] [--hide-topology [--allow-node N]...\n"
               "                    [--kfd-root DIR]] [--best-effort] -- CMD ARGS...\n       tk8s-gpujail --probe\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  std::set<long> allow_nodes, allow_render;
  std::string kfd_root = "/sys/devices/virtual/kfd/kfd/topology/nodes", dri_root = "/dev/dri";
  bool best_effort = false, probe = false, hide_topology = false;
  int i = 1;
  for (; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) throw std::invalid_argument(a + " needs a value");
      return argv[++i];
    };
    try {
      if (a == "--") { ++i; break; }
      if (a == "--allow-node") allow_nodes.insert(std::stol(next()));
      else if (a == "--allow-render") allow_render.insert(std::stol(next()));
      else if (a == "--kfd-root") kfd_root = next();
      else if (a == "--dri-root") dri_root = next();
      else if (a == "--best-effort") best_effort = true;
      else if (a == "--hide-topology") hide_topology = true;
      else if (a == "--probe") probe = true;
      else return usage();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "tk8s-gpujail: %s\n", e.what());
      return usage();
    }
  }
  const int abi = landlock_abi();
  if (probe) {
    std::printf("{\"landlock_abi\": %d, \"usable\": %s%s}\n", abi > 0 ? abi : 0, abi > 0 ? "true" : "false",
                abi > 0 ? "" : (std::string(", \"error\": \"") + std::strerror(-abi) + "\"").c_str());
    return abi > 0 ? 0 : 1;
  }
  if (i >= argc) return usage();

  std::string mode;
  if (abi <= 0) {
    mode = std::string("none:landlock unavailable (") + std::strerror(-abi) + ")";
    if (!best_effort) {
      std::fprintf(stderr, "tk8s-gpujail: %s\n", mode.c_str());
      return 125;
    }
  } else {
    // what this pod must not open: the other GPUs' topology nodes and DRM device nodes
    std::set<std::string> deny;
    const std::string kroot = hide_topology ? real(kfd_root) : std::string();
    if (!kroot.empty()) {
      for (const auto& n : list_dir(kroot)) {
        char* end = nullptr;
        const long id = std::strtol(n.c_str(), &end, 10);
        if (end == n.c_str() || *end) continue;
        if (allow_nodes.count(id) || is_cpu_node(kroot + "/" + n)) continue;
        deny.insert(kroot + "/" + n);
      }
    }
    const std::string droot = real(dri_root);
    if (!droot.empty()) {
      for (const auto& n : list_dir(droot)) {
        if (n == "by-path") continue;  // links only: opening through them checks their targets
        if (n.rfind("renderD", 0) == 0 && allow_render.count(std::strtol(n.c_str() + 7, nullptr, 10))) continue;
        deny.insert(droot + "/" + n);
      }
    }
    Jail j;
    landlock_ruleset_attr attr{};
    attr.handled_access_fs = j.rights;
    j.fd = static_cast<int>(ll_create(&attr, sizeof(attr), 0));
    if (j.fd < 0) {
      mode = std::string("none:landlock_create_ruleset: ") + std::strerror(errno);
    } else {
      if (!deny.empty()) j.grant_except("/", deny);
      else j.grant("/");
      if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0) != 0 || ll_restrict(j.fd, 0) != 0) {
        mode = std::string("none:landlock_restrict_self: ") + std::strerror(errno);
      } else {
        mode = "landlock:abi" + std::to_string(abi) + ":denied=" + std::to_string(deny.size());
      }
      close(j.fd);
    }
    if (mode.rfind("none:", 0) == 0 && !best_effort) {
      std::fprintf(stderr, "tk8s-gpujail: %s\n", mode.c_str());
      return 125;
    }
  }
  setenv("TK8S_GPU_ISOLATION", mode.c_str(), 1);
  execvp(argv[i], argv + i);
  std::fprintf(stderr, "tk8s-gpujail: exec %s: %s\n", argv[i], std::strerror(errno));
  return 127;
}
