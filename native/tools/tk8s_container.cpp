// tk8s-container: run a pod's container from an image root file system (agent/images.py).
//
//   tk8s-container --rootfs DIR [--upper DIR] [--workdir D] [--hostname H] [--pid-ns]
//                  [--bind|--bind-ro SRC:DST]... [jail options, gpujail.h] [--no-gpu-jail] -- ARGV...
//   tk8s-container --exec-in PID [--workdir D] [jail options] -- ARGV...   (kubectl exec)
//   tk8s-container --probe      {"usable": bool, "how": "root"|"userns", "error": ...}
//
// The reference's workloads ran in Docker containers (ansible/roles/rancherhost/tasks/main.yml:
// 26-34, dockersetup/tasks/main.yml:42-46). This is the part of a container runtime a tk8s node
// needs, with no daemon:
//
//   1. a mount namespace (and a user namespace when not root; a PID namespace with --pid-ns),
//   2. the image's root file system, as an overlay whose upper layer is the pod's own (--upper:
//      writes stay with the pod, the unpacked image stays pristine; the image itself when the
//      kernel refuses the overlay), with the host's /dev, /sys and /proc inside -- a GPU pod
//      needs /dev/kfd, its render node, /dev/shm (RCCL) and the KFD topology -- plus --bind mounts
//      (e.g. the host's /opt/rocm, like the kubeadm RCCL Job's hostPath),
//   3. chroot + chdir, then the GPU jail of gpujail.h built on the container's own paths (a
//      rule on a host directory above the root file system would grant everything bound under
//      it), then exec of the container's command with the environment it was given.
//
// GPU pods keep the host PID namespace (HIP/RCCL IPC identifies peers by pid). Exit status: the
// command's; 125 = the container could not be set up (message on stderr); 127 = exec failed.
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mount.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "gpujail.h"

namespace {

[[noreturn]] void die(const std::string& what) {
  std::fprintf(stderr, "tk8s-container: %s: %s\n", what.c_str(), std::strerror(errno));
  std::fflush(stderr);
  _exit(125);
}

void write_file(const std::string& path, const std::string& text) {
  const int fd = open(path.c_str(), O_WRONLY | O_CLOEXEC);
  if (fd < 0 || write(fd, text.data(), text.size()) != static_cast<ssize_t>(text.size())) die("write " + path);
  close(fd);
}

void mkdirs(const std::string& path, bool as_file = false) {
  std::string cur;
  size_t pos = 0;
  while (pos != std::string::npos) {
    pos = path.find('/', pos + 1);
    cur = path.substr(0, pos);
    if (cur.empty()) continue;
    if (pos == std::string::npos && as_file) {
      const int fd = open(cur.c_str(), O_CREAT | O_WRONLY | O_CLOEXEC, 0644);
      if (fd >= 0) close(fd);
    } else {
      mkdir(cur.c_str(), 0755);
    }
  }
}

void bind(const std::string& src, const std::string& dst, bool read_only = false) {
  struct stat st {};
  if (stat(src.c_str(), &st) != 0) die("bind source " + src);
  mkdirs(dst, !S_ISDIR(st.st_mode));
  if (mount(src.c_str(), dst.c_str(), nullptr, MS_BIND | MS_REC, nullptr) != 0) die("bind " + src + " -> " + dst);
  // a bind mount takes MS_RDONLY only on a remount of itself
  if (read_only && mount(nullptr, dst.c_str(), nullptr, MS_BIND | MS_REMOUNT | MS_RDONLY, nullptr) != 0)
    die("read-only bind " + dst);
}

// Enter the namespaces: a user namespace mapping this uid/gid to itself when not root (it gives
// the capabilities mount and chroot need, inside it only).
std::string enter(bool pid_ns) {
  const uid_t uid = geteuid();
  const gid_t gid = getegid();
  // its own UTS namespace too: the pod's hostname is set in there, never on the host
  int flags = CLONE_NEWNS | CLONE_NEWUTS | (pid_ns ? CLONE_NEWPID : 0);
  if (uid != 0) flags |= CLONE_NEWUSER;
  if (unshare(flags) != 0) die(uid == 0 ? "unshare(mount namespace)" : "unshare(user + mount namespaces)");
  if (uid != 0) {
    write_file("/proc/self/setgroups", "deny");
    write_file("/proc/self/uid_map", std::to_string(uid) + " " + std::to_string(uid) + " 1");
    write_file("/proc/self/gid_map", std::to_string(gid) + " " + std::to_string(gid) + " 1");
  }
  if (mount(nullptr, "/", nullptr, MS_REC | MS_PRIVATE, nullptr) != 0) die("make / private");
  return uid == 0 ? "root" : "userns";
}

int probe() {
  const pid_t pid = fork();
  if (pid == 0) {
    // quiet: the probe only asks whether the namespaces can be had
    const int devnull = open("/dev/null", O_WRONLY);
    if (devnull >= 0) dup2(devnull, 2);
    enter(false);
    _exit(0);
  }
  int st = 0;
  waitpid(pid, &st, 0);
  const bool ok = WIFEXITED(st) && WEXITSTATUS(st) == 0;
  std::printf("{\"usable\": %s, \"how\": \"%s\"%s}\n", ok ? "true" : "false", geteuid() == 0 ? "root" : "userns",
              ok ? "" : ", \"error\": \"no mount namespace for this user (not root, and user namespaces are off)\"");
  return ok ? 0 : 1;
}

// --exec-in PID: run a command inside a running image pod (kubectl exec): its user, mount and
// PID namespaces, its root, the same GPU jail. PID is the pod's tk8s-container process; with a
// PID namespace that process only waits, and the container is its child.
int exec_in(pid_t pid, const std::string& workdir, const tk8s::jail::Policy& policy, bool jail, char** argv) {
  auto root_of = [](pid_t p) {
    char buf[PATH_MAX];
    const ssize_t n = readlink(("/proc/" + std::to_string(p) + "/root").c_str(), buf, sizeof(buf) - 1);
    return n > 0 ? std::string(buf, n) : std::string();
  };
  if (root_of(pid) == "/") {  // the relaying parent: the container is its first child
    std::ifstream kids("/proc/" + std::to_string(pid) + "/task/" + std::to_string(pid) + "/children");
    pid_t child = 0;
    if (!(kids >> child) || child <= 0) {
      errno = ESRCH;
      die("no container process under pid " + std::to_string(pid));
    }
    pid = child;
  }
  const std::string proc = "/proc/" + std::to_string(pid);
  const int rootfd = open((proc + "/root").c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (rootfd < 0) die("open " + proc + "/root");
  auto join = [&](const char* ns, int type) {
    struct stat mine {}, theirs {};
    if (stat((proc + "/ns/" + ns).c_str(), &theirs) != 0) die(std::string("stat ns ") + ns);
    if (stat((std::string("/proc/self/ns/") + ns).c_str(), &mine) == 0 && mine.st_ino == theirs.st_ino) return;
    const int fd = open((proc + "/ns/" + ns).c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0 || setns(fd, type) != 0) die(std::string("setns ") + ns);
    close(fd);
  };
  join("user", CLONE_NEWUSER);
  join("uts", CLONE_NEWUTS);
  join("mnt", CLONE_NEWNS);
  join("pid", CLONE_NEWPID);
  if (fchdir(rootfd) != 0 || chroot(".") != 0 || chdir("/") != 0) die("enter the container's root");
  close(rootfd);
  const pid_t child = fork();  // a joined PID namespace takes effect for children only
  if (child < 0) die("fork");
  if (child > 0) {
    for (int s : {SIGTERM, SIGINT, SIGHUP}) signal(s, [](int) {});
    int st = 0;
    while (waitpid(child, &st, 0) < 0 && errno == EINTR) {
    }
    return WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
  }
  prctl(PR_SET_PDEATHSIG, SIGKILL);
  std::string mode = "none:--no-gpu-jail";
  if (jail) {
    mode = tk8s::jail::apply(policy);
    if (mode.rfind("none:", 0) == 0) {
      std::fprintf(stderr, "tk8s-container: GPU jail: %s\n", mode.c_str());
      _exit(125);
    }
  }
  if (chdir(workdir.c_str()) != 0) die("chdir " + workdir);
  setenv("TK8S_GPU_ISOLATION", mode.c_str(), 1);
  execvp(argv[0], argv);
  std::fprintf(stderr, "tk8s-container: exec %s: %s\n", argv[0], std::strerror(errno));
  _exit(127);
}

int usage() {
  std::fprintf(stderr,
               "usage: tk8s-container --rootfs DIR [--upper DIR] [--workdir D] [--hostname H] [--pid-ns]\n"
               "                      [--bind|--bind-ro SRC:DST]... [--allow-render M]... [--no-gpu-jail] -- ARGV...\n"
               "       tk8s-container --exec-in PID [--workdir D] [--allow-render M]... -- ARGV...\n"
               "       tk8s-container --probe\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  std::string rootfs, upper, workdir = "/", hostname;
  struct Bind {
    std::string src, dst;
    bool read_only;
  };
  std::vector<Bind> binds;
  bool pid_ns = false, jail = true;
  pid_t exec_pid = 0;
  tk8s::jail::Policy policy;
  int i = 1;
  for (; i < argc; ++i) {
    const std::string a = argv[i];
    try {
      auto next = [&]() -> std::string {
        if (i + 1 >= argc) throw std::invalid_argument(a + " needs a value");
        return argv[++i];
      };
      if (a == "--") {
        ++i;
        break;
      }
      if (tk8s::jail::parse_option(policy, argc, argv, i)) continue;
      if (a == "--probe") return probe();
      if (a == "--rootfs") rootfs = next();
      else if (a == "--upper") upper = next();
      else if (a == "--workdir") workdir = next();
      else if (a == "--hostname") hostname = next();
      else if (a == "--pid-ns") pid_ns = true;
      else if (a == "--no-gpu-jail") jail = false;
      else if (a == "--exec-in") exec_pid = static_cast<pid_t>(std::stol(next()));
      else if (a == "--bind" || a == "--bind-ro") {
        const std::string v = next();
        const auto c = v.find(':');
        if (c == std::string::npos) throw std::invalid_argument(a + " needs SRC:DST");
        binds.push_back({v.substr(0, c), v.substr(c + 1), a == "--bind-ro"});
      } else {
        return usage();
      }
    } catch (const std::exception& e) {
      std::fprintf(stderr, "tk8s-container: %s\n", e.what());
      return usage();
    }
  }
  if (exec_pid > 0 && i < argc) return exec_in(exec_pid, workdir, policy, jail, argv + i);
  if (rootfs.empty() || i >= argc) return usage();
  rootfs = tk8s::jail::real(rootfs);
  if (rootfs.empty()) die("--rootfs");

  const std::string how = enter(pid_ns);
  if (pid_ns) {  // the command becomes pid 1 of its namespace; this process waits and relays
    const pid_t child = fork();
    if (child < 0) die("fork");
    if (child > 0) {
      for (int s : {SIGTERM, SIGINT, SIGHUP}) signal(s, [](int) {});  // reach the child through the group
      int st = 0;
      while (waitpid(child, &st, 0) < 0 && errno == EINTR) {
      }
      return WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
    }
    prctl(PR_SET_PDEATHSIG, SIGKILL);
  }
  std::string root = rootfs, fs_mode = "image";
  if (!upper.empty()) {  // the pod's writes go to its own layer
    const std::string up = upper + "/upper", work = upper + "/work", merged = upper + "/merged";
    mkdirs(up);
    mkdirs(work);
    mkdirs(merged);
    const std::string opts = "lowerdir=" + rootfs + ",upperdir=" + up + ",workdir=" + work;
    if (mount("overlay", merged.c_str(), "overlay", 0, opts.c_str()) == 0) {
      root = merged;
      fs_mode = "overlay";
    } else {
      fs_mode = std::string("image (overlay refused: ") + std::strerror(errno) + ")";
    }
  }
  bind("/dev", root + "/dev");
  bind("/sys", root + "/sys");
  if (pid_ns) {
    mkdirs(root + "/proc");
    if (mount("proc", (root + "/proc").c_str(), "proc", MS_NOSUID | MS_NODEV | MS_NOEXEC, nullptr) != 0)
      die("mount /proc");
  } else {
    bind("/proc", root + "/proc");
  }
  mkdirs(root + "/tmp");
  for (const auto& b : binds) bind(b.src, root + "/" + b.dst, b.read_only);
  if (!hostname.empty() && sethostname(hostname.c_str(), hostname.size()) != 0) die("sethostname");
  if (chroot(root.c_str()) != 0) die("chroot " + root);
  if (chdir("/") != 0) die("chdir /");
  std::string mode = "none:--no-gpu-jail";
  if (jail) {
    mode = tk8s::jail::apply(policy);  // on the container's own paths (see the header comment)
    if (mode.rfind("none:", 0) == 0) {
      std::fprintf(stderr, "tk8s-container: GPU jail: %s\n", mode.c_str());
      return 125;
    }
  }
  if (chdir(workdir.c_str()) != 0) die("chdir " + workdir);
  setenv("TK8S_GPU_ISOLATION", mode.c_str(), 1);
  setenv("TK8S_CONTAINER", ("namespaces:" + how + (pid_ns ? "+pid" : "") + ";rootfs:" + fs_mode).c_str(), 1);
  execvp(argv[i], argv + i);
  std::fprintf(stderr, "tk8s-container: exec %s: %s\n", argv[i], std::strerror(errno));
  return 127;
}
