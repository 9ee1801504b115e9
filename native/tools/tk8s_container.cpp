// tk8s-container: run a pod's container from an image root file system (agent/images.py).
//
//   tk8s-container --rootfs DIR [--upper DIR] [--workdir D] [--hostname H] [--pid-ns]
//                  [--bind|--bind-ro SRC:DST]... [jail options, gpujail.h] [--no-gpu-jail] -- ARGV...
//   tk8s-container --exec-in PID [--workdir D] [jail options] -- ARGV...   (kubectl exec)
//   tk8s-container --probe      {"usable": bool, "how": "root"|"userns"|"ptrace", "error": ...}
//   --mode auto|namespaces|ptrace (before the others; default auto: namespaces when this user
//   can make them, else ptrace)
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
//   3. pivot_root into it (the host's root is detached, so there is no way back up, unlike a
//      chroot), a capability bounding set cut to Docker's default set (a root pod keeps no
//      CAP_SYS_ADMIN, CAP_SYS_PTRACE, CAP_SYS_MODULE ...), then the GPU jail of gpujail.h built
//      on the container's own paths (a rule on a host directory above the root file system would
//      grant everything bound under it), then exec of the container's command with the
//      environment it was given.
//
// Mount points inside the image are resolved inside it (openat2 RESOLVE_IN_ROOT, the image's own
// symlinks followed within the image: Debian's /var/run -> /run lands on the image's /run, never
// the host's), created as needed, and mounted onto through /proc/self/fd -- no path is ever
// looked up in the host's tree on the image's say-so.
//
// GPU pods keep the host PID namespace (HIP/RCCL IPC identifies peers by pid). Exit status: the
// command's; 125 = the container could not be set up (message on stderr); 127 = exec failed.
//
// Where no mount namespace can be had (not root and user namespaces off: the MI355X GPU tier),
// the "ptrace" mode gives the pod the same view by path translation (ptrace_root.h): the pod's
// own tree of hard links to the image with copy-up on write, the host's /dev /proc /sys and the
// volumes at their paths, the image's own loader and interpreters -- and, since the host's tree
// is not detached there, the jail's path layers (--deny/--read-only/--allow, the process pods'
// rules) plus the host's "/" read-only outside the pod's directory. In namespace mode those
// layers are dropped: inside the container they would name the image's paths, not the host's.
#include <fcntl.h>
#include <linux/capability.h>
#include <linux/openat2.h>
#include <sched.h>
#include <sys/syscall.h>
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
#include "ptrace_root.h"

namespace {

// tty: true (agent/runtime.py gives the pod a pty as its controlling terminal): a PID
// namespace hides the relay's process group from the container, and a shell in there reads the
// terminal's foreground group at start to hand the terminal back at exit -- it sees 0, and dash
// ends with "Cannot set tty process group" (exit 2). So the container's first process leads a
// group of its own and takes the foreground before it execs (`term`: decided by the relay before
// the fork, while both see the same groups).
bool owns_terminal() { return isatty(STDIN_FILENO) && tcgetpgrp(STDIN_FILENO) == getpgrp(); }

void take_terminal() {
  if (setpgid(0, 0) != 0) return;
  struct sigaction ign {}, old {};
  ign.sa_handler = SIG_IGN;
  sigaction(SIGTTOU, &ign, &old);  // a background group may still set the foreground
  (void)tcsetpgrp(STDIN_FILENO, getpgrp());
  sigaction(SIGTTOU, &old, nullptr);
}

// The relay's stop signals: the pod's group is signalled as a whole, which reaches the container
// while it is in that group; once it leads a group of its own (a terminal, or a shell's job
// control) the signal is passed on to it.
volatile pid_t g_relay_child = 0;
void relay_signal(int sig) {
  const pid_t c = g_relay_child;
  if (c > 0 && getpgid(c) != getpgrp()) kill(c, sig);
}

void relay_signals(pid_t child) {
  g_relay_child = child;
  for (int s : {SIGTERM, SIGINT, SIGHUP}) signal(s, relay_signal);
}

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

void mkdirs(const std::string& path) {  // a host path of this tool's own choosing (--upper)
  std::string cur;
  size_t pos = 0;
  while (pos != std::string::npos) {
    pos = path.find('/', pos + 1);
    cur = path.substr(0, pos);
    if (!cur.empty()) mkdir(cur.c_str(), 0755);
  }
}

int open_in_root(int rootfd, const std::string& rel, int flags) {
  open_how how{};
  how.flags = static_cast<__u64>(flags | O_CLOEXEC);
  how.resolve = RESOLVE_IN_ROOT | RESOLVE_NO_MAGICLINKS;
  return static_cast<int>(syscall(SYS_openat2, rootfd, rel.empty() ? "." : rel.c_str(), &how, sizeof(how)));
}

// An O_PATH fd of `rel` (a path inside the image) resolved inside it, creating what is missing
// on the way: directories, and the last component as an empty file when `as_file`. A dangling
// symlink on the way is followed (inside the image) and its target created.
int ensure_in_root(int rootfd, std::string rel, bool as_file, int depth = 0) {
  if (depth > 40) {
    errno = ELOOP;
    return -1;
  }
  std::vector<std::string> parts;
  for (size_t i = 0; i <= rel.size();) {
    const size_t j = rel.find('/', i);
    const std::string c = rel.substr(i, j == std::string::npos ? std::string::npos : j - i);
    if (!c.empty() && c != ".") parts.push_back(c);
    if (j == std::string::npos) break;
    i = j + 1;
  }
  std::string cur;
  for (size_t k = 0; k < parts.size(); ++k) {
    const std::string next = cur.empty() ? parts[k] : cur + "/" + parts[k];
    const bool last = k + 1 == parts.size();
    int fd = open_in_root(rootfd, next, O_PATH);
    if (fd < 0 && errno == ENOENT) {
      const int dir = open_in_root(rootfd, cur, O_PATH | O_DIRECTORY);
      if (dir < 0) return -1;
      int rc = 0;
      if (last && as_file) {
        const int f = openat(dir, parts[k].c_str(), O_CREAT | O_WRONLY | O_NOFOLLOW | O_CLOEXEC, 0644);
        rc = f < 0 ? -1 : close(f);
      } else {
        rc = mkdirat(dir, parts[k].c_str(), 0755);
      }
      if (rc != 0 && errno == EEXIST) {  // a dangling symlink: make its target, inside the image
        char buf[PATH_MAX];
        const ssize_t n = readlinkat(dir, parts[k].c_str(), buf, sizeof(buf) - 1);
        close(dir);
        if (n <= 0) return -1;
        std::string target(buf, static_cast<size_t>(n));
        target = target[0] == '/' ? target.substr(1) : (cur.empty() ? target : cur + "/" + target);
        for (size_t r = k + 1; r < parts.size(); ++r) target += "/" + parts[r];
        return ensure_in_root(rootfd, target, as_file, depth + 1);
      }
      close(dir);
      if (rc != 0) return -1;
      fd = open_in_root(rootfd, next, O_PATH);
    }
    if (fd < 0) return -1;
    if (last) return fd;
    close(fd);
    cur = next;
  }
  return open_in_root(rootfd, "", O_PATH | O_DIRECTORY);
}

// Bind host path `src` onto `dst`, a path inside the image (resolved inside it).
void bind(int rootfd, const std::string& src, const std::string& dst, bool read_only = false) {
  struct stat st {};
  if (stat(src.c_str(), &st) != 0) die("bind source " + src);
  const int fd = ensure_in_root(rootfd, dst, !S_ISDIR(st.st_mode));
  if (fd < 0) die("mount point " + dst + " in the image");
  const std::string at = "/proc/self/fd/" + std::to_string(fd);
  if (mount(src.c_str(), at.c_str(), nullptr, MS_BIND | MS_REC, nullptr) != 0) die("bind " + src + " -> " + dst);
  close(fd);
  if (read_only) {  // a bind mount takes MS_RDONLY only on a remount of itself: look it up again (the
                    // fd above still names the directory it now covers)
    const int top = open_in_root(rootfd, dst, O_PATH);
    if (top < 0 || mount(nullptr, ("/proc/self/fd/" + std::to_string(top)).c_str(), nullptr,
                         MS_BIND | MS_REMOUNT | MS_RDONLY, nullptr) != 0)
      die("read-only bind " + dst);
    close(top);
  }
}

// Docker's default capability set: what a container's root keeps. Everything else leaves the
// bounding set, so no process of the pod can ever hold it (CAP_SYS_ADMIN, CAP_SYS_PTRACE,
// CAP_SYS_MODULE, CAP_SYS_RAWIO, CAP_DAC_READ_SEARCH, ...).
void drop_capabilities() {
  const int keep[] = {CAP_CHOWN,  CAP_DAC_OVERRIDE, CAP_FSETID,           CAP_FOWNER,      CAP_MKNOD,
                      CAP_NET_RAW, CAP_SETGID,      CAP_SETUID,           CAP_SETFCAP,     CAP_SETPCAP,
                      CAP_NET_BIND_SERVICE,          CAP_SYS_CHROOT,       CAP_KILL,        CAP_AUDIT_WRITE};
  for (int c = 0; c <= CAP_LAST_CAP; ++c) {
    bool kept = false;
    for (int k : keep) kept |= k == c;
    if (!kept && prctl(PR_CAPBSET_DROP, c, 0, 0, 0) != 0 && errno != EINVAL) die("drop capability " + std::to_string(c));
  }
}

// Make `root` the root of this mount namespace and detach the old one.
void pivot_into(const std::string& root) {
  if (mount(root.c_str(), root.c_str(), nullptr, MS_BIND | MS_REC, nullptr) != 0) die("bind " + root + " onto itself");
  if (chdir(root.c_str()) != 0) die("chdir " + root);
  if (syscall(SYS_pivot_root, ".", ".") != 0) die("pivot_root " + root);  // the old root stacks under the new
  if (umount2(".", MNT_DETACH) != 0) die("detach the host's root");
  if (chdir("/") != 0) die("chdir /");
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

bool namespaces_usable() {
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
  return WIFEXITED(st) && WEXITSTATUS(st) == 0;
}

std::string json_str(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    if (static_cast<unsigned char>(c) >= 0x20) o += c;
  }
  return o + "\"";
}

// "namespaces" or "ptrace" for --mode auto|namespaces|ptrace; "" when neither can be had (`why`).
std::string pick_mode(const std::string& mode, std::string* why) {
  if (mode != "ptrace" && namespaces_usable()) return "namespaces";
  if (mode == "namespaces") {
    *why = "no mount namespace for this user (not root, and user namespaces are off)";
    return "";
  }
  const std::string p = tk8s::troot::probe();
  if (p.empty()) return "ptrace";
  *why = (mode == "ptrace" ? "" : "no mount namespace for this user, and ") + std::string("no ptrace supervision: ") + p;
  return "";
}

int probe(const std::string& mode) {
  std::string why;
  const std::string m = pick_mode(mode, &why);
  const std::string how = m == "ptrace" ? "ptrace" : geteuid() == 0 ? "root" : "userns";
  std::printf("{\"usable\": %s, \"how\": \"%s\"%s}\n", m.empty() ? "false" : "true", how.c_str(),
              m.empty() ? (", \"error\": " + json_str(why)).c_str() : "");
  return m.empty() ? 1 : 0;
}

// --exec-in PID: run a command inside a running image pod (kubectl exec): its user, mount and
// PID namespaces, its root, the same GPU jail. PID is the pod's tk8s-container process; with a
// PID namespace that process only waits, and the container is its child.
int exec_in(pid_t pid, const std::string& workdir, const tk8s::jail::Policy& policy, bool jail, char** argv) {
  auto relays = [](pid_t p) {  // unshared a PID namespace for its children, not itself in it
    struct stat own {}, kids {};
    const std::string ns = "/proc/" + std::to_string(p) + "/ns/";
    return stat((ns + "pid").c_str(), &own) == 0 && stat((ns + "pid_for_children").c_str(), &kids) == 0 &&
           own.st_ino != kids.st_ino;
  };
  if (relays(pid)) {  // the relaying parent (--pid-ns): the container is its first child
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
  // every namespace is opened before any is joined: inside the container's mount namespace,
  // /proc is its own (a PID namespace's), where the host pid above names nothing
  struct Ns {
    const char* name;
    int type;
    int fd;
  };
  Ns nss[] = {{"user", CLONE_NEWUSER, -1}, {"uts", CLONE_NEWUTS, -1}, {"mnt", CLONE_NEWNS, -1}, {"pid", CLONE_NEWPID, -1}};
  for (auto& n : nss) {
    struct stat mine {}, theirs {};
    if (stat((proc + "/ns/" + n.name).c_str(), &theirs) != 0) die(std::string("stat ns ") + n.name);
    if (stat((std::string("/proc/self/ns/") + n.name).c_str(), &mine) == 0 && mine.st_ino == theirs.st_ino) continue;
    n.fd = open((proc + "/ns/" + n.name).c_str(), O_RDONLY | O_CLOEXEC);
    if (n.fd < 0) die(std::string("open ns ") + n.name);
  }
  for (auto& n : nss) {
    if (n.fd < 0) continue;
    if (setns(n.fd, n.type) != 0) die(std::string("setns ") + n.name);
    close(n.fd);
  }
  if (fchdir(rootfd) != 0 || chroot(".") != 0 || chdir("/") != 0) die("enter the container's root");
  close(rootfd);
  const bool term = owns_terminal();
  const pid_t child = fork();  // a joined PID namespace takes effect for children only
  if (child < 0) die("fork");
  if (child > 0) {
    relay_signals(child);
    int st = 0;
    while (waitpid(child, &st, 0) < 0 && errno == EINTR) {
    }
    return WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
  }
  prctl(PR_SET_PDEATHSIG, SIGKILL);
  if (term) take_terminal();
  drop_capabilities();  // what the container's own processes may hold, no more
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

struct Bind {
  std::string src, dst;
  bool read_only;
};

// ptrace mode (ptrace_root.h): the pod's own tree, the jail with the host's "/" read-only outside
// it, the command under a supervisor that translates its paths.
int run_traced(const std::string& rootfs, const std::string& upper, const std::string& workdir,
               const std::string& hostname, const std::vector<Bind>& binds, tk8s::jail::Policy policy, bool jail,
               char** argv) {
  if (upper.empty()) {
    errno = EINVAL;
    die("ptrace mode needs --upper (the pod's own tree)");
  }
  tk8s::troot::View view;
  if (const std::string e = tk8s::troot::make_farm(view, rootfs, upper + "/farm"); !e.empty()) {
    std::fprintf(stderr, "tk8s-container: %s\n", e.c_str());
    return 125;
  }
  view.hostname = hostname;
  for (const char* d : {"/dev", "/proc", "/sys"}) view.add_mount(d, d);
  if (!hostname.empty()) {  // what a UTS namespace would answer there (uname is answered by the supervisor)
    const std::string hf = upper + "/hostname";
    const int fd = open(hf.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0 || write(fd, (hostname + "\n").data(), hostname.size() + 1) != static_cast<ssize_t>(hostname.size() + 1))
      die("write " + hf);
    close(fd);
    view.add_mount("/proc/sys/kernel/hostname", hf);
    view.add_mount("/etc/hostname", hf);
  }
  for (const auto& b : binds) {
    const std::string src = tk8s::jail::real(b.src);
    if (src.empty()) die("bind source " + b.src);
    // the mount point resolved inside the image, as in namespace mode (Debian's /var/run -> /run
    // puts /var/run/secrets/... at /run/secrets/...), and made in the pod's tree so listings show it
    std::string at = b.dst, h;
    if (view.resolve(b.dst, true, &h) == 0 && tk8s::troot::under(view.farm, h)) {
      at = view.to_guest(h);
      struct stat st {};
      const bool dir = stat(src.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
      std::string cur = view.farm;
      const auto parts = tk8s::troot::split_path(at);
      for (size_t k = 0; k < parts.size(); ++k) {
        cur += "/" + parts[k];
        if (k + 1 < parts.size() || dir) {
          mkdir(cur.c_str(), 0755);
        } else if (const int fd = open(cur.c_str(), O_WRONLY | O_CREAT | O_NOFOLLOW | O_CLOEXEC, 0644); fd >= 0) {
          close(fd);
        }
      }
    }
    view.add_mount(at, src);
    (b.read_only ? policy.read_only_paths : policy.allow_paths).push_back(src);
  }
  // the host's tree stays in view: read-only, but for the pod's own tree and its GPU nodes
  // (the deny set still takes the other GPUs' render nodes and the node's secrets)
  policy.read_only_paths.push_back("/");
  policy.allow_paths.push_back(view.farm);
  policy.allow_paths.push_back("/dev");
  std::string host_wd;
  if (view.resolve(workdir, true, &host_wd) != 0) die("workdir " + workdir);
  int pfd[2];
  if (pipe2(pfd, O_CLOEXEC) != 0) die("pipe");
  const pid_t child = fork();
  if (child < 0) die("fork");
  if (child == 0) {
    close(pfd[1]);
    prctl(PR_SET_PDEATHSIG, SIGKILL);
    if (geteuid() == 0) drop_capabilities();
    std::string mode = "none:--no-gpu-jail";
    if (jail) {
      mode = tk8s::jail::apply(policy);
      if (mode.rfind("none:", 0) == 0) {
        std::fprintf(stderr, "tk8s-container: GPU jail: %s\n", mode.c_str());
        _exit(125);
      }
    }
    if (chdir(host_wd.c_str()) != 0) die("chdir " + workdir);
    setenv("TK8S_GPU_ISOLATION", mode.c_str(), 1);
    setenv("TK8S_CONTAINER", (std::string("ptrace:") + (geteuid() == 0 ? "root" : "user") + ";rootfs:farm").c_str(), 1);
    char c;
    if (read(pfd[0], &c, 1) != 1) _exit(125);  // released once the supervisor traces this process
    if (const int rc = tk8s::troot::install_filter(); rc != 0) {
      errno = -rc;
      die("seccomp filter");
    }
    execvp(argv[0], argv);
    std::fprintf(stderr, "tk8s-container: exec %s: %s\n", argv[0], std::strerror(errno));
    _exit(127);
  }
  close(pfd[0]);
  relay_signals(child);  // the pod's group gets them; a child that leads its own group, from here
  FILE* log = nullptr;
  if (const char* lp = getenv("TK8S_PTRACE_LOG"); lp != nullptr && *lp) log = std::fopen(lp, "a");
  tk8s::troot::Tracer tracer(view, log);
  const int rc = tracer.run(child, pfd[1]);
  if (rc < 0) {
    kill(child, SIGKILL);
    waitpid(child, nullptr, 0);
    errno = -rc;
    die("supervise the container");
  }
  return rc;
}

// A running pod in ptrace mode: its tk8s-container process shares our mount namespace (it made
// none) and was started with --rootfs. Its settings come from its command line.
bool traced_pod(pid_t pid, std::string* rootfs, std::string* upper, std::string* hostname, std::vector<Bind>* binds) {
  struct stat mine {}, theirs {};
  const std::string proc = "/proc/" + std::to_string(pid);
  if (stat((proc + "/ns/mnt").c_str(), &theirs) != 0 || stat("/proc/self/ns/mnt", &mine) != 0 ||
      mine.st_ino != theirs.st_ino)
    return false;
  std::ifstream f(proc + "/cmdline", std::ios::binary);
  std::vector<std::string> args;
  for (std::string a; std::getline(f, a, '\0');) args.push_back(a);
  bool found = false;
  for (size_t k = 1; k + 1 < args.size(); ++k) {
    const std::string& a = args[k];
    if (a == "--") break;
    if (a == "--rootfs") *rootfs = args[++k], found = true;
    else if (a == "--upper") *upper = args[++k];
    else if (a == "--hostname") *hostname = args[++k];
    else if (a == "--bind" || a == "--bind-ro") {
      const std::string v = args[++k];
      const auto c = v.find(':');
      if (c != std::string::npos) binds->push_back({v.substr(0, c), v.substr(c + 1), a == "--bind-ro"});
    }
  }
  return found && !upper->empty();
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
  std::string rootfs, upper, workdir = "/", hostname, mode = "auto";
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
      if (a == "--probe") return probe(mode);
      if (a == "--mode") {
        mode = next();
        if (mode != "auto" && mode != "namespaces" && mode != "ptrace") throw std::invalid_argument("--mode auto|namespaces|ptrace");
        continue;
      }
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
  // the pod's cgroups and CPUs first, while their host paths are still in view
  if (const std::string why = tk8s::jail::join_limits(policy); !why.empty()) {
    std::fprintf(stderr, "tk8s-container: %s\n", why.c_str());
    return 125;
  }
  if (exec_pid > 0 && i < argc) {
    std::string r, u, h;
    std::vector<Bind> b;
    if (traced_pod(exec_pid, &r, &u, &h, &b)) return run_traced(r, u, workdir, h, b, policy, jail, argv + i);
    policy.deny_paths.clear(), policy.read_only_paths.clear(), policy.allow_paths.clear();  // host paths
    return exec_in(exec_pid, workdir, policy, jail, argv + i);
  }
  if (rootfs.empty() || i >= argc) return usage();
  rootfs = tk8s::jail::real(rootfs);
  if (rootfs.empty()) die("--rootfs");
  std::string why;
  const std::string picked = pick_mode(mode, &why);
  if (picked.empty()) {
    std::fprintf(stderr, "tk8s-container: %s\n", why.c_str());
    return 125;
  }
  if (picked == "ptrace") return run_traced(rootfs, upper, workdir, hostname, binds, policy, jail, argv + i);
  // namespaces: the path layers name host paths, which the container's root does not show
  policy.deny_paths.clear(), policy.read_only_paths.clear(), policy.allow_paths.clear();

  const std::string how = enter(pid_ns);
  if (pid_ns) {  // the command becomes pid 1 of its namespace; this process waits and relays
    const bool term = owns_terminal();
    const pid_t child = fork();
    if (child < 0) die("fork");
    if (child > 0) {
      relay_signals(child);
      int st = 0;
      while (waitpid(child, &st, 0) < 0 && errno == EINTR) {
      }
      return WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
    }
    prctl(PR_SET_PDEATHSIG, SIGKILL);
    if (term) take_terminal();
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
  const int rootfd = open(root.c_str(), O_PATH | O_DIRECTORY | O_CLOEXEC);
  if (rootfd < 0) die("open " + root);
  bind(rootfd, "/dev", "dev");
  bind(rootfd, "/sys", "sys", /*read_only=*/true);  // as Docker: sysfs is the host's, read-only
  if (pid_ns) {
    const int fd = ensure_in_root(rootfd, "proc", false);
    if (fd < 0 || mount("proc", ("/proc/self/fd/" + std::to_string(fd)).c_str(), "proc", MS_NOSUID | MS_NODEV | MS_NOEXEC,
                        nullptr) != 0)
      die("mount /proc");
    close(fd);
  } else {
    bind(rootfd, "/proc", "proc");
  }
  if (how == "root") bind(rootfd, "/proc/sys", "proc/sys", /*read_only=*/true);  // no sysctl writes from a root pod
  if (const int fd = ensure_in_root(rootfd, "tmp", false); fd >= 0) close(fd);
  for (const auto& b : binds) bind(rootfd, b.src, b.dst, b.read_only);
  close(rootfd);
  if (!hostname.empty() && sethostname(hostname.c_str(), hostname.size()) != 0) die("sethostname");
  pivot_into(root);
  drop_capabilities();
  std::string jail_mode = "none:--no-gpu-jail";
  if (jail) {
    jail_mode = tk8s::jail::apply(policy);  // on the container's own paths (see the header comment)
    if (jail_mode.rfind("none:", 0) == 0) {
      std::fprintf(stderr, "tk8s-container: GPU jail: %s\n", jail_mode.c_str());
      return 125;
    }
  }
  if (chdir(workdir.c_str()) != 0) die("chdir " + workdir);
  setenv("TK8S_GPU_ISOLATION", jail_mode.c_str(), 1);
  setenv("TK8S_CONTAINER", ("namespaces:" + how + (pid_ns ? "+pid" : "") + ";rootfs:" + fs_mode).c_str(), 1);
  execvp(argv[i], argv + i);
  std::fprintf(stderr, "tk8s-container: exec %s: %s\n", argv[i], std::strerror(errno));
  return 127;
}
