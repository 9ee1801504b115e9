// An image pod's root file system without namespaces: tk8s-container's "ptrace" mode.
//
// On a node where this user may make no mount namespace (not root, user namespaces off -- the
// MI355X GPU tier: gpurun_out/r6_ptrace.json, profiles/r6_ptrace/) the container's view of the
// file system is made by path translation instead of mounts, the way PRoot does it, with two
// differences that matter for a multi-tenant GPU node:
//
//   * only the syscalls that name paths stop: a seccomp filter returns SECCOMP_RET_TRACE for them
//     and lets everything else run untraced -- the GPU runtime's ioctls, mmaps and reads never
//     stop, so a GPU pod pays for path lookups only;
//   * containment is not the translation's job: the pod also runs under the Landlock jail of
//     gpujail.h with the host's tree read-only except the pod's own directory (and its GPU
//     nodes, /dev/shm, read-write volumes) and the node's secrets denied, exactly as a process
//     pod. A path the translation does not see (a symlink swapped between the supervisor's
//     lookup and the kernel's, /proc/<pid>/root) reaches at most what a process pod reaches.
//
// The view (View): the guest's "/" is the pod's own tree (its "farm": the image's directories
// made afresh, its symlinks copied, its files HARD-LINKED -- no data copied, unpacked image
// untouched), with the host's /dev, /proc, /sys and the pod's volumes at their guest paths.
// Every path argument is resolved component by component inside the farm -- the image's own
// symlinks, absolute ones included, followed inside it, ".." stopping at its root -- and
// replaced by the host path it names. A write to a file still shared with the image (an open
// for writing, truncate, chmod, chown, utimes, xattrs) first copies it up: the farm entry becomes
// a private copy, so the image's inode is never written (the overlay's copy-up, by the supervisor).
// Results that carry host paths are mapped back: getcwd, readlink of /proc links
// (/proc/self/exe names the program, not its loader), uname's node name is the pod's hostname.
//
// execve: the kernel would load a script's interpreter and an ELF's PT_INTERP from the HOST's
// tree, so the supervisor does what binfmt does, inside the image: "#!" lines are expanded and
// a dynamic executable is started through the image's own loader (`ld.so [--argv0 A] PROG ...`).
//
// Memory for translated strings comes from one anonymous mapping per traced thread, made by
// injecting mmap into the thread at its first translated syscall (the syscall is then restarted):
// nothing is written below a thread's stack pointer (a goroutine's stack is small), and a thread
// whose syscall is still reading its strings is never overwritten by another's.
//
// PTRACE_SEIZE (of a child blocked on a pipe until it is traced): group-stops are told from
// signal-delivery-stops (PTRACE_LISTEN), so the agent's
// SIGSTOP/SIGCONT CPU duty cycle (agent/resources.py) still stops and resumes a traced pod.
// PTRACE_O_EXITKILL: the pod cannot outlive its supervisor untraced, and a filtered syscall
// with no tracer fails (ENOSYS) rather than running untranslated.
//
// x86-64 only; an i386 (int 0x80) syscall kills the process, an x32 one fails with ENOSYS.
// Not emulated: PID and UTS namespaces (the pod sees host pids), openat2 (ENOSYS; callers fall
// back to openat), mount/chroot/pivot_root (EPERM). Reference: the workloads of
// ansible/roles/rancherhost/tasks/main.yml:26-34 ran in Docker containers.
#pragma once

#if !defined(__x86_64__)
#error "ptrace_root.h translates x86-64 syscalls"
#endif

#include <dirent.h>
#include <elf.h>
#include <fcntl.h>
#include <linux/audit.h>
#include <linux/filter.h>
#include <linux/seccomp.h>
#include <signal.h>
#include <stddef.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/ptrace.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <sys/un.h>
#include <sys/user.h>
#include <sys/utsname.h>
#include <sys/wait.h>
#include <sys/xattr.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace tk8s::troot {

#ifndef SYS_fchmodat2
constexpr long SYS_fchmodat2 = 452;
#endif

inline std::vector<std::string> split_path(const std::string& p) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i <= p.size()) {
    const size_t j = p.find('/', i);
    const std::string c = p.substr(i, j == std::string::npos ? std::string::npos : j - i);
    if (!c.empty() && c != ".") out.push_back(c);
    if (j == std::string::npos) break;
    i = j + 1;
  }
  return out;
}

inline bool under(const std::string& prefix, const std::string& p) {  // p is prefix or beneath it
  if (prefix == "/") return !p.empty() && p[0] == '/';
  return p.compare(0, prefix.size(), prefix) == 0 && (p.size() == prefix.size() || p[prefix.size()] == '/');
}

// A host directory or file at a guest path (the host's /dev, /proc, /sys; a volume).
struct Mount {
  std::string guest, host;
};

class View {
 public:
  std::string farm;            // host path of the guest's "/" (canonical)
  std::vector<Mount> mounts;   // longest guest path first
  std::string hostname;
  dev_t image_dev = 0;
  std::unordered_set<ino_t> image_inodes;  // files the farm still shares with the image

  void add_mount(const std::string& guest, const std::string& host) {
    std::string g = "/";
    for (const auto& c : split_path(guest)) g += (g.size() > 1 ? "/" : "") + c;
    mounts.push_back({g, host});
    std::stable_sort(mounts.begin(), mounts.end(),
                     [](const Mount& a, const Mount& b) { return a.guest.size() > b.guest.size(); });
  }

  const Mount* mount_for(const std::string& guest) const {
    for (const auto& m : mounts)
      if (m.guest != "/" && under(m.guest, guest)) return &m;
    return nullptr;
  }

  // The host path of absolute guest path `guest`; -errno (ELOOP) when it cannot be resolved.
  // `follow`: whether a symlink as the last component is followed.
  int resolve(const std::string& guest, bool follow, std::string* host) const {
    std::vector<std::string> todo = split_path(guest);
    std::reverse(todo.begin(), todo.end());
    std::vector<std::string> cur;
    int links = 0;
    auto joined = [&]() {
      std::string g;
      for (const auto& c : cur) g += "/" + c;
      return g.empty() ? std::string("/") : g;
    };
    auto rest = [&]() {
      std::string r;
      for (auto it = todo.rbegin(); it != todo.rend(); ++it) r += "/" + *it;
      return r;
    };
    while (!todo.empty()) {
      const std::string c = todo.back();
      todo.pop_back();
      if (c == "..") {
        if (!cur.empty()) cur.pop_back();
        continue;
      }
      cur.push_back(c);
      const std::string g = joined();
      if (const Mount* m = mount_for(g)) {  // a host tree: the host's kernel resolves the rest --
        const std::string full = g + rest();  // but a mount beneath it (/proc/sys/kernel/hostname) wins
        const Mount* best = mount_for(full);
        if (best == nullptr || best->guest.size() < m->guest.size()) best = m;
        *host = best->host + full.substr(best->guest.size());
        return 0;
      }
      if (todo.empty() && !follow) break;
      const std::string h = farm + g;
      struct stat st {};
      if (lstat(h.c_str(), &st) != 0) break;  // missing (or not a directory): the kernel says which
      if (!S_ISLNK(st.st_mode)) continue;
      if (++links > 40) return -ELOOP;
      char buf[PATH_MAX];
      const ssize_t n = readlink(h.c_str(), buf, sizeof(buf) - 1);
      if (n < 0) return -errno;
      const std::string target(buf, static_cast<size_t>(n));
      cur.pop_back();
      if (!target.empty() && target[0] == '/') cur.clear();
      auto parts = split_path(target);
      for (auto it = parts.rbegin(); it != parts.rend(); ++it) todo.push_back(*it);
    }
    const std::string g = joined();
    *host = (g == "/" ? farm : farm + g) + rest();
    return 0;
  }

  // The guest path of host path `host` (a cwd, a /proc link); `host` itself when outside the view.
  std::string to_guest(const std::string& host) const {
    if (under(farm, host)) return host.size() == farm.size() ? "/" : host.substr(farm.size());
    for (const auto& m : mounts)
      if (under(m.host, host)) return m.guest + host.substr(m.host.size());
    return host;
  }

  bool shared_with_image(const struct stat& st) const {
    return S_ISREG(st.st_mode) && st.st_dev == image_dev && image_inodes.count(st.st_ino) != 0;
  }

  // Make the farm entry `host` the pod's own file if it still shares the image's inode.
  // 0, or -errno.
  int copy_up(const std::string& host) const {
    struct stat st {};
    if (lstat(host.c_str(), &st) != 0 || !shared_with_image(st)) return 0;
    const int in = open(host.c_str(), O_RDONLY | O_CLOEXEC | O_NOFOLLOW);
    if (in < 0) return -errno;
    std::string tmp = host + ".tk8s-cow.XXXXXX";
    std::vector<char> name(tmp.begin(), tmp.end());
    name.push_back('\0');
    const int out = mkstemp(name.data());
    if (out < 0) {
      const int e = errno;
      close(in);
      return -e;
    }
    int rc = 0;
    for (off_t off = 0; off < st.st_size;) {
      const ssize_t n = sendfile(out, in, &off, static_cast<size_t>(std::min<off_t>(st.st_size - off, 1 << 30)));
      if (n <= 0) {
        rc = n < 0 ? -errno : -EIO;
        break;
      }
    }
    if (rc == 0 && fchmod(out, st.st_mode & 07777) != 0) rc = -errno;
    const struct timespec times[2] = {st.st_atim, st.st_mtim};
    if (rc == 0) futimens(out, times);
    close(in);
    close(out);
    if (rc == 0 && rename(name.data(), host.c_str()) != 0) rc = -errno;
    if (rc != 0) unlink(name.data());
    return rc;
  }
};

// ---- the pod's tree --------------------------------------------------------------------

// Walk the unpacked image `src` (an open directory) into `dst`: directories made, symlinks
// copied, regular files hard-linked (copied across file systems), FIFOs made; device nodes and
// sockets are not. Records every image file's inode in `view`.
inline int build_tree(View& view, int src, int dst, bool make) {
  DIR* d = fdopendir(dup(src));
  if (d == nullptr) return -errno;
  int rc = 0;
  while (dirent* e = readdir(d)) {
    const char* n = e->d_name;
    if (!std::strcmp(n, ".") || !std::strcmp(n, "..")) continue;
    struct stat st {};
    if (fstatat(src, n, &st, AT_SYMLINK_NOFOLLOW) != 0) continue;
    if (S_ISDIR(st.st_mode)) {
      if (make && mkdirat(dst, n, 0700) != 0 && errno != EEXIST) {
        rc = -errno;
        break;
      }
      const int s2 = openat(src, n, O_RDONLY | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC);
      const int d2 = make ? openat(dst, n, O_RDONLY | O_DIRECTORY | O_NOFOLLOW | O_CLOEXEC) : -1;
      if (s2 >= 0 && (!make || d2 >= 0)) rc = build_tree(view, s2, d2, make);
      if (make && d2 >= 0) fchmod(d2, st.st_mode & 07777);  // after its entries: a 0555 dir is filled first
      if (s2 >= 0) close(s2);
      if (d2 >= 0) close(d2);
      if (rc != 0) break;
    } else if (S_ISREG(st.st_mode)) {
      view.image_dev = st.st_dev;
      view.image_inodes.insert(st.st_ino);
      if (!make) continue;
      if (linkat(src, n, dst, n, 0) != 0 && errno != EEXIST) {
        const int in = openat(src, n, O_RDONLY | O_CLOEXEC | O_NOFOLLOW);
        const int out = openat(dst, n, O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, st.st_mode & 07777);
        if (in >= 0 && out >= 0) {
          off_t off = 0;
          while (off < st.st_size && sendfile(out, in, &off, static_cast<size_t>(st.st_size - off)) > 0) {
          }
        }
        if (in >= 0) close(in);
        if (out >= 0) close(out);
      }
    } else if (S_ISLNK(st.st_mode)) {
      if (!make) continue;
      char buf[PATH_MAX];
      const ssize_t k = readlinkat(src, n, buf, sizeof(buf) - 1);
      if (k >= 0) {
        buf[k] = '\0';
        if (symlinkat(buf, dst, n) != 0) rc = errno == EEXIST ? 0 : -errno;
      }
    } else if (S_ISFIFO(st.st_mode) && make) {
      mkfifoat(dst, n, st.st_mode & 07777);
    }
  }
  closedir(d);
  return rc;
}

// The pod's tree at `farm` from image `rootfs` (made once; a restarted container keeps its
// writes, as with an overlay's upper layer), plus the directories the host trees are seen at.
inline std::string make_farm(View& view, const std::string& rootfs, const std::string& farm) {
  const std::string done = farm + ".complete";  // beside the tree: the guest's "/" lists only the image's entries
  const bool exists = access(done.c_str(), F_OK) == 0;
  if (!exists) {
    std::string cur;
    for (const auto& c : split_path(farm)) {
      cur += "/" + c;
      mkdir(cur.c_str(), 0755);
    }
  }
  const int src = open(rootfs.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  const int dst = open(farm.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (src < 0 || dst < 0) return "open " + (src < 0 ? rootfs : farm) + ": " + std::strerror(errno);
  const int rc = build_tree(view, src, dst, !exists);
  close(src);
  close(dst);
  if (rc != 0) return "build the pod's tree: " + std::string(std::strerror(-rc));
  if (!exists) {
    for (const char* d : {"dev", "proc", "sys", "tmp"}) mkdirat(AT_FDCWD, (farm + "/" + d).c_str(), d[0] == 't' ? 01777 : 0755);
    const int f = open(done.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0600);
    if (f >= 0) close(f);
  }
  char buf[PATH_MAX];
  if (realpath(farm.c_str(), buf) == nullptr) return "realpath " + farm;
  view.farm = buf;
  return "";
}

// ---- the filter ----------------------------------------------------------------------

// The syscalls that name paths (or return them): the only ones that stop.
inline const std::vector<long>& traced_syscalls() {
  static const std::vector<long> nrs = {
      SYS_open, SYS_openat, SYS_openat2, SYS_creat, SYS_stat, SYS_lstat, SYS_newfstatat, SYS_statx,
      SYS_access, SYS_faccessat, SYS_faccessat2, SYS_readlink, SYS_readlinkat, SYS_execve, SYS_execveat,
      SYS_chdir, SYS_getcwd, SYS_mkdir, SYS_mkdirat, SYS_rmdir, SYS_unlink, SYS_unlinkat, SYS_rename,
      SYS_renameat, SYS_renameat2, SYS_link, SYS_linkat, SYS_symlink, SYS_symlinkat, SYS_chmod, SYS_fchmodat,
      SYS_fchmodat2, SYS_chown, SYS_lchown, SYS_fchownat, SYS_truncate, SYS_utime, SYS_utimes, SYS_utimensat,
      SYS_futimesat, SYS_mknod, SYS_mknodat, SYS_statfs, SYS_getxattr, SYS_lgetxattr, SYS_setxattr,
      SYS_lsetxattr, SYS_listxattr, SYS_llistxattr, SYS_removexattr, SYS_lremovexattr, SYS_inotify_add_watch,
      SYS_fchmod, SYS_fchown, SYS_fsetxattr, SYS_fremovexattr, SYS_bind, SYS_connect, SYS_uname, SYS_chroot,
      SYS_mount, SYS_umount2, SYS_pivot_root, SYS_name_to_handle_at, SYS_open_tree, SYS_move_mount,
      SYS_fsopen, SYS_fsmount, SYS_fspick, SYS_mount_setattr, SYS_fanotify_mark, SYS_uselib, SYS_acct,
      SYS_swapon, SYS_swapoff, SYS_quotactl};
  return nrs;
}

inline int install_filter() {
  const auto& nrs = traced_syscalls();
  std::vector<sock_filter> f;
  f.push_back(BPF_STMT(BPF_LD | BPF_W | BPF_ABS, offsetof(seccomp_data, arch)));
  f.push_back(BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, AUDIT_ARCH_X86_64, 1, 0));
  f.push_back(BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_KILL_PROCESS));  // int 0x80: no way round the view
  f.push_back(BPF_STMT(BPF_LD | BPF_W | BPF_ABS, offsetof(seccomp_data, nr)));
  f.push_back(BPF_JUMP(BPF_JMP | BPF_JGE | BPF_K, 0x40000000u, 0, 1));  // x32
  f.push_back(BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_ERRNO | ENOSYS));
  const size_t k = nrs.size();
  for (size_t i = 0; i < k; ++i)
    f.push_back(BPF_JUMP(BPF_JMP | BPF_JEQ | BPF_K, static_cast<__u32>(nrs[i]), static_cast<__u8>(k - i), 0));
  f.push_back(BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_ALLOW));
  f.push_back(BPF_STMT(BPF_RET | BPF_K, SECCOMP_RET_TRACE));
  sock_fprog prog{static_cast<unsigned short>(f.size()), f.data()};
  if (prctl(PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0) != 0) return -errno;
  if (syscall(SYS_seccomp, SECCOMP_SET_MODE_FILTER, 0, &prog) != 0) return -errno;
  return 0;
}

// ---- the supervisor ----------------------------------------------------------------------

class Tracer {
 public:
  explicit Tracer(const View& v, FILE* log = nullptr) : view_(v), log_(log) {}

  // Trace `child` (blocked reading `release_fd`'s pipe, its filter not yet installed: it
  // installs it once released, then execs) until it exits, its descendants after it; returns its
  // exit status (128 + signal when killed), -errno if it could not be traced.
  int run(pid_t child, int release_fd) {
    main_ = child;
    const long opts = PTRACE_O_TRACESECCOMP | PTRACE_O_TRACESYSGOOD | PTRACE_O_TRACEFORK | PTRACE_O_TRACEVFORK |
                      PTRACE_O_TRACECLONE | PTRACE_O_TRACEEXEC | PTRACE_O_EXITKILL;
    if (ptrace(PTRACE_SEIZE, child, nullptr, reinterpret_cast<void*>(opts)) != 0) return -errno;
    threads_[child] = fresh(child);
    if (write(release_fd, "g", 1) != 1) return -errno;
    close(release_fd);
    int main_status = 0;
    bool main_done = false;
    for (;;) {
      int st = 0;
      const pid_t pid = waitpid(-1, &st, __WALL);
      if (pid < 0) {
        if (errno == EINTR) continue;
        break;  // ECHILD: every tracee is gone
      }
      if (WIFEXITED(st) || WIFSIGNALED(st)) {
        gone(pid);
        if (pid == main_) {
          main_status = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
          main_done = true;
          for (const auto& [t, _] : threads_) kill(t, SIGKILL);  // the container ends with its main process
        }
        if (main_done && threads_.empty()) break;
        continue;
      }
      if (!WIFSTOPPED(st)) continue;
      stopped(pid, st);
    }
    return main_status;
  }

 private:
  enum class Fix { kNone, kInject, kGetcwd, kReadlink, kUname };
  struct Thread {
    pid_t tgid = 0;
    unsigned long scratch = 0;  // this thread's mapping for translated strings (0: none yet)
    unsigned gen = 0;           // the mm generation the mapping belongs to
    Fix fix = Fix::kNone;
    user_regs_struct saved{};   // kInject: the syscall to restart
    int buf_arg = 0, size_arg = 0;
    std::string link;           // kReadlink: the host path read
    std::string exe, pending_exe;
    std::string trace;          // the log line of the syscall in flight (log_ only)
    bool parked = false;        // a new tracee held at its first stop until its parent's event
  };
  static constexpr unsigned long kScratch = 256 * 1024;
  static Thread fresh(pid_t tgid) {
    Thread t;
    t.tgid = tgid;
    return t;
  }

  const View& view_;
  FILE* log_;  // TK8S_PTRACE_LOG: every stopped syscall, its translation and its result
  pid_t main_ = 0;
  std::unordered_map<pid_t, Thread> threads_;
  std::unordered_map<pid_t, unsigned> gen_;                     // tgid -> exec generation
  std::unordered_map<pid_t, std::vector<unsigned long>> pool_;  // tgid -> mappings of exited threads
  std::map<std::string, bool> argv0_ok_;                       // loader -> understands --argv0

  // ---- registers and memory
  static unsigned long long& arg(user_regs_struct& r, int i) {
    switch (i) {
      case 0: return r.rdi;
      case 1: return r.rsi;
      case 2: return r.rdx;
      case 3: return r.r10;
      case 4: return r.r8;
      default: return r.r9;
    }
  }
  static bool read_mem(pid_t pid, unsigned long addr, void* out, size_t n) {
    iovec l{out, n}, r{reinterpret_cast<void*>(addr), n};
    return process_vm_readv(pid, &l, 1, &r, 1, 0) == static_cast<ssize_t>(n);
  }
  static bool read_str(pid_t pid, unsigned long addr, std::string* out) {
    out->clear();
    if (addr == 0) return false;
    char buf[256];
    while (out->size() < PATH_MAX * 2) {
      const size_t page_left = 4096 - (addr & 4095);
      const size_t n = std::min(sizeof(buf), page_left);
      if (!read_mem(pid, addr, buf, n)) return false;
      if (const void* z = std::memchr(buf, 0, n)) {
        out->append(buf, static_cast<const char*>(z) - buf);
        return true;
      }
      out->append(buf, n);
      addr += n;
    }
    return false;
  }
  static bool write_mem(pid_t pid, unsigned long addr, const void* data, size_t n) {
    iovec l{const_cast<void*>(data), n}, r{reinterpret_cast<void*>(addr), n};
    return process_vm_writev(pid, &l, 1, &r, 1, 0) == static_cast<ssize_t>(n);
  }
  struct Arena {  // bump allocation in a thread's scratch mapping, for one syscall
    pid_t pid;
    unsigned long base, used = 0;
    bool needed = false;  // base 0: the thread has no mapping yet, and this syscall needs one
    unsigned long put(const void* data, size_t n) {
      if (base == 0) {
        needed = true;
        return 1;  // a stand-in: the syscall is restarted once the thread has its mapping
      }
      const unsigned long at = base + used;
      if (used + n + 16 > kScratch || !write_mem(pid, at, data, n)) return 0;
      used += (n + 15) & ~15UL;
      return at;
    }
    unsigned long str(const std::string& s) { return put(s.c_str(), s.size() + 1); }
  };

  // ---- thread bookkeeping
  void gone(pid_t pid) {
    auto it = threads_.find(pid);
    if (it == threads_.end()) return;
    const Thread& t = it->second;
    if (t.scratch && t.gen == gen_[t.tgid] && t.tgid != pid) pool_[t.tgid].push_back(t.scratch);
    if (t.tgid == pid) {  // the process is gone: its pool with it
      pool_.erase(pid);
      gen_.erase(pid);
    }
    threads_.erase(it);
  }

  static pid_t tgid_of(pid_t tid) {
    char path[64];
    std::snprintf(path, sizeof(path), "/proc/%d/status", tid);
    FILE* f = std::fopen(path, "r");
    if (f == nullptr) return tid;
    char line[256];
    pid_t tg = tid;
    while (std::fgets(line, sizeof(line), f))
      if (std::sscanf(line, "Tgid: %d", &tg) == 1) break;
    std::fclose(f);
    return tg;
  }

  void stopped(pid_t pid, int st) {
    const int sig = WSTOPSIG(st);
    const int event = st >> 16;
    auto found = threads_.find(pid);
    if (found == threads_.end()) {
      // a new tracee reporting before its parent's fork/vfork/clone event: held at this first
      // stop until that event says what it inherits -- a vfork child runs on its parent's
      // memory, a fork child on a copy of it. Let go early, it would map strings of its own
      // (into its parent, for a vfork child) and the late event would overwrite its state.
      Thread p = fresh(pid);
      p.parked = true;
      found = threads_.emplace(pid, p).first;
      if (event == PTRACE_EVENT_STOP) return;
      found->second.parked = false;
      found->second.tgid = tgid_of(pid);
    }
    Thread& t = found->second;
    if (event == PTRACE_EVENT_SECCOMP) {
      const bool want_exit = on_entry(pid, t);
      ptrace(want_exit ? PTRACE_SYSCALL : PTRACE_CONT, pid, nullptr, nullptr);
      return;
    }
    if (sig == (SIGTRAP | 0x80)) {  // the exit of a syscall we asked to see
      on_exit(pid, t);
      ptrace(PTRACE_CONT, pid, nullptr, nullptr);
      return;
    }
    if (event == PTRACE_EVENT_FORK || event == PTRACE_EVENT_VFORK || event == PTRACE_EVENT_CLONE) {
      unsigned long msg = 0;
      ptrace(PTRACE_GETEVENTMSG, pid, nullptr, &msg);
      const pid_t child = static_cast<pid_t>(msg);
      Thread c = fresh(event == PTRACE_EVENT_CLONE ? tgid_of(child) : child);
      if (c.tgid != t.tgid) {
        // a new process: a copy of this thread's mapping is at the same address in it (fork), or
        // this very mapping while the parent waits (vfork)
        const bool valid = t.scratch && t.gen == gen_[t.tgid];
        c.scratch = valid ? t.scratch : 0;
        c.gen = gen_.emplace(c.tgid, 0u).first->second;
      } else {
        c.gen = gen_[c.tgid];  // a thread: a mapping of its own on its first translated syscall
      }
      c.exe = t.exe;
      auto prev = threads_.find(child);
      const bool parked = prev != threads_.end() && prev->second.parked;
      threads_[child] = c;
      if (parked) ptrace(PTRACE_CONT, child, nullptr, nullptr);  // its first stop came first
      ptrace(PTRACE_CONT, pid, nullptr, nullptr);
      return;
    }
    if (event == PTRACE_EVENT_EXEC) {
      unsigned long former = 0;
      ptrace(PTRACE_GETEVENTMSG, pid, nullptr, &former);
      if (static_cast<pid_t>(former) != pid) {  // a non-leader thread exec'd: it is the leader now
        auto f = threads_.find(static_cast<pid_t>(former));
        if (f != threads_.end()) {
          t.pending_exe = f->second.pending_exe;
          threads_.erase(f);
        }
      }
      t.tgid = pid;
      t.exe = t.pending_exe.empty() ? t.exe : t.pending_exe;
      t.pending_exe.clear();
      t.scratch = 0;  // a new address space
      t.gen = ++gen_[pid];
      pool_.erase(pid);
      ptrace(PTRACE_CONT, pid, nullptr, nullptr);
      return;
    }
    if (event == PTRACE_EVENT_STOP) {
      if (sig == SIGSTOP || sig == SIGTSTP || sig == SIGTTIN || sig == SIGTTOU) {
        ptrace(PTRACE_LISTEN, pid, nullptr, nullptr);  // a group-stop: stays stopped until SIGCONT
      } else {
        ptrace(PTRACE_CONT, pid, nullptr, nullptr);  // a new tracee's first stop
      }
      return;
    }
    if (event != 0) {
      ptrace(PTRACE_CONT, pid, nullptr, nullptr);
      return;
    }
    ptrace(PTRACE_CONT, pid, nullptr, reinterpret_cast<void*>(static_cast<long>(sig)));  // deliver it
  }

  // Answer the syscall without running it.
  static void answer(pid_t pid, user_regs_struct& r, long result) {
    r.orig_rax = static_cast<unsigned long long>(-1);
    r.rax = static_cast<unsigned long long>(result);
    ptrace(PTRACE_SETREGS, pid, nullptr, &r);
  }

  // A mapping for this thread: one from the process's pool, or inject mmap and restart.
  bool ensure_scratch(pid_t pid, Thread& t, user_regs_struct& r) {
    const unsigned g = gen_[t.tgid];
    if (t.scratch && t.gen == g) return true;
    auto& pool = pool_[t.tgid];
    if (!pool.empty()) {
      t.scratch = pool.back();
      t.gen = g;
      pool.pop_back();
      return true;
    }
    t.saved = r;
    t.fix = Fix::kInject;
    user_regs_struct m = r;
    m.orig_rax = SYS_mmap;
    m.rdi = 0;
    m.rsi = kScratch;
    m.rdx = PROT_READ | PROT_WRITE;
    m.r10 = MAP_PRIVATE | MAP_ANONYMOUS;
    m.r8 = static_cast<unsigned long long>(-1);
    m.r9 = 0;
    ptrace(PTRACE_SETREGS, pid, nullptr, &m);
    return false;
  }

  std::string guest_of_fd(pid_t pid, long fd) const {
    char path[64], buf[PATH_MAX];
    if (fd == AT_FDCWD) std::snprintf(path, sizeof(path), "/proc/%d/cwd", pid);
    else std::snprintf(path, sizeof(path), "/proc/%d/fd/%ld", pid, fd);
    const ssize_t n = readlink(path, buf, sizeof(buf) - 1);
    if (n <= 0 || buf[0] != '/') return "";
    return view_.to_guest(std::string(buf, static_cast<size_t>(n)));
  }

  // Translate the path in argument `pi` (relative to the directory fd in argument `di`; -1: the
  // cwd). 0: done (or nothing to do), else -errno to answer with.
  long path_arg(pid_t pid, user_regs_struct& r, Arena& a, int di, int pi, bool follow, bool cow = false,
                std::string* host_out = nullptr, std::string* guest_out = nullptr) {
    std::string p;
    if (!read_str(pid, arg(r, pi), &p)) return arg(r, pi) == 0 ? 0 : -EFAULT;
    if (p.empty()) return 0;  // AT_EMPTY_PATH or ENOENT: the kernel's answer either way
    std::string guest = p;
    if (p[0] != '/') {
      const long dirfd = di < 0 ? AT_FDCWD : static_cast<int>(arg(r, di));
      const std::string base = guest_of_fd(pid, dirfd);
      if (base.empty()) return 0;  // not a directory we know: the kernel answers (ENOTDIR, EBADF)
      guest = base + "/" + p;
    }
    std::string host;
    if (const int rc = view_.resolve(guest, follow, &host); rc < 0) return rc;
    if (cow) {
      if (const int rc = view_.copy_up(host); rc < 0) return rc;
    }
    if (host_out) *host_out = host;
    if (guest_out) *guest_out = guest;
    if (host == p) return 0;  // the host's own path (/dev, /sys, /proc, a volume at its own path): as is
    const unsigned long at = a.str(host);
    if (at == 0) return -ENAMETOOLONG;
    arg(r, pi) = at;
    return 0;
  }

  static bool open_writes(long flags) { return (flags & O_ACCMODE) != O_RDONLY || (flags & O_TRUNC); }
  static bool open_follows(long flags) {
    return !(flags & O_NOFOLLOW) && !((flags & O_CREAT) && (flags & O_EXCL));
  }

  // fchmod/fchown/futimens/fsetxattr on a file still shared with the image: copy it up and do
  // the call on the copy (the fd keeps naming the image's inode). 1: answered, 0: run it as is.
  int fd_cow(pid_t pid, user_regs_struct& r, long nr) {
    char path[64], buf[PATH_MAX];
    std::snprintf(path, sizeof(path), "/proc/%d/fd/%d", pid, static_cast<int>(r.rdi));
    struct stat st {};
    if (stat(path, &st) != 0 || !view_.shared_with_image(st)) return 0;
    const ssize_t n = readlink(path, buf, sizeof(buf) - 1);
    if (n <= 0) return 0;
    const std::string host(buf, static_cast<size_t>(n));
    long rc = view_.copy_up(host);
    if (rc == 0) {
      if (nr == SYS_fchmod) {
        rc = chmod(host.c_str(), static_cast<mode_t>(r.rsi)) == 0 ? 0 : -errno;
      } else if (nr == SYS_fchown) {
        rc = chown(host.c_str(), static_cast<uid_t>(r.rsi), static_cast<gid_t>(r.rdx)) == 0 ? 0 : -errno;
      } else if (nr == SYS_utimensat) {
        struct timespec ts[2];
        if (r.rdx != 0 && !read_mem(pid, r.rdx, ts, sizeof(ts))) rc = -EFAULT;
        else rc = utimensat(AT_FDCWD, host.c_str(), r.rdx ? ts : nullptr, 0) == 0 ? 0 : -errno;
      } else {
        rc = -EPERM;  // xattrs through an fd of the image's file
      }
    }
    answer(pid, r, rc);
    return 1;
  }

  long sockaddr_arg(pid_t pid, user_regs_struct& r, Arena& a, bool follow) {
    const socklen_t len = static_cast<socklen_t>(r.rdx);
    sockaddr_un su{};
    if (len <= offsetof(sockaddr_un, sun_path) || len > sizeof(su)) return 0;
    if (!read_mem(pid, r.rsi, &su, len) || su.sun_family != AF_UNIX || su.sun_path[0] == '\0') return 0;
    const std::string p(su.sun_path, strnlen(su.sun_path, len - offsetof(sockaddr_un, sun_path)));
    std::string guest = p[0] == '/' ? p : guest_of_fd(pid, AT_FDCWD) + "/" + p, host;
    if (const int rc = view_.resolve(guest, follow, &host); rc < 0) return rc;
    if (host.size() >= sizeof(su.sun_path)) return -ENAMETOOLONG;
    sockaddr_un out{};
    out.sun_family = AF_UNIX;
    std::memcpy(out.sun_path, host.c_str(), host.size() + 1);
    const socklen_t n = static_cast<socklen_t>(offsetof(sockaddr_un, sun_path) + host.size() + 1);
    const unsigned long at = a.put(&out, n);
    if (at == 0) return -ENOMEM;
    r.rsi = at;
    r.rdx = n;
    return 0;
  }

  bool argv0_supported(const std::string& loader_host) {
    auto it = argv0_ok_.find(loader_host);
    if (it != argv0_ok_.end()) return it->second;
    bool ok = false;
    if (FILE* f = std::fopen(loader_host.c_str(), "rb")) {
      std::string data;
      char buf[65536];
      size_t n;
      while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0 && data.size() < (16u << 20)) data.append(buf, n);
      std::fclose(f);
      ok = data.find(std::string("--argv0\0", 8)) != std::string::npos ||
           data.find("argv0") != std::string::npos;
    }
    argv0_ok_[loader_host] = ok;
    return ok;
  }

  // execve/execveat: binfmt inside the image. 0 or -errno.
  long exec_arg(pid_t pid, Thread& t, user_regs_struct& r, Arena& a, bool at) {
    const int di = at ? 0 : -1, pi = at ? 1 : 0, vi = at ? 2 : 1, ei = at ? 3 : 2;
    const long flags = at ? static_cast<long>(r.r8) : 0;
    std::string given;
    if (!read_str(pid, arg(r, pi), &given)) return -EFAULT;
    std::string guest, host;
    if (given.empty() && (flags & AT_EMPTY_PATH)) {  // fexecve
      guest = guest_of_fd(pid, static_cast<long>(arg(r, di)));
      if (guest.empty()) return -EBADF;
    } else if (given.empty()) {
      return -ENOENT;
    } else {
      guest = given[0] == '/' ? given : guest_of_fd(pid, di < 0 ? AT_FDCWD : static_cast<long>(arg(r, di))) + "/" + given;
    }
    if (const int rc = view_.resolve(guest, !(flags & AT_SYMLINK_NOFOLLOW), &host); rc < 0) return rc;
    // the program's argv: pointers kept (untouched strings stay where they are)
    std::vector<unsigned long> ptrs;
    for (unsigned long p = arg(r, vi);; p += 8) {
      unsigned long v = 0;
      if (!read_mem(pid, p, &v, 8)) return -EFAULT;
      if (v == 0) break;
      ptrs.push_back(v);
      if (ptrs.size() > 65536) return -E2BIG;
    }
    bool changed = false;
    std::string name = given;          // what a script's interpreter is handed as the script
    for (int depth = 0; depth < 5; ++depth) {
      // the kernel's own check, made here: what runs in the end may be the loader, not this file
      if (faccessat(AT_FDCWD, host.c_str(), X_OK, AT_EACCESS) != 0) {
        if (errno == EACCES || errno == ENOENT || errno == ENOTDIR || errno == ELOOP) return -errno;
        break;
      }
      char head[256] = {};
      const int fd = open(host.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) break;  // the kernel answers (EACCES, ENOENT)
      const ssize_t n = read(fd, head, sizeof(head) - 1);
      if (n >= 2 && head[0] == '#' && head[1] == '!') {
        close(fd);
        std::string line(head + 2, static_cast<size_t>(n - 2));
        line = line.substr(0, line.find('\n'));
        size_t b = line.find_first_not_of(" \t");
        if (b == std::string::npos) return -ENOEXEC;
        size_t e = line.find_first_of(" \t", b);
        const std::string interp = line.substr(b, e == std::string::npos ? std::string::npos : e - b);
        std::string opt;
        if (e != std::string::npos) {
          const size_t ob = line.find_first_not_of(" \t", e);
          if (ob != std::string::npos) {
            opt = line.substr(ob);
            opt.erase(opt.find_last_not_of(" \t\r") + 1);
          }
        }
        // binfmt_script: argv = interp [opt] script argv[1:]
        std::vector<unsigned long> nf;
        nf.push_back(a.str(interp));
        if (!opt.empty()) nf.push_back(a.str(opt));
        nf.push_back(a.str(name));
        if (!ptrs.empty()) ptrs.erase(ptrs.begin());
        ptrs.insert(ptrs.begin(), nf.begin(), nf.end());
        changed = true;
        name = interp;
        guest = interp[0] == '/' ? interp : guest_of_fd(pid, AT_FDCWD) + "/" + interp;
        if (const int rc = view_.resolve(guest, true, &host); rc < 0) return rc;
        continue;
      }
      // an ELF with a loader: start it through the image's loader
      Elf64_Ehdr eh{};
      std::string interp;
      if (pread(fd, &eh, sizeof(eh), 0) == sizeof(eh) && !std::memcmp(eh.e_ident, ELFMAG, SELFMAG) &&
          eh.e_ident[EI_CLASS] == ELFCLASS64 && eh.e_phentsize == sizeof(Elf64_Phdr) && eh.e_phnum < 256) {
        std::vector<Elf64_Phdr> ph(eh.e_phnum);
        const ssize_t want = static_cast<ssize_t>(ph.size() * sizeof(Elf64_Phdr));
        if (pread(fd, ph.data(), static_cast<size_t>(want), static_cast<off_t>(eh.e_phoff)) == want) {
          for (const auto& h : ph) {
            if (h.p_type != PT_INTERP || h.p_filesz == 0 || h.p_filesz > PATH_MAX) continue;
            interp.resize(h.p_filesz);
            if (pread(fd, interp.data(), h.p_filesz, static_cast<off_t>(h.p_offset)) != static_cast<ssize_t>(h.p_filesz))
              interp.clear();
            interp = interp.c_str();
          }
        }
      }
      close(fd);
      const std::string prog_guest = view_.to_guest(host);
      t.pending_exe = prog_guest;
      if (!interp.empty()) {
        std::string loader;
        if (const int rc = view_.resolve(interp, true, &loader); rc < 0) return rc;
        // ld.so [--argv0 ARGV0] PROGRAM ARGS...
        std::vector<unsigned long> nf{a.str(interp)};
        if (!ptrs.empty() && argv0_supported(loader)) {
          nf.push_back(a.str("--argv0"));
          nf.push_back(ptrs[0]);
        }
        nf.push_back(a.str(prog_guest));
        if (!ptrs.empty()) ptrs.erase(ptrs.begin());
        ptrs.insert(ptrs.begin(), nf.begin(), nf.end());
        changed = true;
        host = loader;
      }
      break;
    }
    for (unsigned long p : ptrs)
      if (p == 0) return -ENOMEM;
    const unsigned long file = a.str(host);
    if (file == 0) return -ENAMETOOLONG;
    unsigned long argv = arg(r, vi);
    if (changed) {
      ptrs.push_back(0);
      argv = a.put(ptrs.data(), ptrs.size() * 8);
      if (argv == 0) return -E2BIG;
    }
    const unsigned long envp = arg(r, ei);
    r.orig_rax = SYS_execve;  // execveat resolved: a plain execve of the host path
    r.rdi = file;
    r.rsi = argv;
    r.rdx = envp;
    return 0;
  }

  // The stop at a filtered syscall's entry. True: stop again at its exit.
  bool on_entry(pid_t pid, Thread& t) {
    if (log_ == nullptr) return entry(pid, t);
    user_regs_struct before{};
    ptrace(PTRACE_GETREGS, pid, nullptr, &before);
    std::string p0;
    read_str(pid, before.rdi, &p0);
    std::string p1;
    read_str(pid, before.rsi, &p1);
    const bool exit_stop = entry(pid, t);
    if (t.fix == Fix::kInject) return exit_stop;
    user_regs_struct after{};
    ptrace(PTRACE_GETREGS, pid, nullptr, &after);
    std::string h0, h1;
    if (after.rdi != before.rdi) read_str(pid, after.rdi, &h0);
    if (after.rsi != before.rsi) read_str(pid, after.rsi, &h1);
    char head[96];
    std::snprintf(head, sizeof(head), "%d nr=%lld", pid, static_cast<long long>(before.orig_rax));
    t.trace = std::string(head) + " a0=\"" + p0.substr(0, 200) + "\"" + (h0.empty() ? "" : " -> \"" + h0 + "\"") +
              " a1=\"" + p1.substr(0, 200) + "\"" + (h1.empty() ? "" : " -> \"" + h1 + "\"");
    if (static_cast<long long>(after.orig_rax) == -1) {  // answered here
      std::fprintf(log_, "%s = %lld (answered)\n", t.trace.c_str(), static_cast<long long>(after.rax));
      std::fflush(log_);
      t.trace.clear();
      return exit_stop;
    }
    return true;  // see its result
  }

  bool entry(pid_t pid, Thread& t) {
    user_regs_struct r{};
    if (ptrace(PTRACE_GETREGS, pid, nullptr, &r) != 0) return false;
    const long nr = static_cast<long>(r.orig_rax);
    switch (nr) {  // answered without translation
      case SYS_openat2:
      case SYS_uselib:
        answer(pid, r, -ENOSYS);
        return false;
      case SYS_chroot:
      case SYS_mount:
      case SYS_umount2:
      case SYS_pivot_root:
      case SYS_open_tree:
      case SYS_move_mount:
      case SYS_fsopen:
      case SYS_fsmount:
      case SYS_fspick:
      case SYS_mount_setattr:
      case SYS_fanotify_mark:
      case SYS_acct:
      case SYS_swapon:
      case SYS_swapoff:
      case SYS_quotactl:
        answer(pid, r, -EPERM);
        return false;
      case SYS_name_to_handle_at:
        answer(pid, r, -EOPNOTSUPP);
        return false;
      case SYS_getcwd:
        t.fix = Fix::kGetcwd;
        return true;
      case SYS_uname:
        if (view_.hostname.empty()) return false;
        t.fix = Fix::kUname;
        return true;
      case SYS_fchmod:
      case SYS_fchown:
      case SYS_fsetxattr:
      case SYS_fremovexattr:
        fd_cow(pid, r, nr);
        return false;
      case SYS_utimensat:
        if (r.rsi == 0) {  // futimens(fd)
          fd_cow(pid, r, nr);
          return false;
        }
        break;
      default:
        break;
    }
    // Translated first with the thread's mapping if it has one; a thread that has none gets
    // one only when a string must be written (paths of the host's own trees need none, so a GPU
    // runtime's threads reading /sys and /dev never map anything): from its process's pool, or
    // by injecting mmap, whose exit restarts this syscall.
    const user_regs_struct orig = r;
    const bool mapped = t.scratch && t.gen == gen_[t.tgid];
    Arena a{pid, mapped ? t.scratch : 0};
    long rc = translate(pid, t, r, a, nr);
    if (rc >= 0 && a.needed) {
      user_regs_struct again = orig;
      t.fix = Fix::kNone;
      if (!ensure_scratch(pid, t, again)) return true;
      r = orig;
      Arena b{pid, t.scratch};
      rc = translate(pid, t, r, b, nr);
    }
    if (rc < 0) {
      t.fix = Fix::kNone;
      answer(pid, r, rc);
      return false;
    }
    if (std::memcmp(&orig, &r, sizeof(r)) != 0) ptrace(PTRACE_SETREGS, pid, nullptr, &r);
    return t.fix != Fix::kNone;
  }

  // The path arguments of syscall `nr` rewritten in `r` (strings in `a`); 0 or -errno.
  long translate(pid_t pid, Thread& t, user_regs_struct& r, Arena& a, long nr) {
    long rc = 0;
    std::string host;
    switch (nr) {
      case SYS_open: rc = path_arg(pid, r, a, -1, 0, open_follows(static_cast<long>(r.rsi)), open_writes(static_cast<long>(r.rsi))); break;
      case SYS_creat: rc = path_arg(pid, r, a, -1, 0, true, true); break;
      case SYS_openat: rc = path_arg(pid, r, a, 0, 1, open_follows(static_cast<long>(r.rdx)), open_writes(static_cast<long>(r.rdx))); break;
      case SYS_stat:
      case SYS_access:
      case SYS_chdir:
      case SYS_statfs:
      case SYS_getxattr:
      case SYS_listxattr: rc = path_arg(pid, r, a, -1, 0, true); break;
      case SYS_truncate:
      case SYS_chmod:
      case SYS_chown:
      case SYS_utime:
      case SYS_utimes:
      case SYS_setxattr:
      case SYS_removexattr: rc = path_arg(pid, r, a, -1, 0, true, true); break;
      case SYS_lstat:
      case SYS_mkdir:
      case SYS_rmdir:
      case SYS_unlink:
      case SYS_mknod:
      case SYS_lgetxattr:
      case SYS_llistxattr: rc = path_arg(pid, r, a, -1, 0, false); break;
      case SYS_lchown:
      case SYS_lsetxattr:
      case SYS_lremovexattr: rc = path_arg(pid, r, a, -1, 0, false, true); break;
      case SYS_readlink:
        rc = path_arg(pid, r, a, -1, 0, false, false, &host);
        if (rc == 0 && under("/proc", host)) {
          t.fix = Fix::kReadlink, t.buf_arg = 1, t.size_arg = 2, t.link = host;
        }
        break;
      case SYS_readlinkat:
        rc = path_arg(pid, r, a, 0, 1, false, false, &host);
        if (rc == 0 && under("/proc", host)) {
          t.fix = Fix::kReadlink, t.buf_arg = 2, t.size_arg = 3, t.link = host;
        }
        break;
      case SYS_inotify_add_watch: rc = path_arg(pid, r, a, -1, 1, !(r.rdx & 0x02000000 /* IN_DONT_FOLLOW */)); break;
      case SYS_rename:
      case SYS_link:
        rc = path_arg(pid, r, a, -1, 0, false);
        if (rc == 0) rc = path_arg(pid, r, a, -1, 1, false);
        break;
      case SYS_symlink: rc = path_arg(pid, r, a, -1, 1, false); break;
      case SYS_newfstatat: rc = path_arg(pid, r, a, 0, 1, !(r.r10 & AT_SYMLINK_NOFOLLOW)); break;
      case SYS_statx: rc = path_arg(pid, r, a, 0, 1, !(r.rdx & AT_SYMLINK_NOFOLLOW)); break;
      case SYS_faccessat: rc = path_arg(pid, r, a, 0, 1, true); break;
      case SYS_faccessat2: rc = path_arg(pid, r, a, 0, 1, !(r.r10 & AT_SYMLINK_NOFOLLOW)); break;
      case SYS_mkdirat:
      case SYS_mknodat:
      case SYS_unlinkat: rc = path_arg(pid, r, a, 0, 1, false); break;
      case SYS_fchownat: rc = path_arg(pid, r, a, 0, 1, !(r.r8 & AT_SYMLINK_NOFOLLOW), true); break;
      case SYS_futimesat:
      case SYS_fchmodat: rc = path_arg(pid, r, a, 0, 1, true, true); break;
      case SYS_fchmodat2: rc = path_arg(pid, r, a, 0, 1, !(r.r10 & AT_SYMLINK_NOFOLLOW), true); break;
      case SYS_utimensat: rc = path_arg(pid, r, a, 0, 1, !(r.r10 & AT_SYMLINK_NOFOLLOW), true); break;
      case SYS_renameat:
      case SYS_renameat2:
        rc = path_arg(pid, r, a, 0, 1, false);
        if (rc == 0) rc = path_arg(pid, r, a, 2, 3, false);
        break;
      case SYS_linkat:
        rc = path_arg(pid, r, a, 0, 1, (r.r8 & AT_SYMLINK_FOLLOW) != 0);
        if (rc == 0) rc = path_arg(pid, r, a, 2, 3, false);
        break;
      case SYS_symlinkat: rc = path_arg(pid, r, a, 1, 2, false); break;
      case SYS_execve: rc = exec_arg(pid, t, r, a, false); break;
      case SYS_execveat: rc = exec_arg(pid, t, r, a, true); break;
      case SYS_bind: rc = sockaddr_arg(pid, r, a, false); break;
      case SYS_connect: rc = sockaddr_arg(pid, r, a, true); break;
      default: break;
    }
    return rc;
  }

  void on_exit(pid_t pid, Thread& t) {
    user_regs_struct r{};
    const Fix fix = t.fix;
    t.fix = Fix::kNone;
    if (ptrace(PTRACE_GETREGS, pid, nullptr, &r) != 0) return;
    const long ret = static_cast<long>(r.rax);
    if (log_ != nullptr && !t.trace.empty() && fix != Fix::kInject) {
      std::fprintf(log_, "%s = %ld%s\n", t.trace.c_str(), ret, ret < 0 && ret > -4096 ? (std::string(" ") + std::strerror(static_cast<int>(-ret))).c_str() : "");
      std::fflush(log_);
      t.trace.clear();
    }
    if (fix == Fix::kInject) {
      user_regs_struct back = t.saved;
      if (ret < 0 && ret > -4096) {  // no mapping: the syscall fails
        back.rax = static_cast<unsigned long long>(-ENOMEM);
      } else {
        t.scratch = static_cast<unsigned long>(ret);
        t.gen = gen_[t.tgid];
        back.rip -= 2;  // re-run the syscall instruction: its entry stops again, with a mapping
        back.rax = back.orig_rax;
      }
      ptrace(PTRACE_SETREGS, pid, nullptr, &back);
      return;
    }
    if (ret < 0) return;
    if (fix == Fix::kGetcwd && ret > 0) {
      std::string cwd;
      if (!read_str(pid, r.rdi, &cwd)) return;
      const std::string g = view_.to_guest(cwd);
      if (g.size() + 1 > r.rsi) {
        r.rax = static_cast<unsigned long long>(-ERANGE);
      } else {
        write_mem(pid, r.rdi, g.c_str(), g.size() + 1);
        r.rax = g.size() + 1;
      }
      ptrace(PTRACE_SETREGS, pid, nullptr, &r);
    } else if (fix == Fix::kReadlink && ret > 0) {
      std::string content(static_cast<size_t>(ret), '\0');
      if (!read_mem(pid, arg(r, t.buf_arg), content.data(), content.size())) return;
      std::string g;
      if (t.link.size() > 4 && t.link.compare(t.link.size() - 4, 4, "/exe") == 0) {
        // /proc/<pid>/exe of a traced process: its program, not the loader it was started by
        const std::string pidpart = t.link.substr(6, t.link.size() - 10);
        const pid_t whose = pidpart == "self" ? t.tgid : static_cast<pid_t>(std::atoi(pidpart.c_str()));
        auto w = threads_.find(whose);
        if (w != threads_.end() && !w->second.exe.empty()) g = w->second.exe;
      }
      if (g.empty()) {
        if (content[0] != '/') return;
        g = view_.to_guest(content);
      }
      const size_t n = std::min<size_t>(g.size(), arg(r, t.size_arg));
      write_mem(pid, arg(r, t.buf_arg), g.data(), n);
      r.rax = n;
      ptrace(PTRACE_SETREGS, pid, nullptr, &r);
    } else if (fix == Fix::kUname) {
      char node[sizeof(utsname::nodename)] = {};
      std::strncpy(node, view_.hostname.c_str(), sizeof(node) - 1);
      write_mem(pid, r.rdi + offsetof(utsname, nodename), node, sizeof(node));
    }
  }
};

// Can this user supervise a child this way (PTRACE_SEIZE of its own child, a seccomp filter that
// traces)? "" if so, else what failed.
inline std::string probe() {
  int pfd[2];
  if (pipe2(pfd, O_CLOEXEC) != 0) return std::string("pipe: ") + std::strerror(errno);
  const pid_t pid = fork();
  if (pid < 0) return std::string("fork: ") + std::strerror(errno);
  if (pid == 0) {
    close(pfd[1]);
    char c;
    if (read(pfd[0], &c, 1) != 1) _exit(2);
    if (install_filter() != 0) _exit(3);
    char buf[PATH_MAX];
    syscall(SYS_getcwd, buf, sizeof(buf));  // stops at the supervisor (whatever it answers)
    _exit(0);
  }
  close(pfd[0]);
  int st = 0;
  if (ptrace(PTRACE_SEIZE, pid, nullptr, reinterpret_cast<void*>(PTRACE_O_TRACESECCOMP | PTRACE_O_EXITKILL)) != 0) {
    const std::string why = std::string("ptrace(PTRACE_SEIZE): ") + std::strerror(errno);
    close(pfd[1]);
    waitpid(pid, &st, 0);
    return why;
  }
  if (write(pfd[1], "g", 1) != 1) return "release the child";
  close(pfd[1]);
  bool saw_seccomp = false;
  for (;;) {
    if (waitpid(pid, &st, __WALL) < 0) return std::string("waitpid: ") + std::strerror(errno);
    if (WIFEXITED(st) || WIFSIGNALED(st)) break;
    const int event = st >> 16;
    if (event == PTRACE_EVENT_SECCOMP) saw_seccomp = true;
    ptrace(PTRACE_CONT, pid, nullptr, reinterpret_cast<void*>(static_cast<long>(event == 0 ? WSTOPSIG(st) : 0)));
  }
  if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) return "the traced child failed (seccomp filter refused?)";
  return saw_seccomp ? "" : "no seccomp stop was seen";
}

}  // namespace tk8s::troot
