// Development probe (not part of the product build): may an ordinary user on this machine trace
// its own child with ptrace(2)? VERDICT r5 #8 asks before a ptrace path-translation rootfs mode
// for tk8s-container is attempted on the GPU tier (no root, no user namespaces there).
//
//   g++ -O2 -o build/ptrace_probe native/bench/ptrace_probe.cpp && build/ptrace_probe
//
// Prints one JSON line: the Yama scope, whether PTRACE_TRACEME + PTRACE_SYSCALL stops worked on a
// child that runs /bin/true, how many syscall stops were seen, and whether PTRACE_O_EXITKILL and
// PTRACE_GETREGS were allowed; plus whether unprivileged user namespaces can be made.
#include <errno.h>
#include <sched.h>
#include <signal.h>
#include <sys/ptrace.h>
#include <sys/user.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>

int main() {
  std::string scope = "absent";
  {
    std::ifstream f("/proc/sys/kernel/yama/ptrace_scope");
    if (f) std::getline(f, scope);
  }
  int traceme_errno = 0, setopt_errno = 0, regs_errno = 0, stops = 0, status_exit = -1;
  const pid_t pid = fork();
  if (pid == 0) {
    if (ptrace(PTRACE_TRACEME, 0, nullptr, nullptr) != 0) _exit(100 + errno % 100);
    raise(SIGSTOP);
    execl("/bin/true", "true", static_cast<char*>(nullptr));
    _exit(127);
  }
  int st = 0;
  waitpid(pid, &st, 0);
  if (WIFEXITED(st)) {
    traceme_errno = WEXITSTATUS(st) - 100;
  } else {
    if (ptrace(PTRACE_SETOPTIONS, pid, nullptr,
               reinterpret_cast<void*>(PTRACE_O_TRACESYSGOOD | PTRACE_O_EXITKILL)) != 0)
      setopt_errno = errno;
    for (int i = 0; i < 10000; ++i) {
      if (ptrace(PTRACE_SYSCALL, pid, nullptr, nullptr) != 0) break;
      if (waitpid(pid, &st, 0) < 0) break;
      if (WIFEXITED(st)) {
        status_exit = WEXITSTATUS(st);
        break;
      }
      if (WIFSTOPPED(st) && WSTOPSIG(st) == (SIGTRAP | 0x80)) {
        ++stops;
        if (stops == 1) {
          user_regs_struct regs;
          if (ptrace(PTRACE_GETREGS, pid, nullptr, &regs) != 0) regs_errno = errno;
        }
      }
    }
  }
  // unprivileged user namespace (the container runtime's other unprivileged path)
  int userns_errno = 0;
  const pid_t c = fork();
  if (c == 0) _exit(unshare(CLONE_NEWUSER) == 0 ? 0 : 100 + errno % 100);
  waitpid(c, &st, 0);
  if (WIFEXITED(st) && WEXITSTATUS(st) >= 100) userns_errno = WEXITSTATUS(st) - 100;
  std::printf(
      "{\"yama_ptrace_scope\":\"%s\",\"traceme_errno\":%d,\"setoptions_errno\":%d,\"getregs_errno\":%d,"
      "\"syscall_stops\":%d,\"child_exit\":%d,\"ptrace_ok\":%s,\"userns_errno\":%d,\"userns_ok\":%s}\n",
      scope.c_str(), traceme_errno, setopt_errno, regs_errno, stops, status_exit,
      (traceme_errno == 0 && stops > 0 && regs_errno == 0 && status_exit == 0) ? "true" : "false", userns_errno,
      userns_errno == 0 ? "true" : "false");
  return 0;
}
