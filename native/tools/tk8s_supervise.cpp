// tk8s-supervise: restart-policy process supervisor (the `docker run --restart=unless-stopped`
// of the reference's rancher/server and rancher/agent containers,
// ansible/roles/ranchermaster/tasks/main.yml:11, rancherhost/tasks/main.yml:26-34).
//
//   tk8s-supervise --pidfile F [--log L] [--restart no|on-failure|always|unless-stopped]
//                  [--max-restarts N] [--backoff-ms M] -- PROGRAM [ARGS...]
//   tk8s-supervise --spawn-list FILE
//
// --spawn-list: start one supervisor per line of FILE (its arguments, tab-separated), each in its
// own session, and exit. The bring-up's CLI hands its node-agent zygotes to this one process
// instead of spawning N supervisors itself: Python's os.posix_spawn keeps the GIL through each
// vfork until the exec, ~5 ms of the CLI's own start at 8 workers (profiles/r6_curve/).
//
// * Starts a new session; the child stays in the supervisor's process group, so one
//   killpg(pgid) from teardown stops both.
// * SIGTERM/SIGINT: stop restarting, forward SIGTERM to the child, wait, exit with its code.
// * Child exit: restart per policy with capped exponential back-off (reset after 10 s up).
// * Pidfile (JSON, atomic rename): {"pid": supervisor, "pgid": pgid, "child": child, "restarts": n}.
// Pure POSIX (no HIP): it never touches the GPU, so it may spawn freely.
#include <fcntl.h>
#include <signal.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

volatile sig_atomic_t g_stop = 0;
volatile pid_t g_child = -1;

void on_signal(int) {
  g_stop = 1;
  if (g_child > 0) kill(g_child, SIGTERM);
}

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// Field 22 of /proc/self/stat (start time, clock ticks since boot): with the pid, the identity
// teardown checks before it signals the group (utils/procs.py pidfile_owner_alive).
long long start_ticks() {
  FILE* f = std::fopen("/proc/self/stat", "r");
  if (!f) return -1;
  char buf[1024];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* p = std::strrchr(buf, ')');
  if (!p) return -1;
  long long v = -1;
  for (int field = 2; p && *p; ++field) {  // field 2 ends at ')'; fields are space separated after it
    p = std::strchr(p, ' ');
    if (!p) break;
    ++p;
    if (field + 1 == 22) {
      v = std::atoll(p);
      break;
    }
  }
  return v;
}

void write_pidfile(const std::string& path, pid_t child, int restarts) {
  if (path.empty()) return;
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "w");
  if (!f) return;
  static const long long start = start_ticks();
  std::fprintf(f, "{\"pid\": %d, \"pgid\": %d, \"child\": %d, \"restarts\": %d, \"supervisor\": \"tk8s-supervise\"",
               static_cast<int>(getpid()), static_cast<int>(getpgrp()), static_cast<int>(child), restarts);
  if (start >= 0) std::fprintf(f, ", \"start\": %lld", start);
  std::fprintf(f, "}\n");
  std::fclose(f);
  std::rename(tmp.c_str(), path.c_str());
}

int spawn_list(const char* list) {
  FILE* f = std::fopen(list, "r");
  if (!f) {
    std::fprintf(stderr, "tk8s-supervise: %s: %s\n", list, std::strerror(errno));
    return 2;
  }
  std::string text;
  char buf[4096];
  for (size_t n; (n = std::fread(buf, 1, sizeof buf, f)) > 0;) text.append(buf, n);
  std::fclose(f);
  int started = 0;
  size_t at = 0;
  while (at < text.size()) {
    size_t eol = text.find('\n', at);
    if (eol == std::string::npos) eol = text.size();
    std::vector<std::string> args{"tk8s-supervise"};
    for (size_t i = at; i <= eol;) {
      size_t tab = text.find('\t', i);
      if (tab == std::string::npos || tab > eol) tab = eol;
      args.push_back(text.substr(i, tab - i));
      i = tab + 1;
    }
    at = eol + 1;
    if (args.size() < 3) continue;  // a blank line
    const pid_t pid = fork();
    if (pid < 0) return 1;
    if (pid == 0) {
      std::vector<char*> av;
      for (auto& a : args) av.push_back(&a[0]);
      av.push_back(nullptr);
      execv("/proc/self/exe", av.data());
      _exit(127);
    }
    ++started;
  }
  return started > 0 ? 0 : 1;
}

int usage() {
  std::fprintf(stderr,
               "usage: tk8s-supervise --pidfile F [--log L] [--restart no|on-failure|always|unless-stopped]\n"
               "                      [--max-restarts N] [--backoff-ms M] -- PROGRAM [ARGS...]\n");
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc == 3 && std::strcmp(argv[1], "--spawn-list") == 0) return spawn_list(argv[2]);
  std::string pidfile, log, policy = "unless-stopped";
  long max_restarts = -1, backoff_ms = 100;
  int i = 1;
  for (; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--") { ++i; break; }
    if (i + 1 >= argc) return usage();
    if (a == "--pidfile") pidfile = argv[++i];
    else if (a == "--log") log = argv[++i];
    else if (a == "--restart") policy = argv[++i];
    else if (a == "--max-restarts") max_restarts = std::strtol(argv[++i], nullptr, 10);
    else if (a == "--backoff-ms") backoff_ms = std::strtol(argv[++i], nullptr, 10);
    else return usage();
  }
  if (i >= argc) return usage();
  if (policy != "no" && policy != "on-failure" && policy != "always" && policy != "unless-stopped")
    return usage();
  std::vector<char*> child_argv(argv + i, argv + argc);
  child_argv.push_back(nullptr);

  if (getpgrp() != getpid()) setsid();
  if (!log.empty()) {
    const int fd = open(log.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd >= 0) {
      dup2(fd, STDOUT_FILENO);
      dup2(fd, STDERR_FILENO);
      close(fd);
    }
  }
  struct sigaction sa;
  std::memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_signal;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  signal(SIGHUP, SIG_IGN);

  int restarts = 0, status = 0;
  long delay = backoff_ms;
  // SIGTERM/SIGINT stay blocked across fork(): a signal landing before the child has reset its
  // handlers would otherwise run on_signal in the child and be lost, and the program then exec'd
  // would never see the stop. Pending signals are delivered after the unblock (in the child:
  // with the default action; in the parent: once g_child names the child).
  sigset_t term_set, old_set;
  sigemptyset(&term_set);
  sigaddset(&term_set, SIGTERM);
  sigaddset(&term_set, SIGINT);
  while (!g_stop) {
    const double started = now_s();
    sigprocmask(SIG_BLOCK, &term_set, &old_set);
    const pid_t pid = fork();
    if (pid < 0) {
      sigprocmask(SIG_SETMASK, &old_set, nullptr);
      std::perror("tk8s-supervise: fork");
      return 1;
    }
    if (pid == 0) {
      signal(SIGTERM, SIG_DFL);
      signal(SIGINT, SIG_DFL);
      signal(SIGHUP, SIG_DFL);
      sigprocmask(SIG_SETMASK, &old_set, nullptr);
      execvp(child_argv[0], child_argv.data());
      std::fprintf(stderr, "tk8s-supervise: exec %s: %s\n", child_argv[0], std::strerror(errno));
      _exit(127);
    }
    g_child = pid;
    sigprocmask(SIG_SETMASK, &old_set, nullptr);
    if (g_stop) kill(pid, SIGTERM);  // stopped before this fork: do not leave the child running
    write_pidfile(pidfile, pid, restarts);
    while (waitpid(pid, &status, 0) < 0 && errno == EINTR) {
    }
    g_child = -1;
    const int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + WTERMSIG(status);
    if (g_stop) break;
    const bool failed = code != 0;
    const bool again = policy == "always" || policy == "unless-stopped" || (policy == "on-failure" && failed);
    if (!again || (max_restarts >= 0 && restarts >= max_restarts)) {
      std::fprintf(stderr, "tk8s-supervise: %s exited with %d; not restarting\n", child_argv[0], code);
      if (!pidfile.empty()) unlink(pidfile.c_str());
      return code;
    }
    if (now_s() - started > 10.0) delay = backoff_ms;  // it ran fine for a while: reset back-off
    std::fprintf(stderr, "tk8s-supervise: %s exited with %d; restart #%d in %ld ms\n", child_argv[0], code,
                 restarts + 1, delay);
    std::fflush(stderr);
    timespec ts{delay / 1000, (delay % 1000) * 1000000L};
    while (nanosleep(&ts, &ts) < 0 && errno == EINTR && !g_stop) {
    }
    delay = delay * 2 > 10000 ? 10000 : delay * 2;
    ++restarts;
  }
  if (!pidfile.empty()) unlink(pidfile.c_str());
  return WIFEXITED(status) ? WEXITSTATUS(status) : 0;
}
