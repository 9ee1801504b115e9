// tk8s-reuse: the validation pod's fast path. The pod's result is normally the node's early GPU
// burn-in (tk8s-probe --out, started while the control plane came up); printing that file must
// not cost a HIP runtime load (~12 ms of exec + dynamic loading of libamdhip64 on the bring-up's
// critical path), so this wrapper links nothing of ROCm. Without a burn-in result it runs the
// probe as its child and exits with its status.
//
//   tk8s-reuse FILE [--wait S] -- PROBE [ARGS...]
#include <spawn.h>
#include <sys/wait.h>

#include <cstdlib>

#include "reuse.h"

extern char** environ;

int main(int argc, char** argv) {
  std::string file;
  double wait_s = 120;
  int dash = -1;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--") {
      dash = i;
      break;
    }
    if (a == "--wait" && i + 1 < argc) {
      wait_s = std::atof(argv[++i]);
    } else if (file.empty()) {
      file = a;
    }
  }
  if (file.empty() || dash < 0 || dash + 1 >= argc) {
    std::fprintf(stderr, "usage: tk8s-reuse FILE [--wait S] -- PROBE [ARGS...]\n");
    return 2;
  }
  const int rc = tk8s::reuse(file, wait_s);
  if (rc >= 0) return rc;
  pid_t pid = 0;  // a child, not an exec: the probe is the process that touches the GPU
  if (posix_spawn(&pid, argv[dash + 1], nullptr, nullptr, argv + dash + 1, environ) != 0) {
    std::perror("tk8s-reuse: spawn");
    return 127;
  }
  int status = 0;
  while (waitpid(pid, &status, 0) < 0 && errno == EINTR) {
  }
  if (WIFEXITED(status)) return WEXITSTATUS(status);
  return 128 + (WIFSIGNALED(status) ? WTERMSIG(status) : 0);
}
