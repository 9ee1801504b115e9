// Pipelined validation, reader side: the result of a GPU burn-in that finished (FILE) or is
// still running (FILE.pending names its launcher's pid), shared by tk8s-probe --reuse and the
// HIP-free tk8s-reuse wrapper the validation pods run.
#pragma once

#include <signal.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>

namespace tk8s {

inline bool exists(const std::string& p) { return access(p.c_str(), F_OK) == 0; }

// The result's own "ok" is its first key (every writer puts it first); whitespace-tolerant.
inline bool ok_of(const std::string& j) {
  auto p = j.find("\"ok\"");
  if (p == std::string::npos) return false;
  p = j.find(':', p + 4);
  if (p == std::string::npos) return false;
  p = j.find_first_not_of(" \t\r\n", p + 1);
  return p != std::string::npos && j.compare(p, 4, "true") == 0;
}

// pid written into FILE.pending by the launcher (0 / absent: unknown, assume alive).
inline bool burnin_alive(const std::string& pending) {
  std::ifstream f(pending);
  long pid = 0;
  if (!(f >> pid) || pid <= 0) return true;
  if (kill(static_cast<pid_t>(pid), 0) != 0 && errno != EPERM) return false;
  // An exited burn-in its launcher has not reaped yet is a zombie: dead for our purpose.
  std::ifstream st("/proc/" + std::to_string(pid) + "/stat");
  std::string line;
  if (!std::getline(st, line)) return true;
  const auto rp = line.rfind(')');
  return rp == std::string::npos || rp + 2 >= line.size() || line[rp + 2] != 'Z';
}

// Print a finished (or still running) burn-in's result. Returns -1 when there is none (no
// burn-in, or it died without writing a result): the caller then probes itself.
// A result is single-use: it is renamed to FILE.consumed before it is read (rename is atomic, so
// of two readers exactly one gets it), and a re-created validation pod -- agent restart,
// --resume, a re-join -- finds nothing and probes the GPU again instead of re-reporting an old pass.
inline int reuse(const std::string& file, double wait_s) {
  const auto t = std::chrono::steady_clock::now();
  auto waited_ms = [&] {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
  };
  while (!exists(file) && exists(file + ".pending") && waited_ms() < wait_s * 1e3) {
    if (!burnin_alive(file + ".pending") && !exists(file)) break;
    std::this_thread::sleep_for(std::chrono::microseconds(500));  // a stat + /proc read: cheap
  }
  const std::string taken = file + ".consumed";
  if (std::rename(file.c_str(), taken.c_str()) != 0) return -1;
  std::ifstream f(taken);
  if (!f) return -1;
  std::stringstream ss;
  ss << f.rdbuf();
  std::string j = ss.str();
  while (!j.empty() && (j.back() == '\n' || j.back() == '\r')) j.pop_back();
  if (j.empty() || j.front() != '{') return -1;
  std::printf("%s\n", j.c_str());
  std::fflush(stdout);
  return ok_of(j) ? 0 : 1;
}

}  // namespace tk8s
