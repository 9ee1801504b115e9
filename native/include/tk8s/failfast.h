// Fail-fast support for the GPU payloads (tk8s-rccl, tk8s-probe, tk8s-hsaprobe): bounded waits,
// a no-progress watchdog, and the native fault points of TK8S_FAULTS.
//
// Why: the reference's readiness loop has no bound at all
// (/root/reference/setup.sh:56-85); the MI355X bring-up must never let one dead peer or wedged
// GPU turn into a hang. Every wait a payload does on the GPU or on another rank therefore runs
// under a deadline, and a watchdog thread ends the process (JSON error line naming the phase,
// exit kWatchdogExit) when the main thread makes no progress at all -- the backstop for calls that block
// inside a library (a communicator init waiting for a rank that never comes).
//
// Fault points (comma-separated in TK8S_FAULTS, the same variable utils/faults.py reads):
//   <tool>.hang@<phase>   the process stops making progress in that phase (host side: it sleeps;
//                         GPU side phases use a stall kernel instead, see gpu_stall in kernels.h)
//   <tool>.exit@<phase>   the process exits (status 3) at the start of that phase: a dead peer
//   <tool>.crash@<phase>  abort() at the start of that phase (SIGABRT, like a GPU fault's abort)
// <tool> is "rccl" or "probe"; phases are the tool's own ("uid", "init", "sweep", "check";
// "peers"). "probe.hang_peers" and "probe.crash" are accepted as shorthands for
// probe.hang@peers and probe.crash@peers. A ":<rank>" suffix (utils/faults.py's argument) arms
// the point in the process holding that rank only (set_fault_ranks), so one rank of a job can
// hang or die while its peers run normally.
//
// HIP-free on purpose: tk8s-hsaprobe (no HIP) includes it too.
#pragma once

#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace tk8s {

// The watchdog's exit status: its own code, not timeout(1)'s 124 -- the process ends itself
// cleanly (_Exit after its JSON line); it is not killed.
constexpr int kWatchdogExit = 4;

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Seconds from an environment variable (positive), else `def`.
inline double env_seconds(const char* name, double def) {
  const char* v = std::getenv(name);
  if (!v || !*v) return def;
  char* end = nullptr;
  const double x = std::strtod(v, &end);
  return (end && *end == '\0' && x > 0) ? x : def;
}

// Bound on one wait for GPU work that is known to be finite (a probe's kernels, one collective):
// TK8S_GPU_SYNC_TIMEOUT_S, default 30 s -- the HSA payload's long-standing bound.
inline double gpu_sync_timeout_s() { return env_seconds("TK8S_GPU_SYNC_TIMEOUT_S", 30.0); }

// Bound on one xGMI pull's wait (TK8S_PEER_SYNC_TIMEOUT_S, default 5 s, never above the general
// bound): a 16-64 MiB pull takes milliseconds even over PCIe, so a link that has not finished by
// then is reported rather than waited for.
inline double peer_sync_timeout_s() {
  const double g = gpu_sync_timeout_s();
  return env_seconds("TK8S_PEER_SYNC_TIMEOUT_S", g < 5.0 ? g : 5.0);
}

// Bound on a payload's whole peer phase (TK8S_PEER_PHASE_TIMEOUT_S, default 20 s): pulls not yet
// started when it has passed are reported as not run.
inline double peer_phase_timeout_s() { return env_seconds("TK8S_PEER_PHASE_TIMEOUT_S", 20.0); }

// ---- TK8S_FAULTS ---------------------------------------------------------------------------
struct FaultEntry {
  std::string point;  // "<tool>.<kind>@<phase>"
  long rank = -1;     // ":<rank>": only the process holding that rank; -1: every process
};

inline const std::vector<FaultEntry>& fault_entries() {
  static const std::vector<FaultEntry> entries = [] {
    std::vector<FaultEntry> out;
    const char* v = std::getenv("TK8S_FAULTS");
    std::stringstream ss(v ? v : "");
    std::string tok;
    while (std::getline(ss, tok, ',')) {
      while (!tok.empty() && tok.front() == ' ') tok.erase(tok.begin());
      while (!tok.empty() && tok.back() == ' ') tok.pop_back();
      FaultEntry e;
      const auto colon = tok.find(':');
      if (colon != std::string::npos) {
        char* end = nullptr;
        const std::string arg = tok.substr(colon + 1);
        const long r = std::strtol(arg.c_str(), &end, 10);
        e.rank = (!arg.empty() && end && *end == '\0' && r >= 0) ? r : -2;  // -2: a malformed rank matches nothing
        tok = tok.substr(0, colon);
      }
      if (tok == "probe.hang_peers") tok = "probe.hang@peers";
      if (tok == "probe.crash") tok = "probe.crash@peers";
      e.point = tok;
      if (!tok.empty()) out.push_back(e);
    }
    return out;
  }();
  return entries;
}

// The ranks this process holds ([first, first + count)); before it is known: none (rank-targeted
// points stay off until then).
inline std::atomic<long>& fault_first_rank() {
  static std::atomic<long> v{-1};
  return v;
}
inline std::atomic<long>& fault_rank_count() {
  static std::atomic<long> v{0};
  return v;
}
inline void set_fault_ranks(long first, long count) {
  fault_first_rank() = first;
  fault_rank_count() = count;
}

// Is "<tool>.<kind>@<phase>" armed (for one of this process's ranks, if it names one)?
inline bool fault_armed(const std::string& tool, const std::string& kind, const std::string& phase) {
  const std::string want = tool + "." + kind + "@" + phase;
  const long first = fault_first_rank(), count = fault_rank_count();
  for (const auto& e : fault_entries()) {
    if (e.point != want) continue;
    if (e.rank == -1 || (e.rank >= 0 && first >= 0 && e.rank >= first && e.rank < first + count)) return true;
  }
  return false;
}

// Sleep "forever" (until a watchdog or a signal ends the process).
[[noreturn]] inline void fault_hang() {
  for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
}

// The host-side fault points of one phase: exit / crash at its start, hang (host) when asked.
// A GPU-side phase passes host_hang=false and arms a stall kernel itself for "hang".
inline void fault_point(const std::string& tool, const std::string& phase, bool host_hang = true) {
  if (fault_armed(tool, "exit", phase)) {
    std::fprintf(stderr, "tk8s-%s: TK8S_FAULTS %s.exit@%s: exiting\n", tool.c_str(), tool.c_str(), phase.c_str());
    std::fflush(stderr);
    std::_Exit(3);
  }
  if (fault_armed(tool, "crash", phase)) {
    std::fprintf(stderr, "tk8s-%s: TK8S_FAULTS %s.crash@%s: aborting\n", tool.c_str(), tool.c_str(), phase.c_str());
    std::fflush(stderr);
    std::abort();
  }
  if (host_hang && fault_armed(tool, "hang", phase)) {
    std::fprintf(stderr, "tk8s-%s: TK8S_FAULTS %s.hang@%s: hanging\n", tool.c_str(), tool.c_str(), phase.c_str());
    std::fflush(stderr);
    fault_hang();
  }
}

// ---- watchdog ------------------------------------------------------------------------------
// The main thread names its phase and how long it may take (arm); the watchdog thread checks
// every 50 ms. On expiry it runs on_expire(phase, seconds) -- which must print the tool's JSON
// error line -- and _Exit(kWatchdogExit)s (no destructors: they could block on the very thing
// that hung).
class Watchdog {
 public:
  using Expire = std::function<void(const std::string& phase, double waited_s)>;

  // The thread shares its state (not `this`): it outlives the object if main returns first.
  explicit Watchdog(Expire on_expire) : st_(std::make_shared<State>()) {
    st_->on_expire = std::move(on_expire);
    std::shared_ptr<State> st = st_;
    std::thread([st] { loop(*st); }).detach();  // lives until the process ends
  }

  // Enter `phase`: it must finish (or re-arm) within `seconds`.
  void arm(const std::string& phase, double seconds) {
    std::lock_guard<std::mutex> lock(st_->mu);
    st_->phase = phase;
    st_->started = now_s();
    st_->deadline = st_->started + seconds;
  }
  void disarm() {
    std::lock_guard<std::mutex> lock(st_->mu);
    st_->deadline = 0;
  }
  std::string phase() {
    std::lock_guard<std::mutex> lock(st_->mu);
    return st_->phase;
  }

 private:
  struct State {
    std::mutex mu;
    std::string phase = "start";
    double started = 0, deadline = 0;
    Expire on_expire;
  };

  static void loop(State& st) {
    for (;;) {
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
      std::string phase;
      double waited = 0;
      {
        std::lock_guard<std::mutex> lock(st.mu);
        if (st.deadline == 0 || now_s() < st.deadline) continue;
        phase = st.phase;
        waited = now_s() - st.started;
      }
      st.on_expire(phase, waited);
      std::fflush(stdout);
      std::fflush(stderr);
      std::_Exit(kWatchdogExit);
    }
  }

  std::shared_ptr<State> st_;
};

// Poll `ready` (true: done) until it holds or `timeout_s` passes; `fail` (optional) is asked
// every poll for an error that ends the wait early (an RCCL async error). Spins with yields for
// the first 2 ms (the common case: GPU work that is about to finish), then sleeps 50 us growing
// to 1 ms. Returns "" on success, else what ended the wait.
inline std::string poll_until(const std::function<bool()>& ready, double timeout_s,
                              const std::function<std::string()>& fail = nullptr) {
  const double t0 = now_s();
  int sleep_us = 50;
  for (;;) {
    if (ready()) return "";
    if (fail) {
      std::string e = fail();
      if (!e.empty()) return e;
    }
    const double dt = now_s() - t0;
    if (dt > timeout_s) {
      char buf[96];
      std::snprintf(buf, sizeof buf, "timed out after %.1f s", dt);
      return buf;
    }
    if (dt < 0.002) {
      std::this_thread::yield();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
      sleep_us = sleep_us < 1000 ? sleep_us * 2 : 1000;
    }
  }
}

}  // namespace tk8s
