// Host-only self-test of tk8s/failfast.h (the payloads' deadlines, watchdog and TK8S_FAULTS
// points), built with -fsanitize=address,undefined by tests/test_failfast.py. No GPU: the GPU
// waits are poll_until over hipStreamQuery, and poll_until itself is what is tested here.
//
//   failfast_selftest armed <tool> <kind> <phase> <first_rank> <rank_count>   -> prints 1 / 0
//   failfast_selftest point <tool> <phase>        -> runs fault_point (exit 3 / abort / hang)
//   failfast_selftest watchdog <seconds>          -> arms a watchdog, then never progresses
//   failfast_selftest poll                        -> poll_until checks; prints "poll ok"
#include <cstdio>
#include <cstdlib>
#include <string>

#include "tk8s/failfast.h"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const std::string mode = argv[1];
  if (mode == "armed" && argc == 7) {
    tk8s::set_fault_ranks(std::atol(argv[5]), std::atol(argv[6]));
    std::printf("%d\n", tk8s::fault_armed(argv[2], argv[3], argv[4]) ? 1 : 0);
    return 0;
  }
  if (mode == "point" && argc == 4) {
    tk8s::set_fault_ranks(0, 1);
    tk8s::fault_point(argv[2], argv[3]);
    std::printf("passed\n");
    return 0;
  }
  if (mode == "watchdog" && argc == 3) {
    tk8s::Watchdog dog([](const std::string& phase, double waited) {
      std::printf("{\"ok\":false,\"phase\":\"%s\",\"waited_s\":%.2f}\n", phase.c_str(), waited);
    });
    dog.arm("sweep", std::atof(argv[2]));
    tk8s::fault_hang();
  }
  if (mode == "poll") {
    int n = 0;
    // ready after 5 polls
    std::string r = tk8s::poll_until([&] { return ++n >= 5; }, 5.0);
    if (!r.empty() || n != 5) return 1;
    // never ready: times out near the bound
    const double t0 = tk8s::now_s();
    r = tk8s::poll_until([] { return false; }, 0.2);
    const double dt = tk8s::now_s() - t0;
    if (r.rfind("timed out", 0) != 0 || dt < 0.2 || dt > 1.0) return 1;
    // an error ends the wait at once
    r = tk8s::poll_until([] { return false; }, 30.0, [] { return std::string("peer died"); });
    if (r != "peer died") return 1;
    std::printf("poll ok\n");
    return 0;
  }
  return 2;
}
