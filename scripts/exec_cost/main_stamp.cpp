// Prints the wall-clock time (unix ms) at main's first line: with the spawn time taken by the
// parent, the cost of exec + dynamic loading + the libraries' static constructors.
#include <chrono>
#include <cstdio>
#ifdef WITH_HSA
#include <hsa/hsa.h>
#endif
int main() {
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::system_clock::now().time_since_epoch()).count();
  std::printf("%.3f\n", ms);
#ifdef WITH_HSA
  if (ms < 0) hsa_init();  // never runs: keeps the library linked
#endif
  return 0;
}
