#include <stdio.h>
#include <time.h>
int main(void) {
  struct timespec ts; clock_gettime(CLOCK_REALTIME, &ts);
  printf("%.3f\n", ts.tv_sec * 1e3 + ts.tv_nsec / 1e6);
  return 0;
}
