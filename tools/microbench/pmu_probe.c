#include <linux/perf_event.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <stdio.h>
#include <string.h>
int main() {
  struct perf_event_attr a; memset(&a, 0, sizeof a);
  a.type = PERF_TYPE_HARDWARE; a.size = sizeof a; a.config = PERF_COUNT_HW_INSTRUCTIONS; a.disabled = 1; a.exclude_kernel = 1;
  int fd = syscall(SYS_perf_event_open, &a, 0, -1, -1, 0);
  printf("fd %d\n", fd);
  if (fd < 0) { perror("perf_event_open"); return 1; }
  ioctl(fd, PERF_EVENT_IOC_ENABLE, 0);
  volatile long x = 0; for (int i = 0; i < 1000000; ++i) x += i;
  ioctl(fd, PERF_EVENT_IOC_DISABLE, 0);
  long long v; read(fd, &v, 8); printf("instructions %lld\n", v);
}
