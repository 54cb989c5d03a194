// H2D copy rate of 75 MB of pinned host memory placed on each NUMA node (mmap + mbind MPOL_BIND + touch +
// hipHostRegister), twice per node in alternating order: does the DMA rate depend on where the host pages live?
// build: hipcc -O2 -std=c++17 -o tools/microbench/numa_h2d tools/microbench/numa_h2d.cpp
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>

static long mbind_(void* a, unsigned long len, int mode, const unsigned long* mask, unsigned long maxnode, unsigned f) {
  return syscall(SYS_mbind, a, len, mode, mask, maxnode, f);
}

static float h2d(uint8_t* p, uint8_t* d, size_t bytes, hipStream_t st) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e9;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, st);
    (void)hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, st);
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  int nodes = 0;
  for (int n = 0; n < 64; ++n) {
    char path[64];
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d", n);
    DIR* dd = opendir(path);
    if (!dd) break;
    closedir(dd);
    ++nodes;
  }
  char buf[64] = {0};
  FILE* f = fopen("/sys/class/kfd/kfd/topology/nodes/1/properties", "r");
  (void)f;
  printf("numa nodes: %d\n", nodes);
  const size_t bytes = 72u << 20;
  uint8_t* d = nullptr;
  (void)hipMalloc((void**)&d, bytes);
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  for (int pass = 0; pass < 2; ++pass)
    for (int k = 0; k < nodes; ++k) {
      const int node = pass ? nodes - 1 - k : k;
      uint8_t* p = (uint8_t*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      unsigned long mask = 1ul << node;
      const long rc = mbind_(p, bytes, 2 /* MPOL_BIND */, &mask, 64, 0);
      memset(p, 1, bytes);
      if (hipHostRegister(p, bytes, hipHostRegisterDefault) != hipSuccess) { printf("register failed\n"); return 1; }
      const float ms = h2d(p, d, bytes, st);
      printf("node %d (mbind %ld): H2D %.3f ms (%.1f GB/s)\n", node, rc, ms, bytes / ms / 1e6);
      (void)hipHostUnregister(p);
      munmap(p, bytes);
    }
  (void)buf;
  return 0;
}
