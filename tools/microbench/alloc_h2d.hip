// Host-side costs on MI355X that bound the key-set install and the replica flush (round 4 probes):
//  1. hipMalloc of large device buffers (the 172-GB key tables), against hipExtMallocWithFlags and
//     hipMallocAsync on the default pool;
//  2. H2D bandwidth from pinned host memory: one stream, two streams (two SDMA queues), several chunk sizes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char** argv) {
  const size_t GB = 1ull << 30;
  const size_t big = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 64) * GB;
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  size_t fr, tot;
  CK(hipMemGetInfo(&fr, &tot));
  printf("free %.1f GB of %.1f GB\n", fr / 1e9, tot / 1e9);
  for (int rep = 0; rep < 2; ++rep) {
    void* p = nullptr;
    auto t = std::chrono::steady_clock::now();
    CK(hipMalloc(&p, big));
    double a = ms_since(t);
    t = std::chrono::steady_clock::now();
    CK(hipFree(p));
    printf("hipMalloc %zu GB: %.1f ms (%.1f GB/s), hipFree %.1f ms\n", big / GB, a, big / 1e6 / a, ms_since(t));
  }
  {
    void* p = nullptr;
    auto t = std::chrono::steady_clock::now();
    CK(hipExtMallocWithFlags(&p, big, hipDeviceMallocUncached));
    double a = ms_since(t);
    CK(hipFree(p));
    printf("hipExtMallocWithFlags(uncached) %zu GB: %.1f ms\n", big / GB, a);
  }
  {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    void* p = nullptr;
    auto t = std::chrono::steady_clock::now();
    CK(hipMallocAsync(&p, big, s));
    CK(hipStreamSynchronize(s));
    double a = ms_since(t);
    t = std::chrono::steady_clock::now();
    CK(hipFreeAsync(p, s));
    CK(hipStreamSynchronize(s));
    printf("hipMallocAsync %zu GB: %.1f ms, hipFreeAsync %.1f ms\n", big / GB, a, ms_since(t));
    CK(hipStreamDestroy(s));
  }
  {  // many 1-GB pieces: is the cost per byte or per call?
    std::vector<void*> ps(16);
    auto t = std::chrono::steady_clock::now();
    for (auto& q : ps) CK(hipMalloc(&q, GB));
    double a = ms_since(t);
    for (auto& q : ps) CK(hipFree(q));
    printf("16 x hipMalloc 1 GB: %.1f ms\n", a);
  }
  // H2D from pinned memory
  const size_t bytes = 72ull << 20;  // ~ a 2^20-vote round in the votes form (70 B per row)
  void *h = nullptr, *d = nullptr;
  CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  CK(hipMalloc(&d, bytes));
  memset(h, 1, bytes);
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  for (size_t chunk : {bytes, bytes / 4, bytes / 16}) {
    for (int streams = 1; streams <= 2; ++streams) {
      double best = 1e9;
      for (int rep = 0; rep < 6; ++rep) {
        CK(hipDeviceSynchronize());
        auto t = std::chrono::steady_clock::now();
        int k = 0;
        for (size_t off = 0; off < bytes; off += chunk, ++k)
          CK(hipMemcpyAsync((char*)d + off, (char*)h + off, chunk, hipMemcpyHostToDevice, (streams == 2 && (k & 1)) ? s1 : s0));
        CK(hipStreamSynchronize(s0));
        CK(hipStreamSynchronize(s1));
        double m = ms_since(t);
        if (m < best) best = m;
      }
      printf("H2D %zu MB in %zu-MB chunks on %d stream(s): %.3f ms = %.1f GB/s\n", bytes >> 20, chunk >> 20, streams,
             best, bytes / 1e6 / best);
    }
  }
  return 0;
}
