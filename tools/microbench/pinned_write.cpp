// Host write bandwidth into host memory from different allocators (the replica's row arena):
// 16 threads write 72-byte rows over 2^20 rows (75 MB) with streaming stores and with plain stores, 5 reps each,
// into malloc'd memory and hipHostMalloc'd memory under several flag sets; then the H2D copy rate of the same 75 MB
// from each (one copy, and 8 back-to-back copies).
// build: hipcc -O2 -std=c++17 -o tools/microbench/pinned_write tools/microbench/pinned_write.cpp -lpthread
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/mman.h>
#include <thread>
#include <vector>

static double run(uint8_t* dst, bool nt, int T) {
  const size_t N = 1u << 20, ROW = 72;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([=] {
      long long v[9];
      for (int q = 0; q < 9; ++q) v[q] = q * 0x0101010101010101ll + t;
      for (size_t i = N * t / T; i < N * (t + 1) / T; ++i) {
        long long* d = (long long*)(dst + ROW * i);
        if (nt) for (int q = 0; q < 9; ++q) _mm_stream_si64(d + q, v[q] + (long long)i);
        else for (int q = 0; q < 9; ++q) d[q] = v[q] + (long long)i;
      }
      _mm_sfence();
    });
  for (auto& x : th) x.join();
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
  const size_t bytes = 72u << 20;
  struct Cfg { const char* name; unsigned flags; bool pinned; bool thp = false; };
  Cfg cfgs[] = {{"malloc", 0, false},
                {"hipHostMalloc Default", hipHostMallocDefault, true},
                {"Portable", hipHostMallocPortable, true},
                {"THP + hipHostRegister", 0, true, true},
                {"Mapped|Coherent", hipHostMallocMapped | hipHostMallocCoherent, true},
                {"Portable|Mapped", hipHostMallocPortable | hipHostMallocMapped, true},
                {"Portable|Mapped|NonCoherent", hipHostMallocPortable | hipHostMallocMapped | hipHostMallocNonCoherent, true},
                {"Portable|Mapped|Coherent", hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent, true}};
  const bool rev = getenv("REVERSE") != nullptr;  // (allocation order: the first pinned buffer may be special)
  const int n_cfg = (int)(sizeof cfgs / sizeof cfgs[0]);
  for (int ci = 0; ci < n_cfg; ++ci) {
    const Cfg& c = cfgs[rev ? n_cfg - 1 - ci : ci];
    uint8_t* p = nullptr;
    if (c.thp) {  // 2 MB-aligned, transparent huge pages asked for, touched, then pinned
      p = (uint8_t*)aligned_alloc(2u << 20, bytes);
      const int m = madvise(p, bytes, MADV_HUGEPAGE);
      memset(p, 0, bytes);
      if (hipHostRegister(p, bytes, hipHostRegisterDefault) != hipSuccess) { printf("%s: register failed\n", c.name); continue; }
      printf("%s: madvise %d\n", c.name, m);
    } else if (c.pinned) {
      if (hipHostMalloc((void**)&p, bytes, c.flags) != hipSuccess) { printf("%s: alloc failed\n", c.name); continue; }
    } else {
      p = (uint8_t*)aligned_alloc(64, bytes);
      memset(p, 0, bytes);
    }
    for (int nt = 1; nt >= 0; --nt) {
      double best = 1e9, sum = 0;
      for (int rep = 0; rep < 5; ++rep) { const double ms = run(p, nt, 16); best = std::min(best, ms); sum += ms; }
      printf("%-30s %s: best %.3f ms, mean %.3f ms (%.1f GB/s best)\n", c.name, nt ? "stream" : "plain ", best, sum / 5,
             bytes / best / 1e6);
    }
    if (c.pinned) {
      uint8_t* d = nullptr;
      (void)hipMalloc((void**)&d, bytes);
      hipStream_t st;
      (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      for (int pieces : {1, 8}) {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
          (void)hipEventRecord(e0, st);
          for (int k = 0; k < pieces; ++k)
            (void)hipMemcpyAsync(d + bytes / pieces * k, p + bytes / pieces * k, bytes / pieces, hipMemcpyHostToDevice, st);
          (void)hipEventRecord(e1, st);
          (void)hipEventSynchronize(e1);
          float ms = 0;
          (void)hipEventElapsedTime(&ms, e0, e1);
          best = std::min(best, ms);
        }
        printf("%-30s H2D %d piece(s): best %.3f ms (%.1f GB/s)\n", c.name, pieces, best, bytes / best / 1e6);
      }
      (void)hipFree(d);
      (void)hipStreamDestroy(st);
      if (c.thp) {
        (void)hipHostUnregister(p);
        free(p);
      } else {
        (void)hipHostFree(p);
      }
    } else {
      free(p);
    }
  }
  return 0;
}
