// Host write bandwidth into host memory from different allocators (the replica's row arena):
// 16 threads write 72-byte rows over 2^20 rows (75 MB) with streaming stores and with plain stores, 5 reps each,
// into malloc'd memory and hipHostMalloc'd memory under several flag sets.
// build: hipcc -O2 -std=c++17 -o tools/microbench/pinned_write tools/microbench/pinned_write.cpp -lpthread
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
  struct Cfg { const char* name; unsigned flags; bool pinned; };
  Cfg cfgs[] = {{"malloc", 0, false},
                {"hipHostMalloc Default", hipHostMallocDefault, true},
                {"Mapped|Coherent", hipHostMallocMapped | hipHostMallocCoherent, true},
                {"Portable|Mapped", hipHostMallocPortable | hipHostMallocMapped, true},
                {"Portable|Mapped|NonCoherent", hipHostMallocPortable | hipHostMallocMapped | hipHostMallocNonCoherent, true},
                {"Portable|Mapped|Coherent", hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent, true}};
  for (const Cfg& c : cfgs) {
    uint8_t* p = nullptr;
    if (c.pinned) {
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
    if (c.pinned) (void)hipHostFree(p); else free(p);
  }
  return 0;
}
