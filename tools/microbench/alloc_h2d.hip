// Host-side costs on MI355X that bound the key-set install and the replica flush (round 4 probes):
//  1. hipMalloc of large device buffers (the 172-GB key tables), against hipExtMallocWithFlags and
//     hipMallocAsync on the default pool;
//  2. H2D bandwidth from pinned host memory: one stream, two streams (two SDMA queues), several chunk sizes;
//  3. H2D of one votes chunk while a kernel occupies every CU (copy engine or blit kernel);
//  4. a kernel reading pinned host memory directly (zero-copy gather of 64-B rows, as a replica's candidate rows
//     would be gathered) into device memory.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// each lane copies one 64-B row (4 x 16 B); rows in 256-row runs at scattered host offsets (a segment table)
__global__ void gather_rows(const uint4* __restrict__ host, const uint32_t* __restrict__ run_src, uint4* __restrict__ dev,
                            uint64_t rows) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  const uint64_t src = (uint64_t)run_src[i >> 8] * 256 + (i & 255);
  const uint4* s = host + 4 * src;
  uint4* d = dev + 4 * i;
  const uint4 a = s[0], b = s[1];
  const uint4 c = s[2], e = s[3];
  d[0] = a; d[1] = b; d[2] = c; d[3] = e;
}

// a compute load that fills every CU for a fixed number of dependent FMAs per lane (bounded: no spin on time)
__global__ void busy_fma(float* out, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 1e-7f;
  for (int i = 0; i < iters; ++i) a = fmaf(a, b, c);
  if (a == 12345.f) out[blockIdx.x] = a;
}

int main(int argc, char** argv) {
  const size_t GB = 1ull << 30;
  const size_t big = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 64) * GB;
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  size_t fr, tot;
  CK(hipMemGetInfo(&fr, &tot));
  printf("free %.1f GB of %.1f GB\n", fr / 1e9, tot / 1e9);
  const bool only_overlap = argc > 2 && !strcmp(argv[2], "overlap");  // usage: alloc_h2d [GB] [overlap]
  if (!only_overlap) {
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
  {  // the verifier's sequence: the 30-GB base-point table, then 172 GB of key tables (n = 256 at 13 positions)
    void *b = nullptr, *k = nullptr;
    auto t = std::chrono::steady_clock::now();
    CK(hipMalloc(&b, 30 * GB));
    double a1 = ms_since(t);
    t = std::chrono::steady_clock::now();
    CK(hipMalloc(&k, 172 * GB));
    double a2 = ms_since(t);
    t = std::chrono::steady_clock::now();
    CK(hipMemsetAsync(k, 0, 172 * GB, 0));
    CK(hipDeviceSynchronize());
    double a3 = ms_since(t);
    t = std::chrono::steady_clock::now();
    CK(hipMemsetAsync(k, 1, 172 * GB, 0));
    CK(hipDeviceSynchronize());
    double a4 = ms_since(t);
    CK(hipFree(k));
    t = std::chrono::steady_clock::now();
    CK(hipMalloc(&k, 172 * GB));
    double a5 = ms_since(t);
    CK(hipFree(k));
    CK(hipFree(b));
    printf("hipMalloc 30 GB %.1f ms, then 172 GB %.1f ms; first memset of the 172 GB %.1f ms, second %.1f ms; "
           "re-allocation after free %.1f ms\n", a1, a2, a3, a4, a5);
  }
  {  // many 1-GB pieces: is the cost per byte or per call?
    std::vector<void*> ps(16);
    auto t = std::chrono::steady_clock::now();
    for (auto& q : ps) CK(hipMalloc(&q, GB));
    double a = ms_since(t);
    for (auto& q : ps) CK(hipFree(q));
    printf("16 x hipMalloc 1 GB: %.1f ms\n", a);
  }
  {  // host writes into pinned staging (the replica's fill): hipHostMalloc default vs non-coherent vs malloc
    const size_t fb = 64ull << 20;
    std::vector<uint8_t> src(fb, 5);
    void *pd = nullptr, *pn = nullptr;
    CK(hipHostMalloc(&pd, fb, hipHostMallocDefault));
    CK(hipHostMalloc(&pn, fb, hipHostMallocNonCoherent));
    void* pm = malloc(fb);
    for (int threads : {1, 16}) {
      for (int kind = 0; kind < 3; ++kind) {
        uint8_t* dst = (uint8_t*)(kind == 0 ? pd : kind == 1 ? pn : pm);
        double best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
          auto t = std::chrono::steady_clock::now();
          std::vector<std::thread> th;
          for (int k = 0; k < threads; ++k)
            th.emplace_back([&, k] {
              const size_t lo = fb * k / threads, hi = fb * (k + 1) / threads;
              for (size_t off = lo; off < hi; off += 16384) memcpy(dst + off, src.data() + off, std::min<size_t>(16384, hi - off));
            });
          for (auto& x : th) x.join();
          const double m = ms_since(t);
          if (m < best) best = m;
        }
        printf("host memcpy 64 MB in 16-KB pieces, %2d threads, into %s: %.3f ms = %.1f GB/s\n", threads,
               kind == 0 ? "hipHostMalloc(default)    " : kind == 1 ? "hipHostMalloc(NonCoherent)" : "malloc                    ",
               best, fb / 1e6 / best);
      }
    }
    CK(hipHostFree(pd));
    CK(hipHostFree(pn));
    free(pm);
  }
  }  // !only_overlap
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
  {  // H2D while a kernel occupies every CU: do the copies overlap compute (SDMA) or queue behind it (blit kernel)?
    float* junk = nullptr;
    CK(hipMalloc(&junk, 4 << 20));
    hipEvent_t e0, e1, e2, e3;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2)); CK(hipEventCreate(&e3));
    const size_t chunk = 18ull << 20;  // one 2^18-row votes chunk
    const dim3 grid(256 * 16), blk(256);
    for (int iters : {20000, 80000}) {
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, s0));
        hipLaunchKernelGGL(busy_fma, grid, blk, 0, s0, junk, iters);
        CK(hipEventRecord(e1, s0));
        CK(hipStreamSynchronize(s0));
        float kern = 0;
        CK(hipEventElapsedTime(&kern, e0, e1));
        // the same kernel, with a chunk copy enqueued on the other stream right after it
        CK(hipDeviceSynchronize());
        auto t = std::chrono::steady_clock::now();
        CK(hipEventRecord(e0, s0));
        hipLaunchKernelGGL(busy_fma, grid, blk, 0, s0, junk, iters);
        CK(hipEventRecord(e1, s0));
        CK(hipEventRecord(e2, s1));
        CK(hipMemcpyAsync(d, h, chunk, hipMemcpyHostToDevice, s1));
        CK(hipEventRecord(e3, s1));
        CK(hipStreamSynchronize(s1));
        const double copy_host = ms_since(t);
        CK(hipStreamSynchronize(s0));
        float kern2 = 0, copy = 0, copy_end = 0;
        CK(hipEventElapsedTime(&kern2, e0, e1));
        CK(hipEventElapsedTime(&copy, e2, e3));
        CK(hipEventElapsedTime(&copy_end, e0, e3));
        printf("H2D 18 MB beside a %d-iter busy kernel: kernel alone %.3f ms, with copy %.3f ms; copy %.3f ms, done "
               "%.3f ms after the kernel started (host saw it at %.3f ms)\n", iters, kern, kern2, copy, copy_end,
               copy_host);
      }
    }
  }
  {  // zero-copy gather: 2^20 rows of 64 B from pinned host memory, runs of 256 rows in a shuffled order
    const uint64_t rows = 1ull << 20;
    uint4 *hs = nullptr, *ds = nullptr;
    uint32_t* runs = nullptr;
    CK(hipHostMalloc(&hs, rows * 64, hipHostMallocDefault));
    CK(hipMalloc(&ds, rows * 64));
    CK(hipMalloc(&runs, 4 * (rows / 256)));
    std::vector<uint32_t> perm(rows / 256);
    for (uint32_t k = 0; k < perm.size(); ++k) perm[k] = k;
    for (uint32_t k = (uint32_t)perm.size() - 1; k > 0; --k) std::swap(perm[k], perm[(k * 2654435761u) % (k + 1)]);
    CK(hipMemcpy(runs, perm.data(), 4 * perm.size(), hipMemcpyHostToDevice));
    memset(hs, 3, rows * 64);
    for (int blk : {256, 1024}) {
      double best = 1e9;
      for (int rep = 0; rep < 8; ++rep) {
        CK(hipDeviceSynchronize());
        auto t = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(gather_rows, dim3((unsigned)((rows + blk - 1) / blk)), dim3(blk), 0, s0, hs, runs, ds, rows);
        CK(hipStreamSynchronize(s0));
        double m = ms_since(t);
        if (m < best) best = m;
      }
      printf("zero-copy gather kernel, 2^20 x 64-B rows (256-row runs, shuffled), block %d: %.3f ms = %.1f GB/s\n",
             blk, best, rows * 64 / 1e6 / best);
    }
  }
  return 0;
}
