// Host memory bandwidth on the GPU box's CPU share (r06: what bounds the replica's push_many): T threads over
// disjoint slices of buffers larger than the L3, three patterns -- read (sum of 64-bit words), streaming write
// (non-temporal 16-byte stores), and the push_many mix (read 149 B, stream-write 72 B per vote: signature + digest +
// kind/view/seq/signer in, the staged row out).  Best of 5 passes per (pattern, T).
// build: gcc -O2 -mavx2 -pthread -o tools/microbench/host_bw tools/microbench/host_bw.c
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

enum { VOTES = 1 << 20, IN_B = 149, OUT_B = 72 };
static uint8_t *src, *dst;
static size_t src_bytes, dst_bytes;
static int pattern, nthreads;
static pthread_barrier_t bar;
static volatile uint64_t sink;
static double t_beg[16], t_end[16];  // per thread (the span: first start .. last end)

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void* worker(void* arg) {
  const size_t t = (size_t)arg;
  pthread_barrier_wait(&bar);
  t_beg[t] = now();
  uint64_t acc = 0;
  if (pattern == 0) {  // read
    const size_t lo = src_bytes / 64 * t / nthreads * 64, hi = src_bytes / 64 * (t + 1) / nthreads * 64;
    for (size_t i = lo; i < hi; i += 64) {
      const uint64_t* p = (const uint64_t*)(src + i);
      acc += p[0] ^ p[1] ^ p[2] ^ p[3] ^ p[4] ^ p[5] ^ p[6] ^ p[7];
    }
  } else if (pattern == 1) {  // streaming write
    const size_t lo = dst_bytes / 64 * t / nthreads * 64, hi = dst_bytes / 64 * (t + 1) / nthreads * 64;
    const __m128i v = _mm_set1_epi32((int)t);
    for (size_t i = lo; i < hi; i += 64) {
      __m128i* q = (__m128i*)(dst + i);
      _mm_stream_si128(q, v); _mm_stream_si128(q + 1, v); _mm_stream_si128(q + 2, v); _mm_stream_si128(q + 3, v);
    }
    _mm_sfence();
  } else {  // push_many mix: per vote, read IN_B bytes, stream-write OUT_B
    const size_t lo = (size_t)VOTES * t / nthreads, hi = (size_t)VOTES * (t + 1) / nthreads;
    for (size_t v = lo; v < hi; ++v) {
      const uint64_t* p = (const uint64_t*)(src + v * 152);  // (152: IN_B rounded to 8)
      uint64_t x = 0;
      for (int k = 0; k < 19; ++k) x ^= p[k];
      acc += x;
      long long* q = (long long*)(dst + v * OUT_B);  // (72-B rows: 8-B aligned, 8-B streaming stores)
      for (int k = 0; k < 9; ++k) _mm_stream_si64(q + k, (long long)(x + k));
    }
    _mm_sfence();
  }
  sink += acc;
  t_end[t] = now();
  pthread_barrier_wait(&bar);
  return NULL;
}

int main(void) {
  src_bytes = (size_t)VOTES * 152;
  dst_bytes = (size_t)VOTES * OUT_B;
  src = aligned_alloc(4096, src_bytes);
  dst = aligned_alloc(4096, dst_bytes);
  if (!src || !dst) return 1;
  memset(src, 1, src_bytes);
  memset(dst, 0, dst_bytes);
  static const char* names[3] = {"read", "stream_write", "push_mix"};
  static const int ts[] = {1, 2, 4, 8, 12, 16};
  printf("# host_bw: GB/s (best of 5), src %.0f MB, dst %.0f MB\n", src_bytes / 1e6, dst_bytes / 1e6);
  for (pattern = 0; pattern < 3; ++pattern)
    for (size_t j = 0; j < sizeof ts / sizeof ts[0]; ++j) {
      nthreads = ts[j];
      double best = 1e9;
      for (int rep = 0; rep < 5; ++rep) {
        pthread_t th[16];
        pthread_barrier_init(&bar, NULL, (unsigned)nthreads + 1);
        for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, worker, (void*)(size_t)t);
        pthread_barrier_wait(&bar);
        pthread_barrier_wait(&bar);
        double b = t_beg[0], e = t_end[0];
        for (int t = 1; t < nthreads; ++t) {
          if (t_beg[t] < b) b = t_beg[t];
          if (t_end[t] > e) e = t_end[t];
        }
        const double dt = e - b;
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
        pthread_barrier_destroy(&bar);
        if (dt < best) best = dt;
      }
      const double bytes = pattern == 0 ? src_bytes : pattern == 1 ? dst_bytes : (double)VOTES * (IN_B + OUT_B);
      printf("%-12s T=%2d  %7.1f GB/s  %.3f ms%s\n", names[pattern], nthreads, bytes / best / 1e9, best * 1e3,
             pattern == 2 ? "  (2^20 votes: 149 B in + 72 B out)" : "");
    }
  return 0;
}
