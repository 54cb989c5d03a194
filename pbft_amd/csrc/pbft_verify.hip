// MI355X (gfx950) batch Ed25519 verifier for PBFT prepare/commit quorums:
// kernels + the C ABI declared in include/pbft_verify.h.
//
// Data layout in HBM (one context = one GPU):
//   tabB   comb table of the base point, WB-bit signed windows
//          (comb<WB>::P positions x comb<WB>::E entries x 128 B)
//   tabA   one comb table of -A per replica key, same geometry with WA
//   keys   raw 32-byte key encodings (hashed as given) + key_ok bytes
//   batch  SoA: R[N][32], S[N][32], key_idx[N] u16, msg[N][stride]
//   bitmap ceil(N/64) u64 words, one per wavefront (ballot)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/pbft_verify.h"
#include "digest_kernels.h"
#include "verify_core.h"

using namespace pbft;

#ifndef PBFT_WB
#define PBFT_WB 8
#endif
#ifndef PBFT_WA
#define PBFT_WA 8
#endif
#define PBFT_ENVELOPE_LEN 85
#define BLOCK 256

static constexpr int WB = PBFT_WB;
static constexpr int WA = PBFT_WA;

// ------------------------------------------------------------------ errors
static thread_local std::string g_last_error;
static int set_err(int code, const char* what) {
  g_last_error = what;
  return code;
}
#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      char _b[256];                                                                     \
      snprintf(_b, sizeof _b, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
               __LINE__);                                                               \
      return set_err(PBFT_EHIP, _b);                                                    \
    }                                                                                   \
  } while (0)

// ------------------------------------------------------------------ kernels

// Comb tables for a set of points given by encoding (negate: table of -P).
// One thread per (key, position, entry).  key_ok[key] = decodes && !small order.
template <int W>
__global__ void __launch_bounds__(BLOCK) build_comb_kernel(const uint32_t* __restrict__ enc, uint32_t n_keys,
                                                           int negate, uint32_t* __restrict__ tables,
                                                           uint8_t* __restrict__ key_ok) {
  constexpr int P = comb<W>::P, E = comb<W>::E;
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t per_key = (uint64_t)P * E;
  if (tid >= per_key * n_keys) return;
  const uint32_t key = (uint32_t)(tid / per_key);
  const uint32_t rem = (uint32_t)(tid % per_key);
  const int pos = rem / E, j = rem % E;
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = enc[8 * key + i];
  ge A;
  const bool dec = ge_decompress(A, w);
  if (rem == 0 && key_ok) key_ok[key] = (dec && !ge_is_small_order(A)) ? 1 : 0;
  niels n;
  if (!dec) {
    niels_identity(n);
  } else {
    if (negate) { ge t; ge_neg(t, A); A = t; }
    comb_entry<W>(n, A, pos, j);
  }
  store_niels(tables + (size_t)key * comb<W>::TABLE_WORDS + (size_t)rem * 32, n);
}

__device__ __forceinline__ void load32(uint32_t w[8], const uint8_t* p) {
  const uint4* q = (const uint4*)p;
  const uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// One signature per lane; wave ballot -> one bitmap word per wavefront.
template <int LEN>
__global__ void __launch_bounds__(BLOCK) verify_kernel(const uint8_t* __restrict__ R, const uint8_t* __restrict__ S,
                                                       const uint16_t* __restrict__ key_idx,
                                                       const uint8_t* __restrict__ msg, uint32_t msg_len,
                                                       uint32_t msg_stride, uint64_t N,
                                                       const uint32_t* __restrict__ tabB,
                                                       const uint32_t* __restrict__ tabA,
                                                       const uint32_t* __restrict__ keys,
                                                       const uint8_t* __restrict__ key_ok, uint32_t n_keys,
                                                       uint64_t* __restrict__ bitmap) {
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool live = i < N;
  const uint64_t ii = live ? i : 0;  // dead lanes recompute lane 0 (no OOB reads)
  uint32_t r[8], s[8], a[8];
  load32(r, R + 32 * ii);
  load32(s, S + 32 * ii);
  uint32_t ki = key_idx[ii];
  bool kok = ki < n_keys;
  if (!kok) ki = 0;
  kok = kok && key_ok[ki];
  const uint4* kp = (const uint4*)(keys + 8 * ki);
  const uint4 k0 = kp[0], k1 = kp[1];
  a[0] = k0.x; a[1] = k0.y; a[2] = k0.z; a[3] = k0.w; a[4] = k1.x; a[5] = k1.y; a[6] = k1.z; a[7] = k1.w;
  const bool ok = verify_lane<WB, WA, LEN>(r, s, a, kok, msg + (size_t)msg_stride * ii, (int)msg_len, tabB,
                                          tabA + (size_t)ki * comb<WA>::TABLE_WORDS);
  const uint64_t vote = __ballot(live && ok);
  if ((threadIdx.x & 63) == 0 && live) bitmap[i >> 6] = vote;
}

// RFC 8032 signing, one signature per lane (replicas sign their own
// Prepare/Commit envelopes; the reference multicasts them unsigned).
template <int LEN>
__global__ void __launch_bounds__(BLOCK) sign_kernel(const uint32_t* __restrict__ seeds,
                                                     const uint16_t* __restrict__ seed_idx,
                                                     const uint8_t* __restrict__ msg, uint32_t msg_len,
                                                     uint32_t msg_stride, uint64_t N,
                                                     const uint32_t* __restrict__ tabB, uint32_t* __restrict__ R,
                                                     uint32_t* __restrict__ S, uint32_t* __restrict__ pub,
                                                     uint32_t n_seeds) {
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= N) return;
  const uint32_t si = seed_idx[i];
  uint32_t seed[8], r[8], s[8], a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) seed[j] = seeds[8 * si + j];
  sign_lane<WB, LEN>(r, s, a, seed, msg + (size_t)msg_stride * i, (int)msg_len, tabB);
#pragma unroll
  for (int j = 0; j < 8; ++j) { R[8 * i + j] = r[j]; S[8 * i + j] = s[j]; }
  (void)n_seeds;
  if (pub) {
#pragma unroll
    for (int j = 0; j < 8; ++j) pub[8 * si + j] = a[j];  // identical values from every lane of a seed
  }
}

// Request digests: one byte string per lane (offsets/lens into a packed buffer).
template <int KIND>  // 0 = Blake2b-512, 1 = SHA-256
__global__ void __launch_bounds__(BLOCK) digest_kernel(const uint8_t* __restrict__ data,
                                                       const uint64_t* __restrict__ offsets,
                                                       const uint32_t* __restrict__ lens, uint64_t N,
                                                       uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= N) return;
  const uint8_t* m = data + offsets[i];
  if (KIND == 0) {
    uint8_t d[64];
    blake2b512(d, m, lens[i]);
#pragma unroll
    for (int j = 0; j < 64; ++j) out[64 * i + j] = d[j];
  } else {
    uint8_t d[32];
    sha256(d, m, lens[i]);
#pragma unroll
    for (int j = 0; j < 32; ++j) out[32 * i + j] = d[j];
  }
}

// ------------------------------------------------------------------ context
struct pbft_ctx {
  int device = -1;
  hipStream_t stream = nullptr;
  uint32_t* d_tabB = nullptr;
  uint32_t* d_tabA = nullptr;
  uint32_t* d_keys = nullptr;
  uint8_t* d_key_ok = nullptr;
  uint32_t n_keys = 0;
  // staging for the host-buffer API
  uint8_t* d_stage = nullptr;
  size_t stage_cap = 0;
  uint64_t* d_bitmap = nullptr;
  size_t bitmap_cap = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_done = nullptr;
  bool in_flight = false;
  uint64_t* async_out = nullptr;
  uint64_t* h_bitmap = nullptr;  // pinned
  uint64_t async_words = 0;
  float last_ms = 0.f;
};

static int ensure_stage(pbft_ctx* c, size_t bytes, size_t words) {
  if (bytes > c->stage_cap) {
    if (c->d_stage) HIP_TRY(hipFree(c->d_stage));
    c->d_stage = nullptr;
    size_t cap = bytes + (bytes >> 2) + 4096;
    if (hipMalloc(&c->d_stage, cap) != hipSuccess) { c->stage_cap = 0; return set_err(PBFT_ENOMEM, "staging alloc"); }
    c->stage_cap = cap;
  }
  if (words > c->bitmap_cap) {
    if (c->d_bitmap) HIP_TRY(hipFree(c->d_bitmap));
    if (c->h_bitmap) HIP_TRY(hipHostFree(c->h_bitmap));
    c->d_bitmap = nullptr; c->h_bitmap = nullptr;
    size_t cap = words + 64;
    if (hipMalloc(&c->d_bitmap, cap * 8) != hipSuccess) return set_err(PBFT_ENOMEM, "bitmap alloc");
    if (hipHostMalloc(&c->h_bitmap, cap * 8, hipHostMallocDefault) != hipSuccess)
      return set_err(PBFT_ENOMEM, "pinned bitmap alloc");
    c->bitmap_cap = cap;
  }
  return PBFT_OK;
}

static int launch_verify(pbft_ctx* c, const uint8_t* dR, const uint8_t* dS, const uint16_t* dK, const uint8_t* dM,
                         uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t* dB, hipStream_t st) {
  if (N == 0) return PBFT_OK;
  const uint64_t blocks = (N + BLOCK - 1) / BLOCK;
  if (blocks > 0x7fffffffull) return set_err(PBFT_EINVAL, "N too large for one launch");
  HIP_TRY(hipEventRecord(c->ev0, st));
  if (msg_len == PBFT_ENVELOPE_LEN)
    hipLaunchKernelGGL(verify_kernel<PBFT_ENVELOPE_LEN>, dim3((unsigned)blocks), dim3(BLOCK), 0, st, dR, dS, dK, dM,
                       msg_len, msg_stride, N, c->d_tabB, c->d_tabA, c->d_keys, c->d_key_ok, c->n_keys, dB);
  else
    hipLaunchKernelGGL(verify_kernel<-1>, dim3((unsigned)blocks), dim3(BLOCK), 0, st, dR, dS, dK, dM, msg_len,
                       msg_stride, N, c->d_tabB, c->d_tabA, c->d_keys, c->d_key_ok, c->n_keys, dB);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(c->ev1, st));
  return PBFT_OK;
}

static bool check_batch_args(const void* R, const void* S, const void* K, const void* M, uint32_t msg_len,
                             uint32_t msg_stride, uint64_t N, const void* out) {
  if (N == 0) return out != nullptr || true;
  if (!R || !S || !K || !out) return false;
  if (msg_len > 0 && !M) return false;
  if (msg_stride < msg_len) return false;
  if (msg_len > (1u << 24)) return false;
  return true;
}

// Copy a host batch into the staging buffer and launch.  Returns device bitmap.
static int stage_and_launch(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint8_t* M,
                            uint32_t msg_len, uint32_t msg_stride, uint64_t N) {
  const uint64_t words = (N + 63) / 64;
  const size_t offS = 32 * N, offK = 64 * N;
  const size_t offM = (offK + 2 * N + 255) & ~(size_t)255;
  const size_t mbytes = (size_t)msg_stride * N;
  const size_t total = offM + mbytes + 64;  // + slack for unaligned message reads
  int rc = ensure_stage(c, total, words);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_stage, R, 32 * N, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_stage + offS, S, 32 * N, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_stage + offK, K, 2 * N, hipMemcpyHostToDevice, c->stream));
  if (mbytes) HIP_TRY(hipMemcpyAsync(c->d_stage + offM, M, mbytes, hipMemcpyHostToDevice, c->stream));
  return launch_verify(c, c->d_stage, c->d_stage + offS, (const uint16_t*)(c->d_stage + offK), c->d_stage + offM,
                       msg_len, msg_stride, N, c->d_bitmap, c->stream);
}

extern "C" {

const char* pbft_last_error(void) { return g_last_error.c_str(); }

const char* pbft_build_info(void) {
  static char buf[160];
  snprintf(buf, sizeof buf, "pbft_verify gfx950 WB=%d WA=%d block=%d entry=128B tabB=%zuB tabA/key=%zuB", WB, WA,
           BLOCK, comb<WB>::TABLE_WORDS * 4, comb<WA>::TABLE_WORDS * 4);
  return buf;
}

int pbft_verify_ctx_create(int device, pbft_ctx** out) {
  if (!out) return set_err(PBFT_EINVAL, "out is null");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return set_err(PBFT_ENODEV, "no HIP device at that ordinal");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    char b[128];
    snprintf(b, sizeof b, "device %d is %s, this library is built for gfx950", device, prop.gcnArchName);
    return set_err(PBFT_ENODEV, b);
  }
  HIP_TRY(hipSetDevice(device));
  pbft_ctx* c = new pbft_ctx();
  c->device = device;
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreate(&c->ev0));
  HIP_TRY(hipEventCreate(&c->ev1));
  HIP_TRY(hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
  // base point B = (x, 4/5), x even
  const uint32_t benc[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                            0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
  uint32_t* d_benc = nullptr;
  HIP_TRY(hipMalloc(&d_benc, 32));
  HIP_TRY(hipMalloc(&c->d_tabB, comb<WB>::TABLE_WORDS * 4));
  HIP_TRY(hipMemcpyAsync(d_benc, benc, 32, hipMemcpyHostToDevice, c->stream));
  const uint64_t threads = (uint64_t)comb<WB>::P * comb<WB>::E;
  hipLaunchKernelGGL(build_comb_kernel<WB>, dim3((unsigned)((threads + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                     c->stream, d_benc, 1u, 0, c->d_tabB, (uint8_t*)nullptr);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipFree(d_benc));
  *out = c;
  return PBFT_OK;
}

int pbft_verify_ctx_destroy(pbft_ctx* c) {
  if (!c) return PBFT_OK;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  hipFree(c->d_tabB); hipFree(c->d_tabA); hipFree(c->d_keys); hipFree(c->d_key_ok);
  hipFree(c->d_stage); hipFree(c->d_bitmap);
  if (c->h_bitmap) hipHostFree(c->h_bitmap);
  if (c->ev0) hipEventDestroy(c->ev0);
  if (c->ev1) hipEventDestroy(c->ev1);
  if (c->ev_done) hipEventDestroy(c->ev_done);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
  return PBFT_OK;
}

int pbft_verify_set_keys(pbft_ctx* c, const uint8_t* A, uint32_t n, uint8_t* key_ok) {
  if (!c || (!A && n)) return set_err(PBFT_EINVAL, "null argument");
  if (n == 0 || n > 65535) return set_err(PBFT_EINVAL, "key count must be 1..65535");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  hipFree(c->d_tabA); hipFree(c->d_keys); hipFree(c->d_key_ok);
  c->d_tabA = nullptr; c->d_keys = nullptr; c->d_key_ok = nullptr; c->n_keys = 0;
  const size_t tab_bytes = comb<WA>::TABLE_WORDS * 4 * (size_t)n;
  if (hipMalloc(&c->d_tabA, tab_bytes) != hipSuccess) return set_err(PBFT_ENOMEM, "key table alloc");
  HIP_TRY(hipMalloc(&c->d_keys, 32 * (size_t)n));
  HIP_TRY(hipMalloc(&c->d_key_ok, n));
  HIP_TRY(hipMemcpyAsync(c->d_keys, A, 32 * (size_t)n, hipMemcpyHostToDevice, c->stream));
  const uint64_t threads = (uint64_t)comb<WA>::P * comb<WA>::E * n;
  hipLaunchKernelGGL(build_comb_kernel<WA>, dim3((unsigned)((threads + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                     c->stream, c->d_keys, n, 1, c->d_tabA, c->d_key_ok);
  HIP_TRY(hipGetLastError());
  if (key_ok) HIP_TRY(hipMemcpyAsync(key_ok, c->d_key_ok, n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->n_keys = n;
  return PBFT_OK;
}

int pbft_verify_batch(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint8_t* M,
                      uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t* out) {
  int rc = pbft_verify_batch_async(c, R, S, K, M, msg_len, msg_stride, N, out);
  if (rc) return rc;
  return pbft_verify_wait(c);
}

int pbft_verify_batch_async(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint8_t* M,
                            uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t* out) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (!check_batch_args(R, S, K, M, msg_len, msg_stride, N, out)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  if (N == 0) return PBFT_OK;
  HIP_TRY(hipSetDevice(c->device));
  int rc = stage_and_launch(c, R, S, K, M, msg_len, msg_stride, N);
  if (rc) return rc;
  const uint64_t words = (N + 63) / 64;
  HIP_TRY(hipMemcpyAsync(c->h_bitmap, c->d_bitmap, words * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipEventRecord(c->ev_done, c->stream));
  c->in_flight = true;
  c->async_out = out;
  c->async_words = words;
  return PBFT_OK;
}

static int finish_async(pbft_ctx* c) {
  memcpy(c->async_out, c->h_bitmap, c->async_words * 8);
  c->in_flight = false;
  hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1);
  return PBFT_OK;
}

int pbft_verify_poll(pbft_ctx* c) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!c->in_flight) return 1;
  hipError_t e = hipEventQuery(c->ev_done);
  if (e == hipErrorNotReady) return 0;
  HIP_TRY(e);
  finish_async(c);
  return 1;
}

int pbft_verify_wait(pbft_ctx* c) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!c->in_flight) return PBFT_OK;
  HIP_TRY(hipEventSynchronize(c->ev_done));
  return finish_async(c);
}

int pbft_verify_batch_device(pbft_ctx* c, const uint8_t* dR, const uint8_t* dS, const uint16_t* dK,
                             const uint8_t* dM, uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t* dB,
                             void* stream) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!check_batch_args(dR, dS, dK, dM, msg_len, msg_stride, N, dB)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  return launch_verify(c, dR, dS, dK, dM, msg_len, msg_stride, N, dB, st);
}

static int run_digest(pbft_ctx* c, int kind, const uint8_t* data, const uint64_t* offsets, const uint32_t* lens,
                      uint64_t N, uint8_t* out) {
  if (!c || (N && (!offsets || !lens || !out))) return set_err(PBFT_EINVAL, "null argument");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (N == 0) return PBFT_OK;
  uint64_t total = 0;
  for (uint64_t i = 0; i < N; ++i) {
    const uint64_t end = offsets[i] + lens[i];
    if (end > total) total = end;
  }
  if (total && !data) return set_err(PBFT_EINVAL, "null data");
  HIP_TRY(hipSetDevice(c->device));
  const size_t outb = (kind == 0 ? 64 : 32) * N;
  const size_t offO = (total + 64 + 255) & ~(size_t)255;
  const size_t offL = offO + ((8 * N + 255) & ~(size_t)255);
  const size_t offOut = offL + ((4 * N + 255) & ~(size_t)255);
  int rc = ensure_stage(c, offOut + outb, 1);
  if (rc) return rc;
  if (total) HIP_TRY(hipMemcpyAsync(c->d_stage, data, total, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_stage + offO, offsets, 8 * N, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_stage + offL, lens, 4 * N, hipMemcpyHostToDevice, c->stream));
  const unsigned blocks = (unsigned)((N + BLOCK - 1) / BLOCK);
  if (kind == 0)
    hipLaunchKernelGGL(digest_kernel<0>, dim3(blocks), dim3(BLOCK), 0, c->stream, c->d_stage,
                       (const uint64_t*)(c->d_stage + offO), (const uint32_t*)(c->d_stage + offL), N,
                       c->d_stage + offOut);
  else
    hipLaunchKernelGGL(digest_kernel<1>, dim3(blocks), dim3(BLOCK), 0, c->stream, c->d_stage,
                       (const uint64_t*)(c->d_stage + offO), (const uint32_t*)(c->d_stage + offL), N,
                       c->d_stage + offOut);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, c->d_stage + offOut, outb, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return PBFT_OK;
}

int pbft_digest_blake2b512(pbft_ctx* c, const uint8_t* data, const uint64_t* offsets, const uint32_t* lens,
                           uint64_t N, uint8_t* out) {
  return run_digest(c, 0, data, offsets, lens, N, out);
}

int pbft_digest_sha256(pbft_ctx* c, const uint8_t* data, const uint64_t* offsets, const uint32_t* lens, uint64_t N,
                       uint8_t* out) {
  return run_digest(c, 1, data, offsets, lens, N, out);
}

int pbft_sign_batch(pbft_ctx* c, const uint8_t* seeds, uint32_t n_seeds, const uint16_t* seed_idx,
                    const uint8_t* msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint8_t* R, uint8_t* S,
                    uint8_t* pub) {
  if (!c || !seeds || n_seeds == 0 || (N && (!seed_idx || !R || !S)) || (msg_len && !msg) || msg_stride < msg_len)
    return set_err(PBFT_EINVAL, "bad sign arguments");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  for (uint64_t i = 0; i < N; ++i)
    if (seed_idx[i] >= n_seeds) return set_err(PBFT_EINVAL, "seed index out of range");
  HIP_TRY(hipSetDevice(c->device));
  const size_t offI = (32 * (size_t)n_seeds + 255) & ~(size_t)255;
  const size_t offM = offI + ((2 * N + 255) & ~(size_t)255);
  const size_t offR = offM + (((size_t)msg_stride * N + 64 + 255) & ~(size_t)255);
  const size_t offS = offR + 32 * N;
  const size_t offP = offS + 32 * N;
  int rc = ensure_stage(c, offP + 32 * (size_t)n_seeds, 1);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_stage, seeds, 32 * (size_t)n_seeds, hipMemcpyHostToDevice, c->stream));
  if (N) HIP_TRY(hipMemcpyAsync(c->d_stage + offI, seed_idx, 2 * N, hipMemcpyHostToDevice, c->stream));
  if (N && msg_len) HIP_TRY(hipMemcpyAsync(c->d_stage + offM, msg, (size_t)msg_stride * N, hipMemcpyHostToDevice, c->stream));
  uint64_t n_launch = N;
  const uint16_t* d_idx = (const uint16_t*)(c->d_stage + offI);
  std::vector<uint16_t> all;
  if (pub && N == 0) n_launch = 0;
  if (n_launch) {
    const unsigned blocks = (unsigned)((n_launch + BLOCK - 1) / BLOCK);
    if (msg_len == PBFT_ENVELOPE_LEN)
      hipLaunchKernelGGL(sign_kernel<PBFT_ENVELOPE_LEN>, dim3(blocks), dim3(BLOCK), 0, c->stream,
                         (const uint32_t*)c->d_stage, d_idx, c->d_stage + offM, msg_len, msg_stride, n_launch,
                         c->d_tabB, (uint32_t*)(c->d_stage + offR), (uint32_t*)(c->d_stage + offS),
                         pub ? (uint32_t*)(c->d_stage + offP) : nullptr, n_seeds);
    else
      hipLaunchKernelGGL(sign_kernel<-1>, dim3(blocks), dim3(BLOCK), 0, c->stream, (const uint32_t*)c->d_stage,
                         d_idx, c->d_stage + offM, msg_len, msg_stride, n_launch, c->d_tabB,
                         (uint32_t*)(c->d_stage + offR), (uint32_t*)(c->d_stage + offS),
                         pub ? (uint32_t*)(c->d_stage + offP) : nullptr, n_seeds);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(R, c->d_stage + offR, 32 * N, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(S, c->d_stage + offS, 32 * N, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (pub) {
    // public keys of seeds that no lane used are derived by a one-lane-per-seed pass
    std::vector<uint16_t> idx(n_seeds);
    for (uint32_t j = 0; j < n_seeds; ++j) idx[j] = (uint16_t)j;
    uint16_t* d_i2 = nullptr;
    uint32_t *d_r2 = nullptr, *d_s2 = nullptr;
    HIP_TRY(hipMalloc(&d_i2, 2 * (size_t)n_seeds));
    HIP_TRY(hipMalloc(&d_r2, 64 * (size_t)n_seeds));
    d_s2 = d_r2 + 8 * (size_t)n_seeds;
    HIP_TRY(hipMemcpyAsync(d_i2, idx.data(), 2 * (size_t)n_seeds, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(sign_kernel<0>, dim3((n_seeds + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, c->stream,
                       (const uint32_t*)c->d_stage, (const uint16_t*)d_i2, (const uint8_t*)nullptr, 0u, 0u,
                       (uint64_t)n_seeds, c->d_tabB, d_r2, d_s2, (uint32_t*)(c->d_stage + offP), n_seeds);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(pub, c->d_stage + offP, 32 * (size_t)n_seeds, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    hipFree(d_i2);
    hipFree(d_r2);
  }
  return PBFT_OK;
}

float pbft_last_kernel_ms(pbft_ctx* c) {
  if (!c) return -1.f;
  float ms = -1.f;
  if (hipEventSynchronize(c->ev1) != hipSuccess) return -1.f;
  if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) return -1.f;
  c->last_ms = ms;
  return ms;
}

}  // extern "C"
