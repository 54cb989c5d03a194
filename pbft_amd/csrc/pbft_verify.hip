// MI355X (gfx950) batch Ed25519 verifier for PBFT prepare/commit quorums:
// kernels + the C ABI declared in include/pbft_verify.h.
//
// Data layout in HBM (one context = one GPU):
//   tabB   comb table of the base point, plan PLB (10 positions of 25/26-bit
//          signed windows, 128-B entries)
//   tabA   one comb table of -A per replica key, same geometry with WA
//   keys   raw 32-byte key encodings (hashed as given) + key_ok bytes
//   batch  SoA: R[N][32], S[N][32], key_idx[N] u16, msg[N][stride]
//   bitmap ceil(N/64) u64 words, one per wavefront (ballot)
#include <dlfcn.h>
#include <sched.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <rccl/rccl.h>  // types only: librccl.so.1 is dlopen'ed by pbft_multi_create
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/pbft_verify.h"
#include "../../include/pbft_wire.h"
#include "digest_kernels.h"
#include "verify_core.h"

using namespace pbft;
#include "verify_kernels.h"
// Finish configuration by batch size (signatures per lane, product tree, waves per SIMD), measured on MI355X
// with the lane-parallel wave inversion (profiles/r03/ab_finish.txt): 131k 0.2115 -> 0.1906 ms (width 2),
// 262k 0.3628 -> 0.3429 (width 4), 2^20 finish kernel 118.6 -> 91.4 us (width 8, tree, 2 waves per SIMD).
#ifndef PBFT_FIN_SMALL_UPTO
#define PBFT_FIN_SMALL_UPTO (1u << 17)
#endif
#ifndef PBFT_FIN_FM_SMALL
#define PBFT_FIN_FM_SMALL 2  // finish signatures per lane for N <= PBFT_FIN_SMALL_UPTO
#endif
#ifndef PBFT_FIN_TINY_UPTO
#define PBFT_FIN_TINY_UPTO (1u << 16)  // one signature per finish lane up to here (r04: 2^16 0.1097 -> 0.1064 ms,
#endif                                 // 2^17 +3 %: profiles/r04/ab_fin_shard.txt)
#ifndef PBFT_FIN_FM_MID
#define PBFT_FIN_FM_MID 4  // ... for PBFT_FIN_SMALL_UPTO < N < 2^19
#endif
#ifndef PBFT_FIN_FM_BIG
#define PBFT_FIN_FM_BIG 8  // ... for N >= 2^19
#endif
#ifndef PBFT_FIN_TREE_MAX_FM
#define PBFT_FIN_TREE_MAX_FM 8  // finish widths up to this use the cross-lane product tree (one inversion per wave)
#endif
#ifndef PBFT_FIN_W_BIG
#define PBFT_FIN_W_BIG 2  // waves per SIMD of the product-tree finish for N >= 2^19
#endif


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
// A replica key set on one device: raw encodings, key_ok bytes and the -A comb
// tables.  Reference-counted so that contexts cloned for extra streams
// (pbft_verify_ctx_clone) serve batches from the same tables.
struct keyset {
  std::atomic<int> refs{1};
  uint32_t* d_tabA = nullptr;
  uint32_t* d_keys = nullptr;
  uint8_t* d_key_ok = nullptr;
  uint32_t n = 0;
  uint32_t cap = 0;      // keys d_keys / d_key_ok hold
  size_t tab_bytes = 0;  // bytes of d_tabA (a later set_keys whose plan's tables fit reuses the buffers)
  int pa = 0;  // positions of the key plan (identifies PLA_HUGE / PLA_BIG / PLA_MID / PLA_SMALL)
};
static size_t plan_table_words(int pa) {
  return pa == PLA_HUGE::P ? PLA_HUGE::TABLE_WORDS
       : pa == PLA_BIG::P  ? PLA_BIG::TABLE_WORDS
       : pa == PLA_MID::P  ? PLA_MID::TABLE_WORDS
                           : PLA_SMALL::TABLE_WORDS;
}
static void keyset_release(keyset* k) {
  if (k && --k->refs == 0) {
    (void)hipFree(k->d_tabA); (void)hipFree(k->d_keys); (void)hipFree(k->d_key_ok);
    delete k;
  }
}

// device staging buffers of the votes chunks (chunk c uses buffer c % VOTES_BUFS; its copy waits for the kernels
// of chunk c - VOTES_BUFS)
static constexpr int VOTES_BUFS = 4;
#ifndef PBFT_VOTES_TWO_STREAMS
#define PBFT_VOTES_TWO_STREAMS 1
#endif

struct pbft_ctx {
  int device = -1;
  hipStream_t stream = nullptr;
  uint32_t* d_tabB = nullptr;
  keyset* ks = nullptr;
  // cached from ks (null / 0 without a key set)
  uint32_t* d_tabA = nullptr;
  uint32_t* d_keys = nullptr;
  uint8_t* d_key_ok = nullptr;
  uint32_t n_keys = 0;
  int pa = 0;  // comb positions of the installed key tables' plan (PLA_HUGE, PLA_BIG, PLA_MID or PLA_SMALL)
  uint64_t split_below = SPLIT_BELOW;  // latency mode below this batch size (env PBFT_SPLIT_BELOW)
  int fin_m = 0;                       // finish-kernel signatures per lane (0 = by batch size)
  int fin_tree = -1;                   // finish cross-lane tree (0: none; 4 / 6: the compiled tree; -1 = by batch size)
  int fin_waves = 0;                   // product-tree finish compiled for 1 or 2 waves per SIMD (0 = by batch size)
  int lat_split = 0;                   // latency-mode lanes per signature (4 / 8; 0 = by batch size)
  int comb_pair = -1;                  // comb_pair_kernel: 1 on, 0 off, -1 by batch size (PBFT_OPT_COMB_PAIR)
  int comb_prio = -1;                  // 8-wave comb blocks with paired wave priorities: 1, 0, -1 by batch size
                                       // (PBFT_OPT_COMB_PRIO)
  int cus = 0;                         // compute units of the device
  // ev0 / ev1 around every launch (pbft_last_kernel_ms).  Off by default since r05: the two event records cost 7.5 us
  // per comb + finish pair, 4.5 % of the 131k shard (profiles/r05/shard/timing_events.txt)
  bool timing = false;
  uint64_t key_budget_mb = 0;          // key-table budget override (0 = env / default)
  pbft_key_stats kstats{};             // the last pbft_verify_set_keys / _update_keys (pbft_verify_key_stats)
  int fault_inject = 0;                // PBFT_OPT_FAULT_INJECT (tests): fail the next pbft_verify_update_keys
  void adopt(keyset* k) {
    keyset_release(ks);
    ks = k;
    d_tabA = k ? k->d_tabA : nullptr; d_keys = k ? k->d_keys : nullptr; d_key_ok = k ? k->d_key_ok : nullptr;
    n_keys = k ? k->n : 0; pa = k ? k->pa : 0;
  }
  // staging for the host-buffer API
  uint8_t* d_stage = nullptr;
  size_t stage_cap = 0;
  uint64_t* d_bitmap = nullptr;
  size_t bitmap_cap = 0;
  // verify workspace: R' limbs [30][N] u32 + flags[N]
  uint8_t* d_work = nullptr;
  size_t work_cap = 0;
  // votes form: per-envelope block-2 SHA-512 schedule (W[t] + K[t], t = 16..79; 512 B per envelope)
  uint64_t* d_wk = nullptr;
  uint64_t wk_cap = 0;  // envelopes
  uint64_t work_n = 0;     // signatures the workspace layout is sized for (offsets use this, not the batch N)
  bool work_two = false;   // two xyz/flags halves (pipelined form)
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_done = nullptr;
  // pipelined device form: comb on the caller's stream, finish on a second stream, two workspace halves
  hipEvent_t ev_comb = nullptr, ev_fin[2] = {nullptr, nullptr};
  bool fin_pending[2] = {false, false};
  int half = 0;
  // host-buffer pipeline: H2D of chunk c+1 (copy stream) overlaps the kernels of chunk c; VOTES_BUFS device
  // staging buffers (the per-signature form uses 2)
  hipStream_t cstream = nullptr;
  hipEvent_t ev_copied[VOTES_BUFS] = {}, ev_consumed[VOTES_BUFS] = {};
  // votes chunks alternate between the context stream and stream2, each with its own workspace, so that the
  // kernels of consecutive chunks may overlap (PBFT_VOTES_TWO_STREAMS)
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_env = nullptr, ev_s2 = nullptr;
  uint8_t* d_work2 = nullptr;
  size_t work2_cap = 0;
  uint64_t work2_n = 0;
  bool v_two = false;
  bool v_s2_ready = false;  // stream2 has waited for this batch's envelope table and schedule (ev_env)
  bool two_streams = PBFT_VOTES_TWO_STREAMS;  // env PBFT_VOTES_TWO_STREAMS
  bool in_flight = false;
  uint64_t* async_out = nullptr;
  uint64_t* h_bitmap = nullptr;      // pinned, fine-grained
  uint64_t* h_bitmap_dev = nullptr;  // the same memory as the kernels address it (export_words)
  uint64_t async_words = 0;
  float last_ms = 0.f;
  // pinned host staging of the non-blocking host-buffer forms (pageable caller buffers are copied here,
  // then DMA'd asynchronously; pbft_verify_votes_stage hands it out for in-place filling)
  uint8_t* h_stage = nullptr;
  uint8_t* h_stage_dev = nullptr;  // the same memory as the kernels address it (the import kernels)
  size_t h_stage_cap = 0;
  uint64_t staged_n = 0;   // pbft_verify_votes_stage: the batch the staging is laid out for
  uint32_t staged_env = 0;
  bool staged = false;
  // votes batch being launched chunk by chunk (stage_votes_and_launch, pbft_verify_votes_submit_begin / _rows)
  uint64_t v_n = 0, v_next = 0, v_chunk = 0;  // batch rows, first row not launched, chunks launched
  uint32_t v_env = 0;
  size_t v_env_bytes = 0;
  const uint64_t* v_wk = nullptr;
  bool v_open = false;      // begun, not every chunk launched
  bool v_readback = false;  // progressive: each chunk's bitmap words come back on their own (ev_rows)
  std::vector<hipEvent_t> ev_rows;  // per chunk: its bitmap words are in h_bitmap
  std::vector<uint64_t> v_ends;     // per launched chunk: its end row
  uint32_t v_env_cap = 0;           // a batch opened in pieces (pbft_verify_votes_open): its envelope capacity
  hipEvent_t ev_envp = nullptr;     // a piece's envelopes copied
  bool v_short_tail = false;        // the batch's schedule ends with a VOTES_TAIL-row chunk (votes_chunk_end)
  uint64_t rows_out = 0;            // rows whose bitmap words are in the caller's bitmap
  uint64_t chunk_out = 0;           // chunks whose bitmap words are in the caller's bitmap
};

#ifndef PBFT_ENV_SCHED
#define PBFT_ENV_SCHED 1  // A/B: 0 = every signature expands its own block-2 schedule
#endif

// Bitmap words [lo, lo + n) to the pinned host copy, written by a kernel over PCIe.  A hipMemcpyAsync D2H of these
// few KB blocked the calling thread for 6-8 ms at times on MI355X (PBFT_LAUNCH_TRACE in the replica's flush:
// profiles/r04/launch_stalls.txt), stalling the launch loop behind it; a kernel launch returns at once.  The host
// copy is fine-grained memory: the stores reach it without a cache writeback, and the event recorded after the
// kernel orders them before the host's read.
__global__ void export_words_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
  __threadfence_system();
}
static hipError_t export_words(pbft_ctx* c, uint64_t lo, uint64_t n, hipStream_t st);
// 16-byte words from host memory the kernels can address (the mapped staging) to device memory: one launch on the
// consuming stream instead of a copy-stream hipMemcpyAsync + event + cross-stream wait (~0.14 ms of host time per
// votes batch, PBFT_LAUNCH_TRACE=30)
__global__ void import16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// Pinned host staging (grow-only: hipHostMalloc costs milliseconds).  Never while a batch is in flight.
// Every user of the staging calls this first: whatever pbft_verify_votes_stage handed out is void from here on
// (a later pbft_verify_votes_submit must not launch what another path wrote there).
static int ensure_host_stage(pbft_ctx* c, size_t bytes) {
  c->staged = false;
  if (bytes <= c->h_stage_cap) return PBFT_OK;
  if (c->h_stage) HIP_TRY(hipHostFree(c->h_stage));
  c->h_stage = nullptr;
  c->h_stage_dev = nullptr;
  c->h_stage_cap = 0;
  const size_t cap = bytes + (bytes >> 2) + 4096;
  // fine-grained: kernels that read it in place see every host write, with no stale L2 lines
  if (hipHostMalloc(&c->h_stage, cap, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    (void)hipGetLastError();
    c->h_stage = nullptr;
    return set_err(PBFT_ENOMEM, "pinned host staging alloc");
  }
  if (hipHostGetDevicePointer((void**)&c->h_stage_dev, c->h_stage, 0) != hipSuccess) {
    (void)hipGetLastError();
    c->h_stage_dev = nullptr;  // (kernels then never read it in place)
  }
  c->h_stage_cap = cap;
  return PBFT_OK;
}

// True if p is host memory the DMA engines can read in place (hipHostMalloc / hipHostRegister).  A pageable
// pointer makes the query fail; the error is cleared so that the next launch's hipGetLastError is clean.
static bool host_pinned(const void* p) {
  if (!p) return true;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}
// The address kernels read pinned host memory p at, or null (pageable, or no device mapping).
static const uint8_t* host_dev(const void* p) {
  if (!p) return nullptr;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer) return nullptr;
  return (const uint8_t*)a.devicePointer + ((const uint8_t*)p - (const uint8_t*)a.hostPointer);
}

// Host-buffer batches up to one chunk: R, S, key_idx and the messages reach the device staging through ONE kernel
// that reads the pinned host memory over PCIe (16 B per lane, line-contiguous per wave), instead of four
// hipMemcpyAsync.  VERDICT r04 item 2: config #5's back-to-back leg had one 7.5-9.4 ms maximum in every bench line;
// PBFT_LAUNCH_TRACE put it inside hipMemcpyAsync H2D of a 4k batch's columns (profiles/r05/stall_probe.txt: the
// calling thread blocked 7-30 ms in h2d_R / h2d_M while a kernel launch never did), the same signature as the D2H
// stalls r04 removed from the votes path.  PBFT_HOST_IMPORT=0 restores the copies (A/B).
struct import_segs {
  const uint8_t* src[4];
  uint64_t dst_off[4];   // 16-B aligned offsets into the destination
  uint64_t len[4];       // bytes
  uint64_t first[5];     // first 16-B piece of each segment; first[4] = total pieces
};
__global__ void __launch_bounds__(256) import_segs_kernel(import_segs s, uint8_t* __restrict__ dst) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= s.first[4]) return;
  const int k = c >= s.first[2] ? (c >= s.first[3] ? 3 : 2) : (c >= s.first[1] ? 1 : 0);
  const uint64_t o = (c - s.first[k]) * 16;
  const uint8_t* src = s.src[k] + o;
  uint8_t* d = dst + s.dst_off[k] + o;
  const uint64_t rem = s.len[k] - o;
  if (rem >= 16 && ((uintptr_t)src & 15) == 0) {
    *(uint4*)d = *(const uint4*)src;
  } else if (rem >= 16 && ((uintptr_t)src & 3) == 0) {
    const uint32_t* q = (const uint32_t*)src;
    *(uint4*)d = uint4{q[0], q[1], q[2], q[3]};
  } else {
    const int m = rem < 16 ? (int)rem : 16;
    for (int b = 0; b < m; ++b) d[b] = src[b];
  }
}
static bool host_import_enabled() {
  static const bool on = [] {
    const char* e = getenv("PBFT_HOST_IMPORT");
    return !e || strtol(e, nullptr, 10) != 0;
  }();
  return on;
}
// Launch the import of up to 4 host segments (device-readable addresses) into dst; false if a source has no device
// mapping (the caller then copies).
static bool launch_import(const uint8_t* const* src_host, const uint64_t* dst_off, const uint64_t* len, int n,
                          uint8_t* dst, hipStream_t st) {
  if (!host_import_enabled()) return false;
  import_segs s{};
  uint64_t pieces = 0;
  for (int k = 0; k < 4; ++k) {
    s.first[k] = pieces;
    if (k < n && len[k]) {
      s.src[k] = host_dev(src_host[k]);
      if (!s.src[k]) return false;
      s.dst_off[k] = dst_off[k];
      s.len[k] = len[k];
      pieces += (len[k] + 15) / 16;
    }
  }
  s.first[4] = pieces;
  if (pieces == 0) return true;
  hipLaunchKernelGGL(import_segs_kernel, dim3((unsigned)((pieces + 255) / 256)), dim3(256), 0, st, s, dst);
  return true;
}

// Pinned layout of a staged votes batch (pbft_verify_votes_stage): n rows of PBFT_VOTES_ROW_BYTES, then the
// envelopes.
static constexpr uint32_t ROW = PBFT_VOTES_ROW_BYTES;
static_assert(PBFT_VOTES_ROW_BYTES % 8 == 0 && PBFT_VOTES_ROW_KEY == 64 && PBFT_VOTES_ROW_ENV % 4 == 0 &&
                  PBFT_VOTES_ROW_ENV + 4 <= PBFT_VOTES_ROW_BYTES, "votes row layout");
struct host_votes_layout {
  size_t offE, bytes;
  host_votes_layout(uint64_t n, uint32_t n_env) {
    offE = (ROW * (size_t)n + 255) & ~(size_t)255;
    bytes = offE + (size_t)PBFT_ENVELOPE_LEN * n_env + 64;  // + read slack of the envelope loads
  }
};
struct host_batch_layout {
  size_t offS, offK, offM, bytes;
  host_batch_layout(uint64_t n, uint32_t msg_stride) {
    offS = 32 * n;
    offK = 64 * n;
    offM = (offK + 2 * n + 255) & ~(size_t)255;
    bytes = offM + (size_t)msg_stride * n + 64;
  }
};

static hipError_t export_words(pbft_ctx* c, uint64_t lo, uint64_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(export_words_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, c->d_bitmap + lo,
                     c->h_bitmap_dev + lo, n);
  return hipGetLastError();
}

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
    c->d_bitmap = nullptr; c->h_bitmap = nullptr; c->h_bitmap_dev = nullptr;
    size_t cap = words + 64;
    if (hipMalloc(&c->d_bitmap, cap * 8) != hipSuccess) return set_err(PBFT_ENOMEM, "bitmap alloc");
    if (hipHostMalloc(&c->h_bitmap, cap * 8, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return set_err(PBFT_ENOMEM, "pinned bitmap alloc");
    HIP_TRY(hipHostGetDevicePointer((void**)&c->h_bitmap_dev, c->h_bitmap, 0));
    c->bitmap_cap = cap;
  }
  return PBFT_OK;
}

// Grow the verify workspace (never inside a stream capture: call
// pbft_verify_reserve first when capturing launches into a graph).
// Workspace per launch of N signatures (Npad = N rounded up to BLOCK):
//   xyz   [30][N] u32   R' limbs, comb -> finish            120 B/sig
//   flags [N] u8                                              1 B/sig
//   eidx  [steps][Npad] u32  per-step table entry indices    4 x steps B/sig
static constexpr int MAX_STEPS = steps<PLB, PLA_SMALL>::N;  // the smallest key plan has the most steps
static_assert(steps<PLB, PLA_SMALL>::N >= steps<PLB, PLA_MID>::N && steps<PLB, PLA_MID>::N >= steps<PLB, PLA_BIG>::N,
              "");
static inline size_t eidx_offset(uint64_t N) { return (121 * (size_t)N + 255) & ~(size_t)255; }
static inline size_t eidx_bytes(uint64_t N) {
  const uint64_t Npad = (N + 2 * BLOCK - 1) / (2 * BLOCK) * (2 * BLOCK);  // (8-wave comb blocks: PBFT_OPT_COMB_PRIO)
  // (latency mode: 4 or 8 lanes per signature, 8-byte entry addresses, ceil(steps / lanes) per lane)
  const size_t split4 = 8 * (size_t)((MAX_STEPS + 3) / 4) * (Npad * 4 + BLOCK);
  const size_t split8 = 8 * (size_t)((MAX_STEPS + 7) / 8) * (Npad * 8 + BLOCK);
  const size_t split = split4 > split8 ? split4 : split8;
  const size_t comb = 4 * (size_t)MAX_STEPS * Npad;
  return ((comb > split ? comb : split) + 255) & ~(size_t)255;
}
// PBFT_LAUNCH_TRACE=1: every HIP call of a votes chunk launch that blocks the host for more than 0.3 ms is reported
// on stderr (the replica's flush timeline showed 6-7 ms stalls inside pbft_verify_votes_submit_rows)
// (PBFT_LAUNCH_TRACE=<n> with n > 1: report calls longer than n microseconds instead)
static double launch_trace_ms() {
  static const double ms = [] {
    const char* e = getenv("PBFT_LAUNCH_TRACE");
    if (!e) return -1.0;
    const double v = strtod(e, nullptr);
    return v > 1 ? v / 1000.0 : 0.3;
  }();
  return ms;
}
static bool launch_trace() { return launch_trace_ms() >= 0; }
#define LT(name, ...)                                                                                              \
  do {                                                                                                             \
    const auto lt_t0 = std::chrono::steady_clock::now();                                                           \
    __VA_ARGS__;                                                                                                   \
    if (launch_trace()) {                                                                                          \
      const double lt_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - lt_t0).count(); \
      if (lt_ms > launch_trace_ms())                                                                            \
        fprintf(stderr, "launch-stall %s chunk %u: %.3f ms\n", name, (unsigned)c->v_chunk, lt_ms);             \
    }                                                                                                              \
  } while (0)

// second xyz/flags half (pipelined form) after the entry-index region
static inline size_t half1_offset(uint64_t N) { return eidx_offset(N) + eidx_bytes(N); }
// the whole workspace: half 0, the entry indices and (pipelined form) half 1
static inline size_t work_bytes(uint64_t W, bool two) {
  return ((two ? half1_offset(W) + eidx_offset(W) : half1_offset(W)) + 255) & ~(size_t)255;
}
// The layout is a function of c->work_n only, never of the batch at hand: a smaller batch must not move
// the entry-index region onto the xyz/flags half a pipelined finish may still be reading.
static int ensure_work(pbft_ctx* c, uint64_t N, bool two_halves = false) {
  if (N <= c->work_n && (!two_halves || c->work_two)) return PBFT_OK;
  const uint64_t W = N > c->work_n ? N : c->work_n;
  const bool two = two_halves || c->work_two;
  const size_t need = work_bytes(W, two);
  // nothing may still read the old workspace: the finishes of earlier pipelined launches, then this stream
  for (int h = 0; h < 2; ++h)
    if (c->fin_pending[h]) { HIP_TRY(hipEventSynchronize(c->ev_fin[h])); c->fin_pending[h] = false; }
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->d_work) HIP_TRY(hipDeviceSynchronize());  // a device-form launch may run on a caller's stream
  if (c->d_work) HIP_TRY(hipFree(c->d_work));
  c->d_work = nullptr;
  c->work_cap = 0;
  c->work_n = 0;
  c->work_two = false;
  if (hipMalloc(&c->d_work, need) != hipSuccess) return set_err(PBFT_ENOMEM, "verify workspace alloc");
  c->work_cap = need;
  c->work_n = W;
  c->work_two = two;
  return PBFT_OK;
}

// The second workspace (votes chunks on stream2): one half, same layout.
static int ensure_work2(pbft_ctx* c, uint64_t N) {
  if (N <= c->work2_n) return PBFT_OK;
  const uint64_t W = N;
  const size_t need = work_bytes(W, false);
  if (c->d_work2) {
    HIP_TRY(hipStreamSynchronize(c->stream2));
    HIP_TRY(hipFree(c->d_work2));
  }
  c->d_work2 = nullptr;
  c->work2_cap = 0;
  c->work2_n = 0;
  if (hipMalloc(&c->d_work2, need) != hipSuccess) return set_err(PBFT_ENOMEM, "verify workspace alloc");
  c->work2_cap = need;
  c->work2_n = W;
  return PBFT_OK;
}

// fst != null: pipelined form -- the finish runs on fst after an event, on one of two
// workspace halves, so the next launch's comb (on st) overlaps it.  slot 1: the second workspace (votes chunks
// on stream2; no timing events, never pipelined).
static int launch_verify(pbft_ctx* c, const uint8_t* dR, const uint8_t* dS, const uint16_t* dK, const uint8_t* dM,
                         uint32_t msg_len, uint32_t msg_stride, uint64_t N, uint64_t* dB, hipStream_t st,
                         uint32_t rs_stride = 32, uint32_t k_stride = 2, hipStream_t fst = nullptr,
                         const uint32_t* dMI = nullptr, uint32_t n_msg = 0, const uint64_t* dWK = nullptr,
                         uint32_t mi_stride = 1, int slot = 0) {
  if (N == 0) return PBFT_OK;
  const uint64_t blocks = (N + BLOCK - 1) / BLOCK;
  if (blocks > 0x7fffffffull) return set_err(PBFT_EINVAL, "N too large for one launch");
  int rc = slot ? ensure_work2(c, N) : ensure_work(c, N, fst != nullptr);
  if (rc) return rc;
  uint8_t* const wbase = slot ? c->d_work2 : c->d_work;
  const bool timing = c->timing && slot == 0;
  int h = 0;
  if (fst) {
    h = c->half;
    c->half ^= 1;
  }
  if (slot == 0 && c->fin_pending[h]) HIP_TRY(hipStreamWaitEvent(st, c->ev_fin[h], 0));  // a pipelined finish still reading half h
  if (timing) LT("rec_ev0", HIP_TRY(hipEventRecord(c->ev0, st)));
  const uint64_t W = slot ? c->work2_n : c->work_n;  // layout (>= N)
  uint8_t* hw = wbase + (h ? half1_offset(W) : 0);
  const bool latency_mode = N < c->split_below;
  comb_launch_args a;
  a.R = dR; a.S = dS; a.K = (const uint8_t*)dK; a.rs_stride = rs_stride; a.k_stride = k_stride;
  a.M = dM; a.msg_len = msg_len; a.msg_stride = msg_stride; a.N = N;
  a.tabB = c->d_tabB; a.tabA = c->d_tabA; a.keys = c->d_keys; a.key_ok = c->d_key_ok; a.n_keys = c->n_keys;
  a.xyz = (uint32_t*)hw;
  a.flags = hw + 120 * N;  // within the half's 121 W bytes
  a.eidx = (uint32_t*)(wbase + eidx_offset(W));
  a.bitmap = dB; a.msg_idx = dMI; a.n_msg = n_msg; a.mi_stride = mi_stride; a.latency_mode = latency_mode; a.lat_split = c->lat_split; a.st = st;
  a.pair = c->comb_pair;
  a.cus = c->cus;
  a.prio = c->comb_prio;
  a.wk = (PBFT_ENV_SCHED && dMI && msg_len == PBFT_ENVELOPE_LEN) ? dWK : nullptr;
  uint32_t* xyz = a.xyz;
  uint8_t* flags = a.flags;
  LT("comb", HIP_TRY(c->pa == PLA_HUGE::P  ? launch_comb_huge(a)
                     : c->pa == PLA_BIG::P ? launch_comb_big(a)
                     : c->pa == PLA_MID::P ? launch_comb_mid(a)
                                           : launch_comb_small(a)));
  HIP_TRY(hipGetLastError());
  if (fst) {
    if (timing) HIP_TRY(hipEventRecord(c->ev1, st));  // pipelined form: last_kernel_ms = the comb (or latency) kernel
    HIP_TRY(hipEventRecord(c->ev_comb, st));
    HIP_TRY(hipStreamWaitEvent(fst, c->ev_comb, 0));
    st = fst;
  }
  if (!latency_mode) {  // (the latency kernel writes the bitmap itself)
    // signatures per finish lane, product tree and waves per SIMD by batch size (PBFT_FIN_* above)
    const bool big = N >= ((uint64_t)1 << 19);
    int fm = big ? PBFT_FIN_FM_BIG : N > PBFT_FIN_SMALL_UPTO ? PBFT_FIN_FM_MID
                                   : N > PBFT_FIN_TINY_UPTO  ? PBFT_FIN_FM_SMALL : 1;
    // cross-lane product tree (one variable-time inversion per 16-lane row since r04, per wave before) where few
    // signatures share a lane: 131k 0.2106 -> 0.2061 ms at fm 4, 0.2467 -> 0.2160 at fm 1; no gain at fm 16
    // (profiles/r02_ab_log.md); lv is a flag here, finish.hip compiles the tree depth (PBFT_FIN_LV)
    int lv = fm <= PBFT_FIN_TREE_MAX_FM ? PBFT_FIN_LV : 0;
    if (c->fin_m) fm = c->fin_m;
    if (c->fin_tree >= 0) lv = c->fin_tree;
    const int fw = c->fin_waves ? c->fin_waves : (big ? PBFT_FIN_W_BIG : 1);
    LT("finish", HIP_TRY(launch_finish(fm, lv, fw, dR, rs_stride, xyz, flags, N, dB, st)));
    HIP_TRY(hipGetLastError());
  }
  if (fst) {
    HIP_TRY(hipEventRecord(c->ev_fin[h], fst));
    c->fin_pending[h] = true;
    return PBFT_OK;
  }
  if (timing) LT("rec_ev1", HIP_TRY(hipEventRecord(c->ev1, st)));
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

// Staging layout of n signatures: R | S | key_idx | msg (+ slack for unaligned message reads).
struct stage_layout {
  size_t offS, offK, offM, bytes;
  stage_layout(uint64_t n, uint32_t msg_stride) {
    offS = 32 * n;
    offK = 64 * n;
    offM = (offK + 2 * n + 255) & ~(size_t)255;
    bytes = (offM + (size_t)msg_stride * n + 64 + 255) & ~(size_t)255;
  }
};

// Host batches above this many signatures are copied and verified in chunks on two
// staging halves: the H2D copy of chunk c+1 (context copy stream) overlaps the
// kernels of chunk c (context stream).  A multiple of 64: chunks own whole
// bitmap words.  2^18 keeps every chunk in the one-lane-per-signature mode.
#ifndef PBFT_PIPE_CHUNK_LOG2
#define PBFT_PIPE_CHUNK_LOG2 18
#endif
#define PBFT_VOTES_CHUNK_LOG2 18  // PBFT_VOTES_CHUNK_ROWS (include/pbft_verify.h: the replica follows the schedule)
static_assert(PBFT_VOTES_CHUNK_ROWS == (1u << PBFT_VOTES_CHUNK_LOG2) && PBFT_VOTES_FIRST_ROWS % 64 == 0, "");
// chunks own whole 64-bit bitmap words (the kernels write d_bitmap + lo / 64, readbacks copy (n + 63) / 64 words)
static_assert(PBFT_PIPE_CHUNK_LOG2 >= 6 && PBFT_VOTES_CHUNK_LOG2 >= 6, "chunks must be multiples of 64 rows");
static constexpr uint64_t PIPE_CHUNK = 1ull << PBFT_PIPE_CHUNK_LOG2;
// the votes form moves 70 B per signature instead of 151: its copies are about as long as the kernels, so a
// smaller chunk shortens the pipeline's fill and drain (PBFT_VOTES_CHUNK_LOG2)
static constexpr uint64_t VOTES_CHUNK = 1ull << PBFT_VOTES_CHUNK_LOG2;

// Copy a host batch into the staging buffer and launch.  Result: the device bitmap.
static int stage_and_launch(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint8_t* M,
                            uint32_t msg_len, uint32_t msg_stride, uint64_t N) {
  const uint64_t words = (N + 63) / 64;
  if (N <= PIPE_CHUNK) {
    const stage_layout L(N, msg_stride);
    int rc = ensure_stage(c, L.bytes, words);
    if (rc) return rc;
    const uint8_t* src[4] = {R, S, (const uint8_t*)K, M};
    const uint64_t off[4] = {0, L.offS, L.offK, L.offM};
    const uint64_t len[4] = {32 * N, 32 * N, 2 * N, (uint64_t)msg_stride * N};
    bool imported = false;
    LT("import", imported = launch_import(src, off, len, 4, c->d_stage, c->stream));
    if (imported) {
      HIP_TRY(hipGetLastError());
    } else {
      LT("h2d_R", HIP_TRY(hipMemcpyAsync(c->d_stage, R, 32 * N, hipMemcpyHostToDevice, c->stream)));
      LT("h2d_S", HIP_TRY(hipMemcpyAsync(c->d_stage + L.offS, S, 32 * N, hipMemcpyHostToDevice, c->stream)));
      LT("h2d_K", HIP_TRY(hipMemcpyAsync(c->d_stage + L.offK, K, 2 * N, hipMemcpyHostToDevice, c->stream)));
      if ((size_t)msg_stride * N)
        LT("h2d_M", HIP_TRY(hipMemcpyAsync(c->d_stage + L.offM, M, (size_t)msg_stride * N, hipMemcpyHostToDevice,
                                           c->stream)));
    }
    return launch_verify(c, c->d_stage, c->d_stage + L.offS, (const uint16_t*)(c->d_stage + L.offK),
                         c->d_stage + L.offM, msg_len, msg_stride, N, c->d_bitmap, c->stream);
  }
  const stage_layout L(PIPE_CHUNK, msg_stride);
  int rc = ensure_stage(c, 2 * L.bytes, words);
  if (rc) return rc;
  uint64_t chunk = 0;
  for (uint64_t lo = 0; lo < N; lo += PIPE_CHUNK, ++chunk) {
    const uint64_t n = N - lo < PIPE_CHUNK ? N - lo : PIPE_CHUNK;
    const int b = (int)(chunk & 1);
    uint8_t* base = c->d_stage + (size_t)b * L.bytes;
    if (chunk >= 2) HIP_TRY(hipStreamWaitEvent(c->cstream, c->ev_consumed[b], 0));  // kernels of chunk-2 done
    HIP_TRY(hipMemcpyAsync(base, R + 32 * lo, 32 * n, hipMemcpyHostToDevice, c->cstream));
    HIP_TRY(hipMemcpyAsync(base + L.offS, S + 32 * lo, 32 * n, hipMemcpyHostToDevice, c->cstream));
    HIP_TRY(hipMemcpyAsync(base + L.offK, K + lo, 2 * n, hipMemcpyHostToDevice, c->cstream));
    if ((size_t)msg_stride * n)
      HIP_TRY(hipMemcpyAsync(base + L.offM, M + (size_t)msg_stride * lo, (size_t)msg_stride * n,
                             hipMemcpyHostToDevice, c->cstream));
    HIP_TRY(hipEventRecord(c->ev_copied[b], c->cstream));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_copied[b], 0));
    rc = launch_verify(c, base, base + L.offS, (const uint16_t*)(base + L.offK), base + L.offM, msg_len, msg_stride,
                       n, c->d_bitmap + lo / 64, c->stream);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c->ev_consumed[b], c->stream));
  }
  return PBFT_OK;
}

// Votes form, once per call: the block-2 SHA-512 schedule of every 85-byte envelope (sha512.h
// sha512_env_sched), read by each signature's challenge hash instead of expanding it again.
__global__ void __launch_bounds__(BLOCK) env_sched_kernel(const uint8_t* __restrict__ env, uint32_t n_env,
                                                          uint64_t* __restrict__ wk) {
  const uint64_t e = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (e >= n_env) return;
  sha512_env_sched(wk + (size_t)SHA_ENV_WORDS * e, env + (size_t)PBFT_ENVELOPE_LEN * e);
}

// (the buffer grows on first use for a bigger table: not inside a stream capture)
static int ensure_wk(pbft_ctx* c, uint32_t n_env) {
  if (n_env > c->wk_cap) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->d_wk) {
      HIP_TRY(hipDeviceSynchronize());  // a device-form launch may still read it on a caller's stream
      HIP_TRY(hipFree(c->d_wk));
    }
    c->d_wk = nullptr;
    c->wk_cap = 0;
    if (hipMalloc(&c->d_wk, (size_t)SHA_ENV_WORDS * 8 * n_env) != hipSuccess)
      return set_err(PBFT_ENOMEM, "envelope schedule alloc");
    c->wk_cap = n_env;
  }
  return PBFT_OK;
}
static int prepare_env_sched(pbft_ctx* c, const uint8_t* dENV, uint32_t n_env, hipStream_t st, const uint64_t** out) {
  int rc = ensure_wk(c, n_env);
  if (rc) return rc;
  hipLaunchKernelGGL(env_sched_kernel, dim3((n_env + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, dENV, n_env, c->d_wk);
  HIP_TRY(hipGetLastError());
  *out = c->d_wk;
  return PBFT_OK;
}

// Votes form (include/pbft_verify.h pbft_verify_votes): R, S, key_idx and a 4-byte envelope index per
// signature (70 B instead of 151 B over PCIe; 72 B as staged rows) + the batch's table of distinct 85-byte
// envelopes.
// One chunk's device staging: R | S | key_idx | env_idx columns (caller columns), or the chunk's rows as staged
// (PBFT_VOTES_ROW_BYTES each, one copy).
struct votes_layout {
  size_t offS, offK, offI, bytes;
  explicit votes_layout(uint64_t n) {
    offS = 32 * n;
    offK = 64 * n;
    offI = (offK + 2 * n + 15) & ~(size_t)15;
    const size_t cols = (offI + 4 * n + 255) & ~(size_t)255, rows = (ROW * (size_t)n + 255) & ~(size_t)255;
    bytes = cols > rows ? cols : rows;
  }
};

// The kernels' address of [p, p + bytes) in the context's mapped staging, else null.
static const uint8_t* zc_map(const pbft_ctx* c, const void* p, size_t bytes) {
  const uint8_t* q = (const uint8_t*)p;
  if (!c->h_stage_dev || q < c->h_stage || q + bytes > c->h_stage + c->h_stage_cap) return nullptr;
  return c->h_stage_dev + (q - c->h_stage);
}

// rs_stride 32: R and S are separate [N][32] host columns (key_idx, env_idx columns too); PBFT_VOTES_ROW_BYTES: R
// = the staged rows (S = R + 32, key_idx at + 64, env_idx at + 68 of each row).
// votes_begin copies the envelope table and launches its schedule; votes_launch then launches every whole chunk
// inside rows [0, rows) (all the rest once rows >= N): the kernels of chunk c run on the context stream after
// its copies (copy stream), overlapping the copies of chunk c+1.
// Chunk schedule of a votes batch: PBFT_VOTES_CHUNK_END, or (v_short_tail: rows that are all in host memory when
// the batch starts, pbft_verify_votes_submit_host) the same with its last chunk cut down to ~VOTES_TAIL rows -- what
// is left once the last copy lands is that chunk's kernels and the caller's application of its rows
// (r05: the replica's flush ended with 64k rows of both).
static constexpr uint64_t VOTES_TAIL = 16384;
static uint64_t votes_chunk_end(const pbft_ctx* c, uint64_t lo, uint64_t N) {
  const uint64_t e = PBFT_VOTES_CHUNK_END(lo, N);
  if (c->v_short_tail && e == N && N > VOTES_CHUNK && N - lo > VOTES_TAIL + 64) return lo + ((N - lo - VOTES_TAIL) & ~(uint64_t)63);
  return e;
}

static int votes_begin(pbft_ctx* c, const uint8_t* ENV, uint32_t n_env, uint64_t N, bool readback,
                       bool short_tail = false) {
  c->v_short_tail = short_tail;
  c->v_env_cap = 0;  // (not a batch in pieces)
  c->v_ends.clear();
  const uint64_t words = (N + 63) / 64;
  const size_t env_bytes = ((size_t)PBFT_ENVELOPE_LEN * n_env + 64 + 255) & ~(size_t)255;  // + read slack
  const uint64_t ch = N < VOTES_CHUNK ? N : VOTES_CHUNK;
  const votes_layout L(ch);
  int rc = ensure_stage(c, env_bytes + (N > VOTES_CHUNK ? VOTES_BUFS : 1) * L.bytes, words);
  if (rc) return rc;
  // more than one chunk: odd chunks' kernels on stream2 (their own workspace), so consecutive chunks' kernels may
  // overlap -- the small first chunks and the last big one leave most of the GPU idle on one stream
  const bool two = c->two_streams && N > PBFT_VOTES_FIRST_ROWS;
  if (two && !c->stream2) {
    HIP_TRY(hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_env, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_s2, hipEventDisableTiming));
  }
  if (readback) {
    uint64_t chunks = 0;
    for (uint64_t lo = 0; lo < N; lo = votes_chunk_end(c, lo, N)) ++chunks;
    while (c->ev_rows.size() < chunks) {
      hipEvent_t e;
      HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      c->ev_rows.push_back(e);
    }
  }
  const size_t env_len = (size_t)PBFT_ENVELOPE_LEN * n_env;
  const uint8_t* zenv = zc_map(c, ENV, env_len + 15);
  if (zenv && ((uintptr_t)zenv & 15) == 0) {  // the table sits in the mapped staging: copied by a kernel
    const uint64_t n16 = (env_len + 15) / 16;
    hipLaunchKernelGGL(import16_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, c->stream,
                       (const uint4*)zenv, (uint4*)c->d_stage, n16);
    LT("import_env", HIP_TRY(hipGetLastError()));
  } else {
    LT("h2d_env", HIP_TRY(hipMemcpyAsync(c->d_stage, ENV, env_len, hipMemcpyHostToDevice, c->cstream)));
    // the envelopes' block-2 schedule on the context stream once the table has landed (ev_copied[0] is
    // re-recorded by chunk 0)
    LT("rec_env", HIP_TRY(hipEventRecord(c->ev_copied[0], c->cstream)));
    LT("wait_env", HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_copied[0], 0)));
  }
  LT("env_sched", rc = prepare_env_sched(c, c->d_stage, n_env, c->stream, &c->v_wk));
  if (rc) return rc;
  // stream2's chunks read the envelope table and its schedule too (it waits at its first chunk: votes_launch)
  if (two) HIP_TRY(hipEventRecord(c->ev_env, c->stream));
  c->v_s2_ready = false;
  c->v_two = two;
  c->v_n = N;
  c->v_next = 0;
  c->v_chunk = 0;
  c->v_env_bytes = env_bytes;
  c->v_env = n_env;
  c->v_open = true;
  c->v_readback = readback;
  c->rows_out = 0;
  c->chunk_out = 0;
  return PBFT_OK;
}

// One chunk of a votes batch: rows [lo, lo + n) -- their copy (or the mapped staging read in place), the kernels
// on the chunk's stream, its bitmap words back (progressive form) -- then v_next / v_chunk advance.
static int votes_chunk(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint32_t* IDX,
                       uint32_t rs_stride, uint64_t lo, uint64_t n) {
  const uint64_t N = c->v_n;
  const votes_layout L(N < VOTES_CHUNK ? N : VOTES_CHUNK);
  const int b = (int)(c->v_chunk % VOTES_BUFS);
  const int slot = c->v_two ? (int)(c->v_chunk & 1) : 0;
  hipStream_t st = slot ? c->stream2 : c->stream;
  if (slot && !c->v_s2_ready) {
    LT("wait_env2", HIP_TRY(hipStreamWaitEvent(c->stream2, c->ev_env, 0)));
    c->v_s2_ready = true;
  }
  if (c->v_readback && c->ev_rows.size() <= c->v_chunk) {  // (pieces: the chunk count is not known up front)
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->ev_rows.push_back(e);
  }
  c->v_ends.push_back(lo + n);
  const bool rows_form = rs_stride == ROW;
  const uint32_t ks = rows_form ? ROW : 2, mis = rows_form ? ROW / 4 : 1;
  uint8_t* base = c->d_stage + c->v_env_bytes + (size_t)b * L.bytes;
  if (c->v_chunk >= VOTES_BUFS) LT("wait_consumed", HIP_TRY(hipStreamWaitEvent(c->cstream, c->ev_consumed[b], 0)));
  if (rows_form) {  // the chunk's rows: one copy
    LT("h2d_rows", HIP_TRY(hipMemcpyAsync(base, R + (size_t)ROW * lo, (size_t)ROW * n, hipMemcpyHostToDevice,
                                          c->cstream)));
  } else {
    HIP_TRY(hipMemcpyAsync(base, R + 32 * lo, 32 * n, hipMemcpyHostToDevice, c->cstream));
    HIP_TRY(hipMemcpyAsync(base + L.offS, S + 32 * lo, 32 * n, hipMemcpyHostToDevice, c->cstream));
    LT("h2d_key", HIP_TRY(hipMemcpyAsync(base + L.offK, K + lo, 2 * n, hipMemcpyHostToDevice, c->cstream)));
    LT("h2d_idx", HIP_TRY(hipMemcpyAsync(base + L.offI, IDX + lo, 4 * n, hipMemcpyHostToDevice, c->cstream)));
  }
  LT("rec_copied", HIP_TRY(hipEventRecord(c->ev_copied[b], c->cstream)));
  LT("wait_copied", HIP_TRY(hipStreamWaitEvent(st, c->ev_copied[b], 0)));
  int rc = 0;
  LT("kernels", rc = launch_verify(c, base, base + (rows_form ? 32 : L.offS),
                                   (const uint16_t*)(base + (rows_form ? PBFT_VOTES_ROW_KEY : L.offK)), c->d_stage,
                                   PBFT_ENVELOPE_LEN, PBFT_ENVELOPE_LEN, n, c->d_bitmap + lo / 64, st,
                                   rs_stride, ks, nullptr,
                                   (const uint32_t*)(base + (rows_form ? PBFT_VOTES_ROW_ENV : L.offI)), c->v_env,
                                   c->v_wk, mis, slot));
  if (rc) return rc;
  LT("rec_consumed", HIP_TRY(hipEventRecord(c->ev_consumed[b], st)));
  if (c->v_readback) {  // this chunk's bitmap words (a few KB) back on their own, for the caller to apply early
    LT("export_bitmap", HIP_TRY(export_words(c, lo / 64, (n + 63) / 64, st)));
    LT("rec_rows", HIP_TRY(hipEventRecord(c->ev_rows[c->v_chunk], st)));
  }
  c->v_next += n;
  ++c->v_chunk;
  return PBFT_OK;
}

// The context stream (ev_done, the final bitmap export) follows stream2's last chunk too
static int votes_join_streams(pbft_ctx* c) {
  if (c->v_two) {
    HIP_TRY(hipEventRecord(c->ev_s2, c->stream2));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_s2, 0));
  }
  return PBFT_OK;
}

static int votes_launch(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint32_t* IDX,
                        uint32_t rs_stride, uint64_t rows) {
  const uint64_t N = c->v_n;
  while (c->v_next < N && (rows >= N || votes_chunk_end(c, c->v_next, N) <= rows)) {
    const uint64_t lo = c->v_next;
    const int rc = votes_chunk(c, R, S, K, IDX, rs_stride, lo, votes_chunk_end(c, lo, N) - lo);
    if (rc) return rc;
  }
  if (c->v_next >= N) {
    c->v_open = false;
    return votes_join_streams(c);
  }
  return PBFT_OK;
}

static int stage_votes_and_launch(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K,
                                  const uint32_t* IDX, const uint8_t* ENV, uint32_t n_env, uint64_t N,
                                  uint32_t rs_stride = 32) {
  int rc = votes_begin(c, ENV, n_env, N, false);
  if (rc) return rc;
  rc = votes_launch(c, R, S, K, IDX, rs_stride, N);
  c->v_open = false;
  return rc;
}

// The base-point comb table is a constant of the curve: one copy per device,
// shared by every context on it (reference-counted; 30 GB with the default plan).
static std::mutex g_tabB_mu;
static uint32_t* g_tabB[64] = {};
static int g_tabB_refs[64] = {};

static int acquire_base_table(int device, hipStream_t st, uint32_t** out) {
  std::lock_guard<std::mutex> lk(g_tabB_mu);
  if (device < 0 || device >= 64) return set_err(PBFT_ENODEV, "device ordinal >= 64");
  if (!g_tabB[device]) {
    // base point B = (x, 4/5), x even
    const uint32_t benc[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                              0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
    uint32_t* d_benc = nullptr;
    uint32_t* tab = nullptr;
    HIP_TRY(hipMalloc(&d_benc, 32));
    if (hipMalloc(&tab, PLB::TABLE_WORDS * 4) != hipSuccess) {
      (void)hipFree(d_benc);
      return set_err(PBFT_ENOMEM, "base-point table alloc");
    }
    HIP_TRY(hipMemcpyAsync(d_benc, benc, 32, hipMemcpyHostToDevice, st));
    int rc = build_comb_tables(0, d_benc, 1u, 0, tab, nullptr, st) == hipSuccess ? PBFT_OK : set_err(PBFT_EHIP, "base table build");
    (void)hipFree(d_benc);
    if (rc) { (void)hipFree(tab); return rc; }
    g_tabB[device] = tab;
  }
  ++g_tabB_refs[device];
  *out = g_tabB[device];
  return PBFT_OK;
}

static void release_base_table(int device) {
  std::lock_guard<std::mutex> lk(g_tabB_mu);
  if (device < 0 || device >= 64 || g_tabB_refs[device] == 0) return;
  if (--g_tabB_refs[device] == 0) {
    (void)hipFree(g_tabB[device]);
    g_tabB[device] = nullptr;
  }
}

extern "C" {

const char* pbft_last_error(void) { return g_last_error.c_str(); }

const char* pbft_build_info(void) {
  static char buf[256];
  snprintf(buf, sizeof buf,
           "pbft_verify gfx950 PB=%d PA=%d|%d|%d|%d block=%d entry=128B tabB=%zuB tabA/key=%zuB|%zuB|%zuB|%zuB",
           PLB::P, PLA_HUGE::P, PLA_BIG::P, PLA_MID::P, PLA_SMALL::P, BLOCK, PLB::TABLE_WORDS * 4,
           PLA_HUGE::TABLE_WORDS * 4, PLA_BIG::TABLE_WORDS * 4, PLA_MID::TABLE_WORDS * 4, PLA_SMALL::TABLE_WORDS * 4);
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
  c->cus = prop.multiProcessorCount;
  if (const char* e = getenv("PBFT_COMB_PRIO")) {
    const long v = strtol(e, nullptr, 10);
    c->comb_prio = (v == 0 || v == 1) ? (int)v : -1;
  }
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  if (const char* e = getenv("PBFT_SPLIT_BELOW")) c->split_below = strtoull(e, nullptr, 10);
  if (const char* e = getenv("PBFT_VOTES_TWO_STREAMS")) c->two_streams = strtol(e, nullptr, 10) != 0;
  if (const char* e = getenv("PBFT_COMB_PAIR")) {
    const long v = strtol(e, nullptr, 10);
    c->comb_pair = (v == 0 || v == 1) ? (int)v : -1;
  }
  HIP_TRY(hipEventCreate(&c->ev0));
  HIP_TRY(hipEventCreate(&c->ev1));
  HIP_TRY(hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming));
  HIP_TRY(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&c->ev_comb, hipEventDisableTiming));
  for (int b = 0; b < 2; ++b) HIP_TRY(hipEventCreateWithFlags(&c->ev_fin[b], hipEventDisableTiming));
  for (int b = 0; b < VOTES_BUFS; ++b) {
    HIP_TRY(hipEventCreateWithFlags(&c->ev_copied[b], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_consumed[b], hipEventDisableTiming));
  }
  int rc = acquire_base_table(device, c->stream, &c->d_tabB);
  if (rc) {
    (void)hipEventDestroy(c->ev0); (void)hipEventDestroy(c->ev1); (void)hipEventDestroy(c->ev_done);
    for (int b = 0; b < 2; ++b) (void)hipEventDestroy(c->ev_fin[b]);
    for (int b = 0; b < VOTES_BUFS; ++b) { (void)hipEventDestroy(c->ev_copied[b]); (void)hipEventDestroy(c->ev_consumed[b]); }
    (void)hipEventDestroy(c->ev_comb);
    (void)hipStreamDestroy(c->cstream);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return rc;
  }
  *out = c;
  return PBFT_OK;
}

int pbft_verify_ctx_destroy(pbft_ctx* c) {
  if (!c) return PBFT_OK;
  // teardown: errors are ignored (nothing useful to report from a destructor)
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  release_base_table(c->device);
  c->adopt(nullptr);
  (void)hipFree(c->d_stage); (void)hipFree(c->d_bitmap); (void)hipFree(c->d_work); (void)hipFree(c->d_wk);
  if (c->h_bitmap) (void)hipHostFree(c->h_bitmap);
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev_done) (void)hipEventDestroy(c->ev_done);
  for (int b = 0; b < 2; ++b) {
    if (c->fin_pending[b]) (void)hipEventSynchronize(c->ev_fin[b]);
    if (c->ev_fin[b]) (void)hipEventDestroy(c->ev_fin[b]);
  }
  for (int b = 0; b < VOTES_BUFS; ++b) {
    if (c->ev_copied[b]) (void)hipEventDestroy(c->ev_copied[b]);
    if (c->ev_consumed[b]) (void)hipEventDestroy(c->ev_consumed[b]);
  }
  if (c->stream2) { (void)hipStreamSynchronize(c->stream2); (void)hipStreamDestroy(c->stream2); }
  if (c->ev_env) (void)hipEventDestroy(c->ev_env);
  if (c->ev_s2) (void)hipEventDestroy(c->ev_s2);
  (void)hipFree(c->d_work2);
  if (c->ev_comb) (void)hipEventDestroy(c->ev_comb);
  for (hipEvent_t e : c->ev_rows) (void)hipEventDestroy(e);
  if (c->ev_envp) (void)hipEventDestroy(c->ev_envp);
  if (c->cstream) { (void)hipStreamSynchronize(c->cstream); (void)hipStreamDestroy(c->cstream); }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return PBFT_OK;
}

static double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// Install a key set.  Where the time of a re-key went: hipMalloc itself is ~0.3 ms even for
// 172 GB, but VRAM that was written and then freed is wiped by the driver (~22 GB/s, tools/microbench/alloc_h2d:
// re-allocating 202 GB right after freeing it took 9.3 s) and the next allocation waits for that -- a plan change
// that freed 69 GB of tables paid 6.2 s in hipMalloc, the table build itself ~0.25 s.  So a key set whose tables
// fit the current allocation (same plan and at most as many keys, or a smaller plan) is rebuilt IN PLACE -- no
// hipFree, no hipMalloc -- when this context alone holds it; pbft_verify_key_stats reports the phases of the
// last call.
int pbft_verify_set_keys(pbft_ctx* c, const uint8_t* A, uint32_t n, uint8_t* key_ok) {
  if (!c || (!A && n)) return set_err(PBFT_EINVAL, "null argument");
  if (n == 0 || n > 65535) return set_err(PBFT_EINVAL, "key count must be 1..65535");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  const auto t_all = std::chrono::steady_clock::now();
  pbft_key_stats ks{};
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  // this context's key set, if no clone shares it: its tables may be overwritten in place
  keyset* own = (c->ks && c->ks->refs.load() == 1) ? c->ks : nullptr;
  const size_t own_bytes = own ? own->tab_bytes : 0;
  // The widest key plan whose tables fit the budget (PBFT_OPT_KEY_TABLE_BUDGET_MB / env, default 70 % of the HBM
  // free once the old key set is gone: ~180 GB on a 288-GB MI355X after the 30-GB base-point table) and the free
  // memory.  Entry indices are 32-bit (n * entries per key < 2^32).
  auto t = std::chrono::steady_clock::now();
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  ks.meminfo_ms = ms_since(t);
  const size_t avail = free_b + own_bytes;  // (a key set shared with clones stays allocated for them)
  size_t budget_mb = avail / 1048576 * 7 / 10;
  if (const char* e = getenv("PBFT_KEY_TABLE_BUDGET_MB")) budget_mb = strtoull(e, nullptr, 10);
  if (c->key_budget_mb) budget_mb = c->key_budget_mb;
  auto fits = [&](size_t table_words, uint64_t entries_per_key) {
    const size_t bytes = table_words * 4 * (size_t)n;
    return (uint64_t)n * entries_per_key < (1ull << 32) && bytes <= budget_mb * (size_t)1048576 &&
           bytes + ((size_t)4 << 30) < avail;
  };
  int pa = PLA_SMALL::P;
  if (fits(PLA_HUGE::TABLE_WORDS, PLA_HUGE::ENTRIES)) pa = PLA_HUGE::P;
  else if (fits(PLA_BIG::TABLE_WORDS, PLA_BIG::ENTRIES)) pa = PLA_BIG::P;
  else if (fits(PLA_MID::TABLE_WORDS, PLA_MID::ENTRIES)) pa = PLA_MID::P;
  const size_t tab_words = plan_table_words(pa);
  keyset* k = nullptr;
  if (own && n <= own->cap && tab_words * 4 * (size_t)n <= own->tab_bytes) {
    // the tables fit the allocation: rebuild in place.  Launches on callers' streams (device forms) may still
    // read the old tables.
    k = own;
    k->pa = pa;
    ks.reused = 1;
    HIP_TRY(hipDeviceSynchronize());
  } else {
    t = std::chrono::steady_clock::now();
    c->adopt(nullptr);  // (hipFree of an own key set: the slow part of a plan change)
    ks.free_ms = ms_since(t);
    t = std::chrono::steady_clock::now();
    k = new keyset();
    k->pa = pa;
    k->cap = n;
    k->tab_bytes = tab_words * 4 * (size_t)n;
    if (hipMalloc(&k->d_tabA, k->tab_bytes) != hipSuccess ||
        hipMalloc(&k->d_keys, 32 * (size_t)n) != hipSuccess || hipMalloc(&k->d_key_ok, n) != hipSuccess) {
      (void)hipGetLastError();
      keyset_release(k);
      c->kstats = ks;
      return set_err(PBFT_ENOMEM, "key table alloc");
    }
    ks.alloc_ms = ms_since(t);
  }
  k->n = n;
  t = std::chrono::steady_clock::now();
  int rc = PBFT_OK;
  if (hipMemcpyAsync(k->d_keys, A, 32 * (size_t)n, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    rc = set_err(PBFT_EHIP, "key upload");
  if (!rc)
    rc = build_comb_tables(pa, k->d_keys, n, 1, k->d_tabA, k->d_key_ok, c->stream) == hipSuccess
             ? PBFT_OK
             : set_err(PBFT_EHIP, "key table build");
  if (!rc && key_ok && hipMemcpyAsync(key_ok, k->d_key_ok, n, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
    rc = set_err(PBFT_EHIP, "key_ok download");
  if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = set_err(PBFT_EHIP, "key table build");
  ks.build_ms = ms_since(t);
  ks.keys_built = n;
  if (rc) {
    if (k == c->ks) c->adopt(nullptr);  // half-rebuilt tables: no key set rather than a wrong one
    else keyset_release(k);
    c->kstats = ks;
    return rc;
  }
  if (k != c->ks) c->adopt(k);
  else c->n_keys = k->n, c->pa = k->pa;  // rebuilt in place: same buffers, new count (and maybe plan)
  ks.table_bytes = k->tab_bytes;
  ks.total_ms = ms_since(t_all);
  c->kstats = ks;
  return PBFT_OK;
}

// Replace m keys of the installed set in place (the reference admits peers one at a time,
// src/behavior.rs:45-61 add_peer via src/network_behaviour_composer.rs:24-33): only their tables are rebuilt.
// The key set is shared by every clone of this context, so is the update.  Failure handling: a failure
// before any table is written (scratch allocation, key upload) changes nothing; one after the build kernels were
// launched clears key_ok of the updated slots in the SHARED key set -- every context that holds it then rejects
// those keys (their tables may be half-written) instead of verifying against them, the other keys keep working.
__global__ void clear_key_ok_kernel(uint8_t* key_ok, const uint32_t* slots, uint32_t m) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) key_ok[slots[i]] = 0;
}
int pbft_verify_update_keys(pbft_ctx* c, const uint32_t* idx, const uint8_t* A, uint32_t m, uint8_t* key_ok) {
  if (!c || (m && (!idx || !A))) return set_err(PBFT_EINVAL, "null argument");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (!c->ks) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  std::vector<uint32_t> sorted(idx, idx + m);
  std::sort(sorted.begin(), sorted.end());
  for (uint32_t i = 0; i < m; ++i)
    if (sorted[i] >= c->n_keys || (i && sorted[i] == sorted[i - 1]))
      return set_err(PBFT_EINVAL, "key index out of range or repeated");
  const auto t_all = std::chrono::steady_clock::now();
  pbft_key_stats ks{};
  ks.reused = 1;
  if (m == 0) { c->kstats = ks; return PBFT_OK; }
  const int inject = c->fault_inject;
  c->fault_inject = 0;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());  // no launch (this context's, a clone's, a device form's) reads the old tables
  keyset* k = c->ks;
  uint8_t* d_tmp = nullptr;  // [m] slots (u32) then [m][32] encodings
  const size_t off_enc = ((size_t)4 * m + 255) & ~(size_t)255;
  if (inject == 1 || hipMalloc(&d_tmp, off_enc + 32 * (size_t)m) != hipSuccess) {
    (void)hipGetLastError();
    return set_err(PBFT_ENOMEM, "update staging alloc");  // nothing written: the key set is unchanged
  }
  int rc = PBFT_OK, wrote = 0;
  if (hipMemcpyAsync(d_tmp, idx, 4 * (size_t)m, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipMemcpyAsync(d_tmp + off_enc, A, 32 * (size_t)m, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    rc = set_err(PBFT_EHIP, "key upload");
  if (!rc && build_comb_tables(k->pa, (const uint32_t*)(d_tmp + off_enc), m, 1, k->d_tabA, k->d_key_ok, c->stream,
                               (const uint32_t*)d_tmp, k->d_keys, &wrote) != hipSuccess)
    rc = set_err(PBFT_EHIP, wrote ? "key table build" : "key table build scratch alloc");
  if (!rc && inject == 2) rc = set_err(PBFT_EHIP, "key table build (injected fault)");
  std::vector<uint8_t> ok_all;
  if (!rc && key_ok) {
    ok_all.resize(k->n);
    if (hipMemcpyAsync(ok_all.data(), k->d_key_ok, k->n, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
      rc = set_err(PBFT_EHIP, "key_ok download");
  }
  if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = set_err(PBFT_EHIP, "key table build");
  if (rc && (wrote || inject == 2)) {
    // the updated slots' tables may be half-written: reject them everywhere the key set is used
    const std::string why = g_last_error;
    (void)hipGetLastError();
    hipLaunchKernelGGL(clear_key_ok_kernel, dim3((m + 255) / 256), dim3(256), 0, c->stream, k->d_key_ok,
                       (const uint32_t*)d_tmp, m);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess)
      c->adopt(nullptr);  // could not even mark them: drop the key set from this context rather than trust it
    g_last_error = why;
  }
  (void)hipStreamSynchronize(c->stream);
  (void)hipFree(d_tmp);
  if (rc) return rc;
  if (key_ok)
    for (uint32_t i = 0; i < m; ++i) key_ok[i] = ok_all[idx[i]];
  ks.keys_built = m;
  ks.build_ms = ks.total_ms = ms_since(t_all);
  ks.table_bytes = plan_table_words(k->pa) * 4 * (size_t)k->cap;
  c->kstats = ks;
  return PBFT_OK;
}

// Slots idx[0..m) of the context's key set reject every signature from now on (key_ok cleared; the tables stay):
// pbft_replica_update_keys uses it to leave no context of a replica verifying a key its PeerId map does not hold
// after an update failed on one of them.  A later set_keys / update_keys of a slot admits it again.
int pbft_verify_revoke_keys(pbft_ctx* c, const uint32_t* idx, uint32_t m) {
  if (!c || (m && !idx)) return set_err(PBFT_EINVAL, "null argument");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (!c->ks) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  for (uint32_t i = 0; i < m; ++i)
    if (idx[i] >= c->n_keys) return set_err(PBFT_EINVAL, "key index out of range");
  if (m == 0) return PBFT_OK;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());  // (no launch of a clone is reading key_ok while it changes)
  uint32_t* d_idx = nullptr;
  HIP_TRY(hipMalloc(&d_idx, 4 * (size_t)m));
  int rc = PBFT_OK;
  if (hipMemcpyAsync(d_idx, idx, 4 * (size_t)m, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    rc = set_err(PBFT_EHIP, "revoke upload");
  if (!rc) {
    hipLaunchKernelGGL(clear_key_ok_kernel, dim3((m + 255) / 256), dim3(256), 0, c->stream, c->ks->d_key_ok,
                       (const uint32_t*)d_idx, m);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess)
      rc = set_err(PBFT_EHIP, "revoke kernel");
  }
  (void)hipStreamSynchronize(c->stream);
  (void)hipFree(d_idx);
  return rc;
}

// An identity of the key set the context verifies against (shared by its clones: pbft_verify_ctx_clone); 0 = none.
int pbft_verify_key_set_id(pbft_ctx* c, uint64_t* id) {
  if (!c || !id) return set_err(PBFT_EINVAL, "null argument");
  *id = (uint64_t)(uintptr_t)c->ks;
  return PBFT_OK;
}

int pbft_verify_key_stats(pbft_ctx* c, pbft_key_stats* out) {
  if (!c || !out) return set_err(PBFT_EINVAL, "null argument");
  *out = c->kstats;
  return PBFT_OK;
}

int pbft_verify_ctx_clone(pbft_ctx* parent, pbft_ctx** out) {
  if (!parent || !out) return set_err(PBFT_EINVAL, "null argument");
  *out = nullptr;
  pbft_ctx* c = nullptr;
  int rc = pbft_verify_ctx_create(parent->device, &c);
  if (rc) return rc;
  if (parent->ks) {
    ++parent->ks->refs;
    c->adopt(parent->ks);
  }
  // the parent's tuning options (pbft_verify_set_option)
  c->split_below = parent->split_below;
  c->fin_m = parent->fin_m;
  c->fin_tree = parent->fin_tree;
  c->fin_waves = parent->fin_waves;
  c->lat_split = parent->lat_split;
  c->timing = parent->timing;
  c->two_streams = parent->two_streams;
  c->comb_pair = parent->comb_pair;
  c->comb_prio = parent->comb_prio;
  c->key_budget_mb = parent->key_budget_mb;
  *out = c;
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
  bool pinned = false;
  LT("pinned_query", pinned = host_pinned(R) && host_pinned(S) && host_pinned(K) && host_pinned(M));
  if (!pinned) {
    // pageable: copy into the pinned staging first, so the DMA below is asynchronous (a pageable
    // hipMemcpyAsync stages through the runtime's buffers and returns only when the copy is done)
    const host_batch_layout L(N, msg_stride);
    int rc = ensure_host_stage(c, L.bytes);
    if (rc) return rc;
    uint8_t* h = c->h_stage;
    memcpy(h, R, 32 * N);
    memcpy(h + L.offS, S, 32 * N);
    memcpy(h + L.offK, K, 2 * N);
    if (M && msg_stride) memcpy(h + L.offM, M, (size_t)msg_stride * N);
    R = h; S = h + L.offS; K = (const uint16_t*)(h + L.offK); M = M ? h + L.offM : M;
  }
  int rc = stage_and_launch(c, R, S, K, M, msg_len, msg_stride, N);
  if (rc) return rc;
  const uint64_t words = (N + 63) / 64;
  LT("export_bitmap", HIP_TRY(export_words(c, 0, words, c->stream)));
  LT("rec_done", HIP_TRY(hipEventRecord(c->ev_done, c->stream)));
  c->in_flight = true;
  c->v_readback = false;
  c->async_out = out;
  c->async_words = words;
  return PBFT_OK;
}

// Wait for an event by polling hipEventQuery instead of hipEventSynchronize.  VERDICT r04 item 2: with the H2D
// copies of a 4k host batch replaced by the import kernel, the back-to-back leg's stall moved into
// hipEventSynchronize (10.8 ms once in 5 one-second reps, profiles/r05/stall_probe.txt): the runtime's blocking
// wait (spin briefly, then sleep on the completion interrupt) sometimes wakes milliseconds late.  A serving
// thread that waits for its batch is latency-critical, so it polls (yielding the core between polls) -- the same
// thing the replica's flush_poll and the bench's poll loops do.  PBFT_SPIN_WAIT=0 restores hipEventSynchronize.
// The core is yielded only once a wait has lasted 2 ms: a sched_yield that lets another runnable thread in gives the
// core back a scheduler tick later, and the back-to-back leg's 1.05-ms maxima were exactly that (interleaved
// processes on one box, profiles/r05/stream_spin.txt: yielding every 64 polls, max 0.37-1.05 ms; never, 0.21-0.53).
// PBFT_SPIN_WAIT=2: never yield; =3: yield every 64 polls (the first r05 form).
static hipError_t wait_event(hipEvent_t e) {
  static const long spin = [] {
    const char* v = getenv("PBFT_SPIN_WAIT");
    return v ? strtol(v, nullptr, 10) : 1L;
  }();
  if (!spin) return hipEventSynchronize(e);
  const auto t0 = std::chrono::steady_clock::now();
  bool polite = spin == 3;
  for (uint32_t k = 0;; ++k) {
    const hipError_t q = hipEventQuery(e);
    if (q != hipErrorNotReady) return q;
    if ((k & 63) == 63) {
      if (!polite && spin == 1 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) polite = true;
      if (polite) sched_yield();
    }
  }
}

static int finish_async(pbft_ctx* c) {
  memcpy(c->async_out, c->h_bitmap, c->async_words * 8);
  c->in_flight = false;
  c->rows_out = c->async_words * 64;
  // (only with timing events: on events never recorded the call fails and would leave an error that the next
  // launch's hipGetLastError reports; a failure here is cleared for the same reason)
  if (c->timing && hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1) != hipSuccess) (void)hipGetLastError();
  return PBFT_OK;
}

int pbft_verify_poll(pbft_ctx* c) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!c->in_flight) return 1;
  if (c->v_open) return 0;  // progressive batch: not every chunk launched yet
  hipError_t e;
  LT("poll_query", e = hipEventQuery(c->ev_done));
  if (e == hipErrorNotReady) return 0;
  if (e != hipSuccess) {
    c->in_flight = false;  // the batch is lost; the context stays usable for the next submit
    HIP_TRY(e);
  }
  finish_async(c);
  return 1;
}

int pbft_verify_wait(pbft_ctx* c) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!c->in_flight) return PBFT_OK;
  if (c->v_open) return set_err(PBFT_EBUSY, "progressive votes batch not fully submitted");
  hipError_t e;
  LT("wait_sync", e = wait_event(c->ev_done));
  if (e != hipSuccess) {
    c->in_flight = false;
    HIP_TRY(e);
  }
  return finish_async(c);
}

// ---- votes form, non-blocking (include/pbft_verify.h) ----
static int votes_submit_from(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint32_t* I,
                             const uint8_t* E, uint32_t n_env, uint64_t N, uint64_t* out, uint32_t rs_stride = 32) {
  int rc = stage_votes_and_launch(c, R, S, K, I, E, n_env, N, rs_stride);
  if (rc) return rc;
  const uint64_t words = (N + 63) / 64;
  HIP_TRY(export_words(c, 0, words, c->stream));
  HIP_TRY(hipEventRecord(c->ev_done, c->stream));
  c->in_flight = true;
  c->v_readback = false;
  c->async_out = out;
  c->async_words = words;
  return PBFT_OK;
}

int pbft_verify_votes_stage(pbft_ctx* c, uint64_t N, uint32_t n_env, pbft_votes_staging* out) {
  if (!c || !out) return set_err(PBFT_EINVAL, "null argument");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (N && n_env == 0) return set_err(PBFT_EINVAL, "votes batch without envelopes");
  HIP_TRY(hipSetDevice(c->device));
  const host_votes_layout L(N, n_env);
  int rc = ensure_host_stage(c, L.bytes);
  if (rc) return rc;
  uint8_t* h = c->h_stage;
  out->sig = h;
  out->key_idx = (uint16_t*)(h + PBFT_VOTES_ROW_KEY);
  out->env_idx = (uint32_t*)(h + PBFT_VOTES_ROW_ENV);
  out->envelopes = h + L.offE;
  out->row_stride = ROW;
  c->staged = true;
  c->staged_n = N;
  c->staged_env = n_env;
  return PBFT_OK;
}

int pbft_verify_votes_submit(pbft_ctx* c, uint64_t N, uint32_t n_env, uint64_t* out) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (!c->staged || N != c->staged_n || n_env != c->staged_env)
    return set_err(PBFT_EINVAL, "pbft_verify_votes_stage was not called for this batch");
  if (N && !out) return set_err(PBFT_EINVAL, "null bitmap");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  c->staged = false;
  if (N == 0) return PBFT_OK;
  HIP_TRY(hipSetDevice(c->device));
  const host_votes_layout L(N, n_env);
  uint8_t* h = c->h_stage;
  return votes_submit_from(c, h, h + 32, (const uint16_t*)(h + PBFT_VOTES_ROW_KEY),
                           (const uint32_t*)(h + PBFT_VOTES_ROW_ENV), h + L.offE, n_env, N, out, ROW);
}

// Progressive form: the caller fills the staging front to back and launches as it goes.
int pbft_verify_votes_submit_begin(pbft_ctx* c, uint64_t N, uint32_t n_env, uint64_t* out) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (!c->staged || N != c->staged_n || n_env != c->staged_env)
    return set_err(PBFT_EINVAL, "pbft_verify_votes_stage was not called for this batch");
  if (N == 0 || !out) return set_err(PBFT_EINVAL, "empty batch or null bitmap");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  c->staged = false;
  HIP_TRY(hipSetDevice(c->device));
  const host_votes_layout L(N, n_env);
  int rc = votes_begin(c, c->h_stage + L.offE, n_env, N, true);
  if (rc) return rc;
  c->in_flight = true;  // (pbft_verify_poll reports "running" until every chunk is launched and done)
  c->async_out = out;
  c->async_words = (N + 63) / 64;
  return PBFT_OK;
}

int pbft_verify_votes_submit_rows(pbft_ctx* c, uint64_t rows) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!c->in_flight || !c->v_open) return set_err(PBFT_EINVAL, "no progressive votes batch open");
  HIP_TRY(hipSetDevice(c->device));
  uint8_t* h = c->h_stage;
  int rc = votes_launch(c, h, h + 32, (const uint16_t*)(h + PBFT_VOTES_ROW_KEY), (const uint32_t*)(h + PBFT_VOTES_ROW_ENV),
                        ROW, rows);
  if (rc == PBFT_OK && !c->v_open)
    rc = hipEventRecord(c->ev_done, c->stream) == hipSuccess ? PBFT_OK : set_err(PBFT_EHIP, "event record");
  if (rc) {  // the batch is lost: drain what was launched, the context stays usable
    (void)hipStreamSynchronize(c->stream);
    if (c->stream2) (void)hipStreamSynchronize(c->stream2);
    (void)hipStreamSynchronize(c->cstream);
    c->in_flight = false;
    c->v_open = false;
  }
  return rc;
}

int pbft_verify_votes_submit_host(pbft_ctx* c, const uint8_t* rows, uint64_t N, const uint8_t* env, uint32_t n_env,
                                  uint64_t* out) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (N == 0 || !rows || !env || n_env == 0 || !out) return set_err(PBFT_EINVAL, "empty batch or null argument");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  c->staged = false;  // (as every host-buffer submit: a pending stage is void)
  HIP_TRY(hipSetDevice(c->device));
  int rc = votes_begin(c, env, n_env, N, true, true);
  if (rc) return rc;
  c->in_flight = true;
  c->async_out = out;
  c->async_words = (N + 63) / 64;
  rc = votes_launch(c, rows, rows + 32, (const uint16_t*)(rows + PBFT_VOTES_ROW_KEY),
                    (const uint32_t*)(rows + PBFT_VOTES_ROW_ENV), ROW, N);
  if (rc == PBFT_OK)
    rc = hipEventRecord(c->ev_done, c->stream) == hipSuccess ? PBFT_OK : set_err(PBFT_EHIP, "event record");
  if (rc) {  // the batch is lost: drain what was launched, the context stays usable
    (void)hipStreamSynchronize(c->stream);
    if (c->stream2) (void)hipStreamSynchronize(c->stream2);
    (void)hipStreamSynchronize(c->cstream);
    c->in_flight = false;
    c->v_open = false;
  }
  return rc;
}

// Anonymous pages pinned with hipHostRegister rather than hipHostMalloc: on the MI355X boxes the copy engine reads
// them at 56.5 GB/s wherever they are placed, while hipHostMalloc buffers after a process's first one read at 46-50
// GB/s (tools/microbench/pinned_write.cpp, numa_h2d.cpp; profiles/r05/pinned_h2d.txt).  One header page in front
// holds the mapping's length for pbft_host_free.
static constexpr size_t HOST_HDR = 4096;
// ---- votes batch in pieces (pbft_verify_votes_open / _piece / _close): the caller's rows and envelopes are
// written while earlier pieces are already being copied and verified (pbft_replica_push_many: r05) ----
int pbft_verify_votes_open(pbft_ctx* c, uint64_t n_cap, uint32_t env_cap, uint64_t* out) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (n_cap == 0 || env_cap == 0 || !out) return set_err(PBFT_EINVAL, "empty batch or null bitmap");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  c->staged = false;
  HIP_TRY(hipSetDevice(c->device));
  const uint64_t words = (n_cap + 63) / 64;
  const size_t env_bytes = ((size_t)PBFT_ENVELOPE_LEN * env_cap + 64 + 255) & ~(size_t)255;
  const votes_layout L(n_cap < VOTES_CHUNK ? n_cap : VOTES_CHUNK);
  int rc = ensure_stage(c, env_bytes + VOTES_BUFS * L.bytes, words);
  if (rc) return rc;
  rc = ensure_wk(c, env_cap);
  if (rc) return rc;
  const bool two = c->two_streams;
  if (two && !c->stream2) {
    HIP_TRY(hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_env, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_s2, hipEventDisableTiming));
  }
  if (!c->ev_envp) HIP_TRY(hipEventCreateWithFlags(&c->ev_envp, hipEventDisableTiming));
  c->v_short_tail = false;
  c->v_ends.clear();
  c->v_s2_ready = true;  // (stream2 waits for every piece's envelopes itself: votes_piece)
  c->v_two = two;
  c->v_n = n_cap;
  c->v_next = 0;
  c->v_chunk = 0;
  c->v_env_bytes = env_bytes;
  c->v_env = 0;
  c->v_env_cap = env_cap;
  c->v_wk = c->d_wk;
  c->v_open = true;
  c->v_readback = true;
  c->rows_out = 0;
  c->chunk_out = 0;
  c->in_flight = true;
  c->async_out = out;
  c->async_words = words;
  return PBFT_OK;
}

static int votes_drop(pbft_ctx* c, int rc) {  // a failed piece: drain what was launched, the batch is lost
  (void)hipStreamSynchronize(c->stream);
  if (c->stream2) (void)hipStreamSynchronize(c->stream2);
  (void)hipStreamSynchronize(c->cstream);
  c->in_flight = false;
  c->v_open = false;
  c->v_env_cap = 0;
  return rc;
}

int pbft_verify_votes_piece(pbft_ctx* c, const uint8_t* rows, uint64_t row_lo, uint64_t row_hi, const uint8_t* envs,
                            uint32_t env_lo, uint32_t env_hi) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!c->in_flight || !c->v_open || c->v_env_cap == 0) return set_err(PBFT_EINVAL, "no votes batch open in pieces");
  if (!rows || row_lo != c->v_next || row_hi < row_lo || row_hi > c->v_n || (row_lo & 63) ||
      env_lo != c->v_env || env_hi < env_lo || env_hi > c->v_env_cap || (env_hi > env_lo && !envs))
    return set_err(PBFT_EINVAL, "piece out of order or out of the opened bounds");
  HIP_TRY(hipSetDevice(c->device));
  if (env_hi > env_lo) {  // the piece's new envelopes and their block-2 schedules, ahead of its rows' kernels
    const uint32_t ne = env_hi - env_lo;
    if (hipMemcpyAsync(c->d_stage + (size_t)PBFT_ENVELOPE_LEN * env_lo, envs + (size_t)PBFT_ENVELOPE_LEN * env_lo,
                       (size_t)PBFT_ENVELOPE_LEN * ne, hipMemcpyHostToDevice, c->cstream) != hipSuccess ||
        hipEventRecord(c->ev_envp, c->cstream) != hipSuccess || hipStreamWaitEvent(c->stream, c->ev_envp, 0) != hipSuccess)
      return votes_drop(c, set_err(PBFT_EHIP, "piece envelopes"));
    hipLaunchKernelGGL(env_sched_kernel, dim3((ne + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, c->stream,
                       c->d_stage + (size_t)PBFT_ENVELOPE_LEN * env_lo, ne, c->d_wk + (size_t)SHA_ENV_WORDS * env_lo);
    if (hipGetLastError() != hipSuccess) return votes_drop(c, set_err(PBFT_EHIP, "piece envelope schedule"));
    if (c->v_two && (hipEventRecord(c->ev_env, c->stream) != hipSuccess ||
                     hipStreamWaitEvent(c->stream2, c->ev_env, 0) != hipSuccess))
      return votes_drop(c, set_err(PBFT_EHIP, "piece envelope event"));
    c->v_env = env_hi;
  }
  for (uint64_t lo = row_lo; lo < row_hi;) {
    const uint64_t n = row_hi - lo > VOTES_CHUNK ? VOTES_CHUNK : row_hi - lo;
    const int rc = votes_chunk(c, rows, rows + 32, (const uint16_t*)(rows + PBFT_VOTES_ROW_KEY),
                               (const uint32_t*)(rows + PBFT_VOTES_ROW_ENV), ROW, lo, n);
    if (rc) return votes_drop(c, rc);
    lo += n;
  }
  return PBFT_OK;
}

int pbft_verify_votes_close(pbft_ctx* c, uint64_t n) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!c->in_flight || !c->v_open || c->v_env_cap == 0) return set_err(PBFT_EINVAL, "no votes batch open in pieces");
  if (n != c->v_next || n == 0) return votes_drop(c, set_err(PBFT_EINVAL, "close: rows submitted differ"));
  HIP_TRY(hipSetDevice(c->device));
  c->v_open = false;
  c->v_env_cap = 0;
  c->v_n = n;
  c->async_words = (n + 63) / 64;
  int rc = votes_join_streams(c);
  if (rc == PBFT_OK && hipEventRecord(c->ev_done, c->stream) != hipSuccess) rc = set_err(PBFT_EHIP, "event record");
  return rc ? votes_drop(c, rc) : PBFT_OK;
}

int pbft_host_alloc(pbft_ctx* c, size_t bytes, void** out) {
  if (!out) return set_err(PBFT_EINVAL, "null argument");
  *out = nullptr;
  if (!c || bytes == 0) return set_err(PBFT_EINVAL, "null context or empty allocation");
  HIP_TRY(hipSetDevice(c->device));
  const size_t len = HOST_HDR + ((bytes + 4095) & ~(size_t)4095);
  void* m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (m == MAP_FAILED) return set_err(PBFT_ENOMEM, "host mmap");
  memcpy(m, &len, sizeof len);
  uint8_t* p = (uint8_t*)m + HOST_HDR;
  if (hipHostRegister(p, len - HOST_HDR, hipHostRegisterPortable) != hipSuccess) {
    (void)hipGetLastError();
    munmap(m, len);
    return set_err(PBFT_ENOMEM, "pinned host register");
  }
  *out = p;
  return PBFT_OK;
}

int pbft_host_free(pbft_ctx* c, void* p) {
  if (!p) return PBFT_OK;
  if (c) HIP_TRY(hipSetDevice(c->device));
  uint8_t* m = (uint8_t*)p - HOST_HDR;
  size_t len;
  memcpy(&len, m, sizeof len);
  HIP_TRY(hipHostUnregister(p));
  munmap(m, len);
  return PBFT_OK;
}

int pbft_verify_poll_rows(pbft_ctx* c, uint64_t* rows_done) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight && c->v_readback) {
    while (c->rows_out < c->v_next) {  // launched chunks whose bitmap words have landed, in order
      const hipError_t e = hipEventQuery(c->ev_rows[c->chunk_out]);
      if (e == hipErrorNotReady) break;
      if (e != hipSuccess) {
        c->in_flight = false;
        c->v_open = false;
        HIP_TRY(e);
      }
      const uint64_t hi = c->v_ends[c->chunk_out];
      memcpy(c->async_out + c->rows_out / 64, c->h_bitmap + c->rows_out / 64, (hi - c->rows_out + 63) / 64 * 8);
      c->rows_out = hi;
      ++c->chunk_out;
    }
    if (c->v_open || c->rows_out < c->v_n) {
      if (rows_done) *rows_done = c->rows_out;
      return 0;
    }
  }
  const bool progressive = c->in_flight && c->v_readback;
  const int st = pbft_verify_poll(c);
  if (rows_done) *rows_done = st == 1 ? c->rows_out : progressive ? c->rows_out : 0;
  return st;
}

int pbft_verify_votes_async(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint32_t* I,
                            const uint8_t* E, uint32_t n_env, uint64_t N, uint64_t* out) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (N && (!R || !S || !K || !I || !out || !E || n_env == 0)) return set_err(PBFT_EINVAL, "bad votes arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  if (N == 0) return PBFT_OK;
  HIP_TRY(hipSetDevice(c->device));
  if (host_pinned(R) && host_pinned(S) && host_pinned(K) && host_pinned(I) && host_pinned(E))
    return votes_submit_from(c, R, S, K, I, E, n_env, N, out);
  pbft_votes_staging st;
  int rc = pbft_verify_votes_stage(c, N, n_env, &st);
  if (rc) return rc;
  for (uint64_t i = 0; i < N; ++i) {
    uint8_t* row = st.sig + (size_t)ROW * i;
    memcpy(row, R + 32 * i, 32);
    memcpy(row + 32, S + 32 * i, 32);
    const uint32_t kp = K[i];  // key_idx, two zero bytes
    memcpy(row + PBFT_VOTES_ROW_KEY, &kp, 4);
    memcpy(row + PBFT_VOTES_ROW_ENV, I + i, 4);
  }
  memcpy(st.envelopes, E, (size_t)PBFT_ENVELOPE_LEN * n_env);
  return pbft_verify_votes_submit(c, N, n_env, out);
}

// One host batch over several contexts (GPUs of this process, or cloned contexts
// of one GPU): contiguous 64-aligned shards, one async launch per context, each
// writing its own bitmap words in place (no exchange needed when
// the bitmaps return to one host process).
int pbft_verify_batch_multi(pbft_ctx* const* ctxs, uint32_t n_ctx, const uint8_t* R, const uint8_t* S,
                            const uint16_t* K, const uint8_t* M, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                            uint64_t* out) {
  if (!ctxs || n_ctx == 0) return set_err(PBFT_EINVAL, "no contexts");
  for (uint32_t i = 0; i < n_ctx; ++i)
    for (uint32_t j = 0; j < i; ++j)
      if (!ctxs[i] || ctxs[i] == ctxs[j]) return set_err(PBFT_EINVAL, "contexts must be distinct and non-null");
  if (!check_batch_args(R, S, K, M, msg_len, msg_stride, N, out)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (N == 0) return PBFT_OK;
  const uint64_t words = (N + 63) / 64, per = (words + n_ctx - 1) / n_ctx;
  int rc = PBFT_OK;
  uint32_t launched = 0;
  for (; launched < n_ctx; ++launched) {
    const uint64_t lo = launched * per * 64;
    if (lo >= N) break;
    const uint64_t hi = lo + per * 64 < N ? lo + per * 64 : N;
    rc = pbft_verify_batch_async(ctxs[launched], R + 32 * lo, S + 32 * lo, K + lo, M ? M + (size_t)msg_stride * lo : M,
                                 msg_len, msg_stride, hi - lo, out + lo / 64);
    if (rc) break;
  }
  for (uint32_t i = 0; i < launched; ++i) {
    const int w = pbft_verify_wait(ctxs[i]);
    if (!rc) rc = w;
  }
  return rc;
}

}  // extern "C"

// ---- single-process multi-GPU round, bitmap all-gather on RCCL (include/pbft_verify.h) ----
// RCCL is resolved at run time (dlopen), so the verifier loads on hosts and in processes without it; in a
// process that already loaded torch's bundled librccl.so.1 the same object is reused (SONAME match).
namespace {
struct rccl_api {
  bool ok = false;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
};
rccl_api* rccl() {
  static rccl_api api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    api.CommInitAll = (decltype(api.CommInitAll))dlsym(h, "ncclCommInitAll");
    api.CommDestroy = (decltype(api.CommDestroy))dlsym(h, "ncclCommDestroy");
    api.AllGather = (decltype(api.AllGather))dlsym(h, "ncclAllGather");
    api.GroupStart = (decltype(api.GroupStart))dlsym(h, "ncclGroupStart");
    api.GroupEnd = (decltype(api.GroupEnd))dlsym(h, "ncclGroupEnd");
    api.GetErrorString = (decltype(api.GetErrorString))dlsym(h, "ncclGetErrorString");
    api.ok = api.CommInitAll && api.CommDestroy && api.AllGather && api.GroupStart && api.GroupEnd &&
             api.GetErrorString;
  });
  return api.ok ? &api : nullptr;
}
int rccl_err(ncclResult_t r, const char* what) {
  char b[256];
  snprintf(b, sizeof b, "%s: %s", what, rccl() ? rccl()->GetErrorString(r) : "RCCL unavailable");
  return set_err(PBFT_EHIP, b);
}
}  // namespace

struct pbft_multi {
  std::vector<pbft_ctx*> ctx;
  std::vector<ncclComm_t> comm;
};

extern "C" {

int pbft_multi_create(pbft_ctx* const* ctxs, uint32_t n_ctx, pbft_multi** out) {
  if (!ctxs || !out || n_ctx == 0) return set_err(PBFT_EINVAL, "no contexts");
  *out = nullptr;
  std::vector<int> devs(n_ctx);
  for (uint32_t i = 0; i < n_ctx; ++i) {
    if (!ctxs[i]) return set_err(PBFT_EINVAL, "null context");
    devs[i] = ctxs[i]->device;
    for (uint32_t j = 0; j < i; ++j)
      if (devs[j] == devs[i]) return set_err(PBFT_EINVAL, "one context per device (distinct devices)");
  }
  rccl_api* api = rccl();
  if (!api) return set_err(PBFT_ENODEV, "librccl.so.1 not loadable");
  pbft_multi* m = new pbft_multi();
  m->ctx.assign(ctxs, ctxs + n_ctx);
  m->comm.assign(n_ctx, nullptr);
  const ncclResult_t r = api->CommInitAll(m->comm.data(), (int)n_ctx, devs.data());
  if (r != ncclSuccess) {
    delete m;
    return rccl_err(r, "ncclCommInitAll");
  }
  *out = m;
  return PBFT_OK;
}

int pbft_multi_destroy(pbft_multi* m) {
  if (!m) return PBFT_OK;
  (void)pbft_multi_sync(m);
  if (rccl_api* api = rccl())
    for (ncclComm_t c : m->comm)
      if (c) (void)api->CommDestroy(c);
  delete m;
  return PBFT_OK;
}

int pbft_multi_sync(pbft_multi* m) {
  if (!m) return set_err(PBFT_EINVAL, "null multi");
  for (pbft_ctx* c : m->ctx) {
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  return PBFT_OK;
}

int pbft_verify_batch_device_multi(pbft_multi* m, const uint8_t* const* dR, const uint8_t* const* dS,
                                   const uint16_t* const* dK, const uint8_t* const* dM, uint32_t msg_len,
                                   uint32_t msg_stride, const uint64_t* n, uint64_t wpr, uint64_t* const* dB) {
  if (!m || !dR || !dS || !dK || !dM || !n || !dB) return set_err(PBFT_EINVAL, "null argument");
  const uint32_t G = (uint32_t)m->ctx.size();
  for (uint32_t r = 0; r < G; ++r) {
    if ((n[r] + 63) / 64 > wpr) return set_err(PBFT_EINVAL, "words_per_rank < ceil(n[r] / 64)");
    if (!dB[r] || !check_batch_args(dR[r], dS[r], dK[r], dM[r], msg_len, msg_stride, n[r], dB[r]))
      return set_err(PBFT_EINVAL, "bad shard arguments");
    if (m->ctx[r]->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  }
  for (uint32_t r = 0; r < G; ++r) {
    pbft_ctx* c = m->ctx[r];
    HIP_TRY(hipSetDevice(c->device));
    uint64_t* mine = dB[r] + (size_t)r * wpr;
    const uint64_t words = (n[r] + 63) / 64;
    if (wpr > words) HIP_TRY(hipMemsetAsync(mine + words, 0, (wpr - words) * 8, c->stream));
    int rc = launch_verify(c, dR[r], dS[r], dK[r], dM[r], msg_len, msg_stride, n[r], mine, c->stream);
    if (rc) return rc;
  }
  rccl_api* api = rccl();
  ncclResult_t e = api->GroupStart();
  if (e != ncclSuccess) return rccl_err(e, "ncclGroupStart");
  for (uint32_t r = 0; r < G; ++r) {
    pbft_ctx* c = m->ctx[r];
    e = api->AllGather(dB[r] + (size_t)r * wpr, dB[r], wpr, ncclUint64, m->comm[r], c->stream);
    if (e != ncclSuccess) break;
  }
  const ncclResult_t e2 = api->GroupEnd();
  if (e != ncclSuccess) return rccl_err(e, "ncclAllGather");
  if (e2 != ncclSuccess) return rccl_err(e2, "ncclGroupEnd");
  return PBFT_OK;
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

int pbft_verify_batch_device_pipelined(pbft_ctx* c, const uint8_t* dR, const uint8_t* dS, const uint16_t* dK,
                                       const uint8_t* dM, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                                       uint64_t* dB, void* stream, void* finish_stream) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (!stream || !finish_stream || stream == finish_stream)
    return set_err(PBFT_EINVAL, "two distinct non-null streams required");
  if (!check_batch_args(dR, dS, dK, dM, msg_len, msg_stride, N, dB)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  HIP_TRY(hipSetDevice(c->device));
  return launch_verify(c, dR, dS, dK, dM, msg_len, msg_stride, N, dB, (hipStream_t)stream, 32, 2,
                       (hipStream_t)finish_stream);
}

int pbft_verify_votes(pbft_ctx* c, const uint8_t* R, const uint8_t* S, const uint16_t* K, const uint32_t* env_idx,
                      const uint8_t* envelopes, uint32_t n_env, uint64_t N, uint64_t* out) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (N && (!R || !S || !K || !env_idx || !out || !envelopes || n_env == 0))
    return set_err(PBFT_EINVAL, "bad votes arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  if (N == 0) return PBFT_OK;
  int rc = pbft_verify_votes_async(c, R, S, K, env_idx, envelopes, n_env, N, out);
  if (rc) return rc;
  return pbft_verify_wait(c);
}

int pbft_verify_votes_device(pbft_ctx* c, const uint8_t* dR, const uint8_t* dS, const uint16_t* dK,
                             const uint32_t* d_env_idx, const uint8_t* d_envelopes, uint32_t n_env, uint64_t N,
                             uint64_t* dB, void* stream) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (N && (!dR || !dS || !dK || !d_env_idx || !d_envelopes || !dB || n_env == 0))
    return set_err(PBFT_EINVAL, "bad votes arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  if (N == 0) return PBFT_OK;
  const uint64_t* dWK = nullptr;
  int rc = prepare_env_sched(c, d_envelopes, n_env, st, &dWK);
  if (rc) return rc;
  return launch_verify(c, dR, dS, dK, d_envelopes, PBFT_ENVELOPE_LEN, PBFT_ENVELOPE_LEN, N, dB, st, 32, 2, nullptr,
                       d_env_idx, n_env, dWK);
}

// Binary wire records (include/pbft_wire.h): R at +0, S at +32, envelope at +64,
// key index at +150, stride 160 -- read in place by the same kernels.
int pbft_verify_records_device(pbft_ctx* c, const uint8_t* d_rec, uint64_t N, uint64_t* dB, void* stream) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (N && (!d_rec || !dB)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (((uintptr_t)d_rec & 15) != 0) return set_err(PBFT_EINVAL, "records must be 16-byte aligned");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  return launch_verify(c, d_rec, d_rec + 32, (const uint16_t*)(d_rec + 150), d_rec + 64, PBFT_ENVELOPE_LEN,
                       PBFT_RECORD_BYTES, N, dB, st, PBFT_RECORD_BYTES, PBFT_RECORD_BYTES);
}

int pbft_verify_records(pbft_ctx* c, const uint8_t* rec, uint64_t N, uint64_t* out) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (c->in_flight) return set_err(PBFT_EBUSY, "async batch in flight");
  if (N && (!rec || !out)) return set_err(PBFT_EINVAL, "bad batch arguments");
  if (c->n_keys == 0) return set_err(PBFT_ENOKEYS, "pbft_verify_set_keys not called");
  if (N == 0) return PBFT_OK;
  HIP_TRY(hipSetDevice(c->device));
  const uint64_t words = (N + 63) / 64;
  int rc = ensure_stage(c, PBFT_RECORD_BYTES * N + 256, words);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_stage, rec, PBFT_RECORD_BYTES * N, hipMemcpyHostToDevice, c->stream));
  rc = pbft_verify_records_device(c, c->d_stage, N, c->d_bitmap, c->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out, c->d_bitmap, words * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return PBFT_OK;
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
      launch_sign(PBFT_ENVELOPE_LEN, dim3(blocks), dim3(BLOCK), 0, c->stream,
                         (const uint32_t*)c->d_stage, d_idx, c->d_stage + offM, msg_len, msg_stride, n_launch,
                         c->d_tabB, (uint32_t*)(c->d_stage + offR), (uint32_t*)(c->d_stage + offS),
                         pub ? (uint32_t*)(c->d_stage + offP) : nullptr, n_seeds);
    else
      launch_sign(-1, dim3(blocks), dim3(BLOCK), 0, c->stream, (const uint32_t*)c->d_stage,
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
    launch_sign(0, dim3((n_seeds + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, c->stream,
                       (const uint32_t*)c->d_stage, (const uint16_t*)d_i2, (const uint8_t*)nullptr, 0u, 0u,
                       (uint64_t)n_seeds, c->d_tabB, d_r2, d_s2, (uint32_t*)(c->d_stage + offP), n_seeds);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(pub, c->d_stage + offP, 32 * (size_t)n_seeds, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    (void)hipFree(d_i2);
    (void)hipFree(d_r2);
  }
  return PBFT_OK;
}

int pbft_verify_reserve(pbft_ctx* c, uint64_t max_n) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  HIP_TRY(hipSetDevice(c->device));
  return ensure_work(c, max_n, true);  // both halves: either device form can then be captured
}

int pbft_verify_set_option(pbft_ctx* c, int option, uint64_t value) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  switch (option) {
    case PBFT_OPT_SPLIT_BELOW: c->split_below = value; return PBFT_OK;
    case PBFT_OPT_FINISH_WIDTH:
      if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8 && value != 16)
        return set_err(PBFT_EINVAL, "finish width");
      c->fin_m = (int)value;
      return PBFT_OK;
    case PBFT_OPT_FINISH_TREE:
      // the one compiled tree depth (PBFT_FIN_LV) or none; the other depth is a build-time A/B (-DPBFT_FIN_LV)
      if ((value == 4 || value == 6) && value != PBFT_FIN_LV) return set_err(PBFT_EINVAL, "finish tree depth not compiled");
      c->fin_tree = (value == 0 || value == PBFT_FIN_LV) ? (int)value : -1;
      return PBFT_OK;
    case PBFT_OPT_FINISH_WAVES: c->fin_waves = (value == 1 || value == 2) ? (int)value : 0; return PBFT_OK;
    case PBFT_OPT_LAT_SPLIT: c->lat_split = (value == 4 || value == 8) ? (int)value : 0; return PBFT_OK;
    case PBFT_OPT_KERNEL_TIMING: c->timing = value != 0; return PBFT_OK;
    case PBFT_OPT_COMB_PAIR: c->comb_pair = value <= 1 ? (int)value : -1; return PBFT_OK;
    case PBFT_OPT_KEY_TABLE_BUDGET_MB: c->key_budget_mb = value; return PBFT_OK;
    case PBFT_OPT_COMB_PRIO: c->comb_prio = value <= 1 ? (int)value : -1; return PBFT_OK;
    case PBFT_OPT_FAULT_INJECT:
      if (value > 2) return set_err(PBFT_EINVAL, "fault injection point");
      c->fault_inject = (int)value;
      return PBFT_OK;
  }
  return set_err(PBFT_EINVAL, "unknown option");
}

int pbft_verify_ctx_info(pbft_ctx* c, uint32_t* pb, uint32_t* pa, uint32_t* n_keys) {
  if (!c) return set_err(PBFT_EINVAL, "null context");
  if (pb) *pb = (uint32_t)PLB::P;
  if (pa) *pa = (uint32_t)c->pa;
  if (n_keys) *n_keys = c->n_keys;
  return PBFT_OK;
}

float pbft_last_kernel_ms(pbft_ctx* c) {
  if (!c || !c->timing) return -1.f;
  float ms = -1.f;
  if (hipEventSynchronize(c->ev1) != hipSuccess) { (void)hipGetLastError(); return -1.f; }
  if (hipEventElapsedTime(&ms, c->ev0, c->ev1) != hipSuccess) { (void)hipGetLastError(); return -1.f; }
  c->last_ms = ms;
  return ms;
}

}  // extern "C"
