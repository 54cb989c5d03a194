// Host-side PBFT verification state machine (include/pbft_replica.h): signed
// envelopes, a (view, seq) round batcher that hands ready sub-windows of many
// rounds to the GPU verifier in one NON-BLOCKING batch (votes form: one 85-byte
// envelope per (kind, view, seq, digest), an envelope index per signature,
// written straight into the verifier's pinned staging), the quorum predicates,
// a watermark-bounded log with garbage collection, and the PeerId -> key binding.
//
// Mirrors src/state.rs (State: logs keyed by (view, seq), one vote per peer,
// last write wins :56, :66) and src/behavior.rs (validate_* :126-195, prepared
// :177-182, committed_local :214-223, the caller inject_node_event :304-412)
// with the paper's thresholds (2f, 2f+1), commits keyed by (view, seq) instead of
// view only (src/state.rs:22-23), and the signature checks the reference leaves
// as TODOs (src/behavior.rs:127, :185).  The reference calls its validators
// synchronously from a single-threaded poll loop (inject_node_event :304, poll
// :416-426); here a flush is split into pbft_replica_flush_submit (build the batch,
// launch, return) and pbft_replica_flush_poll (apply the bitmap, emit events) so
// that the loop never blocks on the GPU.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <array>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <sched.h>
#include <sys/syscall.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../../include/pbft_replica.h"
#include "../../../include/pbft_wire.h"

namespace {

using Key = std::pair<uint64_t, uint64_t>;  // (view, seq)
using Digest = std::array<uint8_t, 64>;


// Candidates of one kind in one round window, as columns in push order (a candidate leaves when its batch
// completes, so between batches every candidate is pending and a batch takes a whole phase).  A candidate's
// signature lives in its staged row (include/pbft_verify.h: R || S, key index, envelope index), written into one of
// the replica's two row arenas when the vote is pushed (the flush then hands the arena to the
// GPU as it is, without a second pass over every vote); the phase keeps the row's reference.  Per signer: the
// candidate count (flood bound) and the accepted digest (HashMap<PeerId, _>::insert, src/state.rs:49-67: the last
// accepted vote of a signer wins).  Phase 0 of a window holds its PrePrepare candidates (signer = primary).
static constexpr uint32_t ROW_ARENA = 1u << 31, ROW_IDX = ROW_ARENA - 1;  // row reference: arena << 31 | index
struct Phase {
  std::vector<uint32_t> row;  // [k] the candidate's row reference
  std::vector<uint16_t> who;  // signer
  std::vector<uint32_t> dix;  // index into digs
  std::vector<Digest> digs;   // distinct digests of the candidates (honest rounds: one)
  std::vector<uint32_t> denv, dgen;  // per digest: its envelope in the arena of generation dgen (row env_idx)
  std::vector<uint8_t> cnt;   // per signer: candidates
  std::vector<uint32_t> acc;  // per signer: 1 + index into acc_digs (0: none)
  std::vector<Digest> acc_digs;
  std::vector<uint32_t> acc_cnt;  // signers per accepted digest
  uint32_t distinct = 0;          // signers with an accepted vote or a candidate
  uint32_t n_pending = 0;         // candidates not yet in a batch
  uint32_t n_flight = 0;          // the first n_flight candidates are in the batch in flight
  uint64_t row_hi = 0;            // 1 + the largest row index of the candidates
  size_t size() const { return who.size(); }
  void init(uint32_t n) {
    if (cnt.empty()) {
      cnt.assign(n, 0);
      acc.assign(n, 0);
    }
  }
  bool has(uint32_t s) const { return !cnt.empty() && (cnt[s] || acc[s]); }
  int64_t find_dig(const uint8_t* d) const {
    for (size_t j = 0; j < digs.size(); ++j)
      if (memcmp(digs[j].data(), d, 64) == 0) return (int64_t)j;
    return -1;
  }
  void append(const uint8_t* d, int64_t j, uint32_t signer, uint32_t rref, uint32_t env, uint32_t gen) {
    if (j < 0) {
      digs.emplace_back();
      memcpy(digs.back().data(), d, 64);
      denv.push_back(env);
      dgen.push_back(gen);
    } else {
      denv[(size_t)j] = env;  // (the envelope of the arena this row went to)
      dgen[(size_t)j] = gen;
    }
    row.push_back(rref);
    who.push_back((uint16_t)signer);
    dix.push_back(j < 0 ? (uint32_t)digs.size() - 1 : (uint32_t)j);
    ++n_pending;
    if ((rref & ROW_IDX) + 1 > row_hi) row_hi = (rref & ROW_IDX) + 1;
  }
  // drop the first k candidates (a completed batch); re-index the digests of the rest
  void drop_front(size_t k) {
    if (k >= size()) {
      clear_columns();
      return;
    }
    row.erase(row.begin(), row.begin() + k);
    who.erase(who.begin(), who.begin() + k);
    dix.erase(dix.begin(), dix.begin() + k);
    n_flight = n_flight > k ? n_flight - (uint32_t)k : 0;
    std::vector<Digest> nd;
    std::vector<uint32_t> ne, ng;
    for (uint32_t& x : dix) {
      size_t j = 0;
      while (j < nd.size() && nd[j] != digs[x]) ++j;
      if (j == nd.size()) nd.push_back(digs[x]), ne.push_back(denv[x]), ng.push_back(dgen[x]);
      x = (uint32_t)j;
    }
    digs.swap(nd);
    denv.swap(ne);
    dgen.swap(ng);
    row_hi = 0;
    for (uint32_t x : row) row_hi = std::max<uint64_t>(row_hi, (x & ROW_IDX) + 1);
  }
  void clear_columns() {
    row.clear(); who.clear(); dix.clear(); digs.clear(); denv.clear(); dgen.clear();
    row_hi = 0;
    n_flight = 0;
  }
  void clear_candidates() {
    clear_columns();
    n_pending = 0;
  }
  // back to a fresh phase, keeping every allocation (recycled windows)
  void reset() {
    clear_candidates();
    std::fill(cnt.begin(), cnt.end(), 0);
    std::fill(acc.begin(), acc.end(), 0);
    acc_digs.clear();
    acc_cnt.clear();
    distinct = 0;
  }
  uint32_t acc_index(const Digest& d) {  // index into acc_digs (appended if new)
    for (size_t j = 0; j < acc_digs.size(); ++j)
      if (acc_digs[j] == d) return (uint32_t)j;
    acc_digs.push_back(d);
    acc_cnt.push_back(0);
    return (uint32_t)acc_digs.size() - 1;
  }
};

// PBFT_STREAM_STORES=0: plain stores for the staged rows push_many writes (and the flush's fill of the staging when
// the arena cannot be handed over as it is); by default both are streaming (non-temporal) stores -- no
// read-for-ownership of lines that are only written here and read next by the DMA engine (r04 A/B on MI355X boxes:
// the flush's fill 1.1 -> 0.6 ms less of the calling thread's time).
static const bool g_stream_stores = !(getenv("PBFT_STREAM_STORES") && atoi(getenv("PBFT_STREAM_STORES")) == 0);
// PBFT_REPLICA_DIRECT=0: never hand a row arena to the GPU as it is (every batch filled into the staging: the r04
// path); read at every flush (A/B within one process)
static bool direct_enabled() {
  const char* e = getenv("PBFT_REPLICA_DIRECT");
  return !(e && atoi(e) == 0);
}

// One staged row (include/pbft_verify.h: R || S, key_idx, two zero bytes, env_idx), streaming stores where available
static inline void put_row(uint8_t* dst, const uint8_t* sig, uint32_t key, uint32_t env, bool nt) {
  const uint64_t meta = (uint64_t)(key & 0xFFFF) | (uint64_t)env << 32;
#if defined(__x86_64__)
  if (nt) {
    long long v[8];
    memcpy(v, sig, 64);  // (sig may be unaligned: a caller's row)
    for (int q = 0; q < 8; ++q) _mm_stream_si64((long long*)dst + q, v[q]);
    _mm_stream_si64((long long*)dst + 8, (long long)meta);
    return;
  }
#endif
  memcpy(dst, sig, 64);
  memcpy(dst + PBFT_VOTES_ROW_KEY, &meta, 8);
}
static inline void stream_fence() {
#if defined(__x86_64__)
  _mm_sfence();
#endif
}
static inline void cpu_relax() {
#if defined(__x86_64__)
  _mm_pause();
#endif
}

struct Window {
  Phase ph[3];  // [0] PrePrepare candidates, [1] Prepare, [2] Commit
  uint64_t seq = 0;        // its (current-view) sequence number: the ring slot seq & ring_mask holds it
  uint64_t push_call = 0;  // the last push_many that routed rows here, and the task it gave the window to
  uint32_t push_owner = 0;
  bool have_pre_prepare = false;
  bool dirty = false;      // in pbft_replica::dirty (events to be re-evaluated)
  Digest digest{};
  bool pre_prepared_reported = false, prepared_reported = false, committed_reported = false;
  void reset() {
    for (Phase& p : ph) p.reset();
    have_pre_prepare = pre_prepared_reported = prepared_reported = committed_reported = dirty = false;
  }
};

// One phase of the in-flight batch: rows [row0, row0 + count) are its first `count` candidates.
struct Seg {
  Window* w;  // valid unless a window was erased while the batch was in flight (then looked up by key)
  Key key;
  uint64_t row0;     // its first row in the staged batch (arena batches: the candidates before it)
  uint64_t row_end;  // every row of its candidates is below this one (the bitmap prefix that completes it)
  uint32_t count;
  uint32_t env0;  // its envelopes: env0 + index into the phase's digs
  uint8_t kind;   // 0 PrePrepare, 1 Prepare, 2 Commit
};

// Worker threads for the batch fill and the bitmap application: one pool per process, started on first use and
// reused by every large batch of every replica (creating 16 threads costs about a millisecond in a process that
// maps the GPU's memory); one job at a time (start() holds the pool until wait()).
// ---- NUMA (r06): the worker threads on the node whose memory they write ----
// The node holding the page at p (get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR)); -1 if unknown.
static int node_of(const void* p) {
#if defined(SYS_get_mempolicy)
  int node = -1;
  if (p && syscall(SYS_get_mempolicy, &node, nullptr, 0UL, p, 3UL) == 0) return node;
#else
  (void)p;
#endif
  return -1;
}
// The CPUs of NUMA node n (sysfs cpulist, e.g. "0-63,128-191") that this process may use; false if none / unknown.
static bool node_cpus(int n, cpu_set_t* out) {
  CPU_ZERO(out);
  if (n < 0) return false;
  char path[96];
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", n);
  FILE* f = fopen(path, "r");
  if (!f) return false;
  char buf[4096];
  const size_t len = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[len] = 0;
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return false;
  for (char* q = buf; *q;) {
    char* e;
    long a = strtol(q, &e, 10);
    if (e == q) break;
    long b = a;
    if (*e == '-') b = strtol(e + 1, &e, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &allowed)) CPU_SET(c, out);
    q = *e == ',' ? e + 1 : e;
    if (*q == '\n') break;
  }
  return CPU_COUNT(out) > 0;
}

class WorkerPool {
 public:
  // Keep the workers on NUMA node n's CPUs (any of them: the scheduler still balances within the node), or let
  // them float again (n < 0); applied to every worker now and at creation.  Call between jobs.
  void bind(int n) {
    if (n == node_) return;
    cpu_set_t set;
    if (n >= 0 && !node_cpus(n, &set)) n = -1;
    if (n < 0 && sched_getaffinity(0, sizeof set, &set) != 0) return;
    std::lock_guard<std::mutex> lk(job_mu_);
    for (std::thread& t : th_) (void)pthread_setaffinity_np(t.native_handle(), sizeof set, &set);
    node_ = n;
    set_ = set;
  }
  static WorkerPool& get() {
    static WorkerPool* p = new WorkerPool();  // never destroyed: idle workers may outlive static destructors
    return *p;
  }
  // run f(0) .. f(T - 1) on T workers; returns at once (wait() joins the round)
  void start(size_t T, std::function<void(size_t)> f) {
    if (pid_ != getpid()) {
      // a fork()ed child inherits the vector but none of the threads (and maybe locked mutexes): start over
      // with fresh state.  The parent's std::thread objects are leaked, not destroyed (destroying a joinable
      // one terminates, and their handles name threads that do not exist in this process).
      new std::vector<std::thread>(std::move(th_));
      th_ = std::vector<std::thread>();
      new (&job_mu_) std::mutex();
      new (&mu_) std::mutex();
      new (&cv_) std::condition_variable();
      new (&done_) std::condition_variable();
      gen_ = 0;
      active_ = pending_ = running_ = 0;
      closed_ = false;
      node_ = -1;
      pid_ = getpid();
    }
    job_mu_.lock();
    while (th_.size() < T) {
      const size_t id = th_.size();
      th_.emplace_back([this, id] { loop(id); });
      if (node_ >= 0) (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof set_, &set_);
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = std::move(f);
      active_ = T;
      pending_ = T;
      running_ = 0;
      closed_ = false;
      ++gen_;
    }
    cv_.notify_all();
  }
  void wait() {
    {
      std::unique_lock<std::mutex> lk(mu_);
      done_.wait(lk, [&] { return pending_ == 0; });
    }
    job_mu_.unlock();
  }
  void run(size_t T, std::function<void(size_t)> f) {
    start(T, std::move(f));
    wait();
  }
  // Retire the job once the caller's own counters say all of its work is done: workers that have not started it by
  // then skip it, and only those still inside it are waited for -- a worker the host deschedules for milliseconds
  // (r06: up to 10 ms on the GPU boxes, push_rows_start_max_ns) no longer holds up the join (instead of wait()).
  void close() {
    {
      std::unique_lock<std::mutex> lk(mu_);
      closed_ = true;
      done_.wait(lk, [&] { return running_ == 0; });
    }
    job_mu_.unlock();
  }
  // f(0) .. f(T - 1) on the workers and f(T) on the calling thread; done() (the job's own counter of finished items,
  // which the f's take dynamically) ends it, then close()
  template <class Done>
  void run_with_caller(size_t T, const std::function<void(size_t)>& f, Done done) {
    start(T, f);
    f(T);
    while (!done()) cpu_relax();
    close();
  }

 private:
  void loop(size_t id) {
    uint64_t seen = 0;
    for (;;) {  // (idle workers wait here until the process exits)
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen && id < active_; });
        seen = gen_;
        if (closed_) {  // retired before this worker got to it
          if (--pending_ == 0) done_.notify_all();
          continue;
        }
        ++running_;
      }
      job_(id);
      std::lock_guard<std::mutex> lk(mu_);
      --running_;
      if (--pending_ == 0 || (closed_ && running_ == 0)) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_;
  std::function<void(size_t)> job_;
  uint64_t gen_ = 0;
  size_t active_ = 0, pending_ = 0, running_ = 0;
  bool closed_ = false;
  int node_ = -1;  // bind(): the NUMA node the workers are kept on (-1: anywhere the process may run)
  cpu_set_t set_;
  pid_t pid_ = getpid();  // the process whose threads th_ holds
};

}  // namespace

// Flush timeline (PBFT_REPLICA_TRACE=1): host timestamps of the submit / fill / launch / land / apply steps of one
// batch, printed to stderr when the batch completes (tools/replica_probe.py reads them).
static const bool g_trace = getenv("PBFT_REPLICA_TRACE") != nullptr;
static const bool g_push_trace = getenv("PBFT_PUSH_TRACE") != nullptr;

struct TraceEv {
  const char* what;
  uint64_t ns, arg;
};
static uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define RTRACE(r, what, arg) \
  do {                       \
    if (g_trace) (r)->trace.push_back({what, now_ns(), (uint64_t)(arg)}); \
  } while (0)

// A row arena: the staged rows of pushed candidates (and the envelopes their env_idx name), in push order, in
// pinned host memory when the replica has a GPU context.  Pushes go to the current arena; a flush whose batch is
// exactly the current arena's live candidates (the common case: every phase ready) hands the arena itself to the GPU
// (pbft_verify_votes_submit_host) and pushes move to the other one while it is in flight.
struct Arena {
  uint8_t* rows = nullptr;  // [cap][PBFT_VOTES_ROW_BYTES]
  uint8_t* envs = nullptr;  // [ecap][PBFT_ENVELOPE_BYTES] + 64 bytes of read slack
  uint64_t cap = 0, n = 0;  // rows allocated / written (candidates' rows, push_many's unused tails, dropped ones)
  uint32_t ecap = 0, ne = 0;
  bool rows_pinned = false, envs_pinned = false;
  mutable std::atomic<int64_t> live{0};  // candidates whose rows are here
  std::atomic<bool> clean{true};         // every row's env_idx names an envelope of this arena
  uint32_t gen = 0;                      // envelope generation (phases' dgen): renewed when the arena restarts
  bool busy = false;                     // the batch in flight reads it
};

struct pbft_replica {
  std::vector<TraceEv> trace;
  Arena arena[2];
  uint32_t cur = 0;        // the arena pushes write to (never busy)
  uint32_t next_gen = 1;
  bool direct = false;     // the batch in flight is arena `busy_arena` as it is (rows = arena rows)
  uint64_t push_calls = 0;  // threaded push_many calls (Window::push_call)
  // push_many's early batch (r05): the current arena's rows verified in pieces while they are pushed
  // (pbft_verify_votes_open / _piece / _close); flush_submit adopts it when the arena is unchanged since
  struct {
    bool active = false;  // a batch covers arena `arena` rows [0, rows) and envelopes [0, envs); bits -> bitmap
    bool done = false;    // waited for: every bit is in r->bitmap
    bool open = false;    // (single pushes, r06) still open on ctx: pieces [0, rows) launched, more may follow
    uint32_t arena = 0;
    uint64_t rows = 0;
    uint32_t envs = 0;
    std::vector<uint64_t> lo;  // context j (ctxs[j]) verifies rows [lo[j], lo[j + 1]) (one context: {0, rows})
  } eu;
  pbft_replica_timings tm{};      // phases of the last push_many / flush (pbft_replica_get_timings)
  uint64_t early_pieces = 0, early_piece_ns = 0;  // the single pushes' early batch since the last flush_submit
  std::chrono::steady_clock::time_point t_submit_end{};
  uint64_t peak_rows = 0;  // the largest arena a flush has taken, and its envelopes (the single pushes' early batch
  uint32_t peak_envs = 0;  // sizes the arena for a whole round before it opens: pieces read it in place)
  uint32_t busy_arena = 0;
  uint64_t applied_upto = 0;  // rows_done at the last progressive application
  bool adopted = false;       // the batch in flight is an early batch (push_many's or the single pushes')
  bool adopt_partial = true;  // ... applied as its pieces land (r06: push_many's rows lie task by task, so a landed
                              // prefix of rows is a prefix of the windows; PBFT_ADOPT_PARTIAL=0: once, when done)
  pbft_ctx* ctx = nullptr;         // ctxs[0]: digests, small batches
  std::vector<pbft_ctx*> ctxs;     // pbft_replica_create_multi: large batches split over these (one per GPU)
  uint32_t n = 0, f = 0, self = 0;
  uint64_t current_view = 1;  // src/view.rs:5-8: the view starts at 1 (no view change)
  uint64_t h = 0;             // low watermark: every seq <= h is done (committed prefix or checkpoint)
  uint64_t log_window = PBFT_DEFAULT_LOG_WINDOW;
  std::vector<uint8_t> keys;
  std::unordered_map<std::string, uint32_t> key_index;
  // Window store (r06): every window is of the current view (the reference has no view change,
  // src/view.rs) and its seq lies in (h, h + log_window], a dense range: a ring of 2^k >= log_window slots indexed by
  // seq holds them, so a lookup, an insertion, the flush's ordered walk and the GC's committed-prefix step are O(1)
  // per window instead of std::map operations.  Live windows' seqs are distinct modulo the ring size because h only
  // moves in gc(), which drops every window <= h in the same call, and the ring never shrinks.
  std::vector<Window*> ring;              // [seq & ring_mask]: the live window of that seq, or null
  uint64_t ring_mask = 0;
  std::vector<std::unique_ptr<Window>> win_pool;  // every window ever allocated (recycled through win_free)
  std::vector<Window*> win_free;
  size_t n_windows = 0;
  uint64_t win_hi = 0;                    // every live window's seq is <= win_hi
  uint64_t gc_h = 0;                      // every window <= gc_h has been dropped
  std::vector<uint64_t> dirty;            // seqs of windows whose events must be (re-)evaluated
  std::deque<pbft_round_event> evq;       // decided, not yet delivered
  std::map<uint64_t, uint64_t> done;      // seqs of current_view committed locally and GC'd: [lo, hi]
  uint64_t last_seq = ~0ull;              // push fast path: the last window looked up
  Window* last_w = nullptr;
  pbft_ctx* dctx = nullptr;               // the replica's own clone of ctx for request digests (r06): a digest
                                          // never waits for the votes batch on ctx (nor pushes an open one out)
  pbft_batch_verify_fn verify_fn = nullptr;
  void* verify_user = nullptr;
  pbft_votes_submit_fn vsub = nullptr;
  pbft_votes_poll_fn vpoll = nullptr;
  void* vuser = nullptr;
  pbft_digest_fn digest_fn = nullptr;
  void* digest_user = nullptr;
  pbft_replica_stats stats{};
  // the batch in flight (at most one)
  bool in_flight = false;
  int in_flight_via = 0;  // 0 GPU context, 1 votes override, 2 SoA override (already complete)
  std::vector<Seg> segs;
  size_t seg_next = 0;            // segments [0, seg_next) already applied (progressive completion)
  std::vector<uint8_t> touched;   // per segment: some candidate accepted
  uint64_t rows = 0;
  uint64_t rows_span = 0;         // rows of the bitmap: rows + the padding that 64-aligns each context's slice
  // multi-context batch: context k verifies rows [slice_lo[k], slice_lo[k + 1]) (its staged rows; the last
  // slice_lo[k + 1] - slice_hi[k] of them padding); slice_end[k]: its rows known verified (bitmap words landed)
  std::vector<uint64_t> slice_lo, slice_hi, slice_end;
  std::vector<uint8_t> slice_fin;
  bool erased_in_flight = false;  // a stable checkpoint erased windows while the batch was in flight
  std::vector<uint64_t> bitmap;
  // host buffers of the verifier overrides (the GPU path fills the context's pinned staging instead)
  std::vector<uint8_t> hSig, hR, hS, hM, hE;
  std::vector<uint16_t> hK;
  std::vector<uint32_t> hI;
};

static uint32_t primary_of(const pbft_replica* r, uint64_t view) { return (uint32_t)(view % r->n); }

// ---- row arenas ----
static constexpr size_t ROWB = PBFT_VOTES_ROW_BYTES;
// ---- push_many's early batch ----
static bool early_enabled() {  // PBFT_REPLICA_EARLY=0: push_many never launches (read per call: A/B in one process)
  const char* e = getenv("PBFT_REPLICA_EARLY");
  return !(e && atoi(e) == 0);
}
// wait for the early batch (the context is needed, or its arena is about to change); its bits stay adoptable
static int eu_settle(pbft_replica* r) {
  if (!r->eu.active || r->eu.done) return PBFT_OK;
  if (r->eu.open) {  // an open batch cannot be waited for: dropped (a close that does not match drains and drops it)
    (void)pbft_verify_votes_close(r->ctx, 0);
    r->eu.open = false;
    r->eu.active = false;
    return PBFT_OK;
  }
  int rc = PBFT_OK;
  for (size_t j = 0; j + 1 < r->eu.lo.size(); ++j) {
    const int w = pbft_verify_wait(r->ctxs[j]);
    if (w && !rc) rc = w;
  }
  if (rc) {
    r->eu.active = false;  // lost: the flush verifies the rows again
    return rc;
  }
  r->eu.done = true;
  return PBFT_OK;
}
static void eu_drop(pbft_replica* r) {
  (void)eu_settle(r);
  r->eu.active = false;
}

static void* host_mem(pbft_replica* r, size_t bytes, bool* pinned) {
  void* p = nullptr;
  *pinned = false;
  if (r->ctx && pbft_host_alloc(r->ctx, bytes, &p) == PBFT_OK && p) {
    *pinned = true;
    return p;
  }
  return aligned_alloc(64, (bytes + 63) / 64 * 64);  // (no GPU context: the overrides read it)
}
static void host_mem_free(pbft_replica* r, void* p, bool pinned) {
  if (!p) return;
  if (pinned) (void)pbft_host_free(r->ctx, p);
  else free(p);
}
// room for `rows` more rows and `envs` more envelopes (the current arena only: never busy)
static bool arena_reserve(pbft_replica* r, Arena& a, uint64_t rows, uint64_t envs) {
  if ((a.n + rows > a.cap || a.ne + envs > a.ecap) && r->eu.active && &r->arena[r->eu.arena] == &a)
    eu_drop(r);  // (the early batch's copies read this arena: finished before it moves)
  if (a.n + rows > a.cap) {
    if (a.n + rows > ROW_IDX) return false;
    const uint64_t c = std::min<uint64_t>(ROW_IDX, std::max<uint64_t>({2 * a.cap, a.n + rows, 1u << 12}));
    bool pin;
    uint8_t* q = (uint8_t*)host_mem(r, ROWB * c, &pin);
    if (!q) return false;
    if (a.n) memcpy(q, a.rows, ROWB * a.n);
    host_mem_free(r, a.rows, a.rows_pinned);
    a.rows = q;
    a.rows_pinned = pin;
    a.cap = c;
  }
  if (a.ne + envs > a.ecap) {
    if (a.ne + envs > ROW_IDX) return false;
    const uint64_t c = std::min<uint64_t>(ROW_IDX, std::max<uint64_t>({2 * (uint64_t)a.ecap, a.ne + envs, 256}));
    bool pin;
    uint8_t* q = (uint8_t*)host_mem(r, (size_t)PBFT_ENVELOPE_BYTES * c + 64, &pin);
    if (!q) return false;
    if (a.ne) memcpy(q, a.envs, (size_t)PBFT_ENVELOPE_BYTES * a.ne);
    host_mem_free(r, a.envs, a.envs_pinned);
    a.envs = q;
    a.envs_pinned = pin;
    a.ecap = (uint32_t)c;
  }
  return true;
}
// Start the arena over (no candidate's row is in it, nothing reads it): envelope 0 is the one of rows no candidate
// references (push_many's unused tails)
static const uint8_t g_zero_digest[64] = {0};
static void arena_restart(pbft_replica* r, Arena& a) {
  if (r->eu.active && &r->arena[r->eu.arena] == &a) eu_drop(r);
  a.n = 0;
  a.ne = 0;
  a.gen = r->next_gen++;
  a.clean.store(true, std::memory_order_relaxed);
  if (arena_reserve(r, a, 0, 1)) {
    pbft_envelope(a.envs, 0, 0, 0, g_zero_digest);
    a.ne = 1;
  } else {
    a.clean.store(false, std::memory_order_relaxed);
  }
}
// the arena pushes write to, restarted first when nothing references it any more
static Arena& push_arena(pbft_replica* r) {
  Arena& a = r->arena[r->cur];
  if (a.gen == 0 || (a.n > 0 && a.live.load(std::memory_order_relaxed) == 0 && !a.busy)) arena_restart(r, a);
  return a;
}
static inline const uint8_t* row_at(const pbft_replica* r, uint32_t rref) {
  return r->arena[rref >> 31].rows + ROWB * (rref & ROW_IDX);
}
// the first k candidates of p leave (their rows are dead from here on): counted into c[arena] (the caller
// subtracts them from the arenas' live counts once -- one atomic per batch, not per phase: 16 threads updating one
// cache line per segment cost the r05 apply ~0.5 ms), or subtracted at once
static void count_rows(const Phase& p, size_t k, int64_t c[2]) {
  // (the sum in a register: ++c[row >> 31] through memory was a store-to-load chain, ~1,000 cycles per 256-candidate
  // segment -- 38 % of the application, r06)
  const size_t m = std::min(k, p.row.size());
  const uint32_t* row = p.row.data();
  int64_t in1 = 0;
  for (size_t i = 0; i < m; ++i) in1 += row[i] >> 31;
  c[1] += in1;
  c[0] += (int64_t)m - in1;
}
static void release_counts(const pbft_replica* r, const int64_t c[2]) {
  for (int a = 0; a < 2; ++a)
    if (c[a]) r->arena[a].live.fetch_sub(c[a], std::memory_order_relaxed);
}
static void release_rows(const pbft_replica* r, const Phase& p, size_t k) {
  int64_t c[2] = {0, 0};
  count_rows(p, k, c);
  release_counts(r, c);
}
static void release_window(const pbft_replica* r, Window& w) {
  for (Phase& p : w.ph) {
    release_rows(r, p, p.size());
    p.clear_candidates();
  }
}

// Where one pusher writes rows and envelopes: the current arena's end (a single push: grows it), or a range of it
// reserved for one push_many thread (sized for the thread's rows; envelopes beyond its share leave the arena
// unclean, which sends the next batch through the staging fill instead).
struct Sink {
  Arena* a;
  uint32_t aid;
  uint64_t row, row_end;
  uint32_t env, env_end;
  bool grow, nt;
  int64_t added = 0;
};
static Sink single_sink(pbft_replica* r) {
  Arena& a = push_arena(r);
  return Sink{&a, r->cur, a.n, ~0ull, a.ne, ~0u, true, g_stream_stores};
}
static void sink_done(Sink& s) {  // (single sinks) the arena's counts
  if (s.grow) {
    s.a->n = s.row;
    s.a->ne = s.env;
  }
  // (single pushes run on the caller's thread with no worker touching the counts: a plain update, not an RMW)
  s.a->live.store(s.a->live.load(std::memory_order_relaxed) + s.added, std::memory_order_relaxed);
  s.added = 0;
}
static uint32_t sink_env(pbft_replica* r, Sink& s, uint8_t kind, uint64_t view, uint64_t seq, const uint8_t* d) {
  if (s.grow) {
    s.a->n = s.row;
    s.a->ne = s.env;
    if (!arena_reserve(r, *s.a, 0, 1)) {
      s.a->clean.store(false, std::memory_order_relaxed);
      return 0;
    }
  } else if (s.env >= s.env_end) {
    s.a->clean.store(false, std::memory_order_relaxed);
    return 0;
  }
  pbft_envelope(s.a->envs + (size_t)PBFT_ENVELOPE_BYTES * s.env, kind, view, seq, d);
  return s.env++;
}
static bool sink_row(pbft_replica* r, Sink& s, uint64_t* idx) {
  if (s.grow) {
    s.a->n = s.row;
    s.a->ne = s.env;
    if (!arena_reserve(r, *s.a, 1, 0)) return false;
  } else if (s.row >= s.row_end) {
    return false;  // (never: a thread's range holds every row it may push)
  }
  *idx = s.row++;
  return true;
}

// ---- the single-message path's early batch (r06) ----
// Messages delivered one at a time (pbft_replica_push, _push_frames, _push_records, on_pre_prepare: the reference's
// inject_node_event, one message per call on its swarm thread, src/behavior.rs:304) write their rows into the current
// arena in arrival order.  Once a piece's worth of rows is in, the arena is opened as a batch in pieces on the context
// (pbft_verify_votes_open) and every further piece is launched (pbft_verify_votes_piece) while the caller keeps
// pushing, so at the flush only the last < piece + 64 rows are left to copy and verify: flush_submit launches them,
// closes the batch and adopts it (one context; a replica over several contexts hands its arena over at the flush).
// PBFT_EARLY_PIECE: rows per piece (default 2^16; read once, at load -- this runs on every push).
static const uint64_t g_early_piece = [] {
  const char* e = getenv("PBFT_EARLY_PIECE");
  const long long v = e ? strtoll(e, nullptr, 10) : (1 << 16);
  return (uint64_t)(v < 4096 ? 4096 : v > (1 << 22) ? (1 << 22) : v) & ~(uint64_t)63;
}();
static inline uint64_t early_piece_rows() { return g_early_piece; }
static void early_single(pbft_replica* r) {
  if (r->eu.active && !r->eu.open) return;  // push_many's batch (closed): nothing to add
  Arena& A = r->arena[r->cur];
  const uint64_t piece = early_piece_rows();
  if (!r->eu.active) {
    // (not before a flush has shown the round's size: the arena is sized for the round before it opens)
    if (A.n < piece || r->peak_rows == 0 || !early_enabled() || !direct_enabled() || !r->ctx || r->ctxs.size() != 1 || r->verify_fn ||
        r->vsub || r->in_flight || A.busy || !A.rows_pinned || !A.envs_pinned || !A.clean.load(std::memory_order_relaxed))
      return;
    // room for the whole round first (the pieces read the arena in place: it must not move while the batch is open)
    const uint64_t want = std::max<uint64_t>(2 * A.n, r->peak_rows + r->peak_rows / 8);
    const uint64_t want_e = std::max<uint64_t>(2 * (uint64_t)A.ne + 256, r->peak_envs + r->peak_envs / 8);
    if (!arena_reserve(r, A, want - A.n, want_e > A.ne ? want_e - A.ne : 0) || !A.rows_pinned || !A.envs_pinned)
      return;
    r->bitmap.assign((A.cap + 63) / 64, 0);
    if (pbft_verify_votes_open(r->ctx, A.cap, A.ecap, r->bitmap.data()) != PBFT_OK) return;
    r->eu.active = true;
    r->eu.open = true;
    r->eu.done = false;
    r->eu.arena = r->cur;
    r->eu.rows = 0;
    r->eu.envs = 0;
    r->eu.lo.assign({0, A.cap});
    RTRACE(r, "early_open", A.n);
  }
  if (r->eu.arena != r->cur || A.n - r->eu.rows < piece) return;
  const uint64_t hi = A.n & ~(uint64_t)63;
  const uint64_t t0 = now_ns();
  stream_fence();  // (the rows' streaming stores are visible before the copy engine reads them)
  const int rc = pbft_verify_votes_piece(r->ctx, A.rows, r->eu.rows, hi, A.envs, r->eu.envs, A.ne);
  r->early_piece_ns += now_ns() - t0;
  ++r->early_pieces;
  if (rc != PBFT_OK) {
    r->eu.active = r->eu.open = false;  // (a failing piece drops the batch; the flush verifies the arena again)
    return;
  }
  r->eu.rows = hi;
  r->eu.envs = A.ne;
}

static bool in_log(const pbft_replica* r, uint64_t seq) { return seq > r->h && seq - r->h <= r->log_window; }

// accepted votes of phase p matching the window's digest (optionally not counting one signer)
static uint32_t matching(const Window& w, const Phase& p, int64_t exclude = -1) {
  if (!w.have_pre_prepare) return 0;
  for (size_t j = 0; j < p.acc_digs.size(); ++j) {
    if (p.acc_digs[j] != w.digest) continue;
    uint32_t c = p.acc_cnt[j];
    if (exclude >= 0 && !p.acc.empty() && p.acc[exclude] == j + 1) --c;
    return c;
  }
  return 0;
}

// prepared(m, v, n, i): pre-prepare + 2f matching prepares from distinct backups
static bool is_prepared(const pbft_replica* r, uint64_t view, const Window& w) {
  return w.have_pre_prepare && matching(w, w.ph[1], primary_of(r, view)) >= 2 * r->f;
}

// committed-local(m, v, n, i): prepared + 2f+1 matching commits (possibly own)
static bool is_committed_local(const pbft_replica* r, uint64_t view, const Window& w) {
  return is_prepared(r, view, w) && matching(w, w.ph[2]) >= 2 * r->f + 1;
}

// A sub-window closes on its own count: enough distinct signers for the quorum
// (2f backups' Prepares / 2f+1 Commits) or every possible signer.
static bool prepare_ready(const pbft_replica* r, uint64_t view, const Window& w) {
  const Phase& p = w.ph[1];
  if (p.n_pending == 0 || w.prepared_reported) return false;
  const uint32_t c = p.distinct - (p.has(primary_of(r, view)) ? 1 : 0);
  return c >= 2 * r->f || c + 1 >= r->n;
}
static bool commit_ready(const pbft_replica* r, const Window& w) {
  const Phase& p = w.ph[2];
  if (p.n_pending == 0 || w.committed_reported) return false;
  return p.distinct >= 2 * r->f + 1 || p.distinct >= r->n;
}

static std::string key_str(const uint8_t* A) { return std::string((const char*)A, 32); }

// ---- window ring ----
static constexpr uint64_t MAX_LOG_WINDOW = 1ull << 24;  // (pbft_replica_set_log_window; the ring's slots are 8 B)
// room for live seqs (h, h + span]: the ring grows to a power of two >= span, re-slotting the live windows
static void ring_reserve(pbft_replica* r, uint64_t span) {
  uint64_t R = 1024;
  while (R < span) R <<= 1;
  if (R <= r->ring.size()) return;
  std::vector<Window*> nr(R, nullptr);
  for (Window* w : r->ring)
    if (w) nr[w->seq & (R - 1)] = w;
  r->ring.swap(nr);
  r->ring_mask = R - 1;
}
// the live window of (view, seq), or null
static inline Window* find_window(const pbft_replica* r, uint64_t view, uint64_t seq) {
  if (view != r->current_view) return nullptr;
  Window* w = r->ring[seq & r->ring_mask];
  return w && w->seq == seq ? w : nullptr;
}
// the window of (current view, seq), created if absent; seq must be in the log (in_log)
static Window& window_at(pbft_replica* r, uint64_t seq) {
  if (r->last_w && r->last_seq == seq) return *r->last_w;
  Window*& s = r->ring[seq & r->ring_mask];
  if (!s) {
    Window* w;
    if (!r->win_free.empty()) {
      w = r->win_free.back();
      r->win_free.pop_back();
      w->reset();
    } else {
      r->win_pool.emplace_back(new Window());
      w = r->win_pool.back().get();
    }
    w->seq = seq;
    s = w;
    ++r->n_windows;
    if (seq > r->win_hi) r->win_hi = seq;
  }
  r->last_seq = seq;
  r->last_w = s;
  return *s;
}

// erase a window, keeping it (and every vector in it) for the next window
static void drop_window(pbft_replica* r, Window* w) {
  if (r->in_flight) r->erased_in_flight = true;
  release_window(r, *w);  // (an in-flight batch skips the window's rows: erased_in_flight)
  r->ring[w->seq & r->ring_mask] = nullptr;
  --r->n_windows;
  w->seq = 0;  // (no seq in the log is 0: a recycled window matches no lookup until it is reused)
  r->win_free.push_back(w);
  if (r->last_w == w) r->last_w = nullptr;
}

// seqs of the current view committed locally whose windows are gone (interval set)
static void record_done(pbft_replica* r, uint64_t seq) {
  auto it = r->done.upper_bound(seq);  // first interval starting after seq
  if (it != r->done.begin()) {
    auto p = std::prev(it);
    if (seq <= p->second) return;  // already in
    if (p->second + 1 == seq) {
      p->second = seq;
      if (it != r->done.end() && it->first == seq + 1) {
        p->second = it->second;
        r->done.erase(it);
      }
      return;
    }
  }
  if (it != r->done.end() && it->first == seq + 1) {
    const uint64_t hi = it->second;
    r->done.erase(it);
    r->done[seq] = hi;
    return;
  }
  r->done[seq] = seq;
}
// record_done for every seq in [lo, hi] at once (the GC's committed prefix: one interval update, not one per seq)
static void record_done_range(pbft_replica* r, uint64_t lo, uint64_t hi) {
  auto it = r->done.upper_bound(lo);  // first interval starting after lo
  std::map<uint64_t, uint64_t>::iterator cur;
  if (it != r->done.begin() && std::prev(it)->second + 1 >= lo) {
    cur = std::prev(it);  // [a, b] with b + 1 >= lo: extend it
    if (cur->second < hi) cur->second = hi;
  } else {
    cur = r->done.emplace_hint(it, lo, hi);
  }
  // absorb the intervals that now touch or overlap
  for (auto nx = std::next(cur); nx != r->done.end() && nx->first <= cur->second + 1; nx = r->done.erase(nx))
    if (nx->second > cur->second) cur->second = nx->second;
}

static bool is_done(const pbft_replica* r, uint64_t view, uint64_t seq) {
  if (view != r->current_view) return false;
  auto it = r->done.upper_bound(seq);
  if (it == r->done.begin()) return false;
  return seq <= std::prev(it)->second;
}

static void gc(pbft_replica* r) {
  r->last_w = nullptr;  // windows may go away
  // committed prefix: h advances over consecutive committed windows (ring slot h + 1, h + 2, ...)
  const uint64_t h0 = r->h;
  for (;;) {
    Window* w = find_window(r, r->current_view, r->h + 1);
    if (!w || !w->committed_reported) break;
    drop_window(r, w);
    ++r->h;
    ++r->stats.windows_gc;
  }
  if (r->h > h0) record_done_range(r, h0 + 1, r->h);
  // anything else at or below h (a stable checkpoint moved it): seqs (gc_h, h], or every slot when that range is
  // longer than the ring; the in-flight rows of an erased window are skipped when the batch completes (a dropped
  // window's dirty entry finds no window at evaluate())
  if (r->h > r->gc_h && r->n_windows) {
    auto drop_low = [r](Window* w) {
      if (w->committed_reported) record_done(r, w->seq);
      drop_window(r, w);
      ++r->stats.windows_gc;
    };
    if (r->h - r->gc_h <= r->ring.size()) {
      for (uint64_t q = r->gc_h + 1; q <= r->h && r->n_windows; ++q) {
        Window* w = r->ring[q & r->ring_mask];
        if (w && w->seq == q) drop_low(w);
      }
    } else {
      for (Window* w : std::vector<Window*>(r->ring))
        if (w && w->seq <= r->h) drop_low(w);
    }
  }
  if (r->h > r->gc_h) r->gc_h = r->h;
}

// The events one window's state now decides (pre-prepared, prepared :177-182, committed_local :214-223), appended
// to `out`; a committed window drops its stragglers (nothing of it may be in flight: callers guarantee that).
template <class Out>
static void evaluate_window(const pbft_replica* r, uint64_t view, uint64_t seq, Window& w, Out& out) {
  if (!w.pre_prepared_reported && w.have_pre_prepare) {
    w.pre_prepared_reported = true;
    out.push_back({view, seq, PBFT_EVENT_PRE_PREPARED});
  }
  if (!w.prepared_reported && is_prepared(r, view, w)) {
    w.prepared_reported = true;
    out.push_back({view, seq, PBFT_EVENT_PREPARED});
  }
  if (!w.committed_reported && is_committed_local(r, view, w)) {
    w.committed_reported = true;
    out.push_back({view, seq, PBFT_EVENT_COMMITTED_LOCAL});
    release_window(r, w);  // decided: stragglers are never needed
  }
}

// Events of every dirty window, in (view, seq) order, into the replica's queue: the decision is recorded whether
// or not the caller has room for it.  (Windows completed by a batch are evaluated as they are applied,
// apply_range; `dirty` holds the rest.)
static void evaluate(pbft_replica* r) {
  if (r->dirty.empty()) return;
  std::sort(r->dirty.begin(), r->dirty.end());
  for (uint64_t q : r->dirty) {
    Window* w = find_window(r, r->current_view, q);
    if (!w || !w->dirty) continue;  // (gone, or already evaluated: a duplicate entry)
    w->dirty = false;
    evaluate_window(r, r->current_view, q, *w, r->evq);
  }
  r->dirty.clear();
}
static void mark_window_dirty(pbft_replica* r, Window& w) {
  if (!w.dirty) {
    w.dirty = true;
    r->dirty.push_back(w.seq);
  }
}

static void drain(pbft_replica* r, pbft_round_event* events, uint32_t max_events, uint32_t* n_events) {
  uint32_t ne = 0;
  while (events && ne < max_events && !r->evq.empty()) {
    events[ne++] = r->evq.front();
    r->evq.pop_front();
  }
  if (n_events) *n_events = ne;
}

// Put every in-flight candidate back to pending (the batch failed: nothing was applied).
static void mark_dirty(pbft_replica* r);
static void revert_segs(pbft_replica* r) {
  for (size_t gi = r->seg_next; gi < r->segs.size(); ++gi) {  // (segments applied before the failure stay)
    const Seg& g = r->segs[gi];
    Window* wp = find_window(r, g.key.first, g.key.second);
    if (!wp) continue;
    Phase& p = wp->ph[g.kind];
    const uint32_t back = std::min<uint32_t>(p.n_flight, (uint32_t)p.size());  // (the batch's: the first ones)
    p.n_pending += back;
    p.n_flight = 0;
  }
  if (r->seg_next) mark_dirty(r);
  r->segs.clear();
  r->seg_next = 0;
  r->in_flight = false;
  r->erased_in_flight = false;
  if (r->direct) r->arena[r->busy_arena].busy = false;
  r->direct = false;
  r->adopted = false;
}

// The finished batch: State::insert_* for accepted candidates (in push order: the last accepted vote of a signer
// wins), the first accepted PrePrepare fixes the window's digest (conflicting ones rejected, :144-151); verified
// candidates leave the windows.  Segments [s0, s1) (whole windows: a window's segments stay on one thread, in
// order); counts into st[3] = accepted, rejected_sig, rejected_digest; touched[g] = some candidate accepted.
// PBFT_APPLY_PREFETCH: how many segments ahead the application prefetches (0: off; default 1; read per call: A/B in
// one process)
static size_t apply_prefetch() {
  const char* e = getenv("PBFT_APPLY_PREFETCH");
  const long v = e ? strtol(e, nullptr, 10) : 1;
  return (size_t)(v < 0 ? 0 : v > 8 ? 8 : v);
}
static inline void prefetch_bytes(const void* p, size_t n) {
  for (size_t o = 0; o < n; o += 64) __builtin_prefetch((const uint8_t*)p + o);
}
static void prefetch_phase(const Phase& p) {
  const size_t k = p.size();
  prefetch_bytes(p.who.data(), 2 * k);
  prefetch_bytes(p.row.data(), 4 * k);
  prefetch_bytes(p.acc.data(), 4 * p.acc.size());
  prefetch_bytes(p.cnt.data(), p.cnt.size());
  if (!p.digs.empty()) prefetch_bytes(p.digs.data(), 64);
}
static void apply_range(pbft_replica* r, size_t s0, size_t s1, uint64_t st_out[3], uint8_t* touched,
                        std::vector<pbft_round_event>& events) {
  std::vector<int64_t> amap;
  std::vector<uint8_t> mism;
  uint64_t st[3] = {0, 0, 0};  // local: the threads' st_out entries share cache lines
  int64_t rel[2] = {0, 0};     // candidates leaving each arena (one atomic update per call)
  const size_t pf = apply_prefetch();
  if (pf > 1 && !r->erased_in_flight)  // (the first pf - 1 segments of the range: the loop fetches pf ahead)
    for (size_t j = s0 + 1; j < std::min(s1, s0 + pf); ++j) prefetch_phase(r->segs[j].w->ph[r->segs[j].kind]);
  for (size_t gi = s0; gi < s1; ++gi) {
    const Seg& g = r->segs[gi];
    // the next segment's columns and per-signer arrays, fetched while this one is applied (a batch handed over as
    // the arena reaches the application with them cold: nothing since the push has touched them)
    if (pf && gi + pf < s1 && !r->erased_in_flight) prefetch_phase(r->segs[gi + pf].w->ph[r->segs[gi + pf].kind]);
    Window* wp = g.w;
    if (r->erased_in_flight) {
      wp = find_window(r, g.key.first, g.key.second);
      if (!wp) continue;  // window erased (stable checkpoint) while the batch was in flight
    }
    Window& w = *wp;
    Phase& p = w.ph[g.kind];
    const uint64_t* bm = r->bitmap.data();
    // candidate i's row: its arena row when the arena went to the GPU as it is, else the staged row0 + i
    const uint32_t* rref = r->direct ? p.row.data() : nullptr;
    const uint64_t row0 = g.row0;
    auto row_of = [rref, row0](uint32_t i) -> uint64_t { return rref ? (uint64_t)(rref[i] & ROW_IDX) : row0 + i; };
    uint32_t acc_n = 0;
    if (g.kind == 0) {
      for (uint32_t i = 0; i < g.count; ++i) {
        const uint64_t row = row_of(i);
        if (!((bm[row >> 6] >> (row & 63)) & 1)) continue;
        ++acc_n;
        const Digest& d = p.digs[p.dix[i]];
        if (!w.have_pre_prepare) {
          w.have_pre_prepare = true;
          w.digest = d;
        } else if (w.digest != d) {
          ++st[2];
        }
      }
    } else {
      amap.assign(p.digs.size(), -1);
      mism.resize(p.digs.size());
      for (size_t j = 0; j < p.digs.size(); ++j) mism[j] = w.have_pre_prepare && p.digs[j] != w.digest;
      const uint16_t* who = p.who.data();
      const uint32_t* dix = p.dix.data();
      uint32_t* acc = p.acc.data();
      uint8_t* cnt = p.cnt.data();
      uint32_t gone = 0;  // signers left with neither a candidate nor an accepted vote
      if (p.digs.size() == 1) {
        // the honest round: one digest -- its accepted-vote count is added once per segment, not per row
        const uint32_t a = p.acc_index(p.digs[0]) + 1;
        uint32_t gained = 0;
        for (uint32_t i = 0; i < g.count; ++i) {
          const uint64_t row = row_of(i);
          const uint32_t s = who[i];
          const uint32_t prev = acc[s];
          if ((bm[row >> 6] >> (row & 63)) & 1) {
            ++acc_n;
            if (prev != a) {
              if (prev) --p.acc_cnt[prev - 1];
              acc[s] = a;
              ++gained;
            }
            --cnt[s];
          } else {
            gone += --cnt[s] == 0 && !prev;
          }
        }
        p.acc_cnt[a - 1] += gained;
        st[2] += mism[0] ? acc_n : 0;
      } else {
        for (uint32_t i = 0; i < g.count; ++i) {
          const uint64_t row = row_of(i);
          const uint32_t s = who[i];
          if ((bm[row >> 6] >> (row & 63)) & 1) {
            ++acc_n;
            const uint32_t d = dix[i];
            if (amap[d] < 0) amap[d] = p.acc_index(p.digs[d]);
            const uint32_t a = (uint32_t)amap[d] + 1;
            if (acc[s] != a) {
              if (acc[s]) --p.acc_cnt[acc[s] - 1];
              acc[s] = a;
              ++p.acc_cnt[a - 1];
            }
            st[2] += mism[d];
          }
          gone += --cnt[s] == 0 && !acc[s];
        }
      }
      p.distinct -= gone;
    }
    st[0] += acc_n;
    st[1] += g.count - acc_n;
    count_rows(p, g.count, rel);
    p.drop_front(g.count);  // pushes that arrived during the flight stay, in order
    touched[gi] = acc_n > 0;
    // the window's last segment of this batch: its events are decided now, on this thread (segments come in
    // (view, seq) order and a window's stay on one thread, so the threads' event lists concatenate in order)
    if (gi + 1 == r->segs.size() || r->segs[gi + 1].key != g.key) {
      bool any = false;
      for (size_t gj = gi + 1; gj-- > 0 && r->segs[gj].key == g.key;) any = any || touched[gj];
      if (any) evaluate_window(r, g.key.first, g.key.second, w, events);
    }
  }
  release_counts(r, rel);
  for (int k = 0; k < 3; ++k) st_out[k] += st[k];
}

// Threads for the batch fill and the bitmap application of large batches: PBFT_REPLICA_THREADS (default 16,
// capped by the host; 16 vs 8: 2^20 round 5.3-5.7 vs 5.8-6.2 ms, profiles/r03/ab_threads.txt).
// (read per call -- once per batch, not per vote: an A/B can vary it round by round in one process)
static size_t host_threads() {
  const char* e = getenv("PBFT_REPLICA_THREADS");
  const long v = e ? strtol(e, nullptr, 10) : 16;
  return (size_t)(v < 1 ? 1 : v > 64 ? 64 : v);
}

// Apply segments [s0, s1) of the batch (rows all verified); large ranges on several threads, cut at window
// boundaries (balanced by rows) into 4 pieces per thread that the threads -- the calling one too -- take as they
// free up (events kept in piece order).
static void apply_segs(pbft_replica* r, size_t s0, size_t s1) {
  if (s1 <= s0) return;
  const uint64_t lo = r->segs[s0].row0, nrows = r->segs[s1 - 1].row0 + r->segs[s1 - 1].count - lo;
  const unsigned hw = std::thread::hardware_concurrency();
  const size_t T = nrows >= (1u << 16) ? std::min<size_t>(std::min<size_t>(hw ? hw : 1, host_threads()), s1 - s0) : 1;
  const size_t C = T <= 1 ? 1 : std::min<size_t>(4 * T, s1 - s0);
  std::vector<std::array<uint64_t, 3>> st(C, {0, 0, 0});
  std::vector<std::vector<pbft_round_event>> ev(C);
  if (T <= 1) {
    apply_range(r, s0, s1, st[0].data(), r->touched.data(), ev[0]);
  } else {
    std::vector<size_t> cut(C + 1, s1);
    cut[0] = s0;
    for (size_t t = 0; t < C && cut[t] < s1; ++t) {
      const uint64_t hi_row = lo + nrows * (t + 1) / C;
      size_t b = cut[t] + 1;
      while (b < s1 && (t + 1 == C || r->segs[b].row0 < hi_row || r->segs[b].key == r->segs[b - 1].key)) ++b;
      cut[t + 1] = b;
    }
    std::atomic<size_t> next{0}, done{0};
    WorkerPool::get().run_with_caller(T - 1, [&](size_t) {
      for (size_t c; (c = next.fetch_add(1, std::memory_order_relaxed)) < C;) {
        if (cut[c + 1] > cut[c]) {
          std::vector<pbft_round_event> e;  // (local: the pieces' vectors share cache lines)
          apply_range(r, cut[c], cut[c + 1], st[c].data(), r->touched.data(), e);
          ev[c] = std::move(e);
        }
        done.fetch_add(1, std::memory_order_release);
      }
    }, [&] { return done.load(std::memory_order_acquire) == C; });
  }
  for (const auto& e : ev) r->evq.insert(r->evq.end(), e.begin(), e.end());
  for (const auto& c : st) {
    r->stats.accepted += c[0];
    r->stats.rejected_sig += c[1];
    r->stats.rejected_digest += c[2];
  }
  r->seg_next = s1;
}

// the batch is done: its windows with accepted candidates are evaluated next
static void mark_dirty(pbft_replica* r) {
  for (size_t gi = 0; gi < r->seg_next; ++gi)
    if (r->touched[gi]) {
      Window* w = find_window(r, r->segs[gi].key.first, r->segs[gi].key.second);
      if (w) mark_window_dirty(r, *w);
    }
}

static void finish_batch(pbft_replica* r) {
  apply_segs(r, r->seg_next, r->segs.size());  // (windows evaluated as their last segments are applied)
  ++r->stats.batches;
  r->stats.verified += r->rows;
  r->segs.clear();
  r->seg_next = 0;
  r->in_flight = false;
  r->erased_in_flight = false;
  if (r->direct) r->arena[r->busy_arena].busy = false;
  r->direct = false;
  r->adopted = false;
}

// Copy the candidates of segments [s0, s1) into the batch: the GPU context's staged votes rows (rs =
// PBFT_VOTES_ROW_BYTES: signature, key index and envelope index side by side, include/pbft_verify.h) or the
// overrides' columns (rs = 0: SIG [N][64], K [N], IDX [N]).
// (base: the batch row SIG's first row holds -- a multi-context slice's start)
static void fill_rows(pbft_replica* r, size_t s0, size_t s1, uint8_t* SIG, uint16_t* K, uint32_t* IDX, size_t rs,
                      uint64_t base = 0) {
  for (size_t gi = s0; gi < s1; ++gi) {
    const Seg& g = r->segs[gi];
    Phase& p = g.w->ph[g.kind];
    const bool one = p.digs.size() == 1;
    if (rs) {
      uint8_t* row = SIG + rs * (g.row0 - base);
      for (uint32_t i = 0; i < g.count; ++i, row += rs)
        put_row(row, row_at(r, p.row[i]), p.who[i], g.env0 + (one ? 0 : p.dix[i]), g_stream_stores);
    } else {
      for (uint32_t i = 0; i < g.count; ++i) memcpy(SIG + 64 * (g.row0 + i), row_at(r, p.row[i]), 64);
      memcpy(K + g.row0, p.who.data(), 2 * (size_t)g.count);
      if (one) {
        std::fill(IDX + g.row0, IDX + g.row0 + g.count, g.env0);
      } else {
        for (uint32_t i = 0; i < g.count; ++i) IDX[g.row0 + i] = g.env0 + p.dix[i];
      }
    }
    p.n_flight = g.count;
    p.n_pending = 0;
  }
}
static_assert(PBFT_VOTES_ROW_ENV == PBFT_VOTES_ROW_KEY + 4 && PBFT_VOTES_ROW_BYTES == PBFT_VOTES_ROW_KEY + 8,
              "fill_rows writes key_idx, pad and env_idx as one 8-byte word");
static void fill_fence() {
#if defined(__x86_64__)
  if (g_stream_stores) _mm_sfence();
#endif
}
static void fill_envs(pbft_replica* r, size_t s0, size_t s1, uint8_t* ENV) {
  for (size_t gi = s0; gi < s1; ++gi) {
    const Seg& g = r->segs[gi];
    const Phase& p = g.w->ph[g.kind];
    for (size_t j = 0; j < p.digs.size(); ++j)
      pbft_envelope(ENV + PBFT_ENVELOPE_BYTES * (size_t)(g.env0 + j), g.kind, g.key.first, g.key.second,
                    p.digs[j].data());
  }
}
static void fill_segs(pbft_replica* r, size_t s0, size_t s1, uint8_t* SIG, uint16_t* K, uint32_t* IDX, uint8_t* ENV,
                      size_t rs) {
  fill_envs(r, s0, s1, ENV);
  fill_rows(r, s0, s1, SIG, K, IDX, rs);
  fill_fence();
}


// GPU path of a large batch: envelopes, then the rows in steps (the library's votes chunks) on T threads while this thread launches
// each step as soon as it is filled (pbft_verify_votes_submit_rows): the fill overlaps the copies and kernels.
static int fill_and_launch(pbft_replica* r, size_t T, uint8_t* SIG, uint16_t* K, uint32_t* IDX, uint8_t* ENV,
                           uint32_t E, size_t rs) {
  const size_t G = r->segs.size();
  const uint64_t N = r->rows;
  // one fill step per chunk of the library's votes schedule (PBFT_VOTES_CHUNK_END, include/pbft_verify.h)
  std::vector<uint64_t> ends;
  for (uint64_t lo = 0; lo < N; lo = PBFT_VOTES_CHUNK_END(lo, N)) ends.push_back(PBFT_VOTES_CHUNK_END(lo, N));
  const size_t W = ends.size();
  std::vector<size_t> cut(W + 1, G);  // step k = segments [cut[k], cut[k+1]): those starting below ends[k]
  cut[0] = 0;
  auto first_at = [&](uint64_t row) {
    return (size_t)(std::lower_bound(r->segs.begin(), r->segs.end(), row,
                                     [](const Seg& g, uint64_t x) { return g.row0 < x; }) - r->segs.begin());
  };
  for (size_t k = 1; k < W; ++k) cut[k] = first_at(ends[k - 1]);
  std::unique_ptr<std::atomic<uint32_t>[]> done(new std::atomic<uint32_t>[W]);
  for (size_t k = 0; k < W; ++k) done[k].store(0, std::memory_order_relaxed);
  std::atomic<uint32_t> envs_done{0};
  // the workers write the envelope table first (their share of the segments: one cache miss per window, 0.6 ms
  // on one thread), then the rows step by step; this thread opens the batch once the table is complete
  WorkerPool::get().start(T, [&](size_t t) {
      fill_envs(r, G * t / T, G * (t + 1) / T, ENV);
      envs_done.fetch_add(1, std::memory_order_release);
      for (size_t k = 0; k < W; ++k) {
        const size_t a = cut[k], b = cut[k + 1];
        if (b > a) {  // part t of the step, balanced by rows
          const uint64_t lo = r->segs[a].row0, hi = b < G ? r->segs[b].row0 : N;
          const size_t x = t == 0 ? a : std::max(a, first_at(lo + (hi - lo) * t / T));
          const size_t y = t + 1 == T ? b : std::min(b, first_at(lo + (hi - lo) * (t + 1) / T));
          if (y > x) fill_rows(r, x, y, SIG, K, IDX, rs);
        }
        fill_fence();  // (streaming stores are weakly ordered: visible before the chunk is launched)
        done[k].fetch_add(1, std::memory_order_release);
      }
  });
  while (envs_done.load(std::memory_order_acquire) < T) std::this_thread::yield();
  RTRACE(r, "envs", E);
  int rc = pbft_verify_votes_submit_begin(r->ctx, N, E, r->bitmap.data());
  RTRACE(r, "begin", N);
  for (size_t k = 0; k < W && rc == PBFT_OK; ++k) {
    while (done[k].load(std::memory_order_acquire) < T) std::this_thread::yield();
    RTRACE(r, "filled", k);
    rc = pbft_verify_votes_submit_rows(r->ctx, cut[k + 1] < G ? r->segs[cut[k + 1]].row0 : N);
    RTRACE(r, "launched", k);
  }
  WorkerPool::get().wait();  // (on failure too: every candidate is then marked in flight, as revert_segs expects)
  return rc;
}

// Multi-context batch (pbft_replica_create_multi): the segments are cut into one contiguous slice per context
// (balanced by rows, at segment boundaries; each slice 64-aligned so that no bitmap word has two writers, the gap
// padded with rows that verify as 0 and are never applied), each context stages its slice and the envelope table
// in its own pinned staging, and the fill steps go round-robin over the contexts' chunk schedules so every GPU
// starts on its first chunk at once.  Returns the contexts that opened a batch in *opened (to be drained on
// failure).
static int fill_and_launch_multi(pbft_replica* r, size_t T, uint32_t E, size_t* opened) {
  *opened = 0;
  const size_t G = r->segs.size();
  const size_t K = r->slice_lo.size() - 1;
  std::vector<size_t> sg(K + 1);  // slice k = segments [sg[k], sg[k + 1])
  {
    size_t gi = 0;
    for (size_t k = 0; k <= K; ++k) {
      while (gi < G && r->segs[gi].row0 < r->slice_lo[k]) ++gi;
      sg[k] = k == K ? G : gi;
    }
  }
  std::vector<pbft_votes_staging> st(K);
  for (size_t k = 0; k < K; ++k) {
    const uint64_t nk = r->slice_lo[k + 1] - r->slice_lo[k];
    int rc = pbft_verify_votes_stage(r->ctxs[k], nk, E, &st[k]);
    if (rc) return rc;
    // padding rows (key 0, envelope 0, zero signature: bit 0, never applied)
    const uint64_t real = r->slice_hi[k] - r->slice_lo[k];
    if (nk > real) memset(st[k].sig + (size_t)st[k].row_stride * real, 0, (size_t)st[k].row_stride * (nk - real));
  }
  // fill steps: chunk c of every context's schedule, then chunk c + 1 ...
  struct Step { size_t k, a, b; uint64_t launch_rows; };
  std::vector<Step> steps;
  {
    std::vector<std::vector<uint64_t>> ends(K);
    size_t W = 0;
    for (size_t k = 0; k < K; ++k) {
      const uint64_t nk = r->slice_lo[k + 1] - r->slice_lo[k];
      for (uint64_t lo = 0; lo < nk; lo = PBFT_VOTES_CHUNK_END(lo, nk)) ends[k].push_back(PBFT_VOTES_CHUNK_END(lo, nk));
      W = std::max(W, ends[k].size());
    }
    std::vector<size_t> next(K);
    for (size_t k = 0; k < K; ++k) next[k] = sg[k];
    for (size_t c = 0; c < W; ++c)
      for (size_t k = 0; k < K; ++k) {
        if (c >= ends[k].size()) continue;
        const uint64_t nk = r->slice_lo[k + 1] - r->slice_lo[k];
        const uint64_t end_abs = r->slice_lo[k] + ends[k][c];
        size_t b = next[k];
        if (c + 1 == ends[k].size()) b = sg[k + 1];
        else while (b < sg[k + 1] && r->segs[b].row0 < end_abs) ++b;
        const uint64_t launch = b < sg[k + 1] ? r->segs[b].row0 - r->slice_lo[k] : nk;
        steps.push_back({k, next[k], b, launch});
        next[k] = b;
      }
  }
  const size_t S = steps.size();
  std::unique_ptr<std::atomic<uint32_t>[]> done(new std::atomic<uint32_t>[S]);
  for (size_t q = 0; q < S; ++q) done[q].store(0, std::memory_order_relaxed);
  std::atomic<uint32_t> envs_done{0};
  auto first_at = [&](uint64_t row) {
    return (size_t)(std::lower_bound(r->segs.begin(), r->segs.end(), row,
                                     [](const Seg& g, uint64_t x) { return g.row0 < x; }) - r->segs.begin());
  };
  uint8_t* const env0 = st[0].envelopes;
  WorkerPool::get().start(T, [&](size_t t) {
    fill_envs(r, G * t / T, G * (t + 1) / T, env0);
    envs_done.fetch_add(1, std::memory_order_release);
    for (size_t q = 0; q < S; ++q) {
      const Step& sp = steps[q];
      if (sp.b > sp.a) {  // part t of the step, balanced by rows
        const uint64_t lo = r->segs[sp.a].row0, hi = r->segs[sp.b - 1].row0 + r->segs[sp.b - 1].count;
        const size_t x = t == 0 ? sp.a : std::max(sp.a, first_at(lo + (hi - lo) * t / T));
        const size_t y = t + 1 == T ? sp.b : std::min(sp.b, first_at(lo + (hi - lo) * (t + 1) / T));
        const size_t rs = st[sp.k].row_stride;
        // rows addressed from the slice's start: row0 - slice_lo[k] in context k's staging
        if (y > x) fill_rows(r, x, y, st[sp.k].sig, nullptr, nullptr, rs, r->slice_lo[sp.k]);
      }
      fill_fence();
      done[q].fetch_add(1, std::memory_order_release);
    }
  });
  while (envs_done.load(std::memory_order_acquire) < T) std::this_thread::yield();
  for (size_t k = 1; k < K; ++k) memcpy(st[k].envelopes, env0, (size_t)PBFT_ENVELOPE_BYTES * E);
  RTRACE(r, "envs", E);
  int rc = PBFT_OK;
  size_t failed = K;  // the context whose call failed (its batch is dropped by that call, or was never opened)
  for (size_t k = 0; k < K && rc == PBFT_OK; ++k) {
    rc = pbft_verify_votes_submit_begin(r->ctxs[k], r->slice_lo[k + 1] - r->slice_lo[k], E,
                                        r->bitmap.data() + r->slice_lo[k] / 64);
    if (rc == PBFT_OK) *opened = k + 1;
    else failed = k;
  }
  RTRACE(r, "begin", r->rows_span);
  for (size_t q = 0; q < S && rc == PBFT_OK; ++q) {
    while (done[q].load(std::memory_order_acquire) < T) std::this_thread::yield();
    rc = pbft_verify_votes_submit_rows(r->ctxs[steps[q].k], steps[q].launch_rows);
    if (rc) failed = steps[q].k;
    RTRACE(r, "launched", q);
  }
  WorkerPool::get().wait();
  if (rc) {
    // the other opened contexts' batches may still be open (not every chunk launched), and
    // pbft_verify_wait refuses an open batch -- they would stay in flight for good.  Their staging is complete now
    // (the workers have joined): launch the rest of each, so the caller's waits drain them.
    for (size_t k = 0; k < *opened; ++k)
      if (k != failed) (void)pbft_verify_votes_submit_rows(r->ctxs[k], r->slice_lo[k + 1] - r->slice_lo[k]);
  }
  return rc;
}

// Cut the batch's segments into one slice per context (balanced by rows, at segment boundaries) and renumber the
// rows so that every slice starts 64-aligned; false if fewer than two non-empty slices result.
static bool plan_slices(pbft_replica* r) {
  const size_t G = r->segs.size(), K = r->ctxs.size();
  const uint64_t N = r->rows;
  std::vector<size_t> cut{0};
  for (size_t k = 1; k < K; ++k) {
    const uint64_t target = N * k / K;
    size_t b = cut.back();
    while (b < G && r->segs[b].row0 < target) ++b;
    if (b > cut.back() && b < G) cut.push_back(b);
  }
  cut.push_back(G);
  if (cut.size() < 3) return false;
  const size_t S = cut.size() - 1;
  r->slice_lo.assign(S + 1, 0);
  r->slice_hi.assign(S, 0);
  uint64_t shift = 0;
  for (size_t k = 0; k < S; ++k) {
    const uint64_t old_lo = r->segs[cut[k]].row0;
    const uint64_t lo = k == 0 ? 0 : (old_lo + shift + 63) / 64 * 64;
    shift = lo - old_lo;
    for (size_t gi = cut[k]; gi < cut[k + 1]; ++gi) r->segs[gi].row0 += shift;
    r->slice_lo[k] = lo;
    r->slice_hi[k] = r->segs[cut[k + 1] - 1].row0 + r->segs[cut[k + 1] - 1].count;
  }
  for (size_t k = 0; k + 1 < S; ++k) r->slice_lo[k + 1] = std::max(r->slice_lo[k + 1], r->slice_hi[k]);
  r->slice_lo[S] = r->slice_hi[S - 1];
  r->rows_span = r->slice_lo[S];
  r->slice_end.assign(S, 0);
  r->slice_fin.assign(S, 0);
  return true;
}

extern "C" {

void pbft_envelope(uint8_t out[PBFT_ENVELOPE_BYTES], uint8_t kind, uint64_t view, uint64_t seq,
                   const uint8_t digest[64]) {
  memcpy(out, "PBFT", 4);
  out[4] = kind;
  for (int i = 0; i < 8; ++i) out[5 + i] = (uint8_t)(view >> (8 * i));
  for (int i = 0; i < 8; ++i) out[13 + i] = (uint8_t)(seq >> (8 * i));
  memcpy(out + 21, digest, 64);
}

int pbft_replica_create(pbft_ctx* ctx, uint32_t n, uint32_t self_id, const uint8_t* keys, pbft_replica** out) {
  return pbft_replica_create_multi(ctx ? &ctx : nullptr, ctx ? 1 : 0, n, self_id, keys, out);
}

int pbft_replica_create_multi(pbft_ctx* const* ctxs, uint32_t n_ctx, uint32_t n, uint32_t self_id,
                              const uint8_t* keys, pbft_replica** out) {
  if (!out || !keys || n < 1 || n > 65535 || self_id >= n || n_ctx > PBFT_MAX_REPLICA_CTX || (n_ctx && !ctxs))
    return PBFT_EINVAL;
  for (uint32_t k = 0; k < n_ctx; ++k) {
    if (!ctxs[k]) return PBFT_EINVAL;
    for (uint32_t j = 0; j < k; ++j)
      if (ctxs[j] == ctxs[k]) return PBFT_EINVAL;  // one batch in flight per context: distinct contexts
  }
  pbft_replica* r = new pbft_replica();
  r->ctxs.assign(ctxs, ctxs + n_ctx);
  r->ctx = n_ctx ? ctxs[0] : nullptr;
  r->n = n;
  r->f = (n - 1) / 3;
  r->self = self_id;
  r->keys.assign(keys, keys + 32 * (size_t)n);
  for (uint32_t i = 0; i < n; ++i) r->key_index.emplace(key_str(keys + 32 * (size_t)i), i);  // first index wins
  ring_reserve(r, r->log_window);
  *out = r;
  return PBFT_OK;
}

int pbft_replica_update_keys(pbft_replica* r, const uint32_t* idx, const uint8_t* A, uint32_t m, uint8_t* key_ok) {
  if (!r || (m && (!idx || !A))) return PBFT_EINVAL;
  if (r->in_flight) return PBFT_EBUSY;
  auto replaced = [&](uint32_t slot) {
    for (uint32_t j = 0; j < m; ++j)
      if (idx[j] == slot) return true;
    return false;
  };
  for (uint32_t i = 0; i < m; ++i) {
    if (idx[i] >= r->n) return PBFT_EINVAL;
    for (uint32_t j = 0; j < i; ++j)
      if (idx[j] == idx[i] || memcmp(A + 32 * (size_t)j, A + 32 * (size_t)i, 32) == 0) return PBFT_EINVAL;
    // a new key another (kept) slot already holds: one of the two would be unreachable by PeerId
    auto it = r->key_index.find(key_str(A + 32 * (size_t)i));
    if (it != r->key_index.end() && it->second != idx[i] && !replaced(it->second)) return PBFT_EINVAL;
  }
  if (r->ctx && m) {
    eu_drop(r);  // (its bits were computed under the old keys)
    // every GPU's key set, once per set (clones share one: ADVICE r05, it used to be rebuilt per context)
    std::vector<uint64_t> sets;
    int rc = PBFT_OK;
    for (size_t k = 0; k < r->ctxs.size() && rc == PBFT_OK; ++k) {
      uint64_t id = 0;
      if (pbft_verify_key_set_id(r->ctxs[k], &id) == PBFT_OK && id &&
          std::find(sets.begin(), sets.end(), id) != sets.end())
        continue;
      rc = pbft_verify_update_keys(r->ctxs[k], idx, A, m, key_ok);
      if (rc == PBFT_OK) sets.push_back(id);
    }
    if (rc) {
      // All or nothing across the replica's contexts (contexts 0..k-1 held the new keys, context
      // k the old or a cleared slot, and the PeerId map the old identity -- a vote's bit depended on its slice): the
      // updated slots are revoked on EVERY context, rebuilt or not, and keys / key_index keep the old identity, so
      // every context rejects the slots' votes until a retry installs the new keys everywhere.
      for (pbft_ctx* c : r->ctxs) (void)pbft_verify_revoke_keys(c, idx, m);
      if (key_ok) memset(key_ok, 0, m);
      return rc;
    }
  } else if (key_ok) {
    memset(key_ok, 1, m);  // (no GPU context: the installed verifier override judges the keys)
  }
  // the old keys' entries: dropped, or handed to a kept slot with the same key (replicas created with duplicates)
  for (uint32_t i = 0; i < m; ++i) {
    const std::string old = key_str(&r->keys[32 * (size_t)idx[i]]);
    auto it = r->key_index.find(old);
    if (it == r->key_index.end() || it->second != idx[i]) continue;
    r->key_index.erase(it);
    for (uint32_t j = 0; j < r->n; ++j)
      if (!replaced(j) && key_str(&r->keys[32 * (size_t)j]) == old) {
        r->key_index.emplace(old, j);
        break;
      }
  }
  for (uint32_t i = 0; i < m; ++i) {
    uint8_t* k = &r->keys[32 * (size_t)idx[i]];
    memcpy(k, A + 32 * (size_t)i, 32);
    r->key_index[key_str(k)] = idx[i];
  }
  return PBFT_OK;
}

int pbft_replica_destroy(pbft_replica* r) {
  if (!r) return PBFT_OK;
  if (r->in_flight && r->in_flight_via == 0) {
    if (!r->slice_lo.empty()) {
      for (size_t k = 0; k < r->slice_fin.size(); ++k)
        if (!r->slice_fin[k]) (void)pbft_verify_wait(r->ctxs[k]);
    } else if (r->ctx) {
      (void)pbft_verify_wait(r->ctx);
    }
  }
  if (r->in_flight && r->in_flight_via == 1 && r->vpoll)
    while (r->vpoll(r->vuser) == 0) std::this_thread::yield();
  eu_drop(r);
  for (Arena& a : r->arena) {
    host_mem_free(r, a.rows, a.rows_pinned);
    host_mem_free(r, a.envs, a.envs_pinned);
  }
  if (r->dctx) (void)pbft_verify_ctx_destroy(r->dctx);
  delete r;
  return PBFT_OK;
}

int pbft_replica_set_verifier(pbft_replica* r, pbft_batch_verify_fn fn, void* user) {
  if (!r) return PBFT_EINVAL;
  if (r->in_flight) return PBFT_EBUSY;
  eu_drop(r);
  r->verify_fn = fn;
  r->verify_user = user;
  if (fn) r->vsub = nullptr, r->vpoll = nullptr;  // the last installed verifier serves the flushes
  return PBFT_OK;
}

int pbft_replica_set_votes_verifier(pbft_replica* r, pbft_votes_submit_fn submit, pbft_votes_poll_fn poll,
                                    void* user) {
  if (!r || (!submit) != (!poll)) return PBFT_EINVAL;
  if (r->in_flight) return PBFT_EBUSY;
  eu_drop(r);
  r->vsub = submit;
  r->vpoll = poll;
  r->vuser = user;
  if (submit) r->verify_fn = nullptr;
  return PBFT_OK;
}

int pbft_replica_set_digest_fn(pbft_replica* r, pbft_digest_fn fn, void* user) {
  if (!r) return PBFT_EINVAL;
  r->digest_fn = fn;
  r->digest_user = user;
  return PBFT_OK;
}

int pbft_replica_set_log_window(pbft_replica* r, uint64_t log_window) {
  if (!r || log_window == 0 || log_window > MAX_LOG_WINDOW) return PBFT_EINVAL;
  ring_reserve(r, log_window);
  r->log_window = log_window;
  return PBFT_OK;
}

// validate_pre_prepare (src/behavior.rs:126-157) + State::insert_pre_prepare (src/state.rs:40-47);
// the signature (TODO :127) is checked by the next flush, batched with the votes.  peer_idx is the
// authenticated sender (inject_node_event's peer_id, src/behavior.rs:304, arm :310-318): only the view's
// primary may fill a window's PrePrepare candidate slots, so a relaying backup cannot crowd out the real one.
int pbft_replica_on_pre_prepare(pbft_replica* r, uint32_t peer_idx, uint64_t view, uint64_t seq, const uint8_t* op,
                                uint32_t op_len, const uint8_t claimed_digest[64], const uint8_t primary_sig[64],
                                uint8_t digest_out[64]) {
  if (!r || (!op && op_len) || !claimed_digest || !primary_sig) return PBFT_EINVAL;
  if (peer_idx != primary_of(r, view)) {  // checked before the digest: a backup's relay costs no hashing
    ++r->stats.pushed;
    ++r->stats.rejected_signer;
    return 0;
  }
  uint8_t d[64];
  int rc;
  if (r->digest_fn) {
    rc = r->digest_fn(r->digest_user, op, op_len, d);
  } else {
    if (!r->ctx) return PBFT_ENODEV;
    // on the replica's own clone of the context (its stream, the shared tables): never behind, nor in the way of,
    // the votes batch on ctx -- an early batch still open or running (the digest used to wait for it and
    // fail with its error)
    if (!r->dctx && (rc = pbft_verify_ctx_clone(r->ctx, &r->dctx)) != PBFT_OK) {
      r->dctx = nullptr;
      return rc;
    }
    const uint64_t off = 0;
    const uint8_t empty = 0;
    rc = pbft_digest_blake2b512(r->dctx, op_len ? op : &empty, &off, &op_len, 1, d);
  }
  if (rc) return rc;
  if (digest_out) memcpy(digest_out, d, 64);
  ++r->stats.pushed;
  if (memcmp(d, claimed_digest, 64) != 0) { ++r->stats.rejected_digest; return 0; }  // validate_digest :139-145
  if (view != r->current_view) { ++r->stats.rejected_view; return 0; }                // :134-141
  if (!in_log(r, seq)) { ++r->stats.rejected_watermark; return 0; }                   // h/H TODO :154
  Window& w = window_at(r, seq);
  if (w.have_pre_prepare) {                                                           // :144-151
    if (memcmp(w.digest.data(), d, 64) != 0) ++r->stats.rejected_digest; else ++r->stats.duplicates;
    return 0;
  }
  Phase& p = w.ph[0];
  const int64_t j = p.find_dig(d);
  if (j >= 0)
    for (size_t i = 0; i < p.size(); ++i)
      if (p.dix[i] == (uint32_t)j && memcmp(row_at(r, p.row[i]), primary_sig, 64) == 0) { ++r->stats.duplicates; return 0; }
  if (p.size() >= PBFT_MAX_CANDIDATES) { ++r->stats.dropped_flood; return 0; }
  Sink s = single_sink(r);
  const uint32_t prim = primary_of(r, view);
  const uint32_t env = j >= 0 && p.dgen[(size_t)j] == s.a->gen ? p.denv[(size_t)j] : sink_env(r, s, 0, view, seq, d);
  uint64_t ri;
  if (!sink_row(r, s, &ri)) { sink_done(s); return PBFT_ENOMEM; }
  put_row(s.a->rows + ROWB * ri, primary_sig, prim, env, s.nt);
  p.append(d, j, prim, s.aid << 31 | (uint32_t)ri, env, s.a->gen);
  ++s.added;
  sink_done(s);
  early_single(r);
  return 1;
}

// Counters one push updates (the replica's own, or a worker thread's share in a parallel push_many).
struct PushCounts {
  uint64_t pushed = 0, rejected_view = 0, rejected_watermark = 0, duplicates = 0, dropped_flood = 0, queued = 0;
};

// The part of a push that touches one window (State::insert_* candidates, src/state.rs:49-67): 1 queued, 0 dropped,
// PBFT_ENOMEM (no arena row).  The candidate's staged row goes to the sink's arena.
static int push_into(pbft_replica* r, Window& w, uint8_t kind, uint64_t view, uint64_t seq, const uint8_t* digest,
                     uint32_t signer, const uint8_t* sig, PushCounts& st, Sink& sk) {
  if (w.committed_reported) { ++st.duplicates; return 0; }  // late vote for a decided round
  Phase& p = w.ph[kind];
  p.init(r->n);
  if (p.acc[signer] && memcmp(p.acc_digs[p.acc[signer] - 1].data(), digest, 64) == 0) {
    ++st.duplicates;
    return 0;
  }
  const int64_t j = p.find_dig(digest);
  if (p.cnt[signer]) {
    if (j >= 0)
      for (size_t i = 0; i < p.size(); ++i)
        if (p.who[i] == signer && p.dix[i] == (uint32_t)j && memcmp(row_at(r, p.row[i]), sig, 64) == 0) {
          ++st.duplicates;
          return 0;
        }
    if (p.cnt[signer] >= PBFT_MAX_CANDIDATES) { ++st.dropped_flood; return 0; }
  }
  if (p.row.capacity() == 0) {  // one allocation per phase for the common case (every signer votes once)
    const size_t c = r->n < 1024 ? r->n : 1024;
    p.row.reserve(c); p.who.reserve(c); p.dix.reserve(c);
  }
  const uint32_t env =
      j >= 0 && p.dgen[(size_t)j] == sk.a->gen ? p.denv[(size_t)j] : sink_env(r, sk, kind, view, seq, digest);
  uint64_t ri;
  if (!sink_row(r, sk, &ri)) return PBFT_ENOMEM;
  put_row(sk.a->rows + ROWB * ri, sig, signer, env, sk.nt);
  if (!p.cnt[signer] && !p.acc[signer]) ++p.distinct;
  p.append(digest, j, signer, sk.aid << 31 | (uint32_t)ri, env, sk.a->gen);
  ++p.cnt[signer];
  ++sk.added;
  ++st.queued;
  return 1;
}

static void add_counts(pbft_replica* r, const PushCounts& c) {
  r->stats.pushed += c.pushed;
  r->stats.rejected_view += c.rejected_view;
  r->stats.rejected_watermark += c.rejected_watermark;
  r->stats.duplicates += c.duplicates;
  r->stats.dropped_flood += c.dropped_flood;
}

// inject_node_event Prepare / Commit arms (src/behavior.rs:340-412): enqueue into the round window
static inline bool eq64(const uint8_t* a, const uint8_t* b) {  // 64 bytes, branch-free
  uint64_t x = 0;
#pragma GCC unroll 8
  for (int q = 0; q < 8; ++q) {
    uint64_t u, v;
    memcpy(&u, a + 8 * q, 8);
    memcpy(&v, b + 8 * q, 8);
    x |= u ^ v;
  }
  return x == 0;
}

// The common single push in one branch-light pass (r06, VERDICT r05 item 1: the reference's ingress is one message
// per call on one thread, so the per-vote cost of this call bounds a replica's ingest): the window is the last one
// looked up or in the ring, its phase already holds exactly this digest with an envelope in the current arena, the
// signer has neither a candidate nor an accepted vote there, and the arena and the phase's columns have room.  The
// outcome is the general path's (push_into) for the same vote; anything else takes the general path.
// (flatten: the columns' push_back and the row's stores inline -- host PMU on the GPU box, r06: ~250 instructions per
// vote through this call with them as calls)
__attribute__((flatten)) static int push_fast(pbft_replica* r, uint8_t kind, uint64_t seq, const uint8_t* digest,
                                              uint32_t signer, const uint8_t* sig) {
  Window* w = r->last_w && r->last_seq == seq ? r->last_w : nullptr;
  if (!w) {
    Window* x = r->ring[seq & r->ring_mask];
    if (!x || x->seq != seq) return -1;
    r->last_seq = seq;
    r->last_w = w = x;
  }
  if (w->committed_reported) return -1;
  Phase& p = w->ph[kind];
  if (p.cnt.empty() || p.digs.size() != 1 || p.cnt[signer] || p.acc[signer] || p.row.size() == p.row.capacity() ||
      !eq64(p.digs[0].data(), digest))
    return -1;
  Arena& A = r->arena[r->cur];
  if (A.gen == 0 || A.n >= A.cap || p.dgen[0] != A.gen || (A.n > 0 && A.live.load(std::memory_order_relaxed) == 0))
    return -1;
  const uint64_t ri = A.n++;
  put_row(A.rows + ROWB * ri, sig, signer, p.denv[0], g_stream_stores);
  A.live.store(A.live.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
  p.row.push_back(r->cur << 31 | (uint32_t)ri);
  p.who.push_back((uint16_t)signer);
  p.dix.push_back(0);
  ++p.n_pending;
  if (ri + 1 > p.row_hi) p.row_hi = ri + 1;
  ++p.distinct;
  ++p.cnt[signer];
  return 1;
}

// The same common case for a push_many thread writing into its sink's reserved rows: push_into's outcome, or -1
// (then push_into decides).
__attribute__((flatten)) static int push_into_fast(Window& w, uint8_t kind, const uint8_t* digest, uint32_t signer,
                                                   const uint8_t* sig, PushCounts& st, Sink& sk) {
  if (w.committed_reported) return -1;
  Phase& p = w.ph[kind];
  if (p.cnt.empty() || p.digs.size() != 1 || p.cnt[signer] || p.acc[signer] || p.row.size() == p.row.capacity() ||
      sk.grow || sk.row >= sk.row_end || p.dgen[0] != sk.a->gen || !eq64(p.digs[0].data(), digest))
    return -1;
  const uint64_t ri = sk.row++;
  put_row(sk.a->rows + ROWB * ri, sig, signer, p.denv[0], sk.nt);
  p.row.push_back(sk.aid << 31 | (uint32_t)ri);
  p.who.push_back((uint16_t)signer);
  p.dix.push_back(0);
  ++p.n_pending;
  if (ri + 1 > p.row_hi) p.row_hi = ri + 1;
  ++p.distinct;
  ++p.cnt[signer];
  ++sk.added;
  ++st.queued;
  return 1;
}

// The single push's every case but the common one (push_fast), out of line: the common case then needs no stack
// frame for the counts and the sink (r06: ~280 instructions per vote through pbft_replica_push, host PMU).
__attribute__((noinline)) static int push_slow(pbft_replica* r, uint8_t kind, uint64_t view, uint64_t seq,
                                               const uint8_t* digest, uint32_t signer, const uint8_t* sig);

int pbft_replica_push(pbft_replica* r, uint8_t kind, uint64_t view, uint64_t seq, const uint8_t digest[64],
                      uint32_t signer, const uint8_t sig[64]) {
  if (!r || !digest || !sig || (kind != PBFT_KIND_PREPARE && kind != PBFT_KIND_COMMIT)) return PBFT_EINVAL;
  if (signer < r->n && view == r->current_view && in_log(r, seq) && push_fast(r, kind, seq, digest, signer, sig) == 1) {
    ++r->stats.pushed;
    const uint64_t n = r->arena[r->cur].n;  // (the early batch's next step is due: every piece's worth of rows)
    if (__builtin_expect(r->eu.open ? n - r->eu.rows >= early_piece_rows()
                                    : (!r->eu.active && n >= early_piece_rows() && r->peak_rows), 0))
      early_single(r);
    return 1;
  }
  return push_slow(r, kind, view, seq, digest, signer, sig);
}

static int push_slow(pbft_replica* r, uint8_t kind, uint64_t view, uint64_t seq, const uint8_t* digest,
                     uint32_t signer, const uint8_t* sig) {
  PushCounts c;
  ++c.pushed;
  int rc = 0;
  if (signer >= r->n || view != r->current_view) ++c.rejected_view;  // validate_commit :187-190
  else if (!in_log(r, seq)) ++c.rejected_watermark;
  else {
    Sink sk = single_sink(r);
    rc = push_into(r, window_at(r, seq), kind, view, seq, digest, signer, sig, c, sk);
    sink_done(sk);
    if (rc == 1) early_single(r);
  }
  add_counts(r, c);
  return rc;
}

// push_many of at least this many rows runs on the worker pool (PBFT_REPLICA_THREADS threads)
static constexpr uint64_t PUSH_PAR_MIN = 1u << 14;
// push_many keeps the worker threads on the NUMA node of the caller's input (the 149 B per vote they read; the GPU
// boxes are two-socket, and the scheduler spread the workers over both: 8 processes interleaved, r06,
// profiles/r06/replica/numa_ab/: round 3.08-3.14 ms bound against 3.03-3.50 ms, push_many 1.97-2.07 against
// 2.05-2.40); PBFT_NUMA_BIND=0 (read per call): anywhere the process may run
static void numa_bind(const void* input) {
  const char* e = getenv("PBFT_NUMA_BIND");
  WorkerPool::get().bind(e && atoi(e) == 0 ? -1 : node_of(input));
}

// push_many's early-batch pieces: rows per piece (PBFT_MANY_PIECE, 2^12..2^22, default 2^17; read per call)
static uint64_t many_piece_rows() {
  const char* e = getenv("PBFT_MANY_PIECE");
  const long long v = e ? strtoll(e, nullptr, 10) : (1 << 17);
  return (uint64_t)(v < 4096 ? 4096 : v > (1 << 22) ? (1 << 22) : v) & ~(uint64_t)63;
}
// push_many's tasks per worker thread (PBFT_PUSH_TASKS, 1..64, default 8; read per call)
static size_t push_tasks_per_thread() {
  const char* e = getenv("PBFT_PUSH_TASKS");
  const long v = e ? strtol(e, nullptr, 10) : 8;
  return (size_t)(v < 1 ? 1 : v > 64 ? 64 : v);
}

int pbft_replica_push_many(pbft_replica* r, uint64_t N, const uint8_t* kind, const uint64_t* view, const uint64_t* seq,
                           const uint8_t* digests, const uint32_t* signer, const uint8_t* sigs, uint64_t* queued) {
  if (!r || (N && (!kind || !view || !seq || !digests || !signer || !sigs))) return PBFT_EINVAL;
  // rows before the first invalid kind are pushed, then PBFT_EINVAL (as N single pushes would)
  uint64_t n_ok = 0;
  while (n_ok < N && (kind[n_ok] == PBFT_KIND_PREPARE || kind[n_ok] == PBFT_KIND_COMMIT)) ++n_ok;
  const unsigned hw = std::thread::hardware_concurrency();
  const size_t T = n_ok >= PUSH_PAR_MIN ? std::min<size_t>(hw ? hw : 1, host_threads()) : 1;
  uint64_t q = 0;
  if (T <= 1) {
    for (uint64_t i = 0; i < n_ok; ++i) {
      const int rc = pbft_replica_push(r, kind[i], view[i], seq[i], digests + 64 * i, signer[i], sigs + 64 * i);
      if (rc < 0) {
        if (queued) *queued = q;
        return rc;
      }
      q += (uint64_t)rc;
    }
  } else {
    // The windows are independent: every window's rows go to ONE thread, in input order (per-window order is
    // all the state machine depends on: the last accepted vote of a signer wins).
    //  1. (threads, by input slices) the per-row checks that need no window, and runs of consecutive rows with
    //     one (view, seq); rejected rows are flagged and do not break a run;
    struct Run { uint64_t lo, hi, seq; Window* w; uint32_t owner; uint64_t good; bool first; };
    RTRACE(r, "push", n_ok);
    numa_bind(digests);
    const uint64_t tp0 = now_ns();
    // (in 8 chunks per thread, taken dynamically: a worker the host deschedules holds up one chunk, not a
    // sixteenth of the call -- the r06 replica leg's slowest round had this pass at 4.1 ms against 0.3)
    const size_t C = T * 8;
    std::vector<std::vector<Run>> slice_runs(C);
    std::vector<uint8_t> bad(n_ok);
    std::vector<PushCounts> cnt(T);
    std::atomic<size_t> next_chunk{0}, chunks_done{0};
    std::vector<uint64_t> t_done(T, 0);
    // (T - 1 workers and this thread; a worker that has not started when the last chunk is done is not waited for)
    WorkerPool::get().run_with_caller(T - 1, [&](size_t t) {
      for (size_t ch; (ch = next_chunk.fetch_add(1, std::memory_order_relaxed)) < C;) {
        const uint64_t lo = n_ok * ch / C, hi = n_ok * (ch + 1) / C;
        std::vector<Run> runs;  // (local, stored once: the chunks' vectors share cache lines)
        // (locals: the byte stores below may alias anything, which would reload every field per row)
        const uint32_t n = r->n;
        const uint64_t cur = r->current_view, h = r->h, win = r->log_window;
        uint64_t rv = 0, rw = 0, run_seq = ~0ull, run_lo = 0, run_good = 0;
        uint8_t* bd = bad.data();
        for (uint64_t i = lo; i < hi; ++i) {
          const uint64_t q = seq[i];
          const bool v_bad = signer[i] >= n || view[i] != cur;
          const bool w_bad = !v_bad && !(q > h && q - h <= win);
          rv += v_bad;
          rw += w_bad;
          bd[i] = v_bad | w_bad;
          if (v_bad | w_bad) continue;
          if (q != run_seq) {
            if (run_seq != ~0ull) runs.push_back({run_lo, i, run_seq, nullptr, 0, run_good, false});
            run_seq = q;
            run_lo = i;
            run_good = 0;
          }
          ++run_good;
        }
        if (run_seq != ~0ull) runs.push_back({run_lo, hi, run_seq, nullptr, 0, run_good, false});
        slice_runs[ch] = std::move(runs);
        cnt[t].pushed += hi - lo;
        cnt[t].rejected_view += rv;
        cnt[t].rejected_watermark += rw;
        chunks_done.fetch_add(1, std::memory_order_release);
      }
      t_done[t] = now_ns();
    }, [&] { return chunks_done.load(std::memory_order_acquire) == C; });
    //  2. (this thread) the windows of the runs -- created here, the only window insertions -- grouped into G tasks
    //     (r06: PBFT_PUSH_TASKS per thread, default 8) by the input position of each window's first run; a task
    //     holds every run of its windows, in input order (per-window order is all the state machine depends on), and
    //     its own range of the arena: a row per row it may push, two envelopes per window whose first run it holds
    //     + 8.  The threads take the tasks in order as they free up, so a worker the host slows (a remote socket, a
    //     busy SMT sibling, an interrupt) takes fewer of them instead of holding the pass up: with one fixed range per
    //     thread, the first worker of a slow round finished in a third of the pass (push_rows_end_min_ns).
    RTRACE(r, "push_checked", T);
    const uint64_t tp1 = now_ns();
    std::vector<Run> runs;
    for (auto& v : slice_runs) runs.insert(runs.end(), v.begin(), v.end());
    const uint64_t call = ++r->push_calls;
    const size_t G = std::max<size_t>(1, std::min<size_t>(T * push_tasks_per_thread(), runs.size()));
    std::vector<uint64_t> g_rows(G, 0), g_envs(G, 8);
    for (Run& u : runs) {
      Window& w = window_at(r, u.seq);
      u.w = &w;
      u.first = w.push_call != call;
      if (u.first) {  // the window's first run in this call: its task
        w.push_call = call;
        w.push_owner = (uint32_t)(u.lo * G / n_ok);
        g_envs[w.push_owner] += 2;
      }
      u.owner = w.push_owner;
      g_rows[u.owner] += u.good;
    }
    std::vector<uint32_t> g_first(G + 1, 0), order(runs.size());  // runs by task, input order within a task
    for (const Run& u : runs) ++g_first[u.owner + 1];
    for (size_t g = 0; g < G; ++g) g_first[g + 1] += g_first[g];
    {
      std::vector<uint32_t> at(g_first.begin(), g_first.end() - 1);
      for (size_t x = 0; x < runs.size(); ++x) order[at[runs[x].owner]++] = (uint32_t)x;
    }
    Arena& A = push_arena(r);
    uint64_t rows_all = 0;
    for (size_t g = 0; g < G; ++g) rows_all += g_rows[g];
    // Early batch (r05): with GPU contexts, no batch in flight and a large call, the arena range of this call is
    // launched in pieces while the threads push (each piece's rows all written: every task below its end done;
    // every task's range starts 64-aligned, so the pieces' bitmap words are their own), so that the copies and
    // kernels of the round run under push_many instead of after flush_submit.  Rows of rejected pushes and each
    // task's padding are rows no candidate references.
    const bool early = early_enabled() && direct_enabled() && r->ctx && !r->verify_fn && !r->vsub &&
                       !r->in_flight && !r->eu.active && A.rows_pinned && A.envs_pinned &&
                       A.clean.load(std::memory_order_relaxed) && rows_all >= (1u << 17);
    std::vector<uint64_t> g_row0(G + 1), g_env0(G + 1);
    {
      uint64_t row = A.n, env = A.ne;
      for (size_t g = 0; g < G; ++g) {
        g_row0[g] = row;
        g_env0[g] = env;
        row += g_rows[g];
        if (early) row = (row + 63) & ~(uint64_t)63;
        env += g_envs[g];
      }
      g_row0[G] = row;
      g_env0[G] = env;
    }
    if (!arena_reserve(r, A, g_row0[G] - A.n, g_env0[G] - A.ne)) return PBFT_ENOMEM;  // (nothing pushed)
    // several contexts (one per GPU): context j takes tasks [tb[j], tb[j + 1]) -- balanced by rows, the first tasks
    // to the first context, whose GPU starts first -- as one batch of its own, its first piece carrying every
    // envelope written so far (its rows may name any of them)
    const size_t K = early ? std::min<size_t>(r->ctxs.size(), G) : 0;
    std::vector<size_t> tb(K + 1, G);
    std::vector<uint64_t> ctx_lo(K + 1);
    if (early) {
      tb[0] = 0;
      const uint64_t span = g_row0[G] - A.n;
      for (size_t j = 1; j < K; ++j) {
        size_t g = tb[j - 1] + 1;
        while (g < G - (K - j) && g_row0[g] - A.n < span * j / K) ++g;
        tb[j] = g;
      }
      for (size_t j = 0; j <= K; ++j) ctx_lo[j] = j == 0 ? 0 : g_row0[tb[j]];
    }
    bool launched = false;
    size_t opened = 0;
    if (early) {  // the batches are opened before the threads start: envelope 0 and the rows pushed before this call
      r->bitmap.assign((g_row0[G] + 63) / 64, 0);
      launched = true;
      for (size_t j = 0; j < K && launched; ++j) {
        launched = pbft_verify_votes_open(r->ctxs[j], ctx_lo[j + 1] - ctx_lo[j], (uint32_t)g_env0[tb[j + 1]],
                                          r->bitmap.data() + ctx_lo[j] / 64) == PBFT_OK;
        if (launched) opened = j + 1;
      }
    }
    std::unique_ptr<std::atomic<uint32_t>[]> g_done(new std::atomic<uint32_t>[G]);
    for (size_t g = 0; g < G; ++g) g_done[g].store(0, std::memory_order_relaxed);
    std::atomic<size_t> next_task{0}, tasks_done{0};
    std::vector<int64_t> added(T, 0);
    RTRACE(r, "push_windows", runs.size());
    const uint64_t tp2 = now_ns();
    //  3. (threads) every task pushes the rows of its windows in input order into its range; the range's unused
    //     rows (rejected pushes, the padding) become rows no candidate references (key 0, envelope 0), its unused
    //     envelopes copies of envelope 0
    static const uint8_t zero_sig[64] = {0};
    std::vector<uint64_t> t_beg(T, 0), t_end(T, 0);
    const std::function<void(size_t)> work = [&](size_t t) {
      t_beg[t] = now_ns();
      // (thread-local copies: the threads' entries of cnt share cache lines, and every row updates them)
      PushCounts c = cnt[t];
      int64_t add = 0;
      for (size_t g; (g = next_task.fetch_add(1, std::memory_order_relaxed)) < G;) {
        Sink sk{&A, r->cur, g_row0[g], g_row0[g] + g_rows[g], (uint32_t)g_env0[g], (uint32_t)(g_env0[g] + g_envs[g]),
                false, g_stream_stores};
        for (uint32_t x = g_first[g]; x < g_first[g + 1]; ++x) {
          const Run& u = runs[order[x]];
          for (uint64_t i = u.lo; i < u.hi; ++i)
            if (!bad[i] && push_into_fast(*u.w, kind[i], digests + 64 * i, signer[i], sigs + 64 * i, c, sk) < 0)
              push_into(r, *u.w, kind[i], view[i], seq[i], digests + 64 * i, signer[i], sigs + 64 * i, c, sk);
        }
        for (uint64_t x = sk.row; x < g_row0[g + 1]; ++x) put_row(A.rows + ROWB * x, zero_sig, 0, 0, g_stream_stores);
        for (; sk.env < sk.env_end; ++sk.env)
          memcpy(A.envs + (size_t)PBFT_ENVELOPE_BYTES * sk.env, A.envs, PBFT_ENVELOPE_BYTES);
        add += sk.added;
        if (early) {
          stream_fence();  // (streaming stores are weakly ordered: visible before the task is marked done)
          g_done[g].store(1, std::memory_order_release);
        }
        tasks_done.fetch_add(1, std::memory_order_acq_rel);
      }
      if (g_stream_stores) stream_fence();  // (drained before the join)
      cnt[t] = c;
      added[t] = add;
      t_end[t] = now_ns();
    };
    if (!early) {  // (T - 1 workers and this thread)
      WorkerPool::get().run_with_caller(T - 1, work, [&] { return tasks_done.load(std::memory_order_acquire) == G; });
    } else {  // (T workers; this thread launches the pieces)
      WorkerPool::get().start(T, work);
      // launch context j's rows in pieces of exactly `piece` rows (2^17 by default: a whole wave generation of the
      // comb at 2 waves per SIMD, as efficient per row as a 2^20 launch -- r06 trace: pieces of ~1/8 of the rows at
      // arbitrary sizes ran comb + finish 20-40 % slower), each as soon as every task below its end is done and
      // carrying the envelopes of every task done so far; the context's odd rows go FIRST, as a short piece (at the
      // end, a short piece's latency-form kernels ran beside the last full one and finished after it)
      const uint64_t piece = many_piece_rows();
      auto first_end = [&](size_t jj) {
        const uint64_t span = ctx_lo[jj + 1] - ctx_lo[jj];
        return ctx_lo[jj] + (span % piece ? span % piece : std::min(piece, span));
      };
      size_t done = 0, j = 0;
      uint64_t plo = 0;   // the context's next piece starts here (absolute row)
      uint64_t pend = K ? first_end(0) : 0;  // ... and ends here
      uint32_t elo = 0;   // ... and its new envelopes start here
      auto launch = [&](uint64_t hi, uint32_t ehi) {
        if (launched && hi > plo)
          launched = pbft_verify_votes_piece(r->ctxs[j], A.rows + ROWB * ctx_lo[j], plo - ctx_lo[j], hi - ctx_lo[j],
                                             A.envs, elo, ehi) == PBFT_OK;
        plo = hi;
        elo = ehi;
      };
      while (j < K) {
        while (done < G && g_done[done].load(std::memory_order_acquire)) ++done;
        const size_t end = std::min(done, tb[j + 1]);
        if (end == tb[j + 1]) {  // the context's rows are all written
          while (plo < ctx_lo[j + 1]) {
            const uint64_t hi = std::min(ctx_lo[j + 1], pend);
            launch(hi, (uint32_t)g_env0[end]);
            pend = hi + piece;
          }
          if (launched) launched = pbft_verify_votes_close(r->ctxs[j], ctx_lo[j + 1] - ctx_lo[j]) == PBFT_OK;
          ++j;
          elo = 0;
          if (j < K) pend = first_end(j);
          continue;
        }
        if (pend < ctx_lo[j + 1] && g_row0[end] >= pend) {
          launch(pend, (uint32_t)g_env0[end]);
          pend += piece;
          continue;
        }
        // (sleeping, not spinning, while most tasks are left: the T workers have the host's cores; the last ones
        // are waited for with pauses, so that the last piece goes out as soon as they are done)
        if (G - done > T) std::this_thread::sleep_for(std::chrono::microseconds(20));
        else for (int s = 0; s < 64; ++s) cpu_relax();
      }
      WorkerPool::get().close();  // (j == K: every task is done)
    }
    A.n = g_row0[G];
    A.ne = (uint32_t)g_env0[G];
    if (early) {
      if (launched) {
        r->eu.active = true;
        r->eu.done = false;
        r->eu.arena = r->cur;
        r->eu.rows = A.n;
        r->eu.envs = A.ne;
        r->eu.lo = ctx_lo;
      } else {
        // (a failed open, piece or close dropped that context's batch; the other opened ones are dropped -- a close
        // that does not match drops a batch still open -- or finished, and forgotten)
        for (size_t jj = 0; jj < opened; ++jj) {
          (void)pbft_verify_votes_close(r->ctxs[jj], 0);
          (void)pbft_verify_wait(r->ctxs[jj]);
        }
      }
      RTRACE(r, "early", launched);
    }
    for (int64_t a : added) A.live.fetch_add(a, std::memory_order_relaxed);
    for (const PushCounts& c : cnt) {
      add_counts(r, c);
      q += c.queued;
    }
    RTRACE(r, "push_done", q);
    r->tm.push_checks_ns = tp1 - tp0;
    r->tm.push_windows_ns = tp2 - tp1;
    r->tm.push_rows_ns = now_ns() - tp2;
    // (workers retired before they started left 0: not counted)
    auto min_set = [](const std::vector<uint64_t>& v, uint64_t t0) {
      uint64_t m = ~0ull;
      for (uint64_t x : v) if (x && x < m) m = x;
      return m == ~0ull ? 0 : m - t0;
    };
    r->tm.push_checks_end_min_ns = min_set(t_done, tp0);
    r->tm.push_rows_start_max_ns = *std::max_element(t_beg.begin(), t_beg.end()) - tp2;
    r->tm.push_rows_end_min_ns = min_set(t_end, tp2);
    if (g_push_trace && r->trace.size() >= 4) {  // PBFT_PUSH_TRACE (with PBFT_REPLICA_TRACE): pass times of this call
      auto at = [&](const char* what) {
        for (size_t x = r->trace.size(); x-- > 0;)
          if (!strcmp(r->trace[x].what, what)) return r->trace[x].ns;
        return (uint64_t)0;
      };
      fprintf(stderr, "push-trace: checks %.3f windows %.3f rows %.3f ms\n", (at("push_checked") - at("push")) / 1e6,
              (at("push_windows") - at("push_checked")) / 1e6, (at("push_done") - at("push_windows")) / 1e6);
      r->trace.clear();
    }
  }
  if (queued) *queued = q;
  return n_ok < N ? PBFT_EINVAL : PBFT_OK;
}

// Verify every READY sub-window (force: every pending candidate) in one batch, asynchronously.
static uint64_t ns_since(std::chrono::steady_clock::time_point t0) {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

// An arena batch's segments: every candidate of each in flight, each segment complete once the rows below its
// phase's last row reference are.  (r06: these walks over every window -- segments, marking, GC -- ran in chunks on
// the pool for a 0.1-ms median gain, until a worker descheduled while holding a chunk held one flush_submit for
// 3.9 ms: profiles/r06/final/; serial again.)
static void mark_arena_segs(pbft_replica* r) {
  for (Seg& g : r->segs) {
    Phase& p = g.w->ph[g.kind];
    g.row_end = p.row_hi;
    p.n_flight = g.count;
    p.n_pending = 0;
  }
}

// The batch is the current arena as it is (flush_submit_impl checked that its live candidates are exactly the
// batch's): rows [0, A.n) -- the candidates' rows, push_many's unused tails and rows of candidates that left before
// the flush, which verify and are never applied -- go to the GPU straight from the pinned arena, over every context
// in 64-aligned slices; the segments read their candidates' bits at their row references.
static int submit_arena(pbft_replica* r, uint64_t N) {
  const uint32_t a = r->cur;
  Arena& A = r->arena[a];
  const uint64_t rows = A.n;
  r->rows = N;
  r->rows_span = rows;
  r->bitmap.assign((rows + 63) / 64, 0);
  r->touched.assign(r->segs.size(), 0);
  r->seg_next = 0;
  r->slice_lo.clear();
  const size_t K = r->ctxs.size();
  int rc = PBFT_OK;
  RTRACE(r, "arena", rows);
  if (K > 1 && rows >= (1u << 16)) {
    r->slice_lo.assign(K + 1, rows);
    for (size_t k = 0; k < K; ++k) r->slice_lo[k] = (rows * k / K) & ~(uint64_t)63;
    r->slice_hi.assign(r->slice_lo.begin() + 1, r->slice_lo.end());
    r->slice_end.assign(K, 0);
    r->slice_fin.assign(K, 0);
    size_t opened = 0;
    for (size_t k = 0; k < K && rc == PBFT_OK; ++k) {
      const uint64_t lo = r->slice_lo[k], hi = r->slice_lo[k + 1];
      rc = pbft_verify_votes_submit_host(r->ctxs[k], A.rows + ROWB * lo, hi - lo, A.envs, A.ne,
                                         r->bitmap.data() + lo / 64);
      if (rc == PBFT_OK) opened = k + 1;
    }
    if (rc) {
      for (size_t k = 0; k < opened; ++k) (void)pbft_verify_wait(r->ctxs[k]);
      r->direct = false;
      revert_segs(r);
      return rc;
    }
  } else {
    rc = pbft_verify_votes_submit_host(r->ctx, A.rows, rows, A.envs, A.ne, r->bitmap.data());
    if (rc) {
      r->direct = false;
      revert_segs(r);
      return rc;
    }
  }
  RTRACE(r, "launched", K);
  // (after the launch: the copies start while this thread marks the batch's candidates)
  mark_arena_segs(r);
  A.busy = true;
  r->busy_arena = a;
  r->direct = true;
  r->cur = a ^ 1;  // (the other arena holds no candidate: restarted by the next push)
  r->in_flight = true;
  r->in_flight_via = 0;
  return PBFT_OK;
}

// The batch is the current arena as push_many's early batch already verifies it (running, or done): this flush only
// marks its candidates; r->bitmap was the early batch's output from the start.
static int adopt_early(pbft_replica* r, uint64_t N) {
  const uint32_t a = r->cur;
  Arena& A = r->arena[a];
  r->rows = N;
  r->rows_span = A.n;
  r->touched.assign(r->segs.size(), 0);
  r->seg_next = 0;
  r->slice_lo.clear();
  mark_arena_segs(r);
  if (r->eu.lo.size() > 2) {  // one slice per context (flush_poll: each context's own prefix)
    const size_t S = r->eu.lo.size() - 1;
    r->slice_lo = r->eu.lo;
    r->slice_hi.assign(r->slice_lo.begin() + 1, r->slice_lo.end());
    r->slice_end.assign(S, 0);
    r->slice_fin.assign(S, 0);
  }
  A.busy = true;
  r->busy_arena = a;
  r->direct = true;
  r->cur = a ^ 1;
  r->in_flight = true;
  r->in_flight_via = 0;
  r->eu.active = false;
  r->adopted = true;
  r->adopt_partial = [] {
    const char* e = getenv("PBFT_ADOPT_PARTIAL");
    return !e || atoi(e) != 0;
  }();
  RTRACE(r, "adopted", A.n);
  return PBFT_OK;
}

static int flush_submit_impl(pbft_replica* r, int force, uint64_t* n_rows);
int pbft_replica_flush_submit(pbft_replica* r, int force, uint64_t* n_rows) {
  if (!r) return PBFT_EINVAL;
  const auto t0 = std::chrono::steady_clock::now();
  const bool busy = r->in_flight;
  const uint64_t pieces = r->early_pieces, piece_ns = r->early_piece_ns;
  const int rc = flush_submit_impl(r, force, n_rows);
  const uint64_t dt = ns_since(t0);
  r->stats.submit_ns += dt;
  if (!busy) {  // (the phases of the batch this call launched; a PBFT_EBUSY call leaves the running one's)
    r->tm.submit_launch_ns = dt > r->tm.submit_segs_ns ? dt - r->tm.submit_segs_ns : 0;
    r->tm.early_pieces = pieces;
    r->tm.early_piece_ns = piece_ns;
    r->early_pieces = r->early_piece_ns = 0;
    r->tm.wait_ns = r->tm.apply_partial_ns = r->tm.apply_final_ns = r->tm.gc_ns = r->tm.polls = 0;
    r->t_submit_end = std::chrono::steady_clock::now();
  }
  RTRACE(r, "submit_end", rc);
  return rc;
}

static int flush_submit_impl(pbft_replica* r, int force, uint64_t* n_rows) {
  if (n_rows) *n_rows = 0;
  if (r->in_flight) return PBFT_EBUSY;
  RTRACE(r, "submit", 0);
  stream_fence();  // (single pushes write their rows with streaming stores: drained before any batch reads them)
  const uint64_t ts0 = now_ns();
  r->tm.submit_segs_ns = 0;
  r->tm.early_last_rows = 0;
  if (!r->verify_fn && !r->vsub && !r->ctx) return PBFT_ENODEV;
  // 1. one segment per ready phase: its candidates (all pending between batches) and its envelopes, one per
  //    distinct (kind, view, seq, digest)
  r->segs.clear();
  uint64_t N = 0;
  uint32_t E = 0;
  const uint64_t view = r->current_view;
  for (uint64_t q = r->h + 1; q <= r->win_hi && r->n_windows; ++q) {  // (the ring in seq order)
    Window* wp = r->ring[q & r->ring_mask];
    if (!wp || wp->seq != q) continue;
    Window& w = *wp;
    const bool rd[3] = {w.ph[0].n_pending > 0, force ? w.ph[1].n_pending > 0 : prepare_ready(r, view, w),
                        force ? w.ph[2].n_pending > 0 : commit_ready(r, w)};
    for (int kind = 0; kind < 3; ++kind) {
      if (!rd[kind]) continue;
      Phase& p = w.ph[kind];
      r->segs.push_back({&w, Key{view, q}, N, N + p.size(), (uint32_t)p.size(), E, (uint8_t)kind});
      N += p.size();
      E += (uint32_t)p.digs.size();
    }
  }
  r->rows = N;
  r->rows_span = N;
  r->slice_lo.clear();
  RTRACE(r, "segs", r->segs.size());
  r->tm.submit_segs_ns = now_ns() - ts0;
  if (n_rows) *n_rows = N;
  if (N == 0) { r->segs.clear(); return PBFT_OK; }
  r->applied_upto = 0;
  {
    // the batch is exactly the current arena's candidates: the arena goes to the GPU as it is
    Arena& A = r->arena[r->cur];
    Arena& B = r->arena[r->cur ^ 1];
    const bool direct = direct_enabled() && r->ctx && !r->verify_fn && !r->vsub && A.rows_pinned && A.envs_pinned &&
                        A.clean.load() && A.gen && B.live.load() == 0 && !B.busy &&
                        (int64_t)N == A.live.load() && A.n <= N + std::max<uint64_t>(4096, N / 16);
    if (direct) {
      r->peak_rows = std::max<uint64_t>(r->peak_rows, A.n);
      r->peak_envs = std::max<uint32_t>(r->peak_envs, A.ne);
    }
    if (r->eu.active && r->eu.open && direct && r->eu.arena == r->cur) {
      // the single pushes' early batch: its last piece (the rows and envelopes since), closed, then adopted
      int rc = PBFT_OK;
      if (A.n > r->eu.rows || A.ne > r->eu.envs)
        rc = pbft_verify_votes_piece(r->ctx, A.rows, r->eu.rows, A.n, A.envs, r->eu.envs, A.ne);
      RTRACE(r, "early_last", A.n - r->eu.rows);
      r->tm.early_last_rows = A.n - r->eu.rows;
      if (rc == PBFT_OK) rc = pbft_verify_votes_close(r->ctx, A.n);
      r->eu.open = false;
      if (rc == PBFT_OK) {
        r->eu.rows = A.n;
        r->eu.envs = A.ne;
        r->eu.lo.assign({0, A.n});
        return adopt_early(r, N);
      }
      r->eu.active = false;  // (the failing call dropped the batch: the arena goes over as it is below)
    }
    if (r->eu.active) {  // push_many's early batch: adopted when it covers exactly this arena as it is now
      if (direct && r->eu.arena == r->cur && A.n == r->eu.rows && A.ne == r->eu.envs) return adopt_early(r, N);
      eu_drop(r);
    }
    if (direct) return submit_arena(r, N);
    // (else the staging fill below; pushes during the flight go to the other arena when nothing is left in it)
    if (B.live.load() == 0 && !B.busy) r->cur ^= 1;
  }
  // several contexts (pbft_replica_create_multi) and a batch large enough for the threaded fill: one slice each
  const bool multi = r->ctxs.size() > 1 && !r->verify_fn && !r->vsub && N >= (1u << 16) && plan_slices(r);
  if (!multi) r->slice_lo.clear();
  for (Seg& g : r->segs) g.row_end = g.row0 + g.count;  // (after plan_slices moved the slices' rows)
  r->bitmap.assign((r->rows_span + 63) / 64, 0);
  // 2. fill the batch: the GPU context's pinned staging (zero-copy votes form) or the overrides' buffers; large
  //    batches with several threads (a memcpy per phase: the replica's side is memory-bound)
  int rc = PBFT_OK;
  uint8_t *SIG, *ENV;
  uint16_t* K;
  uint32_t* IDX;
  size_t rs = 0;  // staged rows' stride (0: the overrides' columns)
  if (multi) {
    const size_t G = r->segs.size();
    r->touched.assign(G, 0);
    r->seg_next = 0;
    const unsigned hw = std::thread::hardware_concurrency();
    const size_t T = std::min<size_t>(std::min<size_t>(hw ? hw : 1, host_threads()), G);
    size_t opened = 0;
    rc = fill_and_launch_multi(r, T < 1 ? 1 : T, E, &opened);
    r->in_flight_via = 0;
    if (rc) {  // drain what was opened (its kernels write this batch's bitmap), then the candidates are pending again
      for (size_t k = 0; k < opened; ++k) (void)pbft_verify_wait(r->ctxs[k]);
      revert_segs(r);
      return rc;
    }
    r->in_flight = true;
    return PBFT_OK;
  }
  if (r->verify_fn || r->vsub) {
    r->hSig.resize(64 * N); r->hK.resize(N); r->hI.resize(N);
    r->hE.assign(PBFT_ENVELOPE_BYTES * (size_t)E + 16, 0);
    SIG = r->hSig.data(); K = r->hK.data(); IDX = r->hI.data(); ENV = r->hE.data();
  } else {
    pbft_votes_staging st{};
    rc = pbft_verify_votes_stage(r->ctx, N, E, &st);
    RTRACE(r, "stage", rc);
    if (rc) { r->segs.clear(); return rc; }
    SIG = st.sig; K = st.key_idx; IDX = st.env_idx; ENV = st.envelopes;
    rs = st.row_stride;
  }
  const size_t G = r->segs.size();
  r->touched.assign(G, 0);
  r->seg_next = 0;
  const unsigned hw = std::thread::hardware_concurrency();
  const size_t T = N >= (1u << 16) ? std::min<size_t>(std::min<size_t>(hw ? hw : 1, host_threads()), G) : 1;
  if (T > 1 && !r->verify_fn && !r->vsub) {
    rc = fill_and_launch(r, T, SIG, K, IDX, ENV, E, rs);
    r->in_flight_via = 0;
    if (rc) { revert_segs(r); return rc; }
    r->in_flight = true;
    return PBFT_OK;
  }
  if (T <= 1) {
    fill_segs(r, 0, G, SIG, K, IDX, ENV, rs);
  } else {
    std::vector<size_t> cut(T + 1, G);
    cut[0] = 0;
    for (size_t t = 0; t < T; ++t) {  // balanced by rows
      const uint64_t hi_row = N * (t + 1) / T;
      size_t s1 = cut[t];
      while (s1 < G && (t + 1 == T || r->segs[s1].row0 < hi_row)) ++s1;
      cut[t + 1] = s1;
    }
    WorkerPool::get().run(T, [&](size_t t) {
      if (cut[t + 1] > cut[t]) fill_segs(r, cut[t], cut[t + 1], SIG, K, IDX, ENV, rs);
    });
  }
  // 3. launch
  if (r->verify_fn) {  // synchronous per-signature override: R, S columns and one envelope per signature
    r->hR.resize(32 * N); r->hS.resize(32 * N);
    r->hM.assign(PBFT_ENVELOPE_BYTES * N + 16, 0);  // + read slack
    for (uint64_t i = 0; i < N; ++i) {
      memcpy(&r->hR[32 * i], SIG + 64 * i, 32);
      memcpy(&r->hS[32 * i], SIG + 64 * i + 32, 32);
      memcpy(&r->hM[PBFT_ENVELOPE_BYTES * i], ENV + PBFT_ENVELOPE_BYTES * (size_t)IDX[i], PBFT_ENVELOPE_BYTES);
    }
    rc = r->verify_fn(r->verify_user, r->hR.data(), r->hS.data(), K, r->hM.data(), PBFT_ENVELOPE_BYTES,
                      PBFT_ENVELOPE_BYTES, N, r->bitmap.data());
    r->in_flight_via = 2;
  } else if (r->vsub) {
    rc = r->vsub(r->vuser, SIG, K, IDX, ENV, E, N, r->bitmap.data());
    r->in_flight_via = 1;
  } else {
    rc = pbft_verify_votes_submit(r->ctx, N, E, r->bitmap.data());
    r->in_flight_via = 0;
  }
  if (rc) { revert_segs(r); return rc; }  // nothing applied: the candidates stay pending
  r->in_flight = true;
  return PBFT_OK;
}

// 1 = no batch in flight any more (the finished one applied; events of every dirty window queued and delivered
// up to max_events -- the rest wait for the next call); 0 = still running; < 0 = the batch failed (its
// candidates are pending again).
int pbft_replica_flush_poll(pbft_replica* r, pbft_round_event* events, uint32_t max_events, uint32_t* n_events) {
  if (!r) return PBFT_EINVAL;
  if (n_events) *n_events = 0;
  if (r->in_flight) {
    int st = 1;
    uint64_t rows_done = 0;
    if (r->in_flight_via == 0 && !r->slice_lo.empty()) {
      // multi-context batch: the prefix of rows known verified -- slice by slice, each context's own prefix
      const size_t S = r->slice_end.size();
      for (size_t k = 0; k < S; ++k) {
        if (r->slice_fin[k]) continue;
        uint64_t d = 0;
        const int sk = pbft_verify_poll_rows(r->ctxs[k], &d);
        if (sk < 0) {
          for (size_t j = 0; j < S; ++j)
            if (j != k && !r->slice_fin[j]) (void)pbft_verify_wait(r->ctxs[j]);
          revert_segs(r);
          return sk;
        }
        r->slice_end[k] = r->slice_lo[k] + std::min<uint64_t>(d, r->slice_lo[k + 1] - r->slice_lo[k]);
        if (sk == 1) r->slice_fin[k] = 1, r->slice_end[k] = r->slice_lo[k + 1];
      }
      st = 1;
      rows_done = 0;
      for (size_t k = 0; k < S; ++k) {
        rows_done = r->slice_end[k];
        if (!r->slice_fin[k]) { st = 0; break; }
      }
    } else if (r->in_flight_via == 0) {
      st = pbft_verify_poll_rows(r->ctx, &rows_done);
    } else if (r->in_flight_via == 1) {
      st = r->vpoll(r->vuser);
    }
    if (st < 0) { revert_segs(r); return st; }
    const auto t0 = std::chrono::steady_clock::now();
    if (st == 0) {
      // a large batch comes back chunk by chunk: apply the segments whose rows are all in while the GPU runs on
      // (a window's segments stay in order: a prefix of the batch)
      const size_t G = r->segs.size();
      // (at least 2^16 more rows in since the last application: the pool wakes for a chunk, not per poll)
      if ((!r->adopted || r->adopt_partial) && r->seg_next < G && rows_done >= r->applied_upto + (1u << 16)) {
        RTRACE(r, "landed", rows_done);
        size_t s1 = r->seg_next;
        while (s1 < G && r->segs[s1].row_end <= rows_done) ++s1;
        if (s1 > r->seg_next) r->applied_upto = rows_done;
        apply_segs(r, r->seg_next, s1);
        r->stats.apply_ns += ns_since(t0);
        r->tm.apply_partial_ns += ns_since(t0);
        RTRACE(r, "applied", s1);
      }
      ++r->tm.polls;
      return 0;
    }
    RTRACE(r, "done", rows_done);
    r->tm.wait_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t0 - r->t_submit_end).count();
    finish_batch(r);
    RTRACE(r, "finish_batch", 0);
    r->tm.apply_final_ns = ns_since(t0);
    const auto t1 = std::chrono::steady_clock::now();
    evaluate(r);
    RTRACE(r, "evaluate", r->evq.size());
    gc(r);
    r->tm.gc_ns = ns_since(t1);
    r->stats.apply_ns += ns_since(t0);
    RTRACE(r, "gc", r->n_windows);
    if (g_trace && !r->trace.empty()) {
      const uint64_t t_0 = r->trace.front().ns;
      fprintf(stderr, "replica-trace:");
      for (const TraceEv& e : r->trace) fprintf(stderr, " %s:%llu@%.3f", e.what, (unsigned long long)e.arg, (e.ns - t_0) * 1e-6);
      fprintf(stderr, "\n");
      r->trace.clear();
    }
  } else {
    evaluate(r);
    gc(r);
  }
  drain(r, events, max_events, n_events);
  return 1;
}

// Blocking flush: poll until done, so that each chunk is applied as it lands (as the non-blocking form's caller
// does) instead of waiting for the whole batch first; the polling thread keeps its core for the first 2 ms of a
// wait and yields after that (the library's own waits do the same: pbft_verify_wait).
struct Backoff {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  uint32_t k = 0;
  void pause() {
    if ((++k & 63) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) std::this_thread::yield();
  }
};
int pbft_replica_flush(pbft_replica* r, int force, pbft_round_event* events, uint32_t max_events,
                       uint32_t* n_events) {
  if (!r) return PBFT_EINVAL;
  if (n_events) *n_events = 0;
  // a batch submitted earlier completes first (its events are queued, not lost)
  Backoff b0;
  while (r->in_flight) {
    const int p = pbft_replica_flush_poll(r, nullptr, 0, nullptr);
    if (p < 0) return p;
    if (p == 0) b0.pause();
  }
  int rc = pbft_replica_flush_submit(r, force, nullptr);
  if (rc) return rc;
  Backoff b1;
  for (;;) {
    const int p = pbft_replica_flush_poll(r, events, max_events, n_events);
    if (p != 0) return p < 0 ? p : PBFT_OK;
    b1.pause();
  }
}

int pbft_replica_in_flight(pbft_replica* r) { return r ? (r->in_flight ? 1 : 0) : PBFT_EINVAL; }

// One connection's byte stream of UviBytes/JSON frames (src/protocol_config.rs:49-69 ->
// src/handler.rs:533-548 -> inject_node_event).  peer_idx = the authenticated peer.
int pbft_replica_push_frames(pbft_replica* r, uint32_t peer_idx, const uint8_t* stream, size_t len,
                             uint64_t* consumed, uint64_t* pushed, uint64_t* dropped) {
  if (!r || !consumed || (!stream && len)) return PBFT_EINVAL;
  static thread_local char arena[1 << 16];  // unescaped strings (the PrePrepare's operation)
  uint64_t np = 0, nd = 0;
  size_t off = 0;
  int rc = 0;
  while (off < len) {
    uint64_t fl;
    size_t hn;
    const int u = pbft_uvi_decode(stream + off, len - off, &fl, &hn);
    if (u == 1) break;  // varint incomplete
    if (u != 0 || fl > PBFT_UVI_MAX_FRAME) { rc = PBFT_EINVAL; break; }
    if (len - off - hn < fl) break;  // incomplete frame: keep for the next read
    const char* js = (const char*)stream + off + hn;
    pbft_wire_msg m;
    const bool parsed = pbft_wire_decode_json(js, (size_t)fl, &m, arena, sizeof arena) == 0;
    off += hn + (size_t)fl;
    int got = 0;
    if (!parsed || !m.digest_ok || !m.has_sig) {
      got = 0;  // not a signed PBFT message (the reference would panic in serde_json .unwrap(), src/message.rs:17-18)
    } else if (m.kind == PBFT_MSG_PREPARE || m.kind == PBFT_MSG_COMMIT) {
      // the signer is the authenticated connection (src/behavior.rs:346, :380), never the frame's field
      if (m.replica != peer_idx) ++r->stats.rejected_signer;
      else got = pbft_replica_push(r, (uint8_t)m.kind, m.view, m.seq, m.digest, peer_idx, m.sig);
    } else if (m.kind == PBFT_MSG_PREPREPARE) {
      // only on the primary's own connection (the reference receives it from the primary, src/behavior.rs:89-95):
      // a relayed PrePrepare could otherwise fill the window's candidate slots ahead of the real one
      const uint32_t p = r->n ? primary_of(r, m.view) : 0;
      if (r->n == 0 || m.replica != p) ++r->stats.rejected_signer;
      else  // (on_pre_prepare rejects a connection that is not the primary's)
        got = pbft_replica_on_pre_prepare(r, peer_idx, m.view, m.seq, (const uint8_t*)m.operation, m.operation_len,
                                          m.digest, m.sig, nullptr);
    }
    if (got < 0) { rc = got; break; }
    if (got == 1) ++np; else ++nd;
  }
  *consumed = off;
  if (pushed) *pushed = np;
  if (dropped) *dropped = nd;
  return rc;
}

// One connection's stream of 160-byte binary records (include/pbft_wire.h: R || S, the 85-byte signed envelope, the
// signer's key index) -- the zero-copy alternative to the UviBytes/JSON frames above: no
// parsing, the envelope's fields are read in place.  Same rules as the frames: a vote is pushed only when its key index
// is the authenticated connection's peer; a record that is not a Prepare / Commit envelope is dropped (a PrePrepare
// needs its operation bytes: pbft_replica_on_pre_prepare or a JSON frame).
int pbft_replica_push_records(pbft_replica* r, uint32_t peer_idx, const uint8_t* stream, size_t len,
                              uint64_t* consumed, uint64_t* pushed, uint64_t* dropped) {
  if (!r || !consumed || (!stream && len)) return PBFT_EINVAL;
  const size_t n = len / PBFT_RECORD_BYTES;
  uint64_t np = 0, nd = 0;
  int rc = 0;
  size_t i = 0;
  for (; i < n; ++i) {
    const uint8_t* rec = stream + (size_t)PBFT_RECORD_BYTES * i;
    if (i + 4 < n) {  // (a read's records are consumed in order: fetch ahead of the push)
      __builtin_prefetch(rec + 4 * PBFT_RECORD_BYTES);
      __builtin_prefetch(rec + 4 * PBFT_RECORD_BYTES + 64);
      __builtin_prefetch(rec + 4 * PBFT_RECORD_BYTES + 128);
    }
    const uint8_t* env = rec + 64;
    uint16_t key;
    memcpy(&key, rec + 150, 2);
    int got = 0;
    if (memcmp(env, "PBFT", 4) != 0 || (env[4] != PBFT_KIND_PREPARE && env[4] != PBFT_KIND_COMMIT)) {
      got = 0;
    } else if (key != peer_idx) {
      ++r->stats.rejected_signer;  // (the signer is the connection, src/behavior.rs:346, :380)
    } else {
      uint64_t view, seq;
      memcpy(&view, env + 5, 8);
      memcpy(&seq, env + 13, 8);
      got = pbft_replica_push(r, env[4], view, seq, env + 21, peer_idx, rec);
    }
    if (got < 0) { rc = got; break; }
    if (got == 1) ++np; else ++nd;
  }
  *consumed = (uint64_t)PBFT_RECORD_BYTES * i;
  if (pushed) *pushed = np;
  if (dropped) *dropped = nd;
  return rc;
}

int pbft_replica_stable_checkpoint(pbft_replica* r, uint64_t seq) {
  if (!r) return PBFT_EINVAL;
  if (seq > r->h) r->h = seq;
  gc(r);
  return PBFT_OK;
}

// A GC'd seq reports prepared / committed only if THIS replica committed it locally (a stable checkpoint
// moves h without deciding anything here).
int pbft_replica_prepared(pbft_replica* r, uint64_t view, uint64_t seq) {
  if (!r) return PBFT_EINVAL;
  if (const Window* w = find_window(r, view, seq)) return is_prepared(r, view, *w) ? 1 : 0;
  return is_done(r, view, seq) ? 1 : 0;
}

int pbft_replica_committed_local(pbft_replica* r, uint64_t view, uint64_t seq) {
  if (!r) return PBFT_EINVAL;
  if (const Window* w = find_window(r, view, seq)) return is_committed_local(r, view, *w) ? 1 : 0;
  return is_done(r, view, seq) ? 1 : 0;
}

int pbft_replica_get_timings(pbft_replica* r, pbft_replica_timings* out) {
  if (!r || !out) return PBFT_EINVAL;
  *out = r->tm;
  return PBFT_OK;
}

int pbft_replica_get_stats(pbft_replica* r, pbft_replica_stats* out) {
  if (!r || !out) return PBFT_EINVAL;
  r->stats.low_watermark = r->h;
  r->stats.live_windows = r->n_windows;
  *out = r->stats;
  return PBFT_OK;
}

// ---- libp2p PeerId <-> Ed25519 key (src/main.rs:39-40; libp2p-core 0.31 identity) ----
static const uint8_t PEER_PREFIX[6] = {0x00, 0x24, 0x08, 0x01, 0x12, 0x20};

int pbft_key_from_peer_id(const uint8_t* peer_id, size_t len, uint8_t A[32]) {
  if (!peer_id || !A || len != PBFT_PEER_ID_BYTES || memcmp(peer_id, PEER_PREFIX, 6) != 0) return PBFT_EINVAL;
  memcpy(A, peer_id + 6, 32);
  return PBFT_OK;
}

void pbft_peer_id_from_key(const uint8_t A[32], uint8_t peer_id[PBFT_PEER_ID_BYTES]) {
  memcpy(peer_id, PEER_PREFIX, 6);
  memcpy(peer_id + 6, A, 32);
}

int pbft_key_from_peer_id_b58(const char* text, size_t len, uint8_t A[32]) {
  static const char ALPHA[] = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";
  if (!text || !A || len == 0 || len > 64) return PBFT_EINVAL;
  uint8_t num[64] = {0};  // big-endian accumulator
  size_t zeros = 0;
  while (zeros < len && text[zeros] == '1') ++zeros;
  for (size_t i = 0; i < len; ++i) {
    const char* p = (const char*)memchr(ALPHA, text[i], 58);
    if (!p || text[i] == '\0') return PBFT_EINVAL;
    uint32_t carry = (uint32_t)(p - ALPHA);
    for (int j = 63; j >= 0; --j) {
      carry += 58u * num[j];
      num[j] = (uint8_t)carry;
      carry >>= 8;
    }
    if (carry) return PBFT_EINVAL;  // longer than 64 bytes
  }
  size_t lead = 0;
  while (lead < 64 && num[lead] == 0) ++lead;
  const size_t body = 64 - lead, total = zeros + body;
  if (total != PBFT_PEER_ID_BYTES) return PBFT_EINVAL;
  uint8_t raw[PBFT_PEER_ID_BYTES] = {0};
  memcpy(raw + zeros, num + lead, body);
  return pbft_key_from_peer_id(raw, PBFT_PEER_ID_BYTES, A);
}

int pbft_replica_peer_index(pbft_replica* r, const uint8_t* peer_id, size_t len) {
  if (!r) return PBFT_EINVAL;
  uint8_t A[32];
  if (pbft_key_from_peer_id(peer_id, len, A) != PBFT_OK) return PBFT_EINVAL;
  auto it = r->key_index.find(key_str(A));
  return it == r->key_index.end() ? PBFT_EINVAL : (int)it->second;
}

}  // extern "C"
