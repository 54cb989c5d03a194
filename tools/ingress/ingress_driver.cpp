// BENCH INFRASTRUCTURE (not the product): the reference-shaped caller of the replica's ingress, for bench.py's
// replica_ingress_2^20 leg.  The reference receives every message on ONE thread -- the libp2p
// swarm's poll loop hands each decoded message to Pbft::inject_node_event (src/behavior.rs:304, arms :340-412) one at
// a time -- so these loops run on the calling thread only and time themselves around the calls into the product:
//   ingress_push     one pbft_replica_push per vote, in the given order (inject_node_event's Prepare / Commit arms);
//   ingress_streams  per-connection byte streams (PbftHandler -> message_to_handler_event, src/handler.rs:533-548):
//                    the loop visits the connections round-robin and hands each visit's next `per_visit` messages
//                    (UviBytes/JSON frames -> pbft_replica_push_frames, or 160-byte binary records ->
//                    pbft_replica_push_records) to the replica, the connection being the authenticated peer.
// Built by __graft_entry__.build() next to the library it links (tools/ingress/libingress.so).
#include <dlfcn.h>
#include <linux/perf_event.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/pbft_replica.h"
#include "../../include/pbft_wire.h"

static double now_s() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

// bytes of the next k whole UviBytes frames of buf[0, len) (fewer if the buffer ends first)
static size_t frames_bytes(const uint8_t* buf, size_t len, uint32_t k) {
  size_t off = 0;
  for (uint32_t i = 0; i < k && off < len; ++i) {
    uint64_t fl;
    size_t hn;
    if (pbft_uvi_decode(buf + off, len - off, &fl, &hn) != 0 || len - off - hn < fl) break;
    off += hn + (size_t)fl;
  }
  return off;
}

// Host PMU counters around the timed loop (perf_event_open, user space only; every counter 0 where the kernel
// refuses them): cycles, instructions, LLC references, LLC misses, L1D read misses, dTLB read misses.
static constexpr int N_PMU = 6;
struct Pmu {
  int fd[N_PMU];
  Pmu() {
    static const uint32_t type[N_PMU] = {PERF_TYPE_HARDWARE, PERF_TYPE_HARDWARE, PERF_TYPE_HARDWARE,
                                         PERF_TYPE_HARDWARE, PERF_TYPE_HW_CACHE, PERF_TYPE_HW_CACHE};
    static const uint64_t cfg[N_PMU] = {
        PERF_COUNT_HW_CPU_CYCLES, PERF_COUNT_HW_INSTRUCTIONS, PERF_COUNT_HW_CACHE_REFERENCES,
        PERF_COUNT_HW_CACHE_MISSES,
        PERF_COUNT_HW_CACHE_L1D | (PERF_COUNT_HW_CACHE_OP_READ << 8) | (PERF_COUNT_HW_CACHE_RESULT_MISS << 16),
        PERF_COUNT_HW_CACHE_DTLB | (PERF_COUNT_HW_CACHE_OP_READ << 8) | (PERF_COUNT_HW_CACHE_RESULT_MISS << 16)};
    for (int k = 0; k < N_PMU; ++k) {
      perf_event_attr a;
      memset(&a, 0, sizeof a);
      a.type = type[k];
      a.size = sizeof a;
      a.config = cfg[k];
      a.disabled = 1;
      a.exclude_kernel = 1;
      a.exclude_hv = 1;
      // (more events than the core has counters: the kernel time-multiplexes them -- scaled by enabled / running)
      a.read_format = PERF_FORMAT_TOTAL_TIME_ENABLED | PERF_FORMAT_TOTAL_TIME_RUNNING;
      fd[k] = (int)syscall(SYS_perf_event_open, &a, 0, -1, -1, 0);
    }
  }
  void start() {
    for (int k = 0; k < N_PMU; ++k)
      if (fd[k] >= 0) { ioctl(fd[k], PERF_EVENT_IOC_RESET, 0); ioctl(fd[k], PERF_EVENT_IOC_ENABLE, 0); }
  }
  void stop(uint64_t* out) {
    for (int k = 0; k < N_PMU; ++k) {
      uint64_t v = 0, rd[3];
      if (fd[k] >= 0) {
        ioctl(fd[k], PERF_EVENT_IOC_DISABLE, 0);
        if (read(fd[k], rd, sizeof rd) == (ssize_t)sizeof rd && rd[2] > 0)
          v = (uint64_t)((double)rd[0] * (double)rd[1] / (double)rd[2]);
      }
      if (out) out[k] = v;
    }
  }
  ~Pmu() {
    for (int k = 0; k < N_PMU; ++k)
      if (fd[k] >= 0) close(fd[k]);
  }
};

// PBFT_INGRESS_PROFILE=file: a sampling profile of the calling thread around each timed loop (perf_event_open,
// PERF_SAMPLE_IP every 20,000 user-space cycles, a 4-MiB ring read once at the end), appended to `file` as lines
// "count module offset" (tools/ingress_profile.py symbolizes them with llvm-symbolizer).
struct Sampler {
  int fd = -1;
  uint8_t* ring = nullptr;
  size_t pages = 1024, page = 4096;
  const char* out = getenv("PBFT_INGRESS_PROFILE");
  const char* tag;
  explicit Sampler(const char* t) : tag(t) {
    if (!out) return;
    perf_event_attr a;
    memset(&a, 0, sizeof a);
    a.size = sizeof a;
    a.type = PERF_TYPE_HARDWARE;
    a.config = PERF_COUNT_HW_CPU_CYCLES;
    a.sample_period = 20000;
    a.sample_type = PERF_SAMPLE_IP;
    a.exclude_kernel = 1;
    a.exclude_hv = 1;
    a.disabled = 1;
    fd = (int)syscall(SYS_perf_event_open, &a, 0, -1, -1, 0);
    if (fd < 0) return;
    page = (size_t)sysconf(_SC_PAGESIZE);
    void* m = mmap(nullptr, (pages + 1) * page, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) { close(fd); fd = -1; return; }
    ring = (uint8_t*)m;
    ioctl(fd, PERF_EVENT_IOC_RESET, 0);
    ioctl(fd, PERF_EVENT_IOC_ENABLE, 0);
  }
  ~Sampler() {
    if (fd < 0) return;
    ioctl(fd, PERF_EVENT_IOC_DISABLE, 0);
    const perf_event_mmap_page* hdr = (const perf_event_mmap_page*)ring;
    const uint64_t head = __atomic_load_n(&hdr->data_head, __ATOMIC_ACQUIRE), size = pages * page;
    const uint8_t* data = ring + page;
    std::map<std::pair<std::string, uint64_t>, uint64_t> hist;
    uint64_t lost = 0, n = 0;
    for (uint64_t pos = head > size ? head - size : 0; pos + sizeof(perf_event_header) <= head;) {
      perf_event_header h;
      for (size_t b = 0; b < sizeof h; ++b) ((uint8_t*)&h)[b] = data[(pos + b) % size];
      if (h.size == 0) break;
      if (h.type == PERF_RECORD_SAMPLE) {
        uint64_t ip = 0;
        for (size_t b = 0; b < 8; ++b) ((uint8_t*)&ip)[b] = data[(pos + sizeof h + b) % size];
        Dl_info di;
        if (dladdr((void*)ip, &di) && di.dli_fname) ++hist[{di.dli_fname, ip - (uint64_t)di.dli_fbase}];
        else ++hist[{"?", ip}];
        ++n;
      } else if (h.type == PERF_RECORD_LOST) {
        ++lost;
      }
      pos += h.size;
    }
    FILE* f = fopen(out, "a");
    if (f) {
      fprintf(f, "# %s: %llu samples, %llu lost records\n", tag, (unsigned long long)n, (unsigned long long)lost);
      for (const auto& kv : hist)
        fprintf(f, "%llu %s 0x%llx\n", (unsigned long long)kv.second, kv.first.first.c_str(),
                (unsigned long long)kv.first.second);
      fclose(f);
    }
    munmap(ring, (pages + 1) * page);
    close(fd);
  }
};

extern "C" {

int ingress_pmu_counters() { return N_PMU; }

int ingress_push(pbft_replica* r, uint64_t N, const uint8_t* kind, const uint64_t* view, const uint64_t* seq,
                 const uint8_t* digests, const uint32_t* signer, const uint8_t* sigs, uint64_t* queued,
                 double* seconds, uint64_t* pmu) {
  uint64_t q = 0;
  int rc = 0;
  Sampler prof("push");
  Pmu P;
  P.start();
  const double t0 = now_s();
  for (uint64_t i = 0; i < N; ++i) {
    const int p = pbft_replica_push(r, kind[i], view[i], seq[i], digests + 64 * i, signer[i], sigs + 64 * i);
    if (p < 0) { rc = p; break; }
    q += (uint64_t)p;
  }
  *seconds = now_s() - t0;
  P.stop(pmu);
  *queued = q;
  return rc;
}

int ingress_streams(pbft_replica* r, int binary, uint32_t n_conn, const uint8_t* const* streams,
                    const uint64_t* lens, uint32_t per_visit, uint64_t* pushed, uint64_t* dropped, uint64_t* calls,
                    double* seconds, uint64_t* pmu) {
  std::vector<uint64_t> off(n_conn, 0);
  uint64_t np = 0, nd = 0, nc = 0;
  int rc = 0;
  char tag[32];
  snprintf(tag, sizeof tag, "%s_%u", binary ? "records" : "json", per_visit);
  Sampler prof(tag);
  Pmu P;
  P.start();
  const double t0 = now_s();
  for (bool more = true; more && rc == 0;) {
    more = false;
    for (uint32_t c = 0; c < n_conn && rc == 0; ++c) {
      const uint64_t left = lens[c] - off[c];
      if (!left) continue;
      const uint8_t* p = streams[c] + off[c];
      const size_t n = binary ? (size_t)(left < (uint64_t)PBFT_RECORD_BYTES * per_visit ? left
                                                                                     : (uint64_t)PBFT_RECORD_BYTES * per_visit)
                              : frames_bytes(p, left, per_visit);
      uint64_t used = 0, a = 0, b = 0;
      rc = binary ? pbft_replica_push_records(r, c, p, n, &used, &a, &b)
                  : pbft_replica_push_frames(r, c, p, n, &used, &a, &b);
      ++nc;
      if (rc == 0 && used == 0) rc = PBFT_EINVAL;  // (a stream that makes no progress: malformed)
      off[c] += used;
      np += a;
      nd += b;
      more = more || off[c] < lens[c];
    }
  }
  *seconds = now_s() - t0;
  P.stop(pmu);
  *pushed = np;
  *dropped = nd;
  *calls = nc;
  return rc;
}

// The JSON frames decoded only (pbft_wire_decode_json per frame, no replica), visited as ingress_streams visits
// them: the parse's share of the json modes' instructions per vote.
int ingress_decode_only(uint32_t n_conn, const uint8_t* const* streams, const uint64_t* lens, uint32_t per_visit,
                        uint64_t* frames, double* seconds, uint64_t* pmu) {
  std::vector<uint64_t> off(n_conn, 0);
  static thread_local char arena[1 << 16];
  uint64_t nf = 0;
  int rc = 0;
  Pmu P;
  P.start();
  const double t0 = now_s();
  for (bool more = true; more && rc == 0;) {
    more = false;
    for (uint32_t c = 0; c < n_conn && rc == 0; ++c) {
      for (uint32_t k = 0; k < per_visit && off[c] < lens[c]; ++k) {
        uint64_t fl;
        size_t hn;
        const uint8_t* p = streams[c] + off[c];
        if (pbft_uvi_decode(p, lens[c] - off[c], &fl, &hn) != 0) { rc = PBFT_EINVAL; break; }
        pbft_wire_msg m;
        if (pbft_wire_decode_json((const char*)p + hn, (size_t)fl, &m, arena, sizeof arena) != 0 || !m.has_sig) {
          rc = PBFT_EINVAL;
          break;
        }
        off[c] += hn + (size_t)fl;
        ++nf;
      }
      more = more || off[c] < lens[c];
    }
  }
  *seconds = now_s() - t0;
  P.stop(pmu);
  *frames = nf;
  return rc;
}

}  // extern "C"
