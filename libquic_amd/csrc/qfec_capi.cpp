// qfec_capi.cpp — the C-ABI (include/qfec.h): context, argument validation,
// error mapping, the host-pointer (pinned, chunked, overlapped) path and the
// dispatch to the gfx950 kernels in qfec_kernels.hip.
//
// Error behaviour mirrors QuicFramer: a bool-style failure with a QuicErrorCode
// and a detailed string (quic_framer.cc:1128-1135 set_detailed_error +
// RaiseError); QUIC_BUG (quic_bug_tracker.h:10-11) is never used — nothing
// aborts.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/qfec.h"
#include "qfec_internal.h"
#include "quic_fec_wire.h"

namespace {

thread_local char g_tls_error[512] = "";

constexpr int kSlots = 3;                         // host path pipeline depth
constexpr size_t kStageBytes = 64ull << 20;       // per-slot input staging
constexpr uint64_t kDirectGroups = 256;  // mapped batches up to this size: no staging copies
// A slot's completion word sits on a 64-B line of its own (h_flag[slot *
// kFlagStride]), followed by the encode lengths of a direct batch of up to
// kFlagPlens groups: the completion reads the token and the lengths in one
// cache-line transfer instead of two (the lengths otherwise land in h_out)
constexpr uint32_t kFlagStride = 16;
constexpr uint64_t kFlagPlens = 30;
// Device error words (kernel-latched error bits), one per kind of work so
// that collecting one never reads or clears another's: the
// context stream's device-pointer calls, each staging slot's QFEC_ASYNC op,
// and the synchronous host-pointer paths.
constexpr int kErrStream = 0;
constexpr int kErrSlot0 = 1;  // + slot index
constexpr int kErrHost = kErrSlot0 + kSlots;
constexpr int kErrWords = kErrHost + 1;

struct Slot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* d_in = nullptr;   // device input staging
  uint8_t* d_aux = nullptr;  // device parity-in / missing staging
  uint8_t* d_out = nullptr;  // device output staging
  uint8_t* h_in = nullptr;   // pinned input bounce buffer (device-mapped)
  uint8_t* h_aux = nullptr;
  uint8_t* h_out = nullptr;
  uint8_t* h_in_dev = nullptr;  // the same pinned buffers as the device addresses them
  uint8_t* h_aux_dev = nullptr;
  uint8_t* h_out_dev = nullptr;
  bool busy = false;
};

}  // namespace

constexpr size_t kPhaseSyncBytes = 20 * 256;

struct qfec_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  uint32_t* d_err = nullptr;  // kErrWords words
  uint32_t* h_err = nullptr;  // pinned, kErrWords words
  char last_error[512] = "";
  Slot slots[kSlots];
  bool staging_ready = false;
  // small-batch completion (launch_ragged_latency): per-slot device block
  // counters and host-mapped flags the kernel's last workgroup stores to
  uint32_t* d_done = nullptr;
  // sync words of the phased fixed-shape kernel (20 x 256 B; words 0-18 zero
  // between launches, word 19 counts abandoned launches)
  uint32_t* d_phase = nullptr;
  // phased launches of this context share d_phase, so they must not overlap:
  // after each one phase_done is recorded on its stream, and a phased launch
  // on another stream first waits for it
  hipEvent_t phase_done = nullptr;
  hipStream_t phase_stream = nullptr;
  bool phase_recorded = false;
  // contention policy: the last workgroup of a phased launch copies the
  // abandoned-launch count into h_phase (pinned, mapped); a launch that finds
  // it grown (another context / process kept CUs busy) runs the
  // next kPhaseBackoff large batches with the one-pass kernel, then tries the
  // phased one again
  uint32_t* h_phase = nullptr;
  uint32_t* h_phase_dev = nullptr;
  uint32_t phase_seen = 0;
  uint32_t phase_backoff = 0;
  int last_fixed_phased = -1;  // the last device fixed-shape launch: 1 phased, 0 one-pass
  uint32_t last_phase_grid = 0;  // ... its phased grid (workgroups), 0 one-pass
  uint32_t ncu = 0;          // CU count, queried once
  uint32_t phase_extra = 0;  // test hook (qfec_debug_phase)
  uint32_t phase_min = 0;    // test hook (qfec_debug_phase_min)
  uint32_t no_regsteps = 0;  // test hook (qfec_debug_phase_regsteps)
  uint32_t rt_batch = 0;     // test hook (qfec_debug_phase_rtbatch)
  uint32_t phase_reserve = 0;  // test hook (qfec_debug_phase_reserve)
  bool debug_fail = false;   // test hook (qfec_debug_fail_launches)
  uint32_t* h_flag = nullptr;
  uint32_t* h_flag_dev = nullptr;
  uint32_t flag_token = 0;
  // QFEC_ASYNC mapped ragged calls still running, one per staging slot
  // (qfec_complete finishes them in issue order)
  struct AsyncOp {
    bool live = false;
    bool direct = false;   // completion by the host-mapped flag (token)
    bool svc = false;      // ... set by the small-batch service (no event)
    bool recover = false;
    uint32_t token = 0;
    uint64_t cnt = 0;
    uint16_t* parity_len_out = nullptr;  // encode: the caller's lengths, filled at completion
    uint64_t seq = 0;                    // its ticket (qfec_async_ticket)
  } async_ops[kSlots];
  int async_next = 0;
  uint64_t async_seq = 0;
  uint64_t last_ticket = 0;  // of the last ragged mapped call, 0 if it ran synchronously
  // results of async ops finished by a call other than their owner's (a slot
  // reused, a synchronous call draining the slots, qfec_complete), kept for
  // qfec_complete_ticket: each op's code reaches its own ticket's caller.
  // A ring indexed by ticket (a std::map of every op's code, OK
  // ones included, was walked by every qfec_complete -- thousands of node
  // hops per call at the 4096 cap): insert, claim and overwrite are O(1) and
  // allocate nothing; a ticket 4096 newer takes the oldest's place.
  static constexpr uint32_t kKept = 4096;
  struct Kept {
    uint64_t ticket = 0;  // 0: empty / claimed
    int code = QFEC_OK;
  } kept[kKept];
  // the first code of an op finished by another call that qfec_complete has
  // not reported yet (it reports each such code once; OK codes need none)
  int unreported = QFEC_OK;
  // small-batch service (qfec_internal.h SvcJob): a resident worker on a
  // stream of its own takes mapped async batches of <= kSvcGroups groups from
  // a ring in host-mapped memory -- no kernel launch per batch
  hipStream_t svc_stream = nullptr;
  qfec::SvcShared* svc_sh = nullptr;  // host-mapped control words
  qfec::SvcShared* svc_sh_dev = nullptr;
  qfec::SvcJob* svc_ring = nullptr;   // host-mapped job ring
  qfec::SvcJob* svc_ring_dev = nullptr;
  qfec::SvcDev* svc_dev = nullptr;  // the workers' device-memory words
  uint32_t svc_epoch = 0;           // launches of the worker (its leader's tag)
  uint64_t svc_published = 0;
  uint32_t svc_seq = 0;
  uint64_t svc_launches = 0;
  uint64_t svc_rotations = 0;  // workers stopped for their residency bound (svc_submit)
  bool svc_on = true;  // test hook qfec_debug_service
  uint64_t svc_used_ns = 0;  // steady clock of the last service job / warm (other_service_cus)
  uint64_t svc_launch_ns = 0;  // steady clock of the worker's last launch (kSvcMaxResidentNs)
  uint64_t svc_max_resident_ns;  // the residency bound (kSvcMaxResidentNs; test hook)
  uint64_t svc_idle_ticks;       // the worker's idle time (kSvcIdleTicks; test hook)
  // measurement hook (stamps on): the last service call's host stamps, steady
  // ns: entry, published, token seen, return (qfec_debug_service_trace)
  uint64_t svc_hst[4] = {0, 0, 0, 0};
  bool svc_poison_next = false;  // test hook: the next job's ring entry malformed
  // device scratch of the host-pointer xor / protection / entropy calls:
  // grow-only buffers kept for the context's life (no allocation per call)
  std::vector<void*> scratch_p;
  std::vector<size_t> scratch_n;
};

namespace {

int fail(qfec_ctx* ctx, int code, const char* fmt, ...) {
  char* buf = ctx ? ctx->last_error : g_tls_error;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, 512, fmt, ap);
  va_end(ap);
  return code;
}

#define QFEC_HIP(ctx, expr)                                                         \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess)                                                           \
      return fail((ctx), QFEC_ERR_INTERNAL, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

// The calling thread's current device made ctx's, before anything that
// allocates or launches.  (hipGetDevice reads it, ~50 ns; the set only when it
// differs.)  The connection thread's per-turn calls skip it where they touch
// only the context's own streams, events and host-mapped words -- completion
// polls, a warm call that finds the worker running, a small batch handed to
// the running worker (round 6: five binds a loop turn were ~0.2 us per group
// at one connection) -- and bind on their slow paths (first allocations,
// (re)launches, staged copies, error collection).
int bind(qfec_ctx* ctx) {
  if (!ctx) return fail(nullptr, QFEC_ERR_INTERNAL, "null qfec_ctx");
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != ctx->device)
    QFEC_HIP(ctx, hipSetDevice(ctx->device));
  return QFEC_OK;
}

// Ranges this library mapped itself (qfec_host_alloc, qfec_host_register):
// QFEC_PTR_MAPPED's pointer check answers from them without
// hipPointerGetAttributes (a runtime lookup under its lock) -- the connection
// batcher's launches hand over payload-arena slabs, every one of them from
// qfec_host_alloc.  A thread keeps the last range it matched; any free /
// unregister bumps the generation, which drops every thread's copy.
struct MappedRanges {
  std::mutex mu;
  std::vector<std::pair<uintptr_t, size_t>> r;  // [base, base + size)
  std::atomic<uint64_t> gen{1};
};
MappedRanges& mapped_ranges() {
  static MappedRanges* m = new MappedRanges();  // never destroyed (frees at exit)
  return *m;
}
void note_mapped(const void* p, size_t n) {
  MappedRanges& m = mapped_ranges();
  std::lock_guard<std::mutex> g(m.mu);
  m.r.emplace_back(reinterpret_cast<uintptr_t>(p), n);
}
void forget_mapped(const void* p) {
  MappedRanges& m = mapped_ranges();
  std::lock_guard<std::mutex> g(m.mu);
  const uintptr_t b = reinterpret_cast<uintptr_t>(p);
  m.r.erase(std::remove_if(m.r.begin(), m.r.end(),
                           [b](const std::pair<uintptr_t, size_t>& e) { return e.first == b; }),
            m.r.end());
  m.gen.fetch_add(1, std::memory_order_acq_rel);
}
bool known_mapped(const void* p) {
  struct Hit {
    uint64_t gen = 0;
    uintptr_t base = 0;
    size_t n = 0;
  };
  static thread_local Hit hit;
  MappedRanges& m = mapped_ranges();
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  if (hit.gen == m.gen.load(std::memory_order_acquire) && a - hit.base < hit.n) return true;
  std::lock_guard<std::mutex> g(m.mu);
  for (const auto& e : m.r)
    if (a - e.first < e.second) {
      hit = Hit{m.gen.load(std::memory_order_relaxed), e.first, e.second};
      return true;
    }
  return false;
}

bool is_pinned_or_device(const void* p) {
  if (known_mapped(p)) return true;
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeHost || attr.type == hipMemoryTypeDevice ||
         attr.type == hipMemoryTypeManaged;
}

int ensure_staging(qfec_ctx* ctx) {
  if (ctx->staging_ready) return QFEC_OK;
  int rc = bind(ctx);
  if (rc) return rc;
  for (auto& s : ctx->slots) {
    QFEC_HIP(ctx, hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    QFEC_HIP(ctx, hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    QFEC_HIP(ctx, hipMalloc(&s.d_in, kStageBytes));
    QFEC_HIP(ctx, hipMalloc(&s.d_aux, kStageBytes / 8));
    QFEC_HIP(ctx, hipMalloc(&s.d_out, kStageBytes / 4));
    const unsigned fl = hipHostMallocMapped | hipHostMallocPortable;
    QFEC_HIP(ctx, hipHostMalloc(&s.h_in, kStageBytes, fl));
    QFEC_HIP(ctx, hipHostMalloc(&s.h_aux, kStageBytes / 8, fl));
    QFEC_HIP(ctx, hipHostMalloc(&s.h_out, kStageBytes / 4, fl));
    QFEC_HIP(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&s.h_in_dev), s.h_in, 0));
    QFEC_HIP(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&s.h_aux_dev), s.h_aux, 0));
    QFEC_HIP(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&s.h_out_dev), s.h_out, 0));
  }
  QFEC_HIP(ctx, hipMalloc(&ctx->d_done, kSlots * sizeof(uint32_t)));
  QFEC_HIP(ctx, hipMemset(ctx->d_done, 0, kSlots * sizeof(uint32_t)));
  QFEC_HIP(ctx, hipHostMalloc(&ctx->h_flag, kSlots * kFlagStride * sizeof(uint32_t),
                              hipHostMallocMapped | hipHostMallocPortable));
  std::memset(ctx->h_flag, 0, kSlots * kFlagStride * sizeof(uint32_t));
  QFEC_HIP(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->h_flag_dev), ctx->h_flag, 0));
  ctx->staging_ready = true;
  return QFEC_OK;
}

// ---- small-batch service ---------------------------------------------------
// batches up to this size use it (round 5: 64, with the tables inline in the
// ring entry; round 4: 16)
constexpr uint64_t kSvcGroups = 64;
// idle time before the worker leaves: 100 us (100-MHz wall clock) -- below the
// phased kernel's 200-us meeting timeout, so a worker of another context never
// makes a phased launch give up its meetings; a flush loop that comes back
// within it finds the worker resident
constexpr uint64_t kSvcIdleTicks = 10000;

// Process-wide registry of the contexts that run a small-batch service
// (VERDICT r5 item 3): a phased launch on one context leaves the CUs of the
// OTHER contexts' workers on its device out of its grid.  A worker is kSvcWgs
// workgroups of 512 lanes at 252 VGPRs and 57 KiB of LDS: each holds a CU
// whose LDS a phased workgroup (160 KiB) can no longer get, so a full
// one-per-CU grid would not be resident and its meetings would time out
// (round 5: 0.6-0.7x, abandoned).  The model is the reference's: one
// connection thread per QuicConnection (quic_connection.h:14), here one
// context per thread, several per process.
// A context counts while its worker is resident or queued, AND for
// kSvcRecentNs after its last service job or warm: a worker that its
// connection thread relaunches while the phased grid is being dispatched
// would otherwise take CUs the grid was sized for (measured on the box: one
// launch in four abandoned when only resident workers were counted,
// profiles/round6/pytest_service_r6a_registry_resident_only.log).  A context
// whose service has been quiet that long is not counted: leaving 8 of 256 CUs
// out costs the phased kernel 1.4% (encode 0.804 -> 0.793,
// profiles/round6/phase_reserve_ab_r6d.txt).
constexpr uint64_t kSvcRecentNs = 2000000;  // 2 ms: 20x the worker's idle time
std::mutex g_svc_mu;
std::vector<qfec_ctx*> g_svc_ctxs;

uint64_t steady_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// why: bit 0 recent use, bit 1 alive, bit 2 stream busy (OR over the contexts
// counted; the test hook qfec_debug_other_service_cus)
uint32_t other_service_cus(const qfec_ctx* ctx, uint32_t* why = nullptr) {
  const uint64_t now = steady_ns();
  std::lock_guard<std::mutex> lock(g_svc_mu);
  uint32_t n = 0, w = 0;
  for (const qfec_ctx* c : g_svc_ctxs) {
    if (c == ctx || c->device != ctx->device || !c->svc_sh) continue;
    const uint32_t r =
        (__atomic_load_n(&c->svc_on, __ATOMIC_ACQUIRE) &&
                 now - __atomic_load_n(&c->svc_used_ns, __ATOMIC_ACQUIRE) < kSvcRecentNs
             ? 1u
             : 0u) |
        (__atomic_load_n(&c->svc_sh->alive, __ATOMIC_ACQUIRE) != 0u ? 2u : 0u) |
        (hipStreamQuery(c->svc_stream) == hipErrorNotReady ? 4u : 0u);
    if (r) n += qfec::kSvcWgs;
    w |= r;
  }
  if (why) *why = w;
  return n;
}

int ensure_service(qfec_ctx* ctx) {
  if (ctx->svc_stream) return QFEC_OK;
  int rc = bind(ctx);
  if (rc) return rc;
  const unsigned fl = hipHostMallocMapped | hipHostMallocPortable;
  QFEC_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->svc_sh), sizeof(qfec::SvcShared), fl));
  std::memset(static_cast<void*>(ctx->svc_sh), 0, sizeof(qfec::SvcShared));
  QFEC_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->svc_ring),
                              qfec::kSvcRing * sizeof(qfec::SvcJob), fl));
  std::memset(static_cast<void*>(ctx->svc_ring), 0, qfec::kSvcRing * sizeof(qfec::SvcJob));
  for (uint32_t i = 0; i < qfec::kSvcRing; ++i) ctx->svc_ring[i].seq = 0xFFFFFFFFu;  // none yet
  QFEC_HIP(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->svc_sh_dev), ctx->svc_sh, 0));
  QFEC_HIP(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->svc_ring_dev), ctx->svc_ring, 0));
  QFEC_HIP(ctx, hipMalloc(reinterpret_cast<void**>(&ctx->svc_dev), sizeof(qfec::SvcDev)));
  // (The runtime multiplexes a process's streams onto 4 hardware queues;
  // work on a stream that shares the worker's queue waits behind the
  // resident worker: svc_submit bounds its residency, kSvcMaxResidentNs.  A
  // greatest-priority stream instead -- its own pool of queues -- made every
  // phased launch of another context beside a fed worker abandon its
  // meetings: measured and not kept, profiles/round6/pytest_r6j.log.)
  QFEC_HIP(ctx, hipStreamCreateWithFlags(&ctx->svc_stream, hipStreamNonBlocking));
  // zeroed on the worker's own stream (a non-blocking stream is not ordered
  // after the null stream's memset)
  QFEC_HIP(ctx, hipMemsetAsync(ctx->svc_dev, 0, sizeof(qfec::SvcDev), ctx->svc_stream));
  QFEC_HIP(ctx, hipStreamSynchronize(ctx->svc_stream));
  {
    std::lock_guard<std::mutex> lock(g_svc_mu);
    g_svc_ctxs.push_back(ctx);
  }
  return QFEC_OK;
}

// The ring entry the next job goes into (its tables are written straight
// into entry->tab by the caller, then svc_submit publishes it).  The entry of
// job seq - kSvcRing is free: at most kSlots jobs are outstanding (each holds
// a slot until completed) and kSvcRing > kSlots.
qfec::SvcJob* svc_next_entry(qfec_ctx* ctx) {
  static_assert(qfec::kSvcRing > kSlots, "service ring smaller than the slots");
  return &ctx->svc_ring[ctx->svc_seq % qfec::kSvcRing];
}

// Queue batch `a` (payload pointers; its index tables already inline in
// svc_next_entry(ctx)->tab at the offsets given) as one job; its completion
// is token in the slot's flag.  Publishes, then relaunches the worker if it
// has left (or never ran).
struct SvcTabs {
  uint32_t bytes, off, len, ptr, poff, plen, miss, ooff;
};
// Bounded residency (round 6): the runtime multiplexes a process's streams
// onto 4 hardware queues, and work on any stream that shares the worker's
// queue waits behind the resident worker -- for as long as a connection
// thread keeps it fed (measured: another context's phased launch stalled for
// seconds, once for good, beside a worker fed back to back).  So a worker
// that has been resident this long is rotated at the next job: told to leave
// between turns, a successor queued behind whatever the hardware queue took
// meanwhile -- a wait of at most ~2 ms for the other work, one relaunch per
// 2 ms for the service, and no wait on the connection thread.
constexpr uint64_t kSvcMaxResidentNs = 2000000;
// a job of more groups is split over the worker's workgroups (the leader's
// waves take up to this many: qfec_kernels.hip kSvcWaves)
constexpr uint64_t kSvcSplitGroups = 8;
void svc_abandon(qfec_ctx* ctx);

int svc_submit(qfec_ctx* ctx, int slot, const qfec::RaggedArgs& a, bool recover, uint32_t token,
               const SvcTabs& tb) {
  int rc = ensure_service(ctx);
  if (rc) return rc;
  const uint64_t now = steady_ns();
  __atomic_store_n(&ctx->svc_used_ns, now, __ATOMIC_RELEASE);
  qfec::SvcShared* sh = ctx->svc_sh;
  // Not while a split job is outstanding: its followers may still be
  // waiting for CUs (dispatched behind another kernel), the old kernel
  // cannot end before they have done their shares, and its successor -- with
  // every later job -- would wait behind them too.
  bool split_pending = false;
  for (const auto& op : ctx->async_ops)
    split_pending = split_pending || (op.live && op.svc && op.cnt > kSvcSplitGroups);
  if (!split_pending && ctx->svc_launch_ns != 0 &&
      now - ctx->svc_launch_ns >= ctx->svc_max_resident_ns &&
      __atomic_load_n(&sh->alive, __ATOMIC_SEQ_CST) != 0u) {
    // rotate without waiting for it (round 6: a synchronous stop cost the
    // one-connection path ~0.35 us a group, profiles/round6/bench_r6fin2.json):
    // the resident worker -- and a spare queued behind it -- leave at their
    // next look, published jobs or not; the successor launched now runs after
    // them on the worker stream, behind whatever other work the hardware
    // queue took meanwhile, and starts at what they consumed
    if ((rc = bind(ctx))) return rc;
    __atomic_store_n(&sh->rotate, ctx->svc_epoch, __ATOMIC_SEQ_CST);
    __atomic_store_n(&sh->alive, 1u, __ATOMIC_SEQ_CST);
    const hipError_t e = qfec::launch_ragged_service(ctx->svc_sh_dev, ctx->svc_dev,
                                                     ctx->svc_ring_dev, ctx->h_flag_dev,
                                                     ctx->svc_idle_ticks, ++ctx->svc_epoch,
                                                     ctx->svc_stream);
    if (e != hipSuccess) {
      svc_abandon(ctx);  // every worker gone, the ring rewound, the service off
      return fail(ctx, QFEC_ERR_INTERNAL, "small-batch service launch: %s", hipGetErrorString(e));
    }
    ++ctx->svc_launches;
    ++ctx->svc_rotations;
    ctx->svc_launch_ns = now;
  }
  const uint32_t seq = ctx->svc_seq++;
  qfec::SvcJob& j = ctx->svc_ring[seq % qfec::kSvcRing];
  j.a = a;
  j.a.done_count = nullptr;
  j.a.done_flag = nullptr;
  j.start = ctx->svc_published;
  j.recover = recover ? 1u : 0u;
  j.flag_slot = (uint32_t)slot * kFlagStride;
  j.token = token;
  j.tab_bytes = tb.bytes;
  j.t_off = tb.off;
  j.t_len = tb.len;
  j.t_ptr = tb.ptr;
  j.t_poff = tb.poff;
  j.t_plen = tb.plen;
  j.t_miss = tb.miss;
  j.t_ooff = tb.ooff;
  const uint32_t wseq = ctx->svc_poison_next ? seq ^ 0x80000000u : seq;  // test hook
  ctx->svc_poison_next = false;
  __atomic_store_n(&j.head_sum, 0ull, __ATOMIC_RELAXED);
  __atomic_store_n(&j.seq, wseq, __ATOMIC_RELEASE);
  // the hash of the polled head (the entry's first kSvcHead bytes at most)
  // last: the worker's poll takes a job that fits its head from the bytes it
  // already read when they sum to it, and a larger one's size (every
  // workgroup then copies the entry in one pass)
  constexpr uint32_t kHead = (uint32_t)offsetof(qfec::SvcJob, tab);
  __atomic_store_n(&j.head_sum,
                   qfec::svc_head_hash(j, std::min<uint32_t>((kHead + tb.bytes + 15u) & ~15u,
                                                             qfec::kSvcHead)),
                   __ATOMIC_RELEASE);
  ctx->svc_published += a.n_groups;
  __atomic_store_n(&sh->pub_end, ctx->svc_published, __ATOMIC_RELEASE);
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  if (__atomic_load_n(&sh->alive, __ATOMIC_SEQ_CST) == 0u) {
    __atomic_store_n(&sh->alive, 1u, __ATOMIC_SEQ_CST);
    const hipError_t e =
        bind(ctx) != QFEC_OK
            ? hipErrorInvalidDevice
            : qfec::launch_ragged_service(ctx->svc_sh_dev, ctx->svc_dev, ctx->svc_ring_dev,
                                          ctx->h_flag_dev, ctx->svc_idle_ticks, ++ctx->svc_epoch,
                                          ctx->svc_stream);
    if (e != hipSuccess) {
      // no worker runs (none was alive): take the job back, so that no later
      // worker ever runs it over a reused slot buffer
      __atomic_store_n(&sh->alive, 0u, __ATOMIC_SEQ_CST);
      ctx->svc_published -= a.n_groups;
      __atomic_store_n(&sh->pub_end, ctx->svc_published, __ATOMIC_RELEASE);
      __atomic_store_n(&j.seq, 0xFFFFFFFFu, __ATOMIC_RELEASE);
      --ctx->svc_seq;
      return fail(ctx, QFEC_ERR_INTERNAL, "small-batch service launch: %s", hipGetErrorString(e));
    }
    ++ctx->svc_launches;
    ctx->svc_launch_ns = now;
  }
  return QFEC_OK;
}

// Wait for a service job's token; the worker's stream is polled now and then,
// so a worker that faulted or left without the job ends in an error, not a
// hang.
int wait_flag_svc(qfec_ctx* ctx, int si, uint32_t token) {
  const uint32_t* f = ctx->h_flag + si * kFlagStride;
  for (uint32_t spins = 1;; ++spins) {
    if (__atomic_load_n(f, __ATOMIC_ACQUIRE) == token) return QFEC_OK;
    if ((spins & 4095u) == 0) {
      const hipError_t q = hipStreamQuery(ctx->svc_stream);
      if (q == hipSuccess) {
        if (__atomic_load_n(f, __ATOMIC_ACQUIRE) == token) return QFEC_OK;
        if (__atomic_load_n(&ctx->svc_sh->fault, __ATOMIC_ACQUIRE) != 0u)
          return fail(ctx, QFEC_ERR_INTERNAL,
                      "small-batch service: a published group lies in no ring entry (job "
                      "withheld)");
        return fail(ctx, QFEC_ERR_INTERNAL, "small-batch service left without finishing a job");
      }
      if (q != hipErrorNotReady) QFEC_HIP(ctx, q);
    }
  }
}

void stop_service(qfec_ctx* ctx) {
  if (!ctx->svc_stream) return;
  __atomic_store_n(&ctx->svc_sh->quit, 1u, __ATOMIC_SEQ_CST);
  (void)hipStreamSynchronize(ctx->svc_stream);
  __atomic_store_n(&ctx->svc_sh->alive, 0u, __ATOMIC_SEQ_CST);
}

// A service job failed (no token: the worker faulted, missed a ring entry or
// left): stop every worker, rewind the ring to what the workers finished and
// turn the service off for this context -- the failed job's slot is handed
// to the next call, so no later worker may run it over the reused tables.
// The context's small batches then take the direct path.
void svc_abandon(qfec_ctx* ctx) {
  __atomic_store_n(&ctx->svc_on, false, __ATOMIC_RELEASE);
  if (!ctx->svc_sh) return;
  (void)bind(ctx);  // (reached from completion calls, which do not bind)
  stop_service(ctx);
  for (uint32_t i = 0; i < qfec::kSvcRing; ++i)
    __atomic_store_n(&ctx->svc_ring[i].seq, 0xFFFFFFFFu, __ATOMIC_RELEASE);
  const uint64_t consumed = __atomic_load_n(&ctx->svc_sh->consumed, __ATOMIC_ACQUIRE);
  ctx->svc_published = consumed;
  ctx->svc_seq = (uint32_t)__atomic_load_n(&ctx->svc_sh->jobs, __ATOMIC_ACQUIRE);
  __atomic_store_n(&ctx->svc_sh->pub_end, consumed, __ATOMIC_RELEASE);
  __atomic_store_n(&ctx->svc_sh->fault, 0u, __ATOMIC_RELEASE);
  // the workers' device words afresh (a split job's done count
  // left part-way would misalign every later one of its ring entry, and a
  // follower's announcement count must match the leader's); every worker has
  // left (stop_service synchronised the stream)
  if (ctx->svc_dev &&
      hipMemsetAsync(ctx->svc_dev, 0, sizeof(qfec::SvcDev), ctx->svc_stream) == hipSuccess)
    (void)hipStreamSynchronize(ctx->svc_stream);
  __atomic_store_n(&ctx->svc_sh->quit, 0u, __ATOMIC_SEQ_CST);
}

// Wait for a launch_ragged_latency kernel by spinning on its host-mapped
// completion flag (a few us sooner than the event's wait path); the slot's
// event, recorded after the launch, is polled now and then so that a flag
// that never comes ends in an error instead of a hang.
int wait_flag(qfec_ctx* ctx, int si, uint32_t token) {
  const uint32_t* f = ctx->h_flag + si * kFlagStride;
  for (uint32_t spins = 1;; ++spins) {
    if (__atomic_load_n(f, __ATOMIC_ACQUIRE) == token) return QFEC_OK;
    if ((spins & 1023u) == 0) {
      const hipError_t q = hipEventQuery(ctx->slots[si].done);
      if (q == hipSuccess) {
        if (__atomic_load_n(f, __ATOMIC_ACQUIRE) == token) return QFEC_OK;
        return fail(ctx, QFEC_ERR_INTERNAL, "ragged latency kernel finished without its flag");
      }
      if (q != hipErrorNotReady) QFEC_HIP(ctx, q);
    }
  }
}

int collect_error(qfec_ctx* ctx, hipStream_t stream, int word = kErrStream);

// Finish the QFEC_ASYNC op of slot `si`: QFEC_PENDING if it is still running
// and !wait; otherwise its encode lengths are copied out and its error word
// collected (staged batches latch kernel-side errors; direct ones were
// validated on the host).
int complete_async_op(qfec_ctx* ctx, int si, bool wait) {
  qfec_ctx::AsyncOp& op = ctx->async_ops[si];
  if (!op.live) return QFEC_OK;
  Slot& s = ctx->slots[si];
  if (op.svc) {
    if (!wait && __atomic_load_n(ctx->h_flag + si * kFlagStride, __ATOMIC_ACQUIRE) != op.token) {
      // a worker that is gone without the token (fault, ring miss, exit)
      // must end in an error, not QFEC_PENDING forever
      const hipError_t q = hipStreamQuery(ctx->svc_stream);
      if (q == hipErrorNotReady) return QFEC_PENDING;
      if (q != hipSuccess) {
        op.live = false;
        svc_abandon(ctx);
        QFEC_HIP(ctx, q);
      }
      // drained: the flag is final; wait_flag_svc reports a missing token
    }
    op.live = false;
    const int wrc = wait_flag_svc(ctx, si, op.token);
    if (wrc) {
      // the job may still be published in the ring while its slot is handed
      // to the next call: no later worker may run it
      svc_abandon(ctx);
      return wrc;
    }
  } else if (op.direct) {
    if (!wait && __atomic_load_n(ctx->h_flag + si * kFlagStride, __ATOMIC_ACQUIRE) != op.token) {
      const hipError_t q = hipEventQuery(s.done);
      if (q == hipErrorNotReady) return QFEC_PENDING;
      if (q != hipSuccess) {
        op.live = false;
        QFEC_HIP(ctx, q);
      }
    }
    op.live = false;
    const int wrc = wait_flag(ctx, si, op.token);
    if (wrc) return wrc;
  } else {
    if (!wait) {
      const hipError_t q = hipEventQuery(s.done);
      if (q == hipErrorNotReady) return QFEC_PENDING;
    }
    op.live = false;
    QFEC_HIP(ctx, hipEventSynchronize(s.done));
  }
  if (!op.recover && op.parity_len_out)
    std::memcpy(op.parity_len_out,
                op.direct && op.cnt <= kFlagPlens
                    ? static_cast<const void*>(ctx->h_flag + si * kFlagStride + 1)
                    : static_cast<const void*>(s.h_out),
                op.cnt * sizeof(uint16_t));
  return op.direct ? QFEC_OK : collect_error(ctx, s.stream, kErrSlot0 + si);
}

// Keep op `t`'s code for its ticket's qfec_complete_ticket (the last 4096
// tickets' codes; a newer ticket overwrites the one 4096 before it).  A
// non-OK code not yet reported by qfec_complete is remembered for it.
void keep_code(qfec_ctx* ctx, uint64_t t, int rc, bool reported) {
  ctx->kept[t % qfec_ctx::kKept] = qfec_ctx::Kept{t, rc};
  if (!reported && rc != QFEC_OK && ctx->unreported == QFEC_OK) ctx->unreported = rc;
}

// Finish the op of slot `si` (if live) for a caller that does not own it: its
// code is kept for its owner's qfec_complete_ticket.
void retire_async_op(qfec_ctx* ctx, int si) {
  qfec_ctx::AsyncOp& op = ctx->async_ops[si];
  if (!op.live) return;
  const uint64_t t = op.seq;
  const int rc = complete_async_op(ctx, si, true);
  keep_code(ctx, t, rc, false);
}

// Every outstanding op retired (synchronous calls that use the slots).
void drain_async(qfec_ctx* ctx) {
  for (int i = 0; i < kSlots; ++i) retire_async_op(ctx, i);
}

// Complete every outstanding QFEC_ASYNC op in issue order; the first error
// is returned after all have been finished (or QFEC_PENDING when !wait and
// one is still running: the ones before it are finished).
int complete_async(qfec_ctx* ctx, bool wait) {
  int first = QFEC_OK;
  // ops retired by other calls report here too, once; their codes stay
  // claimable by their tickets (QuicFecGroup::Finish on a context
  // another caller completed)
  first = ctx->unreported;
  ctx->unreported = QFEC_OK;
  for (;;) {
    int si = -1;
    for (int i = 0; i < kSlots; ++i)
      if (ctx->async_ops[i].live && (si < 0 || ctx->async_ops[i].seq < ctx->async_ops[si].seq))
        si = i;
    if (si < 0) return first;
    const uint64_t t = ctx->async_ops[si].seq;
    const int rc = complete_async_op(ctx, si, wait);
    if (rc == QFEC_PENDING) return first ? first : QFEC_PENDING;
    keep_code(ctx, t, rc, true);
    if (rc && !first) first = rc;
  }
}

int check_fixed(qfec_ctx* ctx, uint32_t k, uint32_t L, uint64_t row_stride,
                uint64_t group_stride, uint64_t parity_stride, uint64_t out_stride) {
  if (k < 1 || k > QFEC_MAX_GROUP_PACKETS)
    return fail(ctx, QFEC_ERR_INVALID_FEC_DATA, "FEC group size %u outside [1, %u]", k,
                QFEC_MAX_GROUP_PACKETS);
  if (L < 1 || L > QFEC_MAX_PACKET_SIZE)
    return fail(ctx, QFEC_ERR_INVALID_FEC_DATA, "Illegal payload size: %u (max %u)", L,
                QFEC_MAX_PACKET_SIZE);
  if (row_stride < L || (k > 1 && group_stride < (uint64_t)(k - 1) * row_stride + L) ||
      (k == 1 && group_stride < L) || parity_stride < L || out_stride < L)
    return fail(ctx, QFEC_ERR_INVALID_FEC_DATA, "strides smaller than the payload length");
  return QFEC_OK;
}

int latch_error(qfec_ctx* ctx, uint32_t bits) {
  if (bits == 0) return QFEC_OK;
  if (bits & qfec::kErrMissingIndex)
    return fail(ctx, QFEC_ERR_INVALID_FEC_DATA, "missing packet index >= FEC group size");
  if (bits & qfec::kErrGroupSize)
    return fail(ctx, QFEC_ERR_INVALID_FEC_DATA, "FEC group with 0 or more than 255 packets");
  if (bits & qfec::kErrParityLength)
    return fail(ctx, QFEC_ERR_INVALID_FEC_DATA, "Illegal FEC redundancy length");
  return fail(ctx, QFEC_ERR_INVALID_FEC_DATA,
              "Illegal payload size (0, > kMaxPacketSize or > redundancy length)");
}

// Read and clear the device error word after `stream` has drained.
int collect_error(qfec_ctx* ctx, hipStream_t stream, int word) {
  int rc = bind(ctx);  // (reached from completion calls, which do not bind)
  if (rc) return rc;
  QFEC_HIP(ctx, hipMemcpyAsync(ctx->h_err + word, ctx->d_err + word, sizeof(uint32_t),
                               hipMemcpyDeviceToHost, stream));
  QFEC_HIP(ctx, hipStreamSynchronize(stream));
  const uint32_t bits = ctx->h_err[word];
  if (bits) {
    QFEC_HIP(ctx, hipMemsetAsync(ctx->d_err + word, 0, sizeof(uint32_t), stream));
    QFEC_HIP(ctx, hipStreamSynchronize(stream));
  }
  return latch_error(ctx, bits);
}

// ---- host-pointer path for fixed batches ---------------------------------
// Chunks of whole groups rotate over kSlots streams: H2D (rows [+ parity,
// missing]) -> kernel -> D2H on one stream per slot, so chunk c+1's H2D runs
// under chunk c's kernel and D2H.  Caller memory that is already pinned is
// DMA'd directly; pageable memory bounces through the slot's pinned buffers.
int fixed_host(qfec_ctx* ctx, const uint8_t* rows, const uint8_t* parity, const uint8_t* missing,
               uint32_t k, uint32_t L, uint64_t row_stride, uint64_t group_stride,
               uint64_t parity_stride, uint64_t n, uint8_t* out, uint64_t out_stride) {
  int rc = ensure_staging(ctx);
  if (rc) return rc;
  drain_async(ctx);
  const bool recover = parity != nullptr;
  const bool rows_pinned = is_pinned_or_device(rows);
  const bool par_pinned = recover && is_pinned_or_device(parity);
  const bool out_pinned = is_pinned_or_device(out);
  // groups per chunk bounded by every staging buffer
  uint64_t cg = kStageBytes / group_stride;
  cg = std::min<uint64_t>(cg, (kStageBytes / 4) / L);
  if (recover) cg = std::min<uint64_t>(cg, (kStageBytes / 8) / (L + 1));
  if (cg == 0) return fail(ctx, QFEC_ERR_INTERNAL, "staging too small");

  struct Pending {
    uint64_t g0 = 0, cnt = 0;
    bool live = false;
  } pend[kSlots];

  auto finish = [&](int si) -> int {
    Slot& s = ctx->slots[si];
    if (!pend[si].live) return QFEC_OK;
    QFEC_HIP(ctx, hipEventSynchronize(s.done));
    if (!out_pinned) {
      for (uint64_t g = 0; g < pend[si].cnt; ++g)
        std::memcpy(out + (pend[si].g0 + g) * out_stride, s.h_out + g * L, L);
    }
    pend[si].live = false;
    return QFEC_OK;
  };

  int slot = 0;
  for (uint64_t g0 = 0; g0 < n; g0 += cg, slot = (slot + 1) % kSlots) {
    const uint64_t cnt = std::min(cg, n - g0);
    Slot& s = ctx->slots[slot];
    if ((rc = finish(slot))) return rc;
    // rows: packed [cnt][k][L] on the device side
    const uint64_t dgs = (uint64_t)k * L;
    const bool packed = row_stride == L && group_stride == dgs;
    if (rows_pinned && packed) {
      // contiguous pinned caller layout: one DMA for the whole chunk
      QFEC_HIP(ctx, hipMemcpyAsync(s.d_in, rows + g0 * dgs, cnt * dgs, hipMemcpyHostToDevice,
                                   s.stream));
    } else if (rows_pinned && group_stride == (uint64_t)k * row_stride) {
      // uniformly strided rows: one 2-D DMA (pitch row_stride -> L)
      QFEC_HIP(ctx, hipMemcpy2DAsync(s.d_in, L, rows + g0 * group_stride, row_stride, L,
                                     cnt * k, hipMemcpyHostToDevice, s.stream));
    } else if (rows_pinned) {
      for (uint64_t g = 0; g < cnt; ++g)
        QFEC_HIP(ctx, hipMemcpy2DAsync(s.d_in + g * dgs, L, rows + (g0 + g) * group_stride,
                                       row_stride, L, k, hipMemcpyHostToDevice, s.stream));
    } else {
      for (uint64_t g = 0; g < cnt; ++g) {
        const uint8_t* src = rows + (g0 + g) * group_stride;
        if (row_stride == L) {
          std::memcpy(s.h_in + g * dgs, src, dgs);
        } else {
          for (uint32_t i = 0; i < k; ++i)
            std::memcpy(s.h_in + g * dgs + i * L, src + i * row_stride, L);
        }
      }
      QFEC_HIP(ctx, hipMemcpyAsync(s.d_in, s.h_in, cnt * dgs, hipMemcpyHostToDevice, s.stream));
    }
    uint8_t* d_par = nullptr;
    uint8_t* d_miss = nullptr;
    if (recover) {
      d_par = s.d_aux;
      d_miss = s.d_aux + cnt * L;
      if (par_pinned && parity_stride == L) {
        QFEC_HIP(ctx, hipMemcpyAsync(d_par, parity + g0 * L, cnt * L, hipMemcpyHostToDevice,
                                     s.stream));
      } else if (par_pinned) {
        QFEC_HIP(ctx, hipMemcpy2DAsync(d_par, L, parity + g0 * parity_stride, parity_stride, L,
                                       cnt, hipMemcpyHostToDevice, s.stream));
      } else {
        for (uint64_t g = 0; g < cnt; ++g)
          std::memcpy(s.h_aux + g * L, parity + (g0 + g) * parity_stride, L);
      }
      std::memcpy(s.h_aux + cnt * L, missing + g0, cnt);
      if (!par_pinned)
        QFEC_HIP(ctx, hipMemcpyAsync(d_par, s.h_aux, cnt * L + cnt, hipMemcpyHostToDevice,
                                     s.stream));
      else
        QFEC_HIP(ctx, hipMemcpyAsync(d_miss, s.h_aux + cnt * L, cnt, hipMemcpyHostToDevice,
                                     s.stream));
    }
    qfec::FixedArgs a{};
    a.rows = s.d_in;
    a.parity = d_par;
    a.missing = d_miss;
    a.out = s.d_out;
    a.row_stride = L;
    a.group_stride = dgs;
    a.parity_stride = L;
    a.out_stride = L;
    a.n_groups = cnt;
    a.k = k;
    a.L = L;
    a.err = ctx->d_err + kErrHost;
    QFEC_HIP(ctx, qfec::launch_fixed(a, true, s.stream));
    if (out_pinned && out_stride == L) {
      QFEC_HIP(ctx, hipMemcpyAsync(out + g0 * L, s.d_out, cnt * L, hipMemcpyDeviceToHost,
                                   s.stream));
    } else if (out_pinned) {
      QFEC_HIP(ctx, hipMemcpy2DAsync(out + g0 * out_stride, out_stride, s.d_out, L, L, cnt,
                                     hipMemcpyDeviceToHost, s.stream));
    } else {
      QFEC_HIP(ctx, hipMemcpyAsync(s.h_out, s.d_out, cnt * L, hipMemcpyDeviceToHost, s.stream));
    }
    QFEC_HIP(ctx, hipEventRecord(s.done, s.stream));
    pend[slot].g0 = g0;
    pend[slot].cnt = cnt;
    pend[slot].live = true;
  }
  for (int si = 0; si < kSlots; ++si)
    if ((rc = finish(si))) return rc;
  return collect_error(ctx, ctx->slots[0].stream, kErrHost);
}

// ---- QFEC_PTR_MAPPED: payloads in pinned host memory, read in place ---------
// The kernels address the caller's pinned, device-mapped host buffers directly
// (zero-copy over PCIe: tools/tune/tune_zero_copy.hip measures a kernel read of
// pinned host rows at the H2D copy rate, 55-58 GB/s), so the packet bytes
// cross the link exactly once and no host thread copies them.  Only the index
// arrays are staged (10 B per packet + 12-23 B per group), chunked over the
// context's slots so chunk c+1's tables are copied while chunk c runs.
// Groups per mapped-mode chunk: the staging capacity, or fewer when
// QFEC_CHUNK_GROUPS is set (lets the tests run the multi-chunk pipeline on
// small batches; read per call).
uint64_t mapped_chunk_groups(uint64_t cap) {
  const char* e = std::getenv("QFEC_CHUNK_GROUPS");
  const uint64_t v = e ? std::strtoull(e, nullptr, 10) : 0;
  return v ? std::min(v, cap) : cap;
}

int check_mapped(qfec_ctx* ctx, const void* p, const char* what) {
  if (!is_pinned_or_device(p))
    return fail(ctx, QFEC_ERR_INTERNAL,
                "QFEC_PTR_MAPPED: %s is not pinned host (qfec_host_alloc) or device memory", what);
  return QFEC_OK;
}

int fixed_mapped(qfec_ctx* ctx, const uint8_t* rows, const uint8_t* parity, const uint8_t* missing,
                 uint32_t k, uint32_t L, uint64_t row_stride, uint64_t group_stride,
                 uint64_t parity_stride, uint64_t n, uint8_t* out, uint64_t out_stride) {
  int rc = ensure_staging(ctx);
  if (rc) return rc;
  drain_async(ctx);
  const bool recover = parity != nullptr;
  if ((rc = check_mapped(ctx, rows, "rows")) || (rc = check_mapped(ctx, out, "out")) ||
      (recover && (rc = check_mapped(ctx, parity, "parity"))))
    return rc;
  qfec::FixedArgs a{};
  a.rows = rows;
  a.parity = parity;
  a.out = out;
  a.row_stride = row_stride;
  a.group_stride = group_stride;
  a.parity_stride = parity_stride;
  a.out_stride = out_stride;
  a.k = k;
  a.L = L;
  a.err = ctx->d_err + kErrHost;
  // the lost-slot indices are the only staged input (kStageBytes / 8 per chunk);
  // a small batch (one chunk of <= kDirectGroups) is latency-bound: the kernel
  // reads them from the mapped slot buffer itself (no copy), and the error
  // word is not fetched — the host already checked every index the kernel
  // checks (qfec_recover_batch_strided), so the launch cannot latch one
  const uint64_t cg = mapped_chunk_groups(recover ? kStageBytes / 8 : n);
  const bool direct = n <= std::min<uint64_t>(cg, kDirectGroups);
  uint64_t g0_of[kSlots] = {};
  bool live[kSlots] = {};
  int slot = 0;
  for (uint64_t g0 = 0; g0 < n; g0 += cg, slot = (slot + 1) % kSlots) {
    const uint64_t cnt = std::min(cg, n - g0);
    Slot& s = ctx->slots[slot];
    if (live[slot]) QFEC_HIP(ctx, hipEventSynchronize(s.done));  // h_aux free again
    a.rows = rows + g0 * group_stride;
    a.out = out + g0 * out_stride;
    a.n_groups = cnt;
    if (recover) {
      a.parity = parity + g0 * parity_stride;
      std::memcpy(s.h_aux, missing + g0, cnt);
      if (direct) {
        a.missing = s.h_aux_dev;
      } else {
        QFEC_HIP(ctx, hipMemcpyAsync(s.d_aux, s.h_aux, cnt, hipMemcpyHostToDevice, s.stream));
        a.missing = s.d_aux;
      }
    }
    QFEC_HIP(ctx, qfec::launch_fixed(a, true, s.stream));
    QFEC_HIP(ctx, hipEventRecord(s.done, s.stream));
    g0_of[slot] = g0;
    live[slot] = true;
  }
  for (int si = 0; si < kSlots; ++si)
    if (live[si]) QFEC_HIP(ctx, hipEventSynchronize(ctx->slots[si].done));
  (void)g0_of;
  return direct ? QFEC_OK : collect_error(ctx, ctx->slots[0].stream, kErrHost);
}


// A device-pointer fixed-shape launch on the context stream.  Phased launches
// (large nt batches) share the context's sync words: one on a different stream
// than the previous phased launch first waits for that one's completion event
// (they would otherwise update the same counters concurrently and zero each
// other's meetings).  A phased launch that was abandoned since the last look
// (h_phase, copied by the kernel) switches the next kPhaseBackoff large
// batches to the one-pass kernel: a contended GPU runs the phased kernel
// without its meetings anyway, at 4 waves per CU.
constexpr uint32_t kPhaseBackoff = 16;

int fixed_device(qfec_ctx* ctx, qfec::FixedArgs& a, uint32_t flags) {
  const bool nt = (flags & QFEC_CACHED) == 0;
  a.ncu = ctx->ncu;
  a.phase_extra = ctx->phase_extra;
  a.phase_min = ctx->phase_min;
  a.no_regsteps = ctx->no_regsteps;
  a.rt_batch = ctx->rt_batch;
  a.phase_host = ctx->h_phase_dev;
  a.phase_sync = (flags & QFEC_ONE_PASS) ? nullptr : ctx->d_phase;
  uint32_t grid = 0;
  bool phased = a.phase_sync && qfec::fixed_uses_phases(a, nt);
  if (phased) {
    // (the registry only for a batch that would phase at all)
    a.svc_cus = other_service_cus(ctx) + ctx->phase_reserve;
    phased = qfec::fixed_uses_phases(a, nt, &grid);
  }
  if (phased) {
    const uint32_t seen = __atomic_load_n(ctx->h_phase, __ATOMIC_ACQUIRE);
    if (seen != ctx->phase_seen) {
      ctx->phase_seen = seen;
      ctx->phase_backoff = kPhaseBackoff;
    }
    if (ctx->phase_backoff > 0 && ctx->phase_extra == 0) {
      --ctx->phase_backoff;
      a.phase_sync = nullptr;  // one-pass while contention persists
    } else {
      // the phased kernel wants one workgroup on every CU: this context's
      // resident small-batch worker (if any) leaves first (it holds a CU's
      // LDS; a worker of another context leaves within kSvcIdleTicks, below
      // the meetings' timeout)
      // (also when `alive` reads 0 but the worker stream still has work: a
      // worker queued behind one that was leaving)
      if (ctx->svc_sh && (__atomic_load_n(&ctx->svc_sh->alive, __ATOMIC_ACQUIRE) != 0u ||
                          hipStreamQuery(ctx->svc_stream) == hipErrorNotReady)) {
        stop_service(ctx);
        __atomic_store_n(&ctx->svc_sh->quit, 0u, __ATOMIC_SEQ_CST);
      }
      if (ctx->phase_recorded && ctx->phase_stream != ctx->stream)
        QFEC_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->phase_done, 0));
      QFEC_HIP(ctx, qfec::launch_fixed(a, nt, ctx->stream));
      QFEC_HIP(ctx, hipEventRecord(ctx->phase_done, ctx->stream));
      ctx->phase_stream = ctx->stream;
      ctx->phase_recorded = true;
      ctx->last_fixed_phased = 1;
      ctx->last_phase_grid = grid;
      return QFEC_OK;
    }
  }
  a.phase_sync = nullptr;  // (a phased plan refused above: one-pass)
  QFEC_HIP(ctx, qfec::launch_fixed(a, nt, ctx->stream));
  ctx->last_fixed_phased = 0;
  ctx->last_phase_grid = 0;
  return QFEC_OK;
}

}  // namespace

extern "C" {

int qfec_abi_version(void) { return QFEC_ABI_VERSION; }

void* qfec_host_alloc(size_t bytes) {
  void* p = nullptr;
  const hipError_t e =
      hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocMapped | hipHostMallocPortable);
  if (e != hipSuccess) {
    fail(nullptr, QFEC_ERR_INTERNAL, "qfec_host_alloc(%zu): %s", bytes, hipGetErrorString(e));
    return nullptr;
  }
  // QFEC_PTR_MAPPED hands host pointers to the kernels unchanged (as for
  // qfec_host_register): refuse memory the device addresses elsewhere
  void* dev = nullptr;
  const hipError_t d = hipHostGetDevicePointer(&dev, p, 0);
  if (d != hipSuccess || dev != p) {
    (void)hipHostFree(p);
    fail(nullptr, QFEC_ERR_INTERNAL,
         "qfec_host_alloc(%zu): device address %p differs from the host address %p (%s); "
         "QFEC_PTR_MAPPED needs them equal", bytes, dev, p, hipGetErrorString(d));
    return nullptr;
  }
  note_mapped(p, bytes ? bytes : 1);
  return p;
}

void qfec_host_free(void* p) {
  if (!p) return;
  forget_mapped(p);
  (void)hipHostFree(p);
}

int qfec_host_register(void* p, size_t bytes) {
  if (!p || bytes == 0) return fail(nullptr, QFEC_ERR_INTERNAL, "qfec_host_register: empty range");
  hipError_t e = hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable);
  if (e != hipSuccess)
    return fail(nullptr, QFEC_ERR_INTERNAL, "qfec_host_register(%p, %zu): %s", p, bytes,
                hipGetErrorString(e));
  void* dev = nullptr;
  e = hipHostGetDevicePointer(&dev, p, 0);
  if (e != hipSuccess || dev != p) {
    (void)hipHostUnregister(p);
    return fail(nullptr, QFEC_ERR_INTERNAL,
                "qfec_host_register(%p): device address %p differs from the host address (%s); "
                "QFEC_PTR_MAPPED needs them equal", p, dev, hipGetErrorString(e));
  }
  note_mapped(p, bytes);
  return QFEC_OK;
}

int qfec_host_unregister(void* p) {
  forget_mapped(p);
  const hipError_t e = hipHostUnregister(p);
  if (e != hipSuccess)
    return fail(nullptr, QFEC_ERR_INTERNAL, "qfec_host_unregister(%p): %s", p,
                hipGetErrorString(e));
  return QFEC_OK;
}

const char* qfec_strerror(int code) {
  switch (code) {
    case QFEC_OK:
      return "QUIC_NO_ERROR";
    case QFEC_ERR_INTERNAL:
      return "QUIC_INTERNAL_ERROR";
    case QFEC_ERR_INVALID_FEC_DATA:
      return "QUIC_INVALID_FEC_DATA";
    default:
      return "QUIC_UNKNOWN_ERROR";
  }
}

const char* qfec_last_error(const qfec_ctx* ctx) { return ctx ? ctx->last_error : g_tls_error; }

// ---- v<=31 wire format: C wrappers over quic_fec_wire.h ---------------------
size_t qfec_wire_write_private_header(const qfec_fec_header* h, uint8_t* buf, size_t cap) {
  if (!h || !buf) return fail(nullptr, 0, "null buffer"), 0;
  net::FecHeaderFields f;
  f.entropy_flag = h->entropy_flag != 0;
  f.fec_flag = h->fec_flag != 0;
  f.in_fec_group = h->in_fec_group != 0;
  f.fec_group_offset = h->fec_group_offset;
  const size_t n = net::WriteFecPrivateHeader(f, buf, cap);
  if (n == 0) fail(nullptr, 0, "private header does not fit or FEC flag without a group");
  return n;
}

size_t qfec_wire_parse_private_header(const uint8_t* buf, size_t len, int quic_version,
                                      uint64_t packet_number, qfec_fec_header* out) {
  if ((!buf && len) || !out) return fail(nullptr, 0, "null buffer"), 0;
  net::FecHeaderFields f;
  std::string err;
  const size_t n = net::ParseFecPrivateHeader(buf, len, quic_version, packet_number, &f, &err);
  if (n == 0) {
    fail(nullptr, 0, "%s", err.c_str());
    return 0;
  }
  out->entropy_flag = f.entropy_flag;
  out->fec_flag = f.fec_flag;
  out->in_fec_group = f.in_fec_group;
  out->fec_group_offset = f.fec_group_offset;
  return n;
}

size_t qfec_wire_write_revived(const uint64_t* revived, size_t n, size_t packet_number_length,
                               uint8_t* buf, size_t cap) {
  if ((!revived && n) || !buf) return fail(nullptr, 0, "null buffer"), 0;
  std::vector<net::QuicPacketNumber> v(revived, revived + n);
  const size_t w = net::WriteRevivedPackets(v, packet_number_length, buf, cap);
  if (w == 0) fail(nullptr, 0, "revived list does not fit (count > 255, length or capacity)");
  return w;
}

size_t qfec_wire_parse_revived(const uint8_t* buf, size_t len, size_t packet_number_length,
                               uint64_t* revived, size_t* n_out) {
  if ((!buf && len) || !revived || !n_out) return fail(nullptr, 0, "null buffer"), 0;
  std::vector<net::QuicPacketNumber> v;
  std::string err;
  const size_t n = net::ParseRevivedPackets(buf, len, packet_number_length, &v, &err);
  if (n == 0) {
    fail(nullptr, 0, "%s", err.c_str());
    return 0;
  }
  std::copy(v.begin(), v.end(), revived);
  *n_out = v.size();
  return n;
}

size_t qfec_wire_fec_packet_body(uint64_t packet_number, uint64_t fec_group, int entropy_flag,
                                 const uint8_t* redundancy, size_t redundancy_len, uint8_t* buf,
                                 size_t cap) {
  if ((!redundancy && redundancy_len) || !buf) return fail(nullptr, 0, "null buffer"), 0;
  const size_t n = net::SerializeFecPacketBody(
      packet_number, fec_group, entropy_flag != 0,
      net::StringPiece(reinterpret_cast<const char*>(redundancy), redundancy_len), buf, cap);
  if (n == 0)
    fail(nullptr, 0, "FEC packet body: group outside the uint8 offset range, redundancy above "
                     "kMaxPacketSize or capacity too small");
  return n;
}

qfec_ctx* qfec_create(int device) {
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count == 0) {
    fail(nullptr, QFEC_ERR_INTERNAL, "no HIP device available (%s)",
         e != hipSuccess ? hipGetErrorString(e) : "device count 0");
    return nullptr;
  }
  if (device < 0 || device >= count) {
    fail(nullptr, QFEC_ERR_INTERNAL, "device %d out of range [0, %d)", device, count);
    return nullptr;
  }
  qfec_ctx* ctx = new qfec_ctx();
  ctx->device = device;
  bool ok = hipSetDevice(device) == hipSuccess &&
            hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) == hipSuccess &&
            hipMalloc(&ctx->d_err, kErrWords * sizeof(uint32_t)) == hipSuccess &&
            hipMemset(ctx->d_err, 0, kErrWords * sizeof(uint32_t)) == hipSuccess &&
            hipMalloc(&ctx->d_phase, kPhaseSyncBytes) == hipSuccess &&
            hipMemset(ctx->d_phase, 0, kPhaseSyncBytes) == hipSuccess &&
            hipHostMalloc(&ctx->h_err, kErrWords * sizeof(uint32_t), hipHostMallocDefault) ==
                hipSuccess &&
            hipHostMalloc(&ctx->h_phase, sizeof(uint32_t),
                          hipHostMallocMapped | hipHostMallocPortable) == hipSuccess &&
            hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->h_phase_dev), ctx->h_phase,
                                    0) == hipSuccess &&
            hipEventCreateWithFlags(&ctx->phase_done, hipEventDisableTiming) == hipSuccess;
  int ncu = 0;
  ok = ok && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) ==
                 hipSuccess;
  if (!ok) {
    fail(nullptr, QFEC_ERR_INTERNAL, "HIP initialisation failed on device %d", device);
    qfec_destroy(ctx);
    return nullptr;
  }
  *ctx->h_phase = 0;
  ctx->ncu = ncu > 0 ? (uint32_t)ncu : 0;
  ctx->stream = ctx->own_stream;
  ctx->svc_max_resident_ns = kSvcMaxResidentNs;
  ctx->svc_idle_ticks = kSvcIdleTicks;
  // (measurement knob: QFEC_SVC_RESIDENT_US overrides the residency bound)
  if (const char* r = std::getenv("QFEC_SVC_RESIDENT_US"))
    ctx->svc_max_resident_ns = std::strtoull(r, nullptr, 10) * 1000ull;
  return ctx;
}

namespace {
void stop_feeder(qfec_ctx* ctx);  // (a measurement feeder still running on ctx)
}  // namespace

void qfec_destroy(qfec_ctx* ctx) {
  if (!ctx) return;
  stop_feeder(ctx);
  (void)hipSetDevice(ctx->device);
  {
    std::lock_guard<std::mutex> lock(g_svc_mu);
    g_svc_ctxs.erase(std::remove(g_svc_ctxs.begin(), g_svc_ctxs.end(), ctx), g_svc_ctxs.end());
  }
  stop_service(ctx);
  // this context's streams only: a device-wide wait would also wait for
  // another context's resident worker, which a busy connection thread keeps
  // alive indefinitely (round 6)
  if (ctx->own_stream) (void)hipStreamSynchronize(ctx->own_stream);
  if (ctx->stream && ctx->stream != ctx->own_stream) (void)hipStreamSynchronize(ctx->stream);
  for (auto& s : ctx->slots)
    if (s.stream) (void)hipStreamSynchronize(s.stream);
  if (ctx->svc_stream) (void)hipStreamDestroy(ctx->svc_stream);
  if (ctx->svc_sh) (void)hipHostFree(ctx->svc_sh);
  if (ctx->svc_ring) (void)hipHostFree(ctx->svc_ring);
  if (ctx->svc_dev) (void)hipFree(ctx->svc_dev);
  for (auto& s : ctx->slots) {
    if (s.stream) (void)hipStreamDestroy(s.stream);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.d_in) (void)hipFree(s.d_in);
    if (s.d_aux) (void)hipFree(s.d_aux);
    if (s.d_out) (void)hipFree(s.d_out);
    if (s.h_in) (void)hipHostFree(s.h_in);
    if (s.h_aux) (void)hipHostFree(s.h_aux);
    if (s.h_out) (void)hipHostFree(s.h_out);
  }
  if (ctx->d_done) (void)hipFree(ctx->d_done);
  if (ctx->d_phase) (void)hipFree(ctx->d_phase);
  for (void* q : ctx->scratch_p)
    if (q) (void)hipFree(q);
  if (ctx->h_flag) (void)hipHostFree(ctx->h_flag);
  if (ctx->d_err) (void)hipFree(ctx->d_err);
  if (ctx->h_err) (void)hipHostFree(ctx->h_err);
  if (ctx->h_phase) (void)hipHostFree(ctx->h_phase);
  if (ctx->phase_done) (void)hipEventDestroy(ctx->phase_done);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  delete ctx;
}

int qfec_set_stream(qfec_ctx* ctx, void* hip_stream) {
  if (!ctx) return fail(nullptr, QFEC_ERR_INTERNAL, "null qfec_ctx");
  ctx->stream = static_cast<hipStream_t>(hip_stream);
  return QFEC_OK;
}

void* qfec_get_stream(qfec_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

void* qfec_own_stream(qfec_ctx* ctx) { return ctx ? (void*)ctx->own_stream : nullptr; }

int qfec_sync(qfec_ctx* ctx) {
  int rc = bind(ctx);
  if (rc) return rc;
  return collect_error(ctx, ctx->stream);
}

int qfec_complete(qfec_ctx* ctx, int wait) {
  int rc = bind(ctx);
  if (rc) return rc;
  return complete_async(ctx, wait != 0);
}

uint64_t qfec_async_ticket(const qfec_ctx* ctx) { return ctx ? ctx->last_ticket : 0; }

int qfec_complete_ticket(qfec_ctx* ctx, uint64_t ticket, int wait) {
  // no bind: a completion polls the context's own flags, streams and events
  // (collect_error and svc_abandon bind on the slow paths)
  if (!ctx) return fail(nullptr, QFEC_ERR_INTERNAL, "null qfec_ctx");
  qfec_ctx::Kept& f = ctx->kept[ticket % qfec_ctx::kKept];
  if (ticket != 0 && f.ticket == ticket) {
    f.ticket = 0;  // claimed once
    return f.code;
  }
  for (int i = 0; i < kSlots; ++i)
    if (ctx->async_ops[i].live && ctx->async_ops[i].seq == ticket)
      return complete_async_op(ctx, i, wait != 0);
  return fail(ctx, QFEC_ERR_INTERNAL, "unknown or already completed ticket %llu",
              (unsigned long long)ticket);
}

int qfec_encode_batch_strided(qfec_ctx* ctx, const uint8_t* rows, uint32_t k, uint32_t L,
                              uint64_t row_stride, uint64_t group_stride, uint64_t n_groups,
                              uint8_t* parity_out, uint64_t parity_stride, uint32_t flags) {
  int rc = bind(ctx);
  if (rc) return rc;
  if ((rc = check_fixed(ctx, k, L, row_stride, group_stride, parity_stride, parity_stride)))
    return rc;
  if (n_groups == 0) return QFEC_OK;
  if (!rows || !parity_out) return fail(ctx, QFEC_ERR_INTERNAL, "null buffer");
  if ((flags & QFEC_PTR_MAPPED) && (flags & QFEC_PTR_HOST))
    return fail(ctx, QFEC_ERR_INTERNAL, "QFEC_PTR_MAPPED and QFEC_PTR_HOST are exclusive");
  if (flags & QFEC_PTR_MAPPED)
    return fixed_mapped(ctx, rows, nullptr, nullptr, k, L, row_stride, group_stride, 0, n_groups,
                        parity_out, parity_stride);
  if (flags & QFEC_PTR_HOST)
    return fixed_host(ctx, rows, nullptr, nullptr, k, L, row_stride, group_stride, 0, n_groups,
                      parity_out, parity_stride);
  qfec::FixedArgs a{};
  a.rows = rows;
  a.out = parity_out;
  a.row_stride = row_stride;
  a.group_stride = group_stride;
  a.out_stride = parity_stride;
  a.n_groups = n_groups;
  a.k = k;
  a.L = L;
  a.err = ctx->d_err;
  return fixed_device(ctx, a, flags);
}

int qfec_encode_batch(qfec_ctx* ctx, const uint8_t* rows, uint32_t k, uint32_t L,
                      uint64_t n_groups, uint8_t* parity_out, uint32_t flags) {
  return qfec_encode_batch_strided(ctx, rows, k, L, L, (uint64_t)k * L, n_groups, parity_out, L,
                                   flags);
}

int qfec_recover_batch_strided(qfec_ctx* ctx, const uint8_t* rows, const uint8_t* parity,
                               const uint8_t* missing_idx, uint32_t k, uint32_t L,
                               uint64_t row_stride, uint64_t group_stride,
                               uint64_t parity_stride, uint64_t n_groups, uint8_t* out,
                               uint64_t out_stride, uint32_t flags) {
  int rc = bind(ctx);
  if (rc) return rc;
  if ((rc = check_fixed(ctx, k, L, row_stride, group_stride, parity_stride, out_stride)))
    return rc;
  if (n_groups == 0) return QFEC_OK;
  if (!rows || !parity || !missing_idx || !out) return fail(ctx, QFEC_ERR_INTERNAL, "null buffer");
  if ((flags & QFEC_PTR_MAPPED) && (flags & QFEC_PTR_HOST))
    return fail(ctx, QFEC_ERR_INTERNAL, "QFEC_PTR_MAPPED and QFEC_PTR_HOST are exclusive");
  if (flags & (QFEC_PTR_HOST | QFEC_PTR_MAPPED)) {
    for (uint64_t g = 0; g < n_groups; ++g)
      if (missing_idx[g] >= k)
        return fail(ctx, QFEC_ERR_INVALID_FEC_DATA,
                    "missing packet index %u >= FEC group size %u (group %llu)", missing_idx[g],
                    k, (unsigned long long)g);
    if (flags & QFEC_PTR_MAPPED)
      return fixed_mapped(ctx, rows, parity, missing_idx, k, L, row_stride, group_stride,
                          parity_stride, n_groups, out, out_stride);
    return fixed_host(ctx, rows, parity, missing_idx, k, L, row_stride, group_stride,
                      parity_stride, n_groups, out, out_stride);
  }
  qfec::FixedArgs a{};
  a.rows = rows;
  a.parity = parity;
  a.missing = missing_idx;
  a.out = out;
  a.row_stride = row_stride;
  a.group_stride = group_stride;
  a.parity_stride = parity_stride;
  a.out_stride = out_stride;
  a.n_groups = n_groups;
  a.k = k;
  a.L = L;
  a.err = ctx->d_err;
  return fixed_device(ctx, a, flags);
}

int qfec_recover_batch(qfec_ctx* ctx, const uint8_t* rows, const uint8_t* parity,
                       const uint8_t* missing_idx, uint32_t k, uint32_t L, uint64_t n_groups,
                       uint8_t* out, uint32_t flags) {
  return qfec_recover_batch_strided(ctx, rows, parity, missing_idx, k, L, L, (uint64_t)k * L, L,
                                    n_groups, out, L, flags);
}

// In-slot recover: the redundancy sits in the lost
// packet's row, so the lost packet is the XOR of the k rows -- the encode
// kernels over one contiguous stream; in place (out == NULL) the kernels
// write each group's result into its row missing_idx[g].
int qfec_recover_inslot_batch_strided(qfec_ctx* ctx, uint8_t* rows, const uint8_t* missing_idx,
                                      uint32_t k, uint32_t L, uint64_t row_stride,
                                      uint64_t group_stride, uint64_t n_groups, uint8_t* out,
                                      uint64_t out_stride, uint32_t flags) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (out) return qfec_encode_batch_strided(ctx, rows, k, L, row_stride, group_stride, n_groups,
                                            out, out_stride, flags);
  if ((rc = check_fixed(ctx, k, L, row_stride, group_stride, L, L))) return rc;
  if (n_groups == 0) return QFEC_OK;
  if (!rows || !missing_idx) return fail(ctx, QFEC_ERR_INTERNAL, "null buffer");
  if (flags & (QFEC_PTR_HOST | QFEC_PTR_MAPPED))
    return fail(ctx, QFEC_ERR_INTERNAL,
                "in-slot recover in place: device pointers only (pass out for host memory)");
  qfec::FixedArgs a{};
  a.rows = rows;
  a.out = rows;  // unused: every output row is a row of `rows`
  a.inplace_missing = missing_idx;
  a.row_stride = row_stride;
  a.group_stride = group_stride;
  a.parity_stride = L;
  a.out_stride = L;
  a.n_groups = n_groups;
  a.k = k;
  a.L = L;
  a.err = ctx->d_err;
  return fixed_device(ctx, a, flags);
}

int qfec_recover_inslot_batch(qfec_ctx* ctx, uint8_t* rows, const uint8_t* missing_idx, uint32_t k,
                              uint32_t L, uint64_t n_groups, uint8_t* out, uint32_t flags) {
  return qfec_recover_inslot_batch_strided(ctx, rows, missing_idx, k, L, L, (uint64_t)k * L,
                                           n_groups, out, L, flags);
}

// ---- ragged ---------------------------------------------------------------
namespace {

// Host-pointer ragged path (QuicFecGroup::PayloadParity/Revive and the
// connection batches' Flush run through it).  Chunks of whole groups are
// GATHERED on the host into one slot's pinned staging buffer — received
// packets packed back to back, then the chunk's CSR tables rebased to the
// staging layout — moved by ONE H2D, XORed by one ragged launch, and the
// packed outputs come back by one D2H and are scattered to the caller's
// offsets.  Chunks rotate over the context's kSlots streams, so the host
// gathers chunk c+1 while chunk c is on the device.  Nothing is allocated per
// call: the slots' device and pinned buffers (ensure_staging) are reused.
// Only exactly what the device path writes is written: parity_len[g] bytes
// per group (+ parity_len_out on encode).
struct DevBuf {  // a device buffer of a host-pointer call (from the context's scratch)
  void* p = nullptr;
};

// The i-th scratch buffer of a host-pointer call, at least `bytes` long.
// Host-pointer calls are synchronous and a context is used by one thread, so
// the next call may reuse every buffer; a buffer only grows (x2).
hipError_t scratch(qfec_ctx* ctx, size_t i, size_t bytes, void** out) {
  if (ctx->scratch_p.size() <= i) {
    ctx->scratch_p.resize(i + 1, nullptr);
    ctx->scratch_n.resize(i + 1, 0);
  }
  if (ctx->scratch_n[i] < bytes) {
    if (ctx->scratch_p[i]) {
      hipError_t e = hipFree(ctx->scratch_p[i]);
      ctx->scratch_p[i] = nullptr;
      ctx->scratch_n[i] = 0;
      if (e != hipSuccess) return e;
    }
    const size_t want = std::max<size_t>({bytes, 2 * ctx->scratch_n[i], 4096});
    hipError_t e = hipMalloc(&ctx->scratch_p[i], want);
    if (e != hipSuccess) return e;
    ctx->scratch_n[i] = want;
  }
  *out = ctx->scratch_p[i];
  return hipSuccess;
}

struct RaggedChunk {
  uint64_t g0 = 0, n = 0;
  uint64_t np = 0, nbytes = 0, nout = 0, npar = 0;  // staged packets, bytes, output, parity bytes
  bool live = false;
};

inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

struct RaggedLayout {  // byte offsets inside a slot's d_in / h_in (and d_out / h_out)
  uint64_t bytes, off, len, ptr, poff, par, plen, miss, ooff, in_total;
  uint64_t out_plen, out_total;
  RaggedLayout(const RaggedChunk& c, bool recover) {
    bytes = 0;
    off = align_up(c.nbytes, 16);
    len = off + c.np * 8;
    ptr = align_up(len + c.np * 2, 8);
    poff = align_up(ptr + (c.n + 1) * 4, 8);
    par = align_up(poff + c.n * 8, 16);
    plen = align_up(par + (recover ? c.npar : 0), 8);
    miss = plen + (recover ? c.n * 2 : 0);
    ooff = align_up(miss + (recover ? c.n : 0), 8);
    in_total = ooff + (recover ? c.n * 8 : 0);
    out_plen = align_up(c.nout, 8);
    out_total = out_plen + (recover ? 0 : c.n * 2);
  }
};

// Host-side validation of a ragged batch whose tables are host memory (the
// same error words the kernel latches; the kernel re-checks everything else).
int validate_ragged(qfec_ctx* ctx, bool recover, const uint16_t* pkt_len, const uint32_t* grp_ptr,
                    uint64_t n, const uint16_t* parity_len, const uint8_t* missing) {
  uint32_t bits = 0;
  for (uint64_t g = 0; g < n; ++g) {
    if (grp_ptr[g + 1] < grp_ptr[g] || grp_ptr[g + 1] - grp_ptr[g] > QFEC_MAX_GROUP_PACKETS ||
        grp_ptr[g + 1] == grp_ptr[g]) {
      bits |= qfec::kErrGroupSize;
      continue;
    }
    if (recover) {
      if (missing[g] >= grp_ptr[g + 1] - grp_ptr[g]) bits |= qfec::kErrMissingIndex;
      if (parity_len[g] == 0 || parity_len[g] > QFEC_MAX_PACKET_SIZE) bits |= qfec::kErrParityLength;
    }
    for (uint32_t p = grp_ptr[g]; p < grp_ptr[g + 1]; ++p) {
      if (recover && p - grp_ptr[g] == missing[g]) continue;
      if (pkt_len[p] == 0 || pkt_len[p] > QFEC_MAX_PACKET_SIZE ||
          (recover && pkt_len[p] > parity_len[g]))
        bits |= qfec::kErrPacketLength;
    }
  }
  return latch_error(ctx, bits);
}

int ragged_host(qfec_ctx* ctx, bool recover, const uint8_t* bytes, const uint64_t* pkt_off,
                const uint16_t* pkt_len, const uint32_t* grp_ptr, uint64_t n,
                const uint8_t* parity, uint8_t* parity_out, const uint64_t* parity_off,
                const uint16_t* parity_len, uint16_t* parity_len_out, const uint8_t* missing,
                uint8_t* out, const uint64_t* out_off) {
  int rc = ensure_staging(ctx);
  if (rc) return rc;
  drain_async(ctx);
  if ((rc = validate_ragged(ctx, recover, pkt_len, grp_ptr, n, parity_len, missing))) return rc;

  const uint64_t in_cap = kStageBytes, out_cap = kStageBytes / 4;
  RaggedChunk chunk[kSlots];

  auto finish = [&](int si) -> int {
    RaggedChunk& c = chunk[si];
    if (!c.live) return QFEC_OK;
    Slot& s = ctx->slots[si];
    QFEC_HIP(ctx, hipEventSynchronize(s.done));
    const RaggedLayout lay(c, recover);
    const uint16_t* h_plen = reinterpret_cast<const uint16_t*>(s.h_out + lay.out_plen);
    uint64_t o = 0;
    for (uint64_t i = 0; i < c.n; ++i) {
      const uint64_t g = c.g0 + i;
      if (recover) {
        std::memcpy(out + out_off[g], s.h_out + o, parity_len[g]);
        o += parity_len[g];
      } else {
        std::memcpy(parity_out + parity_off[g], s.h_out + o, h_plen[i]);
        parity_len_out[g] = h_plen[i];
        uint16_t mx = 0;
        for (uint32_t p = grp_ptr[g]; p < grp_ptr[g + 1]; ++p) mx = std::max(mx, pkt_len[p]);
        o += mx;
      }
    }
    c.live = false;
    return QFEC_OK;
  };

  int slot = 0;
  uint64_t g = 0;
  while (g < n) {
    // plan the chunk: whole groups while both staging budgets hold
    RaggedChunk c;
    c.g0 = g;
    for (; g < n; ++g) {
      const uint32_t k = grp_ptr[g + 1] - grp_ptr[g];
      uint64_t gb = 0, mx = 0;
      for (uint32_t p = grp_ptr[g]; p < grp_ptr[g + 1]; ++p) {
        if (recover && p - grp_ptr[g] == missing[g]) continue;
        gb += pkt_len[p];
        mx = std::max<uint64_t>(mx, pkt_len[p]);
      }
      const uint64_t gout = recover ? parity_len[g] : mx;
      RaggedChunk t = c;
      t.n += 1;
      t.np += k;
      t.nbytes += gb;
      t.nout += gout;
      t.npar += recover ? parity_len[g] : 0;
      const RaggedLayout lay(t, recover);
      if (c.n > 0 && (lay.in_total > in_cap || lay.out_total > out_cap)) break;
      c = t;
    }
    if ((rc = finish(slot))) return rc;
    Slot& s = ctx->slots[slot];
    const RaggedLayout lay(c, recover);
    uint8_t* h = s.h_in;
    uint64_t* h_off = reinterpret_cast<uint64_t*>(h + lay.off);
    uint16_t* h_len = reinterpret_cast<uint16_t*>(h + lay.len);
    uint32_t* h_ptr = reinterpret_cast<uint32_t*>(h + lay.ptr);
    uint64_t* h_poff = reinterpret_cast<uint64_t*>(h + lay.poff);
    uint16_t* h_plen = reinterpret_cast<uint16_t*>(h + lay.plen);
    uint64_t* h_ooff = reinterpret_cast<uint64_t*>(h + lay.ooff);
    uint64_t b = 0, pb = 0, ob = 0;
    uint32_t q = 0;
    for (uint64_t i = 0; i < c.n; ++i) {
      const uint64_t gg = c.g0 + i;
      h_ptr[i] = q;
      uint16_t mx = 0;
      for (uint32_t p = grp_ptr[gg]; p < grp_ptr[gg + 1]; ++p, ++q) {
        h_len[q] = pkt_len[p];
        if (recover && p - grp_ptr[gg] == missing[gg]) {
          h_off[q] = 0;  // the lost packet's entry is never read
          continue;
        }
        std::memcpy(h + b, bytes + pkt_off[p], pkt_len[p]);
        h_off[q] = b;
        b += pkt_len[p];
        mx = std::max(mx, pkt_len[p]);
      }
      if (recover) {
        std::memcpy(h + lay.par + pb, parity + parity_off[gg], parity_len[gg]);
        h_poff[i] = lay.par + pb;
        pb += parity_len[gg];
        h_plen[i] = parity_len[gg];
        h[lay.miss + i] = missing[gg];
        h_ooff[i] = ob;
        ob += parity_len[gg];
      } else {
        h_poff[i] = ob;
        ob += mx;
      }
    }
    h_ptr[c.n] = q;
    QFEC_HIP(ctx, hipMemcpyAsync(s.d_in, s.h_in, lay.in_total, hipMemcpyHostToDevice, s.stream));
    qfec::RaggedArgs a{};
    a.bytes = s.d_in;
    a.pkt_off = reinterpret_cast<const uint64_t*>(s.d_in + lay.off);
    a.pkt_len = reinterpret_cast<const uint16_t*>(s.d_in + lay.len);
    a.grp_ptr = reinterpret_cast<const uint32_t*>(s.d_in + lay.ptr);
    a.n_groups = c.n;
    a.err = ctx->d_err + kErrHost;
    a.out = s.d_out;
    if (recover) {
      a.parity = s.d_in;  // parity_off is relative to the staging base
      a.parity_off = reinterpret_cast<const uint64_t*>(s.d_in + lay.poff);
      a.parity_len = reinterpret_cast<const uint16_t*>(s.d_in + lay.plen);
      a.missing = s.d_in + lay.miss;
      a.out_off = reinterpret_cast<const uint64_t*>(s.d_in + lay.ooff);
    } else {
      a.parity_off = reinterpret_cast<const uint64_t*>(s.d_in + lay.poff);
      a.parity_len_out = reinterpret_cast<uint16_t*>(s.d_out + lay.out_plen);
    }
    // (the chunk's shape is known here: groups of few bytes run two per wave)
    QFEC_HIP(ctx, qfec::launch_ragged(a, recover, s.stream,
                                      c.nbytes < qfec::kRaggedSmallGroupBytes * c.n));
    QFEC_HIP(ctx, hipMemcpyAsync(s.h_out, s.d_out, lay.out_total, hipMemcpyDeviceToHost,
                                 s.stream));
    QFEC_HIP(ctx, hipEventRecord(s.done, s.stream));
    c.live = true;
    chunk[slot] = c;
    slot = (slot + 1) % kSlots;
  }
  for (int i = 0; i < kSlots; ++i)
    if ((rc = finish((slot + i) % kSlots))) return rc;
  return collect_error(ctx, ctx->slots[0].stream, kErrHost);
}


int ragged_mapped(qfec_ctx* ctx, bool recover, const uint8_t* bytes, const uint64_t* pkt_off,
                  const uint16_t* pkt_len, const uint32_t* grp_ptr, uint64_t n,
                  const uint8_t* parity, uint8_t* parity_out, const uint64_t* parity_off,
                  const uint16_t* parity_len, uint16_t* parity_len_out, const uint8_t* missing,
                  uint8_t* out, const uint64_t* out_off, bool async) {
  const bool hst = ctx->svc_sh && ctx->svc_sh->stamp_on;  // (measurement hook)
  if (hst) ctx->svc_hst[0] = steady_ns();
  int rc = ensure_staging(ctx);
  if (rc) return rc;
  if ((rc = check_mapped(ctx, bytes, "bytes")) ||
      (rc = check_mapped(ctx, recover ? out : parity_out, recover ? "out" : "parity_out")) ||
      (recover && (rc = check_mapped(ctx, parity, "parity"))))
    return rc;
  if ((rc = validate_ragged(ctx, recover, pkt_len, grp_ptr, n, parity_len, missing))) return rc;
  // per-chunk table layout in a slot's d_in / h_in (offsets in bytes)
  struct Tab {
    uint64_t off, len, ptr, poff, plen, miss, ooff, total;
    Tab(uint64_t np, uint64_t ng, bool rec) {
      off = 0;
      len = off + np * 8;
      ptr = align_up(len + np * 2, 8);
      poff = align_up(ptr + (ng + 1) * 4, 8);
      ooff = poff + ng * 8;
      plen = ooff + (rec ? ng * 8 : 0);
      miss = plen + (rec ? ng * 2 : 0);
      total = miss + (rec ? ng : 0);
    }
  };
  struct Pend {
    uint64_t g0 = 0, cnt = 0;
    uint32_t token = 0;  // direct: the completion flag's value
    bool svc = false;    // ... set by the small-batch service
    bool live = false;
  } pend[kSlots];
  auto finish = [&](int si) -> int {
    Pend& c = pend[si];
    if (!c.live) return QFEC_OK;
    if (c.token) {
      const int wrc = c.svc ? wait_flag_svc(ctx, si, c.token) : wait_flag(ctx, si, c.token);
      if (hst && c.svc) ctx->svc_hst[2] = steady_ns();
      if (wrc) {
        c.live = false;
        if (c.svc) svc_abandon(ctx);  // no later worker may run the failed job
        return wrc;
      }
    } else {
      QFEC_HIP(ctx, hipEventSynchronize(ctx->slots[si].done));
    }
    if (!recover)
      std::memcpy(parity_len_out + c.g0,
                  c.token != 0u && c.cnt <= kFlagPlens  // (a direct batch: token set)
                      ? static_cast<const void*>(ctx->h_flag + si * kFlagStride + 1)
                      : static_cast<const void*>(ctx->slots[si].h_out),
                  c.cnt * sizeof(uint16_t));
    c.live = false;
    return QFEC_OK;
  };
  const uint64_t out_cap = mapped_chunk_groups((kStageBytes / 4) / sizeof(uint16_t));
  // QFEC_ASYNC: a batch whose tables fit one slot returns once it is queued
  // and completes in qfec_complete; a larger one runs synchronously.  The
  // other calls that use the slots finish the async ones first.
  async = async && n <= out_cap && Tab(grp_ptr[n] - grp_ptr[0], n, recover).total <= kStageBytes;
  int slot = 0;
  if (async) {
    slot = ctx->async_next;
    retire_async_op(ctx, slot);
  } else {
    drain_async(ctx);
  }
  // A batch whose tables fit one slot (every batch a connection thread
  // flushes) runs DIRECT: the kernel reads the tables from the mapped slot
  // buffer and writes the encode lengths straight into the mapped output
  // buffer, and its last workgroup stores a completion token into
  // host-mapped memory -- no staging copies, no event, one launch -- and the
  // error word is not fetched: validate_ragged checked every condition the
  // kernel latches.  Up to kDirectGroups groups the small-batch kernel (one
  // wave per group, every load of a group in flight at once: latency over
  // PCIe), above that the block kernel.  (Round 3 staged the tables of
  // batches above kDirectGroups to the device and waited on an event.)
  const bool direct =
      n <= out_cap && Tab(grp_ptr[n] - grp_ptr[0], n, recover).total <= kStageBytes;
  // a large chunk's shape (the host holds the tables): groups of few bytes
  // run two per wave (launch_ragged small_groups)
  auto small_groups = [&](uint64_t p0, uint64_t np, uint64_t cnt) {
    uint64_t nb = 0;
    for (uint64_t p = p0; p < p0 + np; ++p) nb += pkt_len[p];
    return nb < qfec::kRaggedSmallGroupBytes * cnt;
  };
  uint64_t g = 0;
  while (g < n) {
    const uint64_t g0 = g;
    for (; g < n; ++g) {  // whole groups while the tables fit
      const Tab t(grp_ptr[g + 1] - grp_ptr[g0], g + 1 - g0, recover);
      if (g > g0 && (t.total > kStageBytes || g + 1 - g0 > out_cap)) break;
    }
    const uint64_t cnt = g - g0, p0 = grp_ptr[g0], np = grp_ptr[g] - p0;
    const Tab t(np, cnt, recover);
    if ((rc = finish(slot))) return rc;
    Slot& s = ctx->slots[slot];
    // a few groups go to the resident service worker, their index tables
    // written INLINE into its ring entry (the worker reads entry and tables
    // in one round trip); everything else through the slot's mapped buffer
    bool svc = direct && ctx->svc_on && cnt <= kSvcGroups && t.total <= qfec::kSvcTab &&
               ensure_service(ctx) == QFEC_OK;
    if (!svc && (rc = bind(ctx))) return rc;  // (a launch follows; the service binds itself)
    qfec::SvcJob* je = svc ? svc_next_entry(ctx) : nullptr;
    uint8_t* h = svc ? je->tab : s.h_in;
    std::memcpy(h + t.off, pkt_off + p0, np * 8);  // payloads stay where they are
    std::memcpy(h + t.len, pkt_len + p0, np * 2);
    uint32_t* h_ptr = reinterpret_cast<uint32_t*>(h + t.ptr);
    for (uint64_t i = 0; i <= cnt; ++i) h_ptr[i] = grp_ptr[g0 + i] - (uint32_t)p0;
    std::memcpy(h + t.poff, parity_off + g0, cnt * 8);
    if (recover) {
      std::memcpy(h + t.ooff, out_off + g0, cnt * 8);
      std::memcpy(h + t.plen, parity_len + g0, cnt * 2);
      std::memcpy(h + t.miss, missing + g0, cnt);
    }
    uint8_t* tab = s.h_in_dev;  // direct: the device reads the tables where they are
    if (!direct) {
      QFEC_HIP(ctx, hipMemcpyAsync(s.d_in, h, t.total, hipMemcpyHostToDevice, s.stream));
      tab = s.d_in;
    }
    qfec::RaggedArgs a{};
    a.bytes = bytes;
    a.pkt_off = reinterpret_cast<const uint64_t*>(tab + t.off);
    a.pkt_len = reinterpret_cast<const uint16_t*>(tab + t.len);
    a.grp_ptr = reinterpret_cast<const uint32_t*>(tab + t.ptr);
    a.parity_off = reinterpret_cast<const uint64_t*>(tab + t.poff);
    a.n_groups = cnt;
    a.err = ctx->d_err + (async ? kErrSlot0 + slot : kErrHost);
    if (recover) {
      a.parity = parity;
      a.parity_len = reinterpret_cast<const uint16_t*>(tab + t.plen);
      a.missing = tab + t.miss;
      a.out_off = reinterpret_cast<const uint64_t*>(tab + t.ooff);
      a.out = out;
    } else {
      a.parity_len_out = reinterpret_cast<uint16_t*>(
          !direct ? s.d_out
                  : cnt <= kFlagPlens ? reinterpret_cast<uint8_t*>(ctx->h_flag_dev + slot * kFlagStride + 1)
                                      : s.h_out_dev);
      a.out = parity_out;
    }
    uint32_t token = 0;
    if (direct) {
      token = ++ctx->flag_token ? ctx->flag_token : ++ctx->flag_token;  // never 0
      a.done_count = ctx->d_done + slot;
      a.done_flag = ctx->h_flag_dev + slot * kFlagStride;
      a.done_token = token;
      // a few groups: the resident service worker takes them from its ring
      // (no launch); a flag is all their completion needs
      const SvcTabs tb{(uint32_t)t.total, (uint32_t)t.off, (uint32_t)t.len, (uint32_t)t.ptr,
                       (uint32_t)t.poff, (uint32_t)t.plen, (uint32_t)t.miss, (uint32_t)t.ooff};
      const bool sub_fail = svc && svc_submit(ctx, slot, a, recover, token, tb) != QFEC_OK;
      if (hst && svc) ctx->svc_hst[1] = steady_ns();
      if (sub_fail) {
        // the service could not be set up or (re)launched: off for this
        // context, this batch launched as before (same flag and token), its
        // tables moved from the ring entry to the slot buffer the launch reads
        __atomic_store_n(&ctx->svc_on, false, __ATOMIC_RELEASE);
        svc = false;
        std::memcpy(s.h_in, je->tab, t.total);
        if ((rc = bind(ctx))) return rc;
      }
      if (!svc) {
        if (cnt <= kDirectGroups)
          QFEC_HIP(ctx, qfec::launch_ragged_latency(a, recover, s.stream));
        else
          QFEC_HIP(ctx, qfec::launch_ragged(a, recover, s.stream, small_groups(p0, np, cnt)));
      }
    } else {
      QFEC_HIP(ctx, qfec::launch_ragged(a, recover, s.stream, small_groups(p0, np, cnt)));
    }
    if (!recover && !direct)
      QFEC_HIP(ctx, hipMemcpyAsync(s.h_out, s.d_out, cnt * sizeof(uint16_t),
                                   hipMemcpyDeviceToHost, s.stream));
    if (!svc) QFEC_HIP(ctx, hipEventRecord(s.done, s.stream));
    if (async) {  // the whole batch in this slot: completed by qfec_complete
      qfec_ctx::AsyncOp& op = ctx->async_ops[slot];
      op.live = true;
      op.direct = direct;
      op.svc = svc;
      op.recover = recover;
      op.token = token;
      op.cnt = cnt;
      op.parity_len_out = recover ? nullptr : parity_len_out;
      op.seq = ++ctx->async_seq;
      ctx->last_ticket = op.seq;
      ctx->async_next = (slot + 1) % kSlots;
      return QFEC_OK;
    }
    pend[slot].g0 = g0;
    pend[slot].cnt = cnt;
    pend[slot].token = token;
    pend[slot].svc = svc;
    pend[slot].live = true;
    slot = (slot + 1) % kSlots;
  }
  for (int i = 0; i < kSlots; ++i)
    if ((rc = finish((slot + i) % kSlots))) return rc;
  if (hst) ctx->svc_hst[3] = steady_ns();
  return direct ? QFEC_OK : collect_error(ctx, ctx->slots[0].stream, kErrHost);
}

}  // namespace

int qfec_encode_ragged(qfec_ctx* ctx, const uint8_t* bytes, const uint64_t* pkt_off,
                       const uint16_t* pkt_len, const uint32_t* grp_ptr, uint64_t n_groups,
                       uint8_t* parity_out, const uint64_t* parity_off,
                       uint16_t* parity_len_out, uint32_t flags) {
  // (mapped batches bind where they launch: ragged_mapped)
  int rc = (flags & QFEC_PTR_MAPPED) && ctx ? QFEC_OK : bind(ctx);
  if (rc) return rc;
  ctx->last_ticket = 0;
  if (ctx->debug_fail)
    return fail(ctx, QFEC_ERR_INTERNAL, "launch failure injected (qfec_debug_fail_launches)");
  if (n_groups == 0) return QFEC_OK;
  if (!bytes || !pkt_off || !pkt_len || !grp_ptr || !parity_out || !parity_off || !parity_len_out)
    return fail(ctx, QFEC_ERR_INTERNAL, "null buffer");
  if ((flags & QFEC_PTR_MAPPED) && (flags & QFEC_PTR_HOST))
    return fail(ctx, QFEC_ERR_INTERNAL, "QFEC_PTR_MAPPED and QFEC_PTR_HOST are exclusive");
  if (flags & QFEC_PTR_MAPPED)
    return ragged_mapped(ctx, false, bytes, pkt_off, pkt_len, grp_ptr, n_groups, nullptr,
                         parity_out, parity_off, nullptr, parity_len_out, nullptr, nullptr,
                         nullptr, (flags & QFEC_ASYNC) != 0);
  if (flags & QFEC_PTR_HOST)
    return ragged_host(ctx, false, bytes, pkt_off, pkt_len, grp_ptr, n_groups, nullptr,
                       parity_out, parity_off, nullptr, parity_len_out, nullptr, nullptr,
                       nullptr);
  qfec::RaggedArgs a{};
  a.bytes = bytes;
  a.pkt_off = pkt_off;
  a.pkt_len = pkt_len;
  a.grp_ptr = grp_ptr;
  a.parity_off = parity_off;
  a.parity_len_out = parity_len_out;
  a.out = parity_out;
  a.n_groups = n_groups;
  a.err = ctx->d_err;
  QFEC_HIP(ctx, qfec::launch_ragged(a, false, ctx->stream, (flags & QFEC_SMALL_GROUPS) != 0));
  return QFEC_OK;
}

int qfec_recover_ragged(qfec_ctx* ctx, const uint8_t* bytes, const uint64_t* pkt_off,
                        const uint16_t* pkt_len, const uint32_t* grp_ptr, uint64_t n_groups,
                        const uint8_t* parity, const uint64_t* parity_off,
                        const uint16_t* parity_len, const uint8_t* missing_idx, uint8_t* out,
                        const uint64_t* out_off, uint32_t flags) {
  // (mapped batches bind where they launch: ragged_mapped)
  int rc = (flags & QFEC_PTR_MAPPED) && ctx ? QFEC_OK : bind(ctx);
  if (rc) return rc;
  ctx->last_ticket = 0;
  if (ctx->debug_fail)
    return fail(ctx, QFEC_ERR_INTERNAL, "launch failure injected (qfec_debug_fail_launches)");
  if (n_groups == 0) return QFEC_OK;
  if (!bytes || !pkt_off || !pkt_len || !grp_ptr || !parity || !parity_off || !parity_len ||
      !missing_idx || !out || !out_off)
    return fail(ctx, QFEC_ERR_INTERNAL, "null buffer");
  if ((flags & QFEC_PTR_MAPPED) && (flags & QFEC_PTR_HOST))
    return fail(ctx, QFEC_ERR_INTERNAL, "QFEC_PTR_MAPPED and QFEC_PTR_HOST are exclusive");
  if (flags & (QFEC_PTR_HOST | QFEC_PTR_MAPPED)) {
    for (uint64_t g = 0; g < n_groups; ++g) {
      const uint32_t k = grp_ptr[g + 1] - grp_ptr[g];
      if (grp_ptr[g + 1] < grp_ptr[g] || k == 0 || k > QFEC_MAX_GROUP_PACKETS)
        return fail(ctx, QFEC_ERR_INVALID_FEC_DATA, "FEC group %llu has %u packets",
                    (unsigned long long)g, k);
      if (missing_idx[g] >= k)
        return fail(ctx, QFEC_ERR_INVALID_FEC_DATA, "missing packet index %u >= %u",
                    missing_idx[g], k);
      if (parity_len[g] == 0 || parity_len[g] > QFEC_MAX_PACKET_SIZE)
        return fail(ctx, QFEC_ERR_INVALID_FEC_DATA, "Illegal FEC redundancy length %u",
                    parity_len[g]);
    }
    if (flags & QFEC_PTR_MAPPED)
      return ragged_mapped(ctx, true, bytes, pkt_off, pkt_len, grp_ptr, n_groups, parity,
                           nullptr, parity_off, parity_len, nullptr, missing_idx, out, out_off,
                           (flags & QFEC_ASYNC) != 0);
    return ragged_host(ctx, true, bytes, pkt_off, pkt_len, grp_ptr, n_groups, parity, nullptr,
                       parity_off, parity_len, nullptr, missing_idx, out, out_off);
  }
  qfec::RaggedArgs a{};
  a.bytes = bytes;
  a.pkt_off = pkt_off;
  a.pkt_len = pkt_len;
  a.grp_ptr = grp_ptr;
  a.parity = parity;
  a.parity_off = parity_off;
  a.parity_len = parity_len;
  a.missing = missing_idx;
  a.out = out;
  a.out_off = out_off;
  a.n_groups = n_groups;
  a.err = ctx->d_err;
  QFEC_HIP(ctx, qfec::launch_ragged(a, true, ctx->stream, (flags & QFEC_SMALL_GROUPS) != 0));
  return QFEC_OK;
}

int qfec_xor_into(qfec_ctx* ctx, const uint8_t* in, uint64_t n, uint8_t* out, uint32_t flags) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (n == 0) return QFEC_OK;
  if (!in || !out) return fail(ctx, QFEC_ERR_INTERNAL, "null buffer");
  if ((flags & QFEC_PTR_MAPPED) && (flags & QFEC_PTR_HOST))
    return fail(ctx, QFEC_ERR_INTERNAL, "QFEC_PTR_MAPPED and QFEC_PTR_HOST are exclusive");
  if (flags & QFEC_PTR_MAPPED) {
    if ((rc = check_mapped(ctx, in, "in")) || (rc = check_mapped(ctx, out, "out"))) return rc;
    QFEC_HIP(ctx, qfec::launch_xor_into(in, n, out, ctx->stream));
    QFEC_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return QFEC_OK;
  }
  if (flags & QFEC_PTR_HOST) {
    DevBuf d_in, d_out;
    size_t si = 0;
    QFEC_HIP(ctx, scratch(ctx, si++, n, &d_in.p));
    QFEC_HIP(ctx, scratch(ctx, si++, n, &d_out.p));
    QFEC_HIP(ctx, hipMemcpyAsync(d_in.p, in, n, hipMemcpyHostToDevice, ctx->stream));
    QFEC_HIP(ctx, hipMemcpyAsync(d_out.p, out, n, hipMemcpyHostToDevice, ctx->stream));
    QFEC_HIP(ctx, qfec::launch_xor_into(static_cast<const uint8_t*>(d_in.p), n,
                                        static_cast<uint8_t*>(d_out.p), ctx->stream));
    QFEC_HIP(ctx, hipMemcpyAsync(out, d_out.p, n, hipMemcpyDeviceToHost, ctx->stream));
    QFEC_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return QFEC_OK;
  }
  QFEC_HIP(ctx, qfec::launch_xor_into(in, n, out, ctx->stream));
  return QFEC_OK;
}

// ---- packet protection -----------------------------------------------------
namespace {

// Host-pointer path: stage the byte span the batch touches, its index arrays
// and the output span through device allocations.
// aead == nullptr: NULL protection; otherwise its key table / per-packet
// arrays (host pointers) are staged too and the ChaCha20-Poly1305 kernels run.
struct AeadHost {
  const uint8_t* keys;
  const uint8_t* prefixes;
  const uint32_t* key_idx;
  const uint64_t* packet_number;
  const uint8_t* path_id;
  bool aes;  // AES-128-GCM (16-B keys) instead of ChaCha20-Poly1305 (32-B keys)
};

int protect_host(qfec_ctx* ctx, bool decrypt, const uint8_t* bytes, const uint64_t* ad_off,
                 const uint16_t* ad_len, const uint64_t* in_off, const uint16_t* in_len,
                 uint64_t n, uint8_t* out, const uint64_t* out_off, uint8_t* ok,
                 const AeadHost* aead = nullptr) {
  uint64_t lo = UINT64_MAX, hi = 0, olo = UINT64_MAX, ohi = 0;
  for (uint64_t p = 0; p < n; ++p) {
    lo = std::min({lo, ad_off[p], in_off[p]});
    hi = std::max({hi, ad_off[p] + ad_len[p], in_off[p] + in_len[p]});
    const uint64_t olen = decrypt ? (in_len[p] >= 12 ? in_len[p] - 12u : 0u) : in_len[p] + 12u;
    olo = std::min(olo, out_off[p]);
    ohi = std::max(ohi, out_off[p] + olen);
  }
  std::vector<uint64_t> aoff(n), ioff(n), ooff(n);
  for (uint64_t p = 0; p < n; ++p) {
    aoff[p] = ad_off[p] - lo;
    ioff[p] = in_off[p] - lo;
    ooff[p] = out_off[p] - olo;
  }
  hipStream_t st = ctx->stream;
  DevBuf d_bytes, d_aoff, d_alen, d_ioff, d_ilen, d_out, d_ooff, d_ok;
  size_t si = 0;
  QFEC_HIP(ctx, scratch(ctx, si++, std::max<uint64_t>(hi - lo, 1), &d_bytes.p));
  QFEC_HIP(ctx, scratch(ctx, si++, n * 8, &d_aoff.p));
  QFEC_HIP(ctx, scratch(ctx, si++, n * 2, &d_alen.p));
  QFEC_HIP(ctx, scratch(ctx, si++, n * 8, &d_ioff.p));
  QFEC_HIP(ctx, scratch(ctx, si++, n * 2, &d_ilen.p));
  QFEC_HIP(ctx, scratch(ctx, si++, std::max<uint64_t>(ohi - olo, 1), &d_out.p));
  QFEC_HIP(ctx, scratch(ctx, si++, n * 8, &d_ooff.p));
  QFEC_HIP(ctx, hipMemcpyAsync(d_bytes.p, bytes + lo, hi - lo, hipMemcpyHostToDevice, st));
  QFEC_HIP(ctx, hipMemcpyAsync(d_aoff.p, aoff.data(), n * 8, hipMemcpyHostToDevice, st));
  QFEC_HIP(ctx, hipMemcpyAsync(d_alen.p, ad_len, n * 2, hipMemcpyHostToDevice, st));
  QFEC_HIP(ctx, hipMemcpyAsync(d_ioff.p, ioff.data(), n * 8, hipMemcpyHostToDevice, st));
  QFEC_HIP(ctx, hipMemcpyAsync(d_ilen.p, in_len, n * 2, hipMemcpyHostToDevice, st));
  QFEC_HIP(ctx, hipMemcpyAsync(d_ooff.p, ooff.data(), n * 8, hipMemcpyHostToDevice, st));
  // seed the output span with the caller's bytes (gaps and failed packets stay)
  QFEC_HIP(ctx, hipMemcpyAsync(d_out.p, out + olo, ohi - olo, hipMemcpyHostToDevice, st));
  if (decrypt) QFEC_HIP(ctx, scratch(ctx, si++, n, &d_ok.p));
  qfec::ProtectArgs a{};
  a.bytes = static_cast<const uint8_t*>(d_bytes.p);
  a.ad_off = static_cast<const uint64_t*>(d_aoff.p);
  a.ad_len = static_cast<const uint16_t*>(d_alen.p);
  a.in_off = static_cast<const uint64_t*>(d_ioff.p);
  a.in_len = static_cast<const uint16_t*>(d_ilen.p);
  a.out = static_cast<uint8_t*>(d_out.p);
  a.out_off = static_cast<const uint64_t*>(d_ooff.p);
  a.ok = static_cast<uint8_t*>(d_ok.p);
  a.n = n;
  if (aead) {
    uint32_t nkeys = 0;
    for (uint64_t p = 0; p < n; ++p) nkeys = std::max(nkeys, aead->key_idx[p] + 1u);
    DevBuf d_keys, d_pre, d_kidx, d_pn, d_path;
    const uint64_t ksz = aead->aes ? 16ull : 32ull;
    QFEC_HIP(ctx, scratch(ctx, si++, ksz * nkeys, &d_keys.p));
    QFEC_HIP(ctx, scratch(ctx, si++, 4ull * nkeys, &d_pre.p));
    QFEC_HIP(ctx, scratch(ctx, si++, n * 4, &d_kidx.p));
    QFEC_HIP(ctx, scratch(ctx, si++, n * 8, &d_pn.p));
    QFEC_HIP(ctx, hipMemcpyAsync(d_keys.p, aead->keys, ksz * nkeys, hipMemcpyHostToDevice, st));
    QFEC_HIP(ctx, hipMemcpyAsync(d_pre.p, aead->prefixes, 4ull * nkeys, hipMemcpyHostToDevice, st));
    QFEC_HIP(ctx, hipMemcpyAsync(d_kidx.p, aead->key_idx, n * 4, hipMemcpyHostToDevice, st));
    QFEC_HIP(ctx, hipMemcpyAsync(d_pn.p, aead->packet_number, n * 8, hipMemcpyHostToDevice, st));
    if (aead->path_id) {
      QFEC_HIP(ctx, scratch(ctx, si++, n, &d_path.p));
      QFEC_HIP(ctx, hipMemcpyAsync(d_path.p, aead->path_id, n, hipMemcpyHostToDevice, st));
    }
    qfec::AeadArgs aa{};
    aa.io = a;
    aa.keys = static_cast<const uint8_t*>(d_keys.p);
    aa.prefixes = static_cast<const uint8_t*>(d_pre.p);
    aa.key_idx = static_cast<const uint32_t*>(d_kidx.p);
    aa.packet_number = static_cast<const uint64_t*>(d_pn.p);
    aa.path_id = static_cast<const uint8_t*>(d_path.p);
    QFEC_HIP(ctx, aead->aes ? qfec::launch_aes128gcm(aa, decrypt, st)
                            : qfec::launch_chacha20poly1305(aa, decrypt, st));
    QFEC_HIP(ctx, hipMemcpyAsync(out + olo, d_out.p, ohi - olo, hipMemcpyDeviceToHost, st));
    if (decrypt) QFEC_HIP(ctx, hipMemcpyAsync(ok, d_ok.p, n, hipMemcpyDeviceToHost, st));
    QFEC_HIP(ctx, hipStreamSynchronize(st));
    return QFEC_OK;
  }
  QFEC_HIP(ctx, qfec::launch_null_protect(a, decrypt, st));
  QFEC_HIP(ctx, hipMemcpyAsync(out + olo, d_out.p, ohi - olo, hipMemcpyDeviceToHost, st));
  if (decrypt) QFEC_HIP(ctx, hipMemcpyAsync(ok, d_ok.p, n, hipMemcpyDeviceToHost, st));
  QFEC_HIP(ctx, hipStreamSynchronize(st));
  return QFEC_OK;
}

int null_protect(qfec_ctx* ctx, bool decrypt, const uint8_t* bytes, const uint64_t* ad_off,
                 const uint16_t* ad_len, const uint64_t* in_off, const uint16_t* in_len,
                 uint64_t n, uint8_t* out, const uint64_t* out_off, uint8_t* ok,
                 uint32_t flags) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (n == 0) return QFEC_OK;
  if (!bytes || !ad_off || !ad_len || !in_off || !in_len || !out || !out_off || (decrypt && !ok))
    return fail(ctx, QFEC_ERR_INTERNAL, "null buffer");
  if (flags & QFEC_PTR_HOST)
    return protect_host(ctx, decrypt, bytes, ad_off, ad_len, in_off, in_len, n, out, out_off, ok);
  qfec::ProtectArgs a{};
  a.bytes = bytes;
  a.ad_off = ad_off;
  a.ad_len = ad_len;
  a.in_off = in_off;
  a.in_len = in_len;
  a.out = out;
  a.out_off = out_off;
  a.ok = ok;
  a.n = n;
  a.scratch_out = (flags & QFEC_SCRATCH_OUTPUT) ? 1u : 0u;
  QFEC_HIP(ctx, qfec::launch_null_protect(a, decrypt, ctx->stream));
  return QFEC_OK;
}

}  // namespace

int aead_protect(qfec_ctx* ctx, bool aes, bool decrypt, const uint8_t* keys, const uint8_t* prefixes,
                   const uint32_t* key_idx, const uint64_t* packet_number, const uint8_t* path_id,
                   const uint8_t* bytes, const uint64_t* ad_off, const uint16_t* ad_len,
                   const uint64_t* in_off, const uint16_t* in_len, uint64_t n, uint8_t* out,
                   const uint64_t* out_off, uint8_t* ok, uint32_t flags) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (n == 0) return QFEC_OK;
  if (!keys || !prefixes || !key_idx || !packet_number || !bytes || !ad_off || !ad_len ||
      !in_off || !in_len || !out || !out_off || (decrypt && !ok))
    return fail(ctx, QFEC_ERR_INTERNAL, "null buffer");
  if (flags & QFEC_PTR_HOST) {
    const AeadHost h{keys, prefixes, key_idx, packet_number, path_id, aes};
    return protect_host(ctx, decrypt, bytes, ad_off, ad_len, in_off, in_len, n, out, out_off, ok,
                        &h);
  }
  qfec::AeadArgs a{};
  a.io.bytes = bytes;
  a.io.ad_off = ad_off;
  a.io.ad_len = ad_len;
  a.io.in_off = in_off;
  a.io.in_len = in_len;
  a.io.out = out;
  a.io.out_off = out_off;
  a.io.ok = ok;
  a.io.n = n;
  a.io.scratch_out = (decrypt && (flags & QFEC_SCRATCH_OUTPUT)) ? 1u : 0u;
  a.keys = keys;
  a.prefixes = prefixes;
  a.key_idx = key_idx;
  a.packet_number = packet_number;
  a.path_id = path_id;
  QFEC_HIP(ctx, aes ? qfec::launch_aes128gcm(a, decrypt, ctx->stream)
                    : qfec::launch_chacha20poly1305(a, decrypt, ctx->stream));
  return QFEC_OK;
}

int qfec_null_encrypt_batch(qfec_ctx* ctx, const uint8_t* bytes, const uint64_t* ad_off,
                            const uint16_t* ad_len, const uint64_t* in_off,
                            const uint16_t* in_len, uint64_t n_packets, uint8_t* out,
                            const uint64_t* out_off, uint32_t flags) {
  return null_protect(ctx, false, bytes, ad_off, ad_len, in_off, in_len, n_packets, out, out_off,
                      nullptr, flags);
}

int qfec_null_decrypt_batch(qfec_ctx* ctx, const uint8_t* bytes, const uint64_t* ad_off,
                            const uint16_t* ad_len, const uint64_t* in_off,
                            const uint16_t* in_len, uint64_t n_packets, uint8_t* out,
                            const uint64_t* out_off, uint8_t* ok, uint32_t flags) {
  return null_protect(ctx, true, bytes, ad_off, ad_len, in_off, in_len, n_packets, out, out_off,
                      ok, flags);
}

int qfec_chacha20poly1305_seal_batch(qfec_ctx* ctx, const uint8_t* keys, const uint8_t* prefixes,
                                     const uint32_t* key_idx, const uint64_t* packet_number,
                                     const uint8_t* path_id, const uint8_t* bytes,
                                     const uint64_t* ad_off, const uint16_t* ad_len,
                                     const uint64_t* in_off, const uint16_t* in_len,
                                     uint64_t n_packets, uint8_t* out, const uint64_t* out_off,
                                     uint32_t flags) {
  return aead_protect(ctx, false, false, keys, prefixes, key_idx, packet_number, path_id, bytes,
                        ad_off, ad_len, in_off, in_len, n_packets, out, out_off, nullptr, flags);
}

int qfec_chacha20poly1305_open_batch(qfec_ctx* ctx, const uint8_t* keys, const uint8_t* prefixes,
                                     const uint32_t* key_idx, const uint64_t* packet_number,
                                     const uint8_t* path_id, const uint8_t* bytes,
                                     const uint64_t* ad_off, const uint16_t* ad_len,
                                     const uint64_t* in_off, const uint16_t* in_len,
                                     uint64_t n_packets, uint8_t* out, const uint64_t* out_off,
                                     uint8_t* ok, uint32_t flags) {
  return aead_protect(ctx, false, true, keys, prefixes, key_idx, packet_number, path_id, bytes,
                        ad_off, ad_len, in_off, in_len, n_packets, out, out_off, ok, flags);
}

int qfec_aes128gcm_seal_batch(qfec_ctx* ctx, const uint8_t* keys, const uint8_t* prefixes,
                              const uint32_t* key_idx, const uint64_t* packet_number,
                              const uint8_t* path_id, const uint8_t* bytes, const uint64_t* ad_off,
                              const uint16_t* ad_len, const uint64_t* in_off,
                              const uint16_t* in_len, uint64_t n_packets, uint8_t* out,
                              const uint64_t* out_off, uint32_t flags) {
  return aead_protect(ctx, true, false, keys, prefixes, key_idx, packet_number, path_id, bytes,
                      ad_off, ad_len, in_off, in_len, n_packets, out, out_off, nullptr, flags);
}

int qfec_aes128gcm_open_batch(qfec_ctx* ctx, const uint8_t* keys, const uint8_t* prefixes,
                              const uint32_t* key_idx, const uint64_t* packet_number,
                              const uint8_t* path_id, const uint8_t* bytes, const uint64_t* ad_off,
                              const uint16_t* ad_len, const uint64_t* in_off,
                              const uint16_t* in_len, uint64_t n_packets, uint8_t* out,
                              const uint64_t* out_off, uint8_t* ok, uint32_t flags) {
  return aead_protect(ctx, true, true, keys, prefixes, key_idx, packet_number, path_id, bytes,
                      ad_off, ad_len, in_off, in_len, n_packets, out, out_off, ok, flags);
}

int qfec_stream_probe(qfec_ctx* ctx, const uint8_t* src, uint64_t n, uint8_t* dst, int mode) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (!src || !dst) return fail(ctx, QFEC_ERR_INTERNAL, "null buffer");
  if (mode != 0 && mode != 1) return fail(ctx, QFEC_ERR_INTERNAL, "probe mode %d", mode);
  QFEC_HIP(ctx, qfec::launch_stream_probe(src, n, dst, mode == 1, ctx->stream));
  return QFEC_OK;
}

int qfec_phase_abandons(qfec_ctx* ctx, uint32_t* count) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (!count) return fail(ctx, QFEC_ERR_INTERNAL, "null count");
  QFEC_HIP(ctx, hipStreamSynchronize(ctx->stream));
  QFEC_HIP(ctx, hipMemcpy(count, ctx->d_phase + 64 * 19, sizeof(uint32_t), hipMemcpyDeviceToHost));
  return QFEC_OK;
}

int qfec_phase_backoff(qfec_ctx* ctx) { return ctx ? (int)ctx->phase_backoff : -1; }

int qfec_last_fixed_phased(const qfec_ctx* ctx) { return ctx ? ctx->last_fixed_phased : -1; }

uint32_t qfec_debug_last_phase_grid(const qfec_ctx* ctx) { return ctx ? ctx->last_phase_grid : 0u; }

int qfec_service_warm(qfec_ctx* ctx) {
  // the worker already running (a loop turn's usual case): no runtime call;
  // the warm count it polls restarts its idle time (a turn that takes most
  // of the 100 us to assemble its batch still finds it resident)
  if (ctx && ctx->svc_on && ctx->svc_sh &&
      __atomic_load_n(&ctx->svc_sh->alive, __ATOMIC_SEQ_CST) != 0u) {
    const uint64_t now = steady_ns();
    __atomic_store_n(&ctx->svc_used_ns, now, __ATOMIC_RELEASE);
    // (not past the residency bound: warm calls alone, with no job for
    // svc_submit to rotate at, must not keep a worker on its hardware queue)
    if (now - ctx->svc_launch_ns < ctx->svc_max_resident_ns)
      __atomic_store_n(&ctx->svc_sh->warm, ctx->svc_sh->warm + 1u, __ATOMIC_RELEASE);
    return QFEC_OK;
  }
  int rc = bind(ctx);
  if (rc) return rc;
  if (!ctx->svc_on) return QFEC_OK;
  if ((rc = ensure_staging(ctx)) || (rc = ensure_service(ctx))) return rc;
  __atomic_store_n(&ctx->svc_used_ns, steady_ns(), __ATOMIC_RELEASE);
  qfec::SvcShared* sh = ctx->svc_sh;
  if (__atomic_load_n(&sh->alive, __ATOMIC_SEQ_CST) != 0u) return QFEC_OK;
  // nothing is published here, so a worker that is leaving needs no second
  // look: a spare one queued behind it on the stream idles out in turn
  __atomic_store_n(&sh->alive, 1u, __ATOMIC_SEQ_CST);
  const hipError_t e = qfec::launch_ragged_service(ctx->svc_sh_dev, ctx->svc_dev, ctx->svc_ring_dev,
                                                   ctx->h_flag_dev, ctx->svc_idle_ticks, ++ctx->svc_epoch,
                                                   ctx->svc_stream);
  if (e != hipSuccess) {
    __atomic_store_n(&sh->alive, 0u, __ATOMIC_SEQ_CST);
    __atomic_store_n(&ctx->svc_on, false, __ATOMIC_RELEASE);
    return fail(ctx, QFEC_ERR_INTERNAL, "small-batch service launch: %s", hipGetErrorString(e));
  }
  ++ctx->svc_launches;
  ctx->svc_launch_ns = steady_ns();
  return QFEC_OK;
}

int qfec_debug_service(qfec_ctx* ctx, int on, uint64_t* stats) {
  if (!ctx) return fail(nullptr, QFEC_ERR_INTERNAL, "null qfec_ctx");
  if (on == 2) {
    // test hook: the next job's ring entry is written with
    // a wrong job number, so the worker finds its groups in no entry
    __atomic_store_n(&ctx->svc_on, true, __ATOMIC_RELEASE);
    ctx->svc_poison_next = true;
    if (ctx->svc_sh) __atomic_store_n(&ctx->svc_sh->quit, 0u, __ATOMIC_SEQ_CST);
  } else if (on == 0 || on == 1) {
    __atomic_store_n(&ctx->svc_on, on != 0, __ATOMIC_RELEASE);
    if (!ctx->svc_on) {
      stop_service(ctx);  // a resident worker leaves at once
    } else if (ctx->svc_sh) {
      __atomic_store_n(&ctx->svc_sh->quit, 0u, __ATOMIC_SEQ_CST);
    }
  }
  if (stats) {
    stats[0] = ctx->svc_launches;
    stats[1] = ctx->svc_sh ? __atomic_load_n(&ctx->svc_sh->jobs, __ATOMIC_ACQUIRE) : 0;
    stats[2] = ctx->svc_sh ? __atomic_load_n(&ctx->svc_sh->alive, __ATOMIC_ACQUIRE) : 0;
  }
  if (stats && on == 3) {  // (mode 3: the query plus the registry's view of this context)
    stats[3] = ctx->svc_stream && hipStreamQuery(ctx->svc_stream) == hipErrorNotReady ? 1u : 0u;
    const uint64_t used = __atomic_load_n(&ctx->svc_used_ns, __ATOMIC_ACQUIRE);
    stats[4] = used ? (steady_ns() - used) / 1000u : ~0ull;  // us since its last job / warm
    stats[5] = ctx->svc_rotations;
  }
  return QFEC_OK;
}

int qfec_debug_service_hold(qfec_ctx* ctx, int hold) {
  if (!ctx) return fail(nullptr, QFEC_ERR_INTERNAL, "null qfec_ctx");
  int rc = ensure_service(ctx);
  if (rc) return rc;
  __atomic_store_n(&ctx->svc_sh->hold, hold ? 1u : 0u, __ATOMIC_SEQ_CST);
  return QFEC_OK;
}

int qfec_debug_service_stamps(qfec_ctx* ctx, int on, uint64_t* stamps) {
  if (!ctx) return fail(nullptr, QFEC_ERR_INTERNAL, "null qfec_ctx");
  int rc = ensure_service(ctx);
  if (rc) return rc;
  if (on >= 0) __atomic_store_n(&ctx->svc_sh->stamp_on, on ? 1u : 0u, __ATOMIC_SEQ_CST);
  if (stamps)
    for (int q = 0; q < 6; ++q)
      stamps[q] = __atomic_load_n(&ctx->svc_sh->stamps[q], __ATOMIC_ACQUIRE);
  return QFEC_OK;
}

int qfec_debug_service_trace(qfec_ctx* ctx, uint64_t* out) {
  if (!ctx || !out) return fail(ctx, QFEC_ERR_INTERNAL, "qfec_debug_service_trace: null argument");
  int rc = ensure_service(ctx);
  if (rc) return rc;
  for (int q = 0; q < 8; ++q) out[q] = __atomic_load_n(&ctx->svc_sh->stamps[q], __ATOMIC_ACQUIRE);
  for (uint32_t w = 0; w < qfec::kSvcWgs; ++w)
    for (int q = 0; q < 4; ++q)
      out[8 + 4 * w + q] = __atomic_load_n(&ctx->svc_sh->wg_stamps[w][q], __ATOMIC_ACQUIRE);
  for (int q = 0; q < 4; ++q) out[8 + 4 * qfec::kSvcWgs + q] = ctx->svc_hst[q];
  return QFEC_OK;
}

uint64_t qfec_debug_service_idle(qfec_ctx* ctx, uint64_t us) {
  if (!ctx) return 0;
  const uint64_t prev = ctx->svc_idle_ticks / 100u;
  ctx->svc_idle_ticks = us * 100u;  // 100-MHz ticks
  return prev;
}

uint64_t qfec_debug_service_resident(qfec_ctx* ctx, uint64_t ns) {
  if (!ctx) return 0;
  const uint64_t prev = ctx->svc_max_resident_ns;
  ctx->svc_max_resident_ns = ns;
  return prev;
}

// Measurement hook (round 6, bench leg phase_beside_service): a native
// connection thread that owns ctx until stopped and flushes one-group mapped
// batches back to back, warming the worker at each turn's start -- what an
// event loop with one connection per turn does.  A Python feeder thread
// starved the measuring thread of the GIL for seconds at a time.
namespace {
struct Feeder {
  std::thread th;
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> jobs{0}, wrong{0};
  std::atomic<int> rc{QFEC_OK};
};
std::mutex g_feed_mu;
std::vector<std::pair<qfec_ctx*, Feeder*>> g_feeders;

void stop_feeder(qfec_ctx* ctx) {
  Feeder* f = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_feed_mu);
    auto it = std::find_if(g_feeders.begin(), g_feeders.end(),
                           [ctx](const std::pair<qfec_ctx*, Feeder*>& x) { return x.first == ctx; });
    if (it == g_feeders.end()) return;
    f = it->second;
    g_feeders.erase(it);
  }
  f->stop = true;
  f->th.join();
  delete f;
}
}  // namespace

int qfec_debug_service_feed(qfec_ctx* ctx, int on, uint64_t* stats) {
  if (!ctx) return fail(nullptr, QFEC_ERR_INTERNAL, "null qfec_ctx");
  std::lock_guard<std::mutex> lock(g_feed_mu);
  auto it = std::find_if(g_feeders.begin(), g_feeders.end(),
                         [ctx](const std::pair<qfec_ctx*, Feeder*>& f) { return f.first == ctx; });
  if (on) {
    if (it != g_feeders.end()) return fail(ctx, QFEC_ERR_INTERNAL, "feeder already running");
    Feeder* f = new Feeder();
    f->th = std::thread([ctx, f] {
      constexpr uint32_t k = 10, L = 1350;
      uint8_t* data = static_cast<uint8_t*>(qfec_host_alloc(k * L));
      uint8_t* par = static_cast<uint8_t*>(qfec_host_alloc(L));
      if (!data || !par) {
        f->rc = QFEC_ERR_INTERNAL;
        qfec_host_free(data);
        qfec_host_free(par);
        return;
      }
      uint8_t want[L];
      std::memset(want, 0, L);
      for (uint32_t i = 0; i < k * L; ++i) {
        data[i] = (uint8_t)(i * 131u + 7u);
        want[i % L] ^= data[i];
      }
      uint64_t off[k];
      uint16_t len[k];
      for (uint32_t i = 0; i < k; ++i) {
        off[i] = (uint64_t)i * L;
        len[i] = (uint16_t)L;
      }
      const uint32_t ptr[2] = {0u, k};
      const uint64_t poff = 0;
      uint16_t plen = 0;
      while (!f->stop.load(std::memory_order_relaxed)) {
        // a loop turn's other work: 20 us without runtime calls (a feeder
        // calling into the HIP runtime back to back stalled the measuring
        // thread's launches and event waits for seconds)
        const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(20);
        while (std::chrono::steady_clock::now() < t_end) {
        }
        (void)qfec_service_warm(ctx);  // the turn's start
        const int r = qfec_encode_ragged(ctx, data, off, len, ptr, 1, par, &poff, &plen,
                                         QFEC_PTR_MAPPED);
        if (r != QFEC_OK) {
          f->rc = r;
          break;
        }
        if (plen != L || std::memcmp(par, want, L) != 0) f->wrong.fetch_add(1);
        f->jobs.fetch_add(1, std::memory_order_relaxed);
      }
      qfec_host_free(data);
      qfec_host_free(par);
    });
    g_feeders.emplace_back(ctx, f);
    // back once the first batch is done (the worker resident and the
    // context registered), or the thread failed
    while (f->jobs.load() == 0 && f->rc.load() == QFEC_OK) std::this_thread::yield();
    return QFEC_OK;
  }
  if (it == g_feeders.end()) return fail(ctx, QFEC_ERR_INTERNAL, "no feeder running");
  Feeder* f = it->second;
  g_feeders.erase(it);
  f->stop = true;
  f->th.join();
  if (stats) {
    stats[0] = f->jobs.load();
    stats[1] = f->wrong.load();
  }
  const int rc = f->rc.load();
  delete f;
  return rc;
}

int qfec_debug_fail_launches(qfec_ctx* ctx, int on) {
  if (!ctx) return fail(nullptr, QFEC_ERR_INTERNAL, "null qfec_ctx");
  ctx->debug_fail = on != 0;
  return QFEC_OK;
}

int qfec_debug_phase(qfec_ctx* ctx, uint32_t extra, int reset_backoff) {
  int rc = bind(ctx);
  if (rc) return rc;
  QFEC_HIP(ctx, hipStreamSynchronize(ctx->stream));
  ctx->phase_extra = std::min<uint32_t>(extra, 64u);
  if (reset_backoff) {
    ctx->phase_seen = __atomic_load_n(ctx->h_phase, __ATOMIC_ACQUIRE);
    ctx->phase_backoff = 0;
  }
  return QFEC_OK;
}

int qfec_debug_phase_min(qfec_ctx* ctx, uint32_t min_phases) {
  int rc = bind(ctx);
  if (rc) return rc;
  ctx->phase_min = min_phases;
  return QFEC_OK;
}

int qfec_debug_phase_regsteps(qfec_ctx* ctx, int on) {
  int rc = bind(ctx);
  if (rc) return rc;
  ctx->no_regsteps = on ? 0u : 1u;
  return QFEC_OK;
}

int qfec_debug_phase_rtbatch(qfec_ctx* ctx, uint32_t batch) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (batch != 0u && batch != 16u && batch != 32u)
    return fail(ctx, QFEC_ERR_INTERNAL, "qfec_debug_phase_rtbatch: batch 0, 16 or 32");
  ctx->rt_batch = batch;
  return QFEC_OK;
}

uint32_t qfec_debug_other_service_cus(qfec_ctx* ctx, uint32_t* why) {
  if (!ctx) return 0;
  return other_service_cus(ctx, why);
}

int qfec_debug_phase_reserve(qfec_ctx* ctx, uint32_t cus) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (cus > 64u) return fail(ctx, QFEC_ERR_INTERNAL, "qfec_debug_phase_reserve: at most 64 CUs");
  ctx->phase_reserve = cus;
  return QFEC_OK;
}

int qfec_synth_fixed(qfec_ctx* ctx, uint8_t* rows, uint32_t k, uint32_t L, uint64_t row_stride,
                     uint64_t group_stride, uint64_t g0, uint64_t n_groups, uint64_t seed) {
  int rc = bind(ctx);
  if (rc) return rc;
  if ((rc = check_fixed(ctx, k, L, row_stride, group_stride, L, L))) return rc;
  if (g0 + n_groups > (1ull << 24))
    return fail(ctx, QFEC_ERR_INVALID_FEC_DATA, "synthetic group index beyond 2^24");
  QFEC_HIP(ctx, qfec::launch_synth_fixed(rows, k, L, row_stride, group_stride, g0, n_groups, seed,
                                         ctx->stream));
  return QFEC_OK;
}

int qfec_synth_ragged(qfec_ctx* ctx, uint8_t* bytes, const uint64_t* pkt_off,
                      const uint16_t* pkt_len, const uint32_t* grp_ptr, uint64_t g0,
                      uint64_t n_groups, uint64_t seed) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (g0 + n_groups > (1ull << 24))
    return fail(ctx, QFEC_ERR_INVALID_FEC_DATA, "synthetic group index beyond 2^24");
  QFEC_HIP(ctx, qfec::launch_synth_ragged(bytes, pkt_off, pkt_len, grp_ptr, g0, n_groups, seed,
                                          ctx->stream));
  return QFEC_OK;
}

int qfec_entropy_cumulative_batch(qfec_ctx* ctx, const uint8_t* entropy, const uint64_t* conn_ptr,
                                  const uint8_t* cum_base, uint64_t n_conns, uint64_t n_packets,
                                  uint8_t* cum, uint32_t flags) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (n_conns == 0) return QFEC_OK;
  if (!entropy || !conn_ptr || !cum) return fail(ctx, QFEC_ERR_INTERNAL, "null buffer");
  qfec::EntropyScanArgs a{entropy, conn_ptr, cum_base, n_conns, cum};
  if (flags & QFEC_PTR_HOST) {
    const uint64_t n = conn_ptr[n_conns];
    DevBuf d_e, d_ptr, d_base, d_cum;
    size_t si = 0;
    QFEC_HIP(ctx, scratch(ctx, si++, n + 1, &d_e.p));
    QFEC_HIP(ctx, scratch(ctx, si++, 8 * (n_conns + 1), &d_ptr.p));
    QFEC_HIP(ctx, scratch(ctx, si++, n + 1, &d_cum.p));
    QFEC_HIP(ctx, hipMemcpyAsync(d_e.p, entropy, n, hipMemcpyHostToDevice, ctx->stream));
    QFEC_HIP(ctx, hipMemcpyAsync(d_ptr.p, conn_ptr, 8 * (n_conns + 1), hipMemcpyHostToDevice,
                                 ctx->stream));
    if (cum_base) {
      QFEC_HIP(ctx, scratch(ctx, si++, n_conns, &d_base.p));
      QFEC_HIP(ctx, hipMemcpyAsync(d_base.p, cum_base, n_conns, hipMemcpyHostToDevice,
                                   ctx->stream));
    }
    a.entropy = static_cast<const uint8_t*>(d_e.p);
    a.conn_ptr = static_cast<const uint64_t*>(d_ptr.p);
    a.cum_base = static_cast<const uint8_t*>(d_base.p);
    a.cum = static_cast<uint8_t*>(d_cum.p);
    QFEC_HIP(ctx, qfec::launch_entropy_scan(a, ctx->stream, n - conn_ptr[0]));
    QFEC_HIP(ctx, hipMemcpyAsync(cum, d_cum.p, n, hipMemcpyDeviceToHost, ctx->stream));
    QFEC_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return QFEC_OK;
  }
  QFEC_HIP(ctx, qfec::launch_entropy_scan(a, ctx->stream, n_packets));
  return QFEC_OK;
}

int qfec_entropy_validate_batch(qfec_ctx* ctx, const uint8_t* cum, const uint64_t* conn_ptr,
                                const uint64_t* first_pn, const uint8_t* cum_base,
                                uint64_t n_conns, const uint32_t* ack_conn,
                                const uint64_t* largest_observed, const uint8_t* claimed,
                                const uint32_t* range_ptr, const uint64_t* range_lo,
                                const uint64_t* range_hi, uint64_t n_acks, uint8_t* ok,
                                uint32_t flags) {
  int rc = bind(ctx);
  if (rc) return rc;
  if (n_acks == 0) return QFEC_OK;
  if (!cum || !conn_ptr || !first_pn || !ack_conn || !largest_observed || !claimed ||
      !range_ptr || !ok || ((!range_lo || !range_hi) && (flags & QFEC_PTR_HOST) &&
                            range_ptr[n_acks] != range_ptr[0]))
    return fail(ctx, QFEC_ERR_INTERNAL, "null buffer");
  qfec::EntropyValidateArgs a{cum, conn_ptr, first_pn, cum_base, n_conns, ack_conn,
                              largest_observed, claimed, range_ptr, range_lo, range_hi, n_acks,
                              ok};
  if (flags & QFEC_PTR_HOST) {
    const uint64_t n = n_conns ? conn_ptr[n_conns] : 0, nr = range_ptr[n_acks];
    DevBuf d_cum, d_ptr, d_first, d_base, d_conn, d_larg, d_claim, d_rptr, d_lo, d_hi, d_ok;
    size_t si = 0;
    struct In {
      DevBuf* d;
      const void* h;
      uint64_t bytes;
    } ins[] = {{&d_cum, cum, n},          {&d_ptr, conn_ptr, 8 * (n_conns + 1)},
               {&d_first, first_pn, 8 * n_conns}, {&d_base, cum_base, cum_base ? n_conns : 0},
               {&d_conn, ack_conn, 4 * n_acks}, {&d_larg, largest_observed, 8 * n_acks},
               {&d_claim, claimed, n_acks},   {&d_rptr, range_ptr, 4 * (n_acks + 1)},
               {&d_lo, range_lo, 8 * nr},      {&d_hi, range_hi, 8 * nr}};
    for (auto& i : ins) {
      if (!i.h) continue;
      QFEC_HIP(ctx, scratch(ctx, si++, i.bytes + 8, &i.d->p));
      if (i.bytes)
        QFEC_HIP(ctx, hipMemcpyAsync(i.d->p, i.h, i.bytes, hipMemcpyHostToDevice, ctx->stream));
    }
    QFEC_HIP(ctx, scratch(ctx, si++, n_acks, &d_ok.p));
    a.cum = static_cast<const uint8_t*>(d_cum.p);
    a.conn_ptr = static_cast<const uint64_t*>(d_ptr.p);
    a.first_pn = static_cast<const uint64_t*>(d_first.p);
    a.cum_base = static_cast<const uint8_t*>(d_base.p);
    a.ack_conn = static_cast<const uint32_t*>(d_conn.p);
    a.largest_observed = static_cast<const uint64_t*>(d_larg.p);
    a.claimed = static_cast<const uint8_t*>(d_claim.p);
    a.range_ptr = static_cast<const uint32_t*>(d_rptr.p);
    a.range_lo = static_cast<const uint64_t*>(d_lo.p);
    a.range_hi = static_cast<const uint64_t*>(d_hi.p);
    a.ok = static_cast<uint8_t*>(d_ok.p);
    QFEC_HIP(ctx, qfec::launch_entropy_validate(a, ctx->stream));
    QFEC_HIP(ctx, hipMemcpyAsync(ok, d_ok.p, n_acks, hipMemcpyDeviceToHost, ctx->stream));
    QFEC_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return QFEC_OK;
  }
  QFEC_HIP(ctx, qfec::launch_entropy_validate(a, ctx->stream));
  return QFEC_OK;
}

}  // extern "C"
