// qfec_internal.h — launch interface between the C-ABI (qfec_capi.cpp) and
// the gfx950 kernels (qfec_kernels.hip).  Not installed; not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace qfec {

// Bits latched into the context's device error word by kernels.
enum : uint32_t {
  kErrMissingIndex = 1u,  // missing_idx >= k
  kErrPacketLength = 2u,  // ragged packet length 0 or > kMaxPacketSize, or > parity_len
  kErrGroupSize = 4u,     // ragged group with 0 or > 255 packets
  kErrParityLength = 8u,  // ragged parity_len 0 or > kMaxPacketSize
};

// Fixed-shape encode / recover.  parity == nullptr selects encode.
// Most workgroups of 256 lanes per launch: an AQL dispatch packet's grid size
// is a 32-bit count of work-items (2^32 / 256 = 2^24 workgroups).
constexpr uint64_t kMaxBlocks256 = (1ull << 24) - 1;

struct FixedArgs {
  const uint8_t* rows;
  const uint8_t* parity;   // recover only: parity rows
  const uint8_t* missing;  // recover only: lost slot per group
  uint8_t* out;
  uint64_t row_stride;
  uint64_t group_stride;
  uint64_t parity_stride;
  uint64_t out_stride;
  uint64_t n_groups;
  uint32_t k;
  uint32_t L;
  uint32_t* err;
  // large nt batches: 19 x 256 B of zeroed sync words for the phased kernel
  // (phase_xor_kernel); nullptr: always the one-pass fixed kernel
  uint32_t* phase_sync = nullptr;
  // phased kernel: the device's CU count (cached by the context: one
  // workgroup per CU), extra workgroups beyond it (test hook: forces the
  // abandon path), and a host-mapped word the last workgroup out copies the
  // abandoned-launch count into (nullable) — the context reads it at the next
  // launch without a synchronisation
  uint32_t ncu = 0;
  uint32_t phase_extra = 0;
  uint32_t* phase_host = nullptr;
  // minimum phase count for the phased kernel (0: kPhMinPhases, about 184K
  // headline groups); test hook qfec_debug_phase_min, for the band study
  uint32_t phase_min = 0;
  // steps per phase of the launch (set by launch_fixed: the batch spread
  // evenly over its phases); 0 = the kernel's full phase
  uint32_t phase_steps = 0;
  // test hook (qfec_debug_phase_regsteps): phased launches without the
  // register-held steps (the A/B of DESIGN.md §4's per-k table)
  uint32_t no_regsteps = 0;
  // CUs held by resident small-batch service workers of OTHER contexts on the
  // device (round 6): the phased grid leaves them free
  uint32_t svc_cus = 0;
  // test hook (qfec_debug_phase_rtbatch): the runtime-k phased body's load
  // batch (0: the per-operation choice, phase_rt_batch; 16 or 32)
  uint32_t rt_batch = 0;
  // in-slot recover written in place (qfec_recover_inslot_batch with out ==
  // NULL; encode form, parity == nullptr): group g's output row is its own
  // row inplace_missing[g], which holds the redundancy on entry; nullptr: out
  const uint8_t* inplace_missing = nullptr;
};

// True if launch_fixed(a, nontemporal, ...) runs the phased kernel; *grid
// (nullable): its workgroup count.
bool fixed_uses_phases(const FixedArgs& a, bool nontemporal, uint32_t* grid = nullptr);

struct RaggedArgs {
  const uint8_t* bytes;
  const uint64_t* pkt_off;
  const uint16_t* pkt_len;
  const uint32_t* grp_ptr;
  const uint8_t* parity;      // recover: parity bytes
  const uint64_t* parity_off; // encode: where to write; recover: where to read
  const uint16_t* parity_len; // recover: lengths in
  uint16_t* parity_len_out;   // encode: lengths out
  const uint8_t* missing;     // recover
  uint8_t* out;               // encode: parity_out; recover: revived packets
  const uint64_t* out_off;    // recover
  uint64_t n_groups;
  uint32_t* err;
  // launch_ragged_latency only (nullptr: none): the last workgroup to finish
  // stores done_token into done_flag (mapped host memory, system scope) after
  // every output is visible; done_count is a zeroed device word it resets
  uint32_t* done_count;
  uint32_t* done_flag;
  uint32_t done_token;
};

// Small-batch service (round 4): one resident workgroup that takes mapped
// ragged batches from a ring in host-mapped memory instead of a kernel launch
// per batch (the launch is most of a small flush's connection-thread cost).
// The host writes a job, then publishes pub_end (the groups published so
// far); the worker processes every published group (one wave per group, the
// small-batch kernel's body), stores each job's token into its slot's flag
// and `consumed`, and exits after idle_ticks without work (alive = 0, then one
// more look at pub_end: the host, after publishing, relaunches it if it
// reads alive == 0 -- each side writes, fences, then reads the other's word).
// Round 5: the job's index tables are written INLINE (tab, at the t_*
// offsets, the direct path's Tab layout), so the worker copies the entry --
// header and tables -- into LDS in one PCIe round trip.  a's table pointers
// are not used by the worker.
constexpr uint32_t kSvcTab = 16384 - 256;  // inline table bytes (64 groups of up to 16 packets)
struct SvcJob {
  RaggedArgs a;       // bytes / parity / out: the mapped payload buffers
  uint64_t start;     // the job's first group in the global group sequence
  uint32_t seq;       // job number (ring index = seq % kSvcRing)
  uint32_t recover;
  uint32_t flag_slot; // index into the context's host-mapped flags
  uint32_t token;
  uint32_t tab_bytes; // table bytes in tab (<= kSvcTab)
  uint32_t t_off, t_len, t_ptr, t_poff, t_plen, t_miss, t_ooff;  // offsets into tab
  // Round 5: svc_head_hash of the entry's first min(entry size, kSvcHead)
  // bytes (this word excluded), stored by the host LAST; the leader reads
  // those bytes in every poll of the ring.  A job it finds whole there (hash,
  // seq and start agree) needs no second PCIe round trip for its entry when
  // it fits them; a larger job's header is then known from the poll, so its
  // size is too, and the rest of its tables is copied in one pass (the
  // followers copy it whole, announced with that size).  0 while the host
  // writes the entry.
  uint64_t head_sum;
  alignas(16) uint8_t tab[kSvcTab];
};
constexpr uint32_t kSvcHead = 1024;  // bytes of the entry read with every poll (64 x 16 B)
constexpr uint32_t kSvcHeadSumWord = (uint32_t)(offsetof(SvcJob, head_sum) / 8u);
static_assert(offsetof(SvcJob, head_sum) % 8u == 0u, "head_sum on a word");
static_assert(offsetof(SvcJob, tab) < kSvcHead, "the header fits the polled bytes");
// Order-free sum over the 8-byte words [0, nbytes / 8) of the entry but
// head_sum's own: each word mixed with its index (splitmix64 finalizer), so a
// torn read -- some 16-B pieces from before the host's writes -- does not sum
// to the stored value (host and device compute the same function).
__host__ __device__ inline uint64_t svc_head_word(uint64_t w, uint32_t i) {
  uint64_t z = w ^ (0x9E3779B97F4A7C15ull * (uint64_t)(i + 1u));
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t svc_head_hash(const SvcJob& j, uint32_t nbytes) {
  const uint64_t* w = reinterpret_cast<const uint64_t*>(&j);
  uint64_t h = 0;
  for (uint32_t i = 0; i < nbytes / 8u; ++i)
    if (i != kSvcHeadSumWord) h += svc_head_word(w[i], i);
  return h | 1ull;  // never 0 (0 = no hash)
}
struct SvcShared {
  // the host's words (the worker reads them) on a cache line of their own:
  // the worker's per-turn stores below would otherwise take the line from
  // the host's cache before every publish
  alignas(64) uint64_t pub_end;  // host: groups published
  uint32_t alive;     // host: 1 when it launches a worker; worker: 1 when it starts,
                      // 0 on its way out
  uint32_t quit;      // host: exit now (context destroyed)
  uint32_t stamp_on;  // host (measurement hook): the worker records stamps[] for each job
  uint32_t hold;      // host (test hook qfec_debug_service_hold): followers wait at
                      // their start while it is 1 (a follower dispatched late)
  uint32_t rotate;    // host: a worker whose launch epoch is at most this leaves at
                      // its next look, published jobs or not -- its successor is
                      // already queued behind it (svc_submit's residency bound)
  uint32_t warm;      // host: bumped by qfec_service_warm on a running worker -- a
                      // batch is coming; the worker's idle time restarts from it
  // the worker's words, stored every turn
  alignas(64) uint64_t consumed;  // worker: groups finished (a new worker starts here)
  uint64_t jobs;      // worker: jobs finished (stats)
  uint32_t fault;     // worker: a published group lay in no ring entry; it left
                      // without finishing (no token for any job of that turn)
  // 100-MHz wall-clock stamps of the last job (qfec_debug_service_stamps):
  // [0] work seen, [1] entry in LDS, [2] wave 0's first group done, [3] every
  // group done, [4] outputs visible (fence), [5] the leader's count / token
  // stored; [6] the token stored (by the last workgroup of a split job), [7]
  // that workgroup (round 6, qfec_debug_service_trace)
  alignas(64) uint64_t stamps[8];
  // round 6: every workgroup's stamps of its share of the last job: [0] its
  // entry in LDS, [1] its groups done, [2] its outputs visible, [3] counted
  uint64_t wg_stamps[8][4];
};
constexpr uint32_t kSvcRing = 8;
// Round 5: the worker is kSvcWgs workgroups.  Workgroup 0 (the leader) polls
// the host's pub_end, walks the published jobs and runs the alive / exit
// protocol above, so only the leader's decisions reach the host.  A job of
// more groups than one workgroup has waves is split over every workgroup;
// each adds itself to its ring entry's done counter after making its outputs
// visible and the last one stores the token.  Smaller jobs are the leader's
// alone.
// Round 6: the leader ANNOUNCES each split job to the followers
// through SvcDev (job number and entry size, in order); a follower takes the
// announcements one by one from its own count `taken`, which outlives the
// launch, and reads no other ring entry.  A follower dispatched late (the CUs
// held by another kernel) therefore still does every split job's share, and
// a split job's entry, whose token waits for every follower, is never reused
// under it.  At most kSlots (3) jobs are outstanding, so kSvcRing
// announcement words never wrap onto one not yet taken.
constexpr uint32_t kSvcWgs = 8;
static_assert(sizeof(SvcShared::wg_stamps) / sizeof(SvcShared::wg_stamps[0]) == kSvcWgs,
              "one stamp row per service workgroup");
struct SvcDev {
  uint32_t exit;             // leader: this launch's epoch when it leaves (after its
                             // last announcement)
  uint32_t done[kSvcRing];   // workgroups finished per ring entry's split job (the
                             // last resets it before the token)
  uint64_t nsplit;           // leader: split jobs announced so far
  uint64_t split[kSvcRing];  // announcement i at i % kSvcRing: job << 32 | entry bytes / 16
  uint64_t taken[kSvcWgs];   // follower w: announcements taken (w = 0 unused)
};
// (the host zeroes SvcDev when it creates the service and when it abandons it)
hipError_t launch_ragged_service(SvcShared* sh, SvcDev* dv, const SvcJob* ring, uint32_t* flags,
                                 uint64_t idle_ticks, uint32_t epoch, hipStream_t s);

// Packet protection batch (qpp_kernels.hip): packet p's associated data (the
// packet header) is ad_len[p] bytes at bytes + ad_off[p], its input payload
// in_len[p] bytes at bytes + in_off[p], its output at out + out_off[p].
struct ProtectArgs {
  const uint8_t* bytes;
  const uint64_t* ad_off;
  const uint16_t* ad_len;
  const uint64_t* in_off;
  const uint16_t* in_len;
  uint8_t* out;
  const uint64_t* out_off;
  uint8_t* ok;  // decrypt: 1 = tag verified and payload written
  uint64_t n;
  // decrypt with QFEC_SCRATCH_OUTPUT: one pass, the output of a packet whose
  // tag fails holds its unverified plaintext (else untouched, two passes)
  uint32_t scratch_out = 0;
};

hipError_t launch_null_protect(const ProtectArgs& a, bool decrypt, hipStream_t s);

// ChaCha20-Poly1305 (QUIC: 12-byte tag, nonce = prefix || LE64(path<<56|pn)).
// Packet p is protected with key key_idx[p] (keys: 32 B each, prefixes: 4 B
// each), packet number packet_number[p], path id path_id[p] (nullptr: 0).
struct AeadArgs {
  ProtectArgs io;
  const uint8_t* keys;
  const uint8_t* prefixes;
  const uint32_t* key_idx;
  const uint64_t* packet_number;
  const uint8_t* path_id;
};

hipError_t launch_chacha20poly1305(const AeadArgs& a, bool decrypt, hipStream_t s);
// AES-128-GCM (QUIC: 12-byte tag; keys are 16 B each).
hipError_t launch_aes128gcm(const AeadArgs& a, bool decrypt, hipStream_t s);

// Packet-entropy bookkeeping (qent_kernels.hip); layout as include/qfec.h.
struct EntropyScanArgs {
  const uint8_t* entropy;
  const uint64_t* conn_ptr;  // n_conns + 1
  const uint8_t* cum_base;   // nullable: 0
  uint64_t n_conns;
  uint8_t* cum;
};

struct EntropyValidateArgs {
  const uint8_t* cum;
  const uint64_t* conn_ptr;
  const uint64_t* first_pn;
  const uint8_t* cum_base;  // nullable: 0
  uint64_t n_conns;
  const uint32_t* ack_conn;
  const uint64_t* largest_observed;
  const uint8_t* claimed;
  const uint32_t* range_ptr;  // n_acks + 1
  const uint64_t* range_lo;
  const uint64_t* range_hi;
  uint64_t n_acks;
  uint8_t* ok;
};

// total_bytes = conn_ptr[n_conns] - conn_ptr[0] (host-known: picks lanes per
// connection), or 0 when unknown.
hipError_t launch_entropy_scan(const EntropyScanArgs& a, hipStream_t s, uint64_t total_bytes);
hipError_t launch_entropy_validate(const EntropyValidateArgs& a, hipStream_t s);

// nontemporal: nt loads and stores (the streaming default; see qfec.h QFEC_CACHED)
hipError_t launch_fixed(const FixedArgs& a, bool nontemporal, hipStream_t s);
// small_groups: the batch's groups carry few bytes each (round 6's band
// table: below kRaggedSmallGroupBytes on average): two groups per wave
// (ragged_multi_kernel) instead of the block kernel.
hipError_t launch_ragged(const RaggedArgs& a, bool recover, hipStream_t s, bool small_groups = false);
// average payload bytes per group below which a large ragged batch runs two
// groups per wave (launch_ragged small_groups; tools/tune/tune_rblock.hip
// mode 2, profiles/round6/ragged_band_r6h.txt)
constexpr uint64_t kRaggedSmallGroupBytes = 4096;
// Small batches whose payloads are read over PCIe (mapped host memory): one
// wave per group, all of a group's loads in flight at once.
hipError_t launch_ragged_latency(const RaggedArgs& a, bool recover, hipStream_t s);
hipError_t launch_stream_probe(const uint8_t* src, uint64_t n, uint8_t* dst, bool copy,
                               hipStream_t s);
hipError_t launch_xor_into(const uint8_t* in, uint64_t n, uint8_t* out, hipStream_t s);
hipError_t launch_synth_fixed(uint8_t* rows, uint32_t k, uint32_t L, uint64_t row_stride,
                              uint64_t group_stride, uint64_t g0, uint64_t n, uint64_t seed,
                              hipStream_t s);
hipError_t launch_synth_ragged(uint8_t* bytes, const uint64_t* pkt_off, const uint16_t* pkt_len,
                               const uint32_t* grp_ptr, uint64_t g0, uint64_t n, uint64_t seed,
                               hipStream_t s);

}  // namespace qfec
