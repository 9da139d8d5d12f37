// qfec_kernels.hip — gfx950 (CDNA4) kernels for the QUIC FEC XOR path.
//
// What they compute (the historical QuicFecGroup whose
// sources are gone from the snapshot, evidence /root/reference/Makefile:5332-5384):
//   encode : parity[j]  = XOR_i p_i[j]                       (zero padded rows)
//   recover: revived[j] = parity[j] XOR_{i != m} p_i[j]
// Both are one streaming pass over HBM with one integer op per byte: the
// roofline is HBM bandwidth (no MFMA — this is a byte-wise XOR reduction).
//
// Layout and mapping:
//  * Fixed shape [G][k][L] (L = 1350 in the headline config).  A row is split
//    into C = ceil(L/16) 16-byte windows; lane t of a group owns the window at
//    byte min(16t, L-16), so the last window ends exactly at the row end and
//    overlaps its neighbour (both lanes store identical bytes there).  No lane
//    ever touches memory outside its rows, no tail branch, no masking.
//    A 256-lane workgroup owns floor(256/C) whole groups (3 at L = 1350), so a
//    wave-instruction reads ~1 KiB of contiguous row bytes and workgroups never
//    split a group.
//  * Rows are only 2-byte aligned at L = 1350 (1350 = 2 mod 4).  gfx950 runs
//    global loads in unaligned-access mode, so every row load is ONE
//    global_load_dwordx4 regardless of alignment (checked in the .s); the
//    L2/TA handle the line crossing.
//  * Recover reads the parity row *in place of* the lost row: k loads per lane,
//    every one unconditional — the lost slot is never read and no lane idles.
//  * Batches of >= 6 phases (about 184K groups at L = 1350) run
//    phase_xor_kernel instead: the same lanes and loads in a persistent
//    one-workgroup-per-CU grid that separates the row reads and the parity
//    writes into grid-wide phases (0.80 of 8 TB/s on any buffer placement).
//  * Ragged CSR batches: eight groups per 4-wave block in one flat window
//    space (ragged_block_kernel; the one-group body below is its exact
//    fallback; the round-1/2 forms, one and two groups per wave, live in
//    tools/tune/ragged_legacy.inc for the A/B record), lanes own 16-byte
//    windows of the packets; a window shorter than 16 bytes is loaded as the
//    16 bytes that end at the packet's last byte and shifted down (zero
//    fill), so again no load leaves the packet.
#include "qfec_internal.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace qfec {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kMaxPacket = 1452;  // kMaxPacketSize, quic_protocol.h:66
constexpr int kBlock = 256;

__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
  u32x4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16t(const uint8_t* p) {
  if constexpr (NT) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  } else {
    return ld16(p);
  }
}

__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) { __builtin_memcpy(p, &v, 16); }

template <bool NT>
__device__ __forceinline__ void st16t(uint8_t* p, u32x4 v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  } else {
    st16(p, v);
  }
}

// A 16-B store with an explicit cache policy (round 6 store-policy probe,
// tools/tune only): 0 nt (the product's st16t<true>), 1 sc1, 2 sc0 sc1,
// 3 nt sc1, 4 nt sc0 sc1 -- vector stores; sc1 drops the line from the XCD's
// L2 (write-through), nt keeps it (MI355X_MICROARCH.md, store flavours).
template <int POL>
__device__ __forceinline__ void st16pol(uint8_t* p, u32x4 v) {
  if constexpr (POL == 0) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  } else if constexpr (POL == 1) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  } else if constexpr (POL == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  } else if constexpr (POL == 3) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
  } else {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
  }
}

// Wave max of 11-bit values by ballots, MSB first (no LDS round trips).
__device__ __forceinline__ uint32_t wave_max11(uint32_t v) {
  uint32_t mx = 0;
#pragma unroll
  for (int b = 10; b >= 0; --b) {
    const uint32_t cand = mx | (1u << b);
    if (__ballot(v >= cand) != 0ull) mx = cand;
  }
  return mx;
}

__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0ull; }

// XCD-aware workgroup order (MI355X_MICROARCH.md, workgroup dispatch: blocks
// b, b + 8, b + 16, ... share an XCD and its L2): maps those blocks onto one
// contiguous share of the grid, bijectively for any n (q = n / 8, r = n % 8).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t n) {
  const uint32_t q = n >> 3, r = n & 7u, x = b & 7u;
  return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + (b >> 3);
}

// N rows r .. r+N-1 of a group, all N loads in flight before the first XOR
// (recover: row m is the parity row `par`).  The runtime-k bodies use it for
// their full batches AND their remainder (a switch on k - r picks N): round
// 4's remainder was a rolled loop, one load in flight per lane, which made
// the runtime-k phased kernel 1.1-2.5x slower than one-pass
// (profiles/round4/phase_k_table_nontemplated_r4o.txt, k = 6: 0.27 vs 0.69).
template <int N, bool RECOVER, bool NT>
__device__ __forceinline__ void xor_rows_n(u32x4& acc, const uint8_t* src, uint64_t row_stride,
                                           uint32_t r, uint32_t m, const uint8_t* par) {
  u32x4 v[N];
#pragma unroll
  for (int w = 0; w < N; ++w) {
    const uint8_t* q = (RECOVER && r + (uint32_t)w == m) ? par : src + (uint64_t)(r + w) * row_stride;
    v[w] = ld16t<NT>(q);
  }
#pragma unroll
  for (int w = 0; w < N; ++w) acc ^= v[w];
}

// Rows [0, k) of a group at runtime k: ceil(k / B) batches of loads in
// flight, their sizes as even as possible (k = 40, B = 32: 20 + 20, not
// 32 + 8 -- a batch is a round trip).  The phased kernel (one wave per SIMD:
// a lane's loads in flight are all the CU has) takes B = 32: round 5's
// B = 16 split k = 20 into 10 + 10 and read at 0.743 / 0.683 of 8 TB/s
// against 0.781 / 0.741 at k = 32 (16 + 16) (profiles/round5/
// phase_k_table_r5b.txt; round 6: profiles/round6/phase_k_table_r6*.txt).
template <int B, bool RECOVER, bool NT>
__device__ __forceinline__ void xor_rows_rt(u32x4& acc, const uint8_t* src, uint64_t row_stride,
                                            uint32_t k, uint32_t m, const uint8_t* par) {
  static_assert(B == 8 || B == 16 || B == 32, "batch of 8, 16 or 32 rows");
  const uint32_t nb = (k + B - 1) / B;
  const uint32_t base = nb ? k / nb : 0u, extra = k - base * nb;
  uint32_t r = 0;
  for (uint32_t b = 0; b < nb; ++b) {
    const uint32_t n = base + (b < extra ? 1u : 0u);
#define QFEC_REM(N)                                                 \
  case N:                                                           \
    xor_rows_n<N, RECOVER, NT>(acc, src, row_stride, r, m, par);    \
    break;
    if (B == 8 || n <= 8u) {
      switch (n) {
        QFEC_REM(1) QFEC_REM(2) QFEC_REM(3) QFEC_REM(4) QFEC_REM(5) QFEC_REM(6) QFEC_REM(7)
        QFEC_REM(8)
        default:
          break;
      }
    } else if constexpr (B >= 16) {
      if (B == 16 || n <= 16u) {
        switch (n) {
          QFEC_REM(9) QFEC_REM(10) QFEC_REM(11) QFEC_REM(12) QFEC_REM(13) QFEC_REM(14)
          QFEC_REM(15) QFEC_REM(16)
          default:
            break;
        }
      } else if constexpr (B == 32) {
        switch (n) {
          QFEC_REM(17) QFEC_REM(18) QFEC_REM(19) QFEC_REM(20) QFEC_REM(21) QFEC_REM(22)
          QFEC_REM(23) QFEC_REM(24) QFEC_REM(25) QFEC_REM(26) QFEC_REM(27) QFEC_REM(28)
          QFEC_REM(29) QFEC_REM(30) QFEC_REM(31) QFEC_REM(32)
          default:
            break;
        }
      }
    }
#undef QFEC_REM
    r += n;
  }
}

// ---------------------------------------------------------------------------
// Fixed shape, L >= 16.
// ---------------------------------------------------------------------------
// SM (recover, gpb <= 8): lost-slot indices by scalar loads, see below.
// INPL (encode form only): the in-slot recover written in place -- the
// group's output row is its own row missing[g] (which held the redundancy);
// a barrier between the loads and the stores keeps a wave from overwriting
// the bytes the overlapping last window of a neighbouring wave still reads.
template <int KC, bool RECOVER, bool NT, bool SM, bool XCD = false, bool INPL = false>
__global__ __launch_bounds__(kBlock) void fixed_xor_kernel(FixedArgs a, uint32_t C,
                                                           uint32_t gpb) {
  static_assert(!(INPL && RECOVER), "in place: the encode form over the k rows");
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;  // group within the workgroup
  const uint32_t t = tid - gl * C;
  const uint64_t gb = (uint64_t)(XCD ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x) * gpb;
  const uint64_t g = gb + gl;
  if constexpr (INPL) {
    // no early return before the barrier: every wave reaches it
    const bool on = gl < gpb && g < a.n_groups;
    const uint64_t gg = on ? g : 0;
    const uint32_t off = min(t * 16u, a.L - 16u);
    const uint8_t* src = a.rows + gg * a.group_stride + off;
    const uint32_t k = KC > 0 ? (uint32_t)KC : a.k;
    const uint32_t m = on ? (uint32_t)a.inplace_missing[gg] : 0u;
    u32x4 acc = {0u, 0u, 0u, 0u};
    if constexpr (KC > 0) {
      xor_rows_n<(KC > 0 ? KC : 1), false, NT>(acc, src, a.row_stride, 0, 0, nullptr);
    } else {
      xor_rows_rt<8, false, NT>(acc, src, a.row_stride, k, 0, nullptr);
    }
    __syncthreads();
    if (on && m < k) st16t<NT>(const_cast<uint8_t*>(src) + (uint64_t)m * a.row_stride, acc);
    if (on && m >= k && t == 0) atomicOr(a.err, kErrMissingIndex);
    return;
  }
  uint64_t mw0 = 0, mw1 = 0;
  if constexpr (RECOVER) {
    // SM: the block's lost-slot indices by (at most) two SCALAR loads of the
    // aligned 8-byte words covering missing[gb .. gb+gpb) (gpb <= 8): every
    // row address below depends on m, and a per-lane byte load here would
    // put a vector-memory round trip in front of all of them (-7% measured).
    // An aligned word holding a valid byte never crosses a page: no fault.
    if constexpr (SM) {
      const uint8_t* mp = a.missing + gb;
      const uint32_t mis = (uint32_t)((uintptr_t)mp & 7u);  // pointer math keeps addrspace(1)
      const uint64_t* wp = reinterpret_cast<const uint64_t*>(mp - mis);
      mw0 = wp[0];
      if (gb + 8u - mis < a.n_groups) mw1 = wp[1];
    }
  }
  if (gl >= gpb || g >= a.n_groups) return;
  const uint32_t off = min(t * 16u, a.L - 16u);
  const uint8_t* src = a.rows + g * a.group_stride + off;
  const uint32_t k = KC > 0 ? (uint32_t)KC : a.k;

  u32x4 acc = {0u, 0u, 0u, 0u};
  if constexpr (RECOVER) {
    uint32_t m;
    if constexpr (SM) {
      const uint32_t sh = gl + (uint32_t)((uintptr_t)(a.missing + gb) & 7u);
      m = (uint32_t)((sh < 8u ? mw0 >> (8u * sh) : mw1 >> (8u * (sh - 8u))) & 0xFFu);
    } else {
      m = a.missing[g];
    }
    if (m >= k) {
      if (t == 0) atomicOr(a.err, kErrMissingIndex);
      return;
    }
    const uint8_t* par = a.parity + g * a.parity_stride + off;
    if constexpr (KC > 0) {
#pragma unroll
      for (uint32_t i = 0; i < (uint32_t)KC; ++i) {
        const uint8_t* p = (i == m) ? par : src + i * a.row_stride;
        acc ^= ld16t<NT>(p);
      }
    } else {
      xor_rows_rt<8, true, NT>(acc, src, a.row_stride, k, m, par);
    }
  } else {
    if constexpr (KC > 0) {
#pragma unroll
      for (uint32_t i = 0; i < (uint32_t)KC; ++i) acc ^= ld16t<NT>(src + i * a.row_stride);
    } else {
      xor_rows_rt<8, false, NT>(acc, src, a.row_stride, k, 0, nullptr);
    }
  }
  st16t<NT>(a.out + g * a.out_stride + off, acc);
}

// ---------------------------------------------------------------------------
// Fixed shape, large batches: the same lanes and loads, phased.
// ---------------------------------------------------------------------------
// The fixed kernel above runs at 0.69-0.81 of 8 TB/s depending on where the
// caller's rows and parity buffers sit in the DRAM relative to each other
// (a property of the (rows, parity) PAIR — the read and write
// streams meeting in the DRAM).  Here a persistent grid of one workgroup per
// CU walks the batch in phases: in phase p every workgroup XORs kPhSteps x gpb
// groups into LDS (160 KiB — the whole CU), the grid meets, every workgroup
// stores its parity rows and goes on to the next phase.  The HBM then sees
// (mostly) separate phases of reads and writes, whatever the placement
// (tools/tune/tune_phase.hip).
// The meetings only shape timing: no workgroup reads what another wrote, so
// every wait is bounded — a workgroup that waits longer than kPhTimeout
// (e.g. the GPU shared with other work, so not all workgroups are resident)
// raises an abandon flag and every workgroup stops waiting for the rest of the
// launch; results are identical either way.
constexpr int kPhSteps = 40;         // 40 x 256 lanes x 16 B = 160 KiB of LDS
// k = 10 (the headline shape): 32 more steps per phase held in VGPRs (one
// wave per SIMD has the register file to itself): 19 phases instead of 35 at
// 2^20 groups, encode +1.6%; recover +0.1-1.3%, +1.7% with the register
// steps' parity rows loaded first (RPF) (tools/tune/tune_phase.hip "40+32",
// profiles/round3/phase/tune_phase_rs*.txt; 40 + 40 / 48 / 64 spill into
// AGPRs and lose).
constexpr int kPhRegSteps = 32;
constexpr int kPhUDefault = 1;       // steps loaded together (k loads in flight per lane)
constexpr uint64_t kPhTimeout = 20000;  // s_memrealtime ticks (100 MHz): 200 us

// sync words, 256 B apart: [0] top, [1..16] sub-counters, [17] exits, [18] abandon,
// [19] abandoned launches so far (never reset: qfec_phase_abandons)
__device__ __forceinline__ uint32_t* ph_word(uint32_t* ps, uint32_t i) { return ps + 64u * i; }

__device__ __forceinline__ uint32_t ph_load(uint32_t* w) {
  return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Meeting number `epoch` (1, 2, ...).  A workgroup adds to one of 16
// sub-counters (one counter for every workgroup cost ~60 us per meeting at
// 1,024 adders); the last adder of a sub-counter in this epoch, told by the
// value its add returned, adds to the top counter, which the waiters poll.
__device__ __forceinline__ void phase_meet(uint32_t* ps, uint32_t epoch) {
  __syncthreads();
  if (threadIdx.x == 0 && ph_load(ph_word(ps, 18)) == 0u) {
    const uint32_t B = gridDim.x, sub = blockIdx.x & 15u, nsub = (B - sub + 15u) / 16u;
    const uint32_t old =
        __hip_atomic_fetch_add(ph_word(ps, 1u + sub), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1u == epoch * nsub)
      __hip_atomic_fetch_add(ph_word(ps, 0), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t target = epoch * min(B, 16u);
    const uint64_t t0 = wall_clock64();
    while (ph_load(ph_word(ps, 0)) < target) {
      if (wall_clock64() - t0 > kPhTimeout) {
        if (__hip_atomic_fetch_or(ph_word(ps, 18), 1u, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT) == 0u)  // count abandoned launches
          __hip_atomic_fetch_add(ph_word(ps, 19), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      if (ph_load(ph_word(ps, 18)) != 0u) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// The last workgroup out zeroes the sync words for the next launch on the
// stream (vector atomics; the launch boundary orders them before it) and
// copies the abandoned-launch count into the context's host-mapped word
// (a vector store at system scope), where the host reads it at the next
// launch without waiting for this one.
__device__ __forceinline__ void phase_exit(uint32_t* ps, uint32_t* host) {
  __syncthreads();
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(ph_word(ps, 17), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
          gridDim.x - 1u) {
    for (uint32_t i = 0; i < 19u; ++i)
      __hip_atomic_store(ph_word(ps, i), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (host)
      __hip_atomic_store(host, ph_load(ph_word(ps, 19)), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Defaults = the product (tools/tune/tune_phase.hip, profiles/round2/phase/
// tune_phase8.txt): one meeting per phase, before the stores (MEET2 adds one
// after them: -3%), one step's k loads in flight per lane (kPhU = 2: -4%);
// FLAT (row pointers as generic pointers: flat loads) changes nothing; XCDW
// (XCD-aware order in the window) +0.5% encode / -3% recover; PARFIRST
// (recover, templated k: the phase's parity rows first, then only the
// received rows) +2.7% recover (tune_phase12.txt); COMPACT (with PARFIRST: the
// k-1 received rows loaded in order, r + (r >= m), so no load instruction runs
// with the lost row's lanes masked off: 17 loads and 22 exec branches per step
// instead of 18 and 32) +2.5% recover, 0.780 vs 0.761 on six buffer pairs
// (profiles/round2/phase/tune_phase_compact.txt).
// RS (encode, tools/tune): RS more steps per phase held in registers after the
// STEPS LDS ones (a longer phase, fewer meetings; one wave per SIMD leaves the
// register file to spare).
template <int KC, bool RECOVER, bool MEET2 = false, bool FLAT = false, int kPhU = kPhUDefault,
          int STEPS = kPhSteps, int NTHR = kBlock, bool XCDW = false, bool PARFIRST = true,
          bool NTLD = true, bool EDGE = false, bool COMPACT = true, int RS = 0, bool RPF = false,
          bool RPFE = false, bool INPL = false, int RTB = 32>
__global__ __launch_bounds__(NTHR) void phase_xor_kernel(FixedArgs a, uint32_t C, uint32_t gpb,
                                                           uint32_t nphase) {
  static_assert(!(INPL && RECOVER), "in place: the encode form over the k rows");
  // (the runtime-k body loads the parity in place of the lost row: parity
  // first with its received rows compact measured 2-6% slower for k = 17-48,
  // profiles/round6/phase_k_table_r6c.txt against r6b)
  constexpr bool PF = RECOVER && PARFIRST && KC > 0;
  static_assert(!RECOVER || STEPS <= 64, "recover: bad-step masks are 64 bits");
  static_assert(RS == 0 || (KC > 0 && kPhU == 1 && !XCDW && RS <= 64 &&
                            (!RECOVER || (PARFIRST && COMPACT))),
                "register steps: templated k, one step at a time (recover: parity first, compact)");
  constexpr int TS = STEPS + RS;  // steps per phase (at most)
  // the launch's steps per phase (launch_fixed spreads the batch evenly over
  // its phases, so the last phase is not a sliver); the LDS steps come first
  const int SP = (kPhU == 1 && a.phase_steps != 0u) ? min((int)a.phase_steps, TS) : TS;
  const int NL = min(STEPS, SP);  // LDS steps in use
  __shared__ u32x4 s_par[STEPS][NTHR];  // lane tid's parity of each step
  const uint32_t tid = threadIdx.x, gl = tid / C, t = tid - gl * C;
  const bool lane_on = gl < gpb;
  const uint32_t off = min(t * 16u, a.L - 16u);
  const uint32_t k = KC > 0 ? (uint32_t)KC : a.k;
  const uint64_t B = gridDim.x;
  for (uint32_t p = 0; p < nphase; ++p) {
    // the kPhU steps from i of phase p cover one contiguous window of
    // B x kPhU gpb groups (the fixed kernel's sliding window); workgroup b
    // owns kPhU gpb of them
    // XCDW: the workgroups of one XCD (b, b+8, ...) take one contiguous share
    // of the window, so the lines two neighbouring groups share stay in one L2
    const uint64_t wb = XCDW ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint64_t base = ((uint64_t)p * (uint64_t)(SP / kPhU) * B + wb) * (gpb * kPhU) + gl;
    // recover: steps whose lost-slot index is out of range (bit i of lo/hi:
    // 32-bit shifts only, STEPS <= 64)
    uint32_t bad_lo = 0, bad_hi = 0;
    auto gidx = [&](int i) {
      return base + (uint64_t)(i / kPhU) * B * gpb * kPhU + (uint64_t)(i % kPhU) * gpb;
    };
    // recover: the lost-slot indices of the next steps are loaded one
    // iteration ahead (every row address depends on them)
    uint32_t m_reg[RS > 0 && RECOVER ? RS : 1];  // register steps' lost slots, loaded early
    if constexpr (RS > 0 && RECOVER) {
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const uint64_t g = gidx(STEPS + j);
        m_reg[j] = lane_on && g < a.n_groups && STEPS + j < SP ? a.missing[g] : 0u;
      }
    }
    uint32_t m_next[kPhU];
    if constexpr (RECOVER) {
#pragma unroll
      for (int u = 0; u < kPhU; ++u) {
        const uint64_t g = gidx(u);
        m_next[u] = lane_on && g < a.n_groups ? a.missing[g] : 0u;
      }
    }
    // RPFE (tools/tune): the register steps' parity rows too, right after the
    // LDS steps' ones -- the phase's whole parity range as one stream
    u32x4 racc[RS > 0 ? RS : 1];
    static_assert(!RPFE || (RS > 0 && RECOVER && RPF && PF), "RPFE: recover register steps, RPF");
    if constexpr (PF) {
      // PARFIRST: the phase's parity rows first, into the accumulators (one
      // stream over the parity buffer), then the received rows only
#pragma unroll 1
      for (int i = 0; i < STEPS; i += 8) {
        u32x4 w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint64_t g = gidx(i + j < NL ? i + j : 0);
          const bool on = i + j < NL && lane_on && g < a.n_groups;
          w[j] = ld16t<NTLD>(a.parity + (on ? g : 0) * a.parity_stride + off);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (i + j < STEPS) s_par[i + j][tid] = w[j];
      }
      if constexpr (RPFE) {
#pragma unroll
        for (int j = 0; j < RS; ++j) {
          const uint64_t g = gidx(STEPS + j);
          const bool on = lane_on && g < a.n_groups && STEPS + j < SP;
          racc[j] = ld16t<NTLD>(a.parity + (on ? g : 0) * a.parity_stride + off);
        }
      }
    }
#pragma unroll 1
    for (int i = 0; i < NL; i += kPhU) {
      u32x4 acc[kPhU];
      uint32_t m[kPhU];
      const uint8_t* src[kPhU];
#pragma unroll
      for (int u = 0; u < kPhU; ++u) {
        const uint64_t g = gidx(i + u);
        const bool on = lane_on && g < a.n_groups;
        src[u] = a.rows + (on ? g : 0) * a.group_stride + off;
        if constexpr (FLAT) asm volatile("" : "+v"(src[u]));
        acc[u] = u32x4{0u, 0u, 0u, 0u};
        m[u] = k;  // encode: no slot replaced
        if constexpr (RECOVER) {
          m[u] = m_next[u];
          if (m[u] >= k) {
            if (on) {
              if (i + u < 32) bad_lo |= 1u << (i + u);
              else bad_hi |= 1u << (i + u - 32);
            }
            m[u] = 0u;  // read something valid; the group is not stored
          }
        }
      }
      if constexpr (PF) {
#pragma unroll
        for (int u = 0; u < kPhU; ++u) {
          u32x4 v[KC];
          if constexpr (COMPACT) {
            // the k-1 received rows in order, every lane on every load (no
            // instruction with the lost row's lanes masked off)
#pragma unroll
            for (int r = 0; r + 1 < KC; ++r)
              v[r] = ld16t<NTLD>(src[u] + ((uint32_t)r + ((uint32_t)r >= m[u] ? 1u : 0u)) * a.row_stride);
            v[KC - 1] = u32x4{0u, 0u, 0u, 0u};
          } else {
#pragma unroll
            for (int r = 0; r < KC; ++r) {
              v[r] = u32x4{0u, 0u, 0u, 0u};
              if ((uint32_t)r != m[u]) v[r] = ld16t<NTLD>(src[u] + r * a.row_stride);
            }
          }
          acc[u] = s_par[i + u][tid];
#pragma unroll
          for (int r = 0; r < KC; ++r) acc[u] ^= v[r];
        }
      } else if constexpr (KC > 0) {
        u32x4 v[kPhU][KC];
#pragma unroll
        for (int u = 0; u < kPhU; ++u) {
          const uint64_t g = gidx(i + u);
          const uint8_t* par = RECOVER ? a.parity + (lane_on && g < a.n_groups ? g : 0) * a.parity_stride + off
                                       : nullptr;
#pragma unroll
          for (int r = 0; r < KC; ++r) {
            const uint8_t* q = (RECOVER && (uint32_t)r == m[u]) ? par : src[u] + r * a.row_stride;
            if constexpr (EDGE) {
              // EDGE: windows in the first / last 128-B line of a row (lines
              // the neighbouring row shares) by default-policy loads, so the
              // second row's load finds the line in L2; nt loads elsewhere
              const uint32_t aw = (uint32_t)(uintptr_t)q;
              const uint32_t rs = (uint32_t)(uintptr_t)(src[u] - off + r * a.row_stride);
              const bool edge = (aw >> 7) == (rs >> 7) || ((aw + 15u) >> 7) == ((rs + a.L - 1u) >> 7);
              v[u][r] = edge ? ld16t<false>(q) : ld16t<true>(q);
            } else {
              v[u][r] = ld16t<NTLD>(q);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < kPhU; ++u)
#pragma unroll
          for (int r = 0; r < KC; ++r) acc[u] ^= v[u][r];
      } else {
        // runtime k (> 16: every k up to 16 is templated): batches of up
        // to RTB loads in flight, as even as possible (xor_rows_rt)
#pragma unroll
        for (int u = 0; u < kPhU; ++u) {
          const uint64_t g = gidx(i + u);
          const uint8_t* par = RECOVER ? a.parity + (lane_on && g < a.n_groups ? g : 0) * a.parity_stride + off
                                       : nullptr;
          xor_rows_rt<RTB, RECOVER, NTLD>(acc[u], src[u], a.row_stride, k, m[u], par);
        }
      }
      if constexpr (RECOVER) {
        if (i + kPhU < NL) {
#pragma unroll
          for (int u = 0; u < kPhU; ++u) {
            const uint64_t g = gidx(i + kPhU + u);
            m_next[u] = lane_on && g < a.n_groups ? a.missing[g] : 0u;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kPhU; ++u) s_par[i + u][tid] = acc[u];
    }
    uint32_t ron[2] = {0u, 0u};  // step j's lane is on: bit j % 32 of word j / 32
    bool rbad = false;           // recover: a register step's lost slot out of range
    if constexpr (RS > 0) {
      // one live row address, advanced step by step (the compiler would
      // otherwise keep every step's address live across the unrolled steps)
      const uint64_t g0r = gidx(STEPS);
      const uint8_t* q = a.rows + g0r * a.group_stride + off;
      const uint64_t dq = B * gpb * a.group_stride;
      const uint8_t* qp = RECOVER ? a.parity + g0r * a.parity_stride + off : nullptr;
      const uint64_t dqp = RECOVER ? B * gpb * a.parity_stride : 0u;
      if constexpr (RECOVER && RPF && !RPFE) {
        // RPF: every register step's parity row first (one stream, as the
        // LDS steps' PARFIRST), then the received rows step by step
#pragma unroll
        for (int j = 0; j < RS; ++j) {
          const uint64_t g = g0r + (uint64_t)j * B * gpb;
          const bool on = lane_on && g < a.n_groups && STEPS + j < SP;
          racc[j] = ld16t<NTLD>(a.parity + (on ? g : 0) * a.parity_stride + off);
        }
      }
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const uint64_t g = g0r + (uint64_t)j * B * gpb;
        bool on = lane_on && g < a.n_groups && STEPS + j < SP;
        u32x4 v[KC];
        if constexpr (RECOVER) {
          uint32_t mj = m_reg[j];
          if (mj >= k) {  // out-of-range lost slot: the group is not stored
            rbad = rbad || on;
            on = false;
            mj = 0u;
          }
          const uint8_t* qq = on ? q : a.rows + off;
          // the parity row, then the k-1 received rows in order (compact)
          if constexpr (RPF) v[0] = racc[j];
          else v[0] = ld16t<NTLD>(on ? qp : a.parity + off);
#pragma unroll
          for (int r = 0; r + 1 < KC; ++r)
            v[r + 1] = ld16t<NTLD>(qq + ((uint32_t)r + ((uint32_t)r >= mj ? 1u : 0u)) * a.row_stride);
        } else {
          const uint8_t* qq = on ? q : a.rows + off;
#pragma unroll
          for (int r = 0; r < KC; ++r) v[r] = ld16t<NTLD>(qq + r * a.row_stride);
        }
        ron[j / 32] |= on ? 1u << (j % 32) : 0u;
        u32x4 x = v[0];
#pragma unroll
        for (int r = 1; r < KC; ++r) x ^= v[r];
        racc[j] = x;
        q += dq;
        // the next step's address waits for this step's XOR: one step's k
        // loads in flight, as in the LDS steps
        asm volatile("" : "+v"(q) : "v"(x));
        if constexpr (RECOVER) {
          qp += dqp;
          asm volatile("" : "+v"(qp) : "v"(x));
        }
      }
    }
    if constexpr (RECOVER) {
      if (((bad_lo | bad_hi) != 0u || rbad) && t == 0u) atomicOr(a.err, kErrMissingIndex);
    }
    phase_meet(a.phase_sync, MEET2 ? 2u * p + 1u : p + 1u);
    // INPL: the output row of group g is its own row missing[g] (the in-slot
    // recover written in place; every read of the phase is done by now, and
    // no other workgroup reads this group).  It runs at 0.73-0.76 of 8 TB/s
    // against 0.80-0.82 out of place: its stores land inside the rows' own
    // allocation, the DRAM placement DESIGN.md §4 measured slow for the
    // one-pass kernel's parity too (prefetching the lost indices before the
    // meeting measured no better: profiles/round5/bench_r5{b,c}.json).
    bool ibad = false;
    auto dst = [&](uint64_t g, bool& on) -> uint8_t* {
      if constexpr (INPL) {
        const uint32_t m = a.inplace_missing[g];
        if (m >= k) {
          ibad = ibad || on;
          on = false;
        }
        return const_cast<uint8_t*>(a.rows) + g * a.group_stride + (uint64_t)m * a.row_stride + off;
      } else {
        return a.out + g * a.out_stride + off;
      }
    };
#pragma unroll 4
    for (int i = 0; i < STEPS; ++i) {
      const uint64_t g = gidx(i);
      const uint32_t skip = RECOVER ? ((i < 32 ? bad_lo >> i : bad_hi >> (i - 32)) & 1u) : 0u;
      bool on = lane_on && g < a.n_groups && !skip && i < NL;
      uint8_t* d = dst(on ? g : 0, on);
      if (on) st16t<true>(d, s_par[i][tid]);
    }
    if constexpr (RS > 0) {
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const uint64_t g = gidx(STEPS + j);
        bool on = ((ron[j / 32] >> (j % 32)) & 1u) != 0u;
        uint8_t* d = dst(on ? g : 0, on);
        if (on) st16t<true>(d, racc[j]);
      }
    }
    if constexpr (INPL) {
      if (ibad && t == 0u) atomicOr(a.err, kErrMissingIndex);
    }
    if constexpr (MEET2) phase_meet(a.phase_sync, 2u * p + 2u);
  }
  phase_exit(a.phase_sync, a.phase_host);
}

// Fixed shape, L < 16 (degenerate tiny packets): one lane per output byte.
template <bool RECOVER>
__global__ __launch_bounds__(kBlock) void fixed_small_kernel(FixedArgs a) {
  const uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t g = e / a.L;
  const uint32_t j = (uint32_t)(e - g * a.L);
  if (g >= a.n_groups) return;
  uint8_t acc = 0;
  const uint8_t* src = a.rows + g * a.group_stride + j;
  if (RECOVER) {
    const uint32_t m = a.missing[g];
    if (m >= a.k) {
      if (j == 0) atomicOr(a.err, kErrMissingIndex);
      return;
    }
    acc = a.parity[g * a.parity_stride + j];
    for (uint32_t i = 0; i < a.k; ++i)
      if (i != m) acc ^= src[i * a.row_stride];
  } else {
    for (uint32_t i = 0; i < a.k; ++i) acc ^= src[i * a.row_stride];
  }
  if (a.inplace_missing) {
    // in-slot recover in place: this lane alone reads and writes byte j
    const uint32_t m = a.inplace_missing[g];
    if (m >= a.k) {
      if (j == 0) atomicOr(a.err, kErrMissingIndex);
      return;
    }
    const_cast<uint8_t*>(src)[(uint64_t)m * a.row_stride] = acc;
    return;
  }
  a.out[g * a.out_stride + j] = acc;
}

// ---------------------------------------------------------------------------
// Ragged CSR: the per-group body (one wave per group) and, below it, the
// two-groups-per-wave product kernel.
// ---------------------------------------------------------------------------
// Bytes [o, o+16) of the 32 bytes lo || hi (o in 0..15), branch-free, in
// 32-bit lanes: two 2-way dword selects (by 8 and by 4 bytes), then one byte
// funnel v_alignbyte_b32 per dword.  No variable 64-bit shift on purpose: on
// gfx950 a v_lshlrev_b64 / v_lshrrev_b64 whose amount sits in the wave's last
// allocated VGPR can shift by v0's value instead (the build
// refuses such code, libquic_amd/isa_guard.py).  Written without multi-way
// selects: the compiler turns those into divergent branches, each of which
// waits for the load (vmcnt(0)) and serialises rows.
__device__ __forceinline__ u32x4 bytes16_at(u32x4 lo, u32x4 hi, uint32_t o) {
  // (named scalars, not arrays: an array here was placed in scratch memory)
  const bool b8 = (o & 8u) != 0u, b4 = (o & 4u) != 0u;
  const uint32_t f0 = b8 ? lo.z : lo.x, f1 = b8 ? lo.w : lo.y, f2 = b8 ? hi.x : lo.z,
                 f3 = b8 ? hi.y : lo.w, f4 = b8 ? hi.z : hi.x, f5 = b8 ? hi.w : hi.y;
  const uint32_t g0 = b4 ? f1 : f0, g1 = b4 ? f2 : f1, g2 = b4 ? f3 : f2, g3 = b4 ? f4 : f3,
                 g4 = b4 ? f5 : f4;
  const uint32_t r = o & 3u;
  return u32x4{__builtin_amdgcn_alignbyte(g1, g0, r), __builtin_amdgcn_alignbyte(g2, g1, r),
               __builtin_amdgcn_alignbyte(g3, g2, r), __builtin_amdgcn_alignbyte(g4, g3, r)};
}

// Right shift of a 16-byte vector by sh bytes (0..15), zero fill.
__device__ __forceinline__ u32x4 shr_bytes_bf(u32x4 v, uint32_t sh) {
  return bytes16_at(v, u32x4{0u, 0u, 0u, 0u}, sh);
}

// Bytes [win, win+16) of a zero-padded packet of `len` bytes, len >= 16.
// Always ONE 16-byte load inside the packet (no exec-masked branch): a window
// that crosses the packet end loads the 16 bytes ending at its last byte and
// shifts them down; a window past the end is zeroed by a select.
template <bool NT>
__device__ __forceinline__ u32x4 window16(const uint8_t* row, uint32_t len, uint32_t win) {
  const bool full = win + 16u <= len;
  const u32x4 v = ld16t<NT>(row + (full ? win : len - 16u));
  // sh = 0 for a full window (shift is then the identity); all-zero mask past the end.
  const uint32_t sh = full ? 0u : min(win + 16u - len, 15u);
  const uint32_t keep = win < len ? 0xFFFFFFFFu : 0u;
  return shr_bytes_bf(v, sh) & keep;
}

// Same for len < 16 (wave-uniform branch per packet; rare).
__device__ __forceinline__ u32x4 window16_small(const uint8_t* row, uint32_t len, uint32_t win) {
  uint8_t b[16];
#pragma unroll
  for (uint32_t x = 0; x < 16; ++x) b[x] = (win + x < len) ? row[win + x] : (uint8_t)0;
  u32x4 v;
  __builtin_memcpy(&v, b, 16);
  return v;
}

// Flat-window ragged kernel: one wave per group.
//
// A group's received packets are cut into 16-byte windows (packet i has
// n_i = ceil(len_i/16); window t covers bytes [16t, 16t+16), the last one
// loaded as the 16 bytes ending at the packet end and shifted down, zero
// filled).  The windows of all packets are numbered consecutively
// (flat index f; packet i owns [S_i, S_i + n_i)) and lane l takes
// f = l, l+64, l+128, ...: every lane of every wave-instruction loads, and
// consecutive lanes read consecutive bytes — across packet boundaries too in a
// packed CSR batch.  Each loaded window is XORed into the group's parity
// accumulator in LDS at byte 16t (ds_xor_b64; two packets' windows can meet
// at the same t inside one instruction, hence the atomic).  The lane's packet
// comes from a bitmask of packet starts (bit S_i set): with M the mask word of
// the wave's 64 windows, packet = starts before + inclusive popcount(M) - 1
// (v_mbcnt), then its offset/length/S from an LDS table.
//
// LDS per wave: accumulator 92 x 16 B, start mask 92 x 8 B, packet table
// 64 x 16 B (3.2 KiB).  Groups of more than 64 received packets run in chunks
// of 64 with the same accumulator.
constexpr int kFlatWaves = kBlock / 64;
constexpr int kParWin = 92;  // ceil(1452/16) = 91 windows (+1 spare)

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// The group's LDS state (accumulator, start mask, packet table) passes data
// between lanes of one wave.  The LDS executes a wave's accesses in program
// order; wavefront-scope fences around a wave barrier keep the compiler from
// moving one lane's access across another lane's (no s_waitcnt emitted).
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Lane src's x (ds_bpermute; src in [0, 64)).  The shuffles below take the
// caller's lane instead of HIP's __shfl*, which recompute it (mbcnt) and
// whose lane-derived addresses the compiler hoists out of a resident loop:
// in the service worker they stayed live through the whole job body and
// spilled to scratch at 256 VGPRs (round 6).
__device__ __forceinline__ uint32_t lane_read(uint32_t x, uint32_t src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)x);
}

// Inclusive prefix sum over the wave.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = lane_read(x, lane >= (uint32_t)d ? lane - (uint32_t)d : lane);
    if (lane >= (uint32_t)d) x += y;
  }
  return x;
}

// The accumulator is only ever accessed as uint32_t (plain and atomic): one
// type, so the compiler cannot reorder the plain initialisation / final reads
// across the atomic XORs on type-based alias grounds.
//   ACC = 0: window t's four dwords at 4t .. 4t+3 (ds_xor_b32 x4; lanes on
//            consecutive windows hit every 4th bank: 4-way conflicts)
//   ACC = 1: component-major, dword c of window t at c*kParWin + t (lanes on
//            consecutive windows hit consecutive banks: conflict-free)
//   ACC = 2: interleaved, 2 x ds_xor_b64.  Its U = 4 build was wrong in ~1%
//            of recover groups — not the atomics: that build's 64-bit funnel
//            shift took its amount from the last VGPR; the
//            funnels are 32-bit now.  Not used (no faster than ACC = 1).
template <int ACC>
__device__ __forceinline__ uint32_t acc_idx(uint32_t t, uint32_t c) {
  return ACC == 1 ? c * (uint32_t)kParWin + t : 4u * t + c;
}
// SCOPE: the lanes that share the accumulator -- one wave (the per-group
// body) or every wave of the block (ragged_block_kernel: 4 waves XOR into the
// same groups).  The DS atomic is the same instruction either way; the scope
// states who may race on the word.
template <int SCOPE = __HIP_MEMORY_SCOPE_WAVEFRONT>
__device__ __forceinline__ void lds_xor_u32(uint32_t* p, uint32_t v) {
  __hip_atomic_fetch_xor(p, v, __ATOMIC_RELAXED, SCOPE);
}
template <int ACC, int SCOPE = __HIP_MEMORY_SCOPE_WAVEFRONT>
__device__ __forceinline__ void lds_xor16(uint32_t* acc, uint32_t t, u32x4 v) {
  if constexpr (ACC == 2) {
    uint64_t* p = reinterpret_cast<uint64_t*>(acc + 4u * t);
    __hip_atomic_fetch_xor(p, (uint64_t)v.x | ((uint64_t)v.y << 32), __ATOMIC_RELAXED, SCOPE);
    __hip_atomic_fetch_xor(p + 1, (uint64_t)v.z | ((uint64_t)v.w << 32), __ATOMIC_RELAXED, SCOPE);
  } else {
    lds_xor_u32<SCOPE>(acc + acc_idx<ACC>(t, 0), v.x);
    lds_xor_u32<SCOPE>(acc + acc_idx<ACC>(t, 1), v.y);
    lds_xor_u32<SCOPE>(acc + acc_idx<ACC>(t, 2), v.z);
    lds_xor_u32<SCOPE>(acc + acc_idx<ACC>(t, 3), v.w);
  }
}
template <int ACC>
__device__ __forceinline__ void lds_put16(uint32_t* acc, uint32_t t, u32x4 v) {
  acc[acc_idx<ACC>(t, 0)] = v.x;
  acc[acc_idx<ACC>(t, 1)] = v.y;
  acc[acc_idx<ACC>(t, 2)] = v.z;
  acc[acc_idx<ACC>(t, 3)] = v.w;
}
template <int ACC>
__device__ __forceinline__ u32x4 lds_get16(const uint32_t* acc, uint32_t t) {
  return u32x4{acc[acc_idx<ACC>(t, 0)], acc[acc_idx<ACC>(t, 1)], acc[acc_idx<ACC>(t, 2)],
               acc[acc_idx<ACC>(t, 3)]};
}

// Bytes [16t, 16t+16) of a zero-padded packet (any len >= 1, 16t < len).
template <bool NT>
__device__ __forceinline__ u32x4 packet_window(const uint8_t* row, uint32_t len, uint32_t t) {
  const uint32_t win = 16u * t;
  if (len >= 16u) {
    const bool full = win + 16u <= len;
    const u32x4 v = ld16t<NT>(row + (full ? win : len - 16u));
    return shr_bytes_bf(v, full ? 0u : win + 16u - len);
  }
  return window16_small(row, len, 0u);  // t == 0 (rare: packets below 16 B)
}

// Window t of a zero-padded row of len >= 16 bytes without a branch: a window
// at or past len loads the row's last 16 bytes and returns zero.
template <bool NT>
__device__ __forceinline__ u32x4 parity_window_bf(const uint8_t* row, uint32_t len, uint32_t t) {
  const uint32_t win = 16u * t;
  const bool in = win < len;
  const bool full = win + 16u <= len;
  const uint32_t at = in && full ? win : len - 16u;
  u32x4 v = shr_bytes_bf(ld16t<NT>(row + at), in && !full ? win + 16u - len : 0u);
  const uint32_t keep = in ? 0xFFFFFFFFu : 0u;
  v.x &= keep;
  v.y &= keep;
  v.z &= keep;
  v.w &= keep;
  return v;
}

// Per-group inputs a wave can fetch one group ahead: the group scalars and,
// for the first 64 received packets, lane r's packet length / offset (and for
// recover the parity row's two windows per lane).
struct GroupPrefetch {
  uint32_t p0, k, m, plen;       // wave-uniform
  uint64_t dst_off;              // parity_off (encode) / out_off (recover)
  uint32_t len, offlo, offhi;    // lane r = received packet r (r < 64)
  u32x4 pw0, pw1;                // recover: parity windows lane, lane + 64
};

template <bool RECOVER>
__device__ __forceinline__ void group_scalars(const RaggedArgs& a, uint64_t g, GroupPrefetch& f) {
  f.p0 = a.grp_ptr[g];
  f.k = a.grp_ptr[g + 1] - f.p0;
  f.m = 0xFFFFFFFFu;
  f.plen = 0;
  if constexpr (RECOVER) {
    f.m = a.missing[g];
    f.plen = a.parity_len[g];
    f.dst_off = a.out_off[g];
  } else {
    f.dst_off = a.parity_off[g];
  }
}

// Vector part (needs the scalars).  Invalid groups load nothing.
template <bool RECOVER, bool NT>
__device__ __forceinline__ void group_vectors(const RaggedArgs& a, uint64_t g, uint32_t lane,
                                              GroupPrefetch& f) {
  f.len = f.offlo = f.offhi = 0;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  f.pw0 = f.pw1 = zero;
  const bool ok = f.k >= 1u && f.k <= 255u && (!RECOVER || (f.m < f.k && f.plen >= 1u &&
                                                             f.plen <= kMaxPacket));
  if (!ok) return;
  const uint32_t kr = RECOVER ? f.k - 1u : f.k;
  if (lane < kr) {
    const uint32_t p = f.p0 + lane + (lane >= f.m ? 1u : 0u);
    f.len = a.pkt_len[p];
    const uint64_t o = a.pkt_off[p];
    f.offlo = (uint32_t)o;
    f.offhi = (uint32_t)(o >> 32);
  }
  if constexpr (RECOVER) {
    const uint8_t* prow = a.parity + a.parity_off[g];
    if (16u * lane < f.plen) f.pw0 = packet_window<NT>(prow, f.plen, lane);
    if (16u * (lane + 64u) < f.plen) f.pw1 = packet_window<NT>(prow, f.plen, lane + 64u);
  }
}

// One group, one wave (see the flat-window description above).
template <bool RECOVER, bool NT, int U, int ACC, bool BF = false>
__device__ __forceinline__ void ragged_group(const RaggedArgs& a, uint64_t g, uint32_t lane,
                                             const GroupPrefetch& f, uint32_t* par,
                                             uint64_t* head, u32x4* meta) {
  const uint32_t p0 = f.p0, k = f.k, m = f.m;
  uint32_t plen = f.plen;
  if (k == 0u || k > 255u) {  // grp_ptr not monotone shows up as k > 255 too
    if (lane == 0) atomicOr(a.err, kErrGroupSize);
    return;
  }
  const u32x4 zero = {0u, 0u, 0u, 0u};
  if constexpr (RECOVER) {
    if (m >= k) {
      if (lane == 0) atomicOr(a.err, kErrMissingIndex);
      return;
    }
    if (plen == 0u || plen > kMaxPacket) {
      if (lane == 0) atomicOr(a.err, kErrParityLength);
      return;
    }
    // accumulator := the parity row (zero past plen), prefetched windows
    lds_put16<ACC>(par, lane, f.pw0);
    if (lane + 64u < kParWin) lds_put16<ACC>(par, lane + 64u, f.pw1);
  } else {
    for (uint32_t t = lane; t < kParWin; t += 64u) lds_put16<ACC>(par, t, zero);
  }
  const uint32_t kr = RECOVER ? k - 1u : k;  // received packets
  const uint32_t lim = RECOVER ? plen : kMaxPacket;
  uint32_t mx = 0;
  for (uint32_t c = 0; c < kr; c += 64u) {
    // packet table of this chunk: lane j = received packet c + j
    const uint32_t r = c + lane;
    uint32_t len = f.len, offlo = f.offlo, offhi = f.offhi;
    if (c > 0) {  // groups of more than 64 received packets: load inline
      len = offlo = offhi = 0;
      if (r < kr) {
        const uint32_t p = p0 + r + (r >= m ? 1u : 0u);
        len = a.pkt_len[p];
        const uint64_t o = a.pkt_off[p];
        offlo = (uint32_t)o;
        offhi = (uint32_t)(o >> 32);
      }
    }
    const bool bad = r < kr && (len == 0u || len > lim);
    if (wave_any(bad)) {
      if (lane == 0) atomicOr(a.err, kErrPacketLength);
      return;
    }
    mx = max(mx, len);
    const uint32_t n = (len + 15u) >> 4;
    const uint32_t incl = wave_incl_scan(n, lane);
    const uint32_t S = incl - n;
    const uint32_t W = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t nit = (W + 63u) >> 6;
    wave_lds_order();  // accumulator initialised / previous chunk's table reads done
    for (uint32_t q = lane; q < nit; q += 64u) head[q] = 0ull;
    wave_lds_order();
    if (r < kr) {
      meta[lane] = u32x4{offlo, offhi, len, S};
      __hip_atomic_fetch_or(&head[S >> 6], 1ull << (S & 63u), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    wave_lds_order();  // packet table and start mask complete
    const uint64_t below = lane == 63u ? ~0ull : ((2ull << lane) - 1ull);
    const uint32_t last = min(kr - c, 64u) - 1u;
    uint32_t before = 0;  // packet starts in earlier wave-iterations
    if (BF && !wave_any(r < kr && len < 16u)) {
      // Branch-free form: every lane loads and XORs on every iteration.  A
      // lane past W loads its packet's last window and XORs ZERO into window
      // `lane` (a no-op, conflict-free) — no exec-masked block, so the
      // compiler cannot sink a load into one and wait on it right there.
      for (uint32_t it = 0; it < nit; it += U) {
        uint64_t M[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint64_t w = head[min(it + (uint32_t)u, (uint32_t)kParWin - 1u)];
          M[u] = it + (uint32_t)u < nit ? w : 0ull;
        }
        u32x4 md[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t pi = min(before + (uint32_t)__popcll(M[u] & below) - 1u, last);
          before += (uint32_t)__popcll(M[u]);
          md[u] = meta[pi];
        }
        u32x4 v[U];
        uint32_t ts[U];  // window (bits 0-15) | shift (bits 16-19) | valid (bit 20)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t fl = 64u * (it + (uint32_t)u) + lane;
          const uint32_t win = 16u * (fl - md[u].w);
          const bool full = win + 16u <= md[u].z;
          v[u] = ld16t<NT>(a.bytes + (((uint64_t)md[u].y << 32) | md[u].x) +
                           (full ? win : md[u].z - 16u));
          const uint32_t sh = full ? 0u : min(win + 16u - md[u].z, 15u);
          ts[u] = fl < W ? ((fl - md[u].w) | (sh << 16) | (1u << 20)) : lane;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          uint32_t keep = (ts[u] >> 20) ? 0xFFFFFFFFu : 0u;
          // opaque to the optimiser: otherwise it proves the XOR of an idle
          // lane to be 0, turns it into a branch and sinks the load into it
          __asm__ volatile("" : "+v"(keep));
          lds_xor16<ACC>(par, ts[u] & 0xFFFFu, shr_bytes_bf(v[u], (ts[u] >> 16) & 15u) & keep);
        }
      }
    } else if (!BF && !wave_any(r < kr && len < 16u)) {
      // Every packet >= 16 B: every lane loads 16 in-packet bytes each
      // iteration (lanes past W re-read their packet's last window and drop
      // it), U iterations' loads in flight before the first XOR.
      for (uint32_t it = 0; it < nit; it += U) {
        // phase 1: the U start-mask words (independent LDS reads)
        uint64_t M[U];
#pragma unroll
        for (int u = 0; u < U; ++u) M[u] = it + u < nit ? head[it + u] : 0ull;
        // phase 2: packet of each window, its table entry
        u32x4 md[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t pi = min(before + (uint32_t)__popcll(M[u] & below) - 1u, last);
          before += (uint32_t)__popcll(M[u]);
          md[u] = meta[pi];
        }
        // phase 3: U in-packet 16-B loads, all in flight
        u32x4 v[U];
        uint32_t tt[U], sh[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t fl = 64u * (it + u) + lane;
          const uint32_t win = 16u * (fl - md[u].w);
          const bool full = win + 16u <= md[u].z;
          v[u] = ld16t<NT>(a.bytes + (((uint64_t)md[u].y << 32) | md[u].x) +
                           (full ? win : md[u].z - 16u));
          sh[u] = full ? 0u : min(win + 16u - md[u].z, 15u);
          tt[u] = fl < W ? fl - md[u].w : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (tt[u] != 0xFFFFFFFFu) lds_xor16<ACC>(par, tt[u], shr_bytes_bf(v[u], sh[u]));
      }
    } else {
      // Some packet below 16 B (rare): generic per-lane windows.
      for (uint32_t it = 0; it < nit; ++it) {
        const uint64_t M = head[it];
        const uint32_t fl = 64u * it + lane;
        const uint32_t pi = min(before + (uint32_t)__popcll(M & below) - 1u, last);
        before += (uint32_t)__popcll(M);
        if (fl < W) {
          const u32x4 md = meta[pi];
          const uint32_t t = fl - md.w;
          lds_xor16<ACC>(par, t, packet_window<false>(a.bytes + (((uint64_t)md.y << 32) | md.x),
                                                  md.z, t));
        }
      }
    }
  }
  if constexpr (!RECOVER) {
    plen = wave_max11(mx);
    if (lane == 0) a.parity_len_out[g] = (uint16_t)plen;
  }
  wave_lds_order();  // every lane's XORs into the accumulator done
  uint8_t* dst = a.out + f.dst_off;
  if (plen >= 16u) {
    const uint32_t nw = (plen + 15u) >> 4;
    for (uint32_t t = lane; t < nw; t += 64u) {
      if (16u * t + 16u <= plen) {
        st16t<NT>(dst + 16u * t, lds_get16<ACC>(par, t));
      } else {
        // tail: the 16 bytes ending at plen, from windows t-1 and t
        const uint32_t o = plen - 16u * t;  // 1..15
        const u32x4 lo = lds_get16<ACC>(par, t - 1u), hi = lds_get16<ACC>(par, t);
        st16t<NT>(dst + plen - 16u, bytes16_at(lo, hi, o));
      }
    }
  } else if (lane < plen) {
    dst[lane] = (uint8_t)(par[acc_idx<ACC>(0, lane >> 2)] >> (8u * (lane & 3u)));
  }
}

// One group's parity accumulator in LDS, component-major (ACC = 1).
constexpr uint32_t kAccWords = 4 * kParWin;

// Ragged CSR, large batches — the PRODUCT kernel (launch_ragged), round 3:
// BLOCK-flat windows.  A short-lived block of WAVES waves owns GPB consecutive
// groups and numbers the 16-B windows of ALL their received packets
// consecutively (the flat-window mapping of ragged_group, widened from one
// wave to the block); lane tid of iteration i takes window NT i + tid
// (NT = 64 WAVES), so one block instruction reads NT/4 KiB of the batch, in
// batch order.  Why: without its parity stores ragged_multi_kernel (each wave
// its own pair of groups, the waves 14 KB apart) read its packets at
// 5.56 TB/s, where 16 waves streaming one chunk (the chunk-phased experiment)
// read at ~6.3 TB/s — fewer, wider streams.  4 waves x 8 groups measured
// +2.5% encode / +4.5% recover over ragged_multi_kernel on three boxes;
// 2 x 4, 2 x 6, 4 x 6, 4 x 10, 4 x 12 less, 8 x 16 and 16 x 32 slower (block
// barriers), U = 1 / 3 no better (profiles/round3/ragged_block/, DESIGN.md
// §4).  One pass of setup per block: the group scalars (wave 0), one
// received packet per lane, a block scan for each packet's first window S, a
// start bitmask and per 64-window block the number of packets starting
// before it (a second block scan).  Blocks that do not fit (more than NT
// received packets or CAPW windows, a packet below 16 B, any invalid field)
// run the per-group body, one wave per group, so outputs and error bits are
// exactly those of the per-group kernel.  Encode parity lengths come from an
// LDS atomicMax.
template <int WAVES>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t lane, uint32_t wv,
                                                    uint32_t* s_w, uint32_t& total) {
  const uint32_t incl = wave_incl_scan(x, lane);
  if (lane == 63u) s_w[wv] = incl;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < WAVES; ++w) {
    const uint32_t v = s_w[w];
    base += (uint32_t)w < wv ? v : 0u;
    tot += v;
  }
  total = tot;
  __syncthreads();  // s_w free again
  return base + incl - x;
}

// PF (recover): the parity windows are loaded into the accumulators before the
// packet table, so their round trip overlaps the table's (measured equal to
// loading them after the scan, profiles/round3/ragged_block/block3.txt).
// DIAG (tools/tune only; bits): 1 = no parity stores (not exact); 2 = output
// rows stored as whole 128-B lines (zeros past the parity length up to the
// line end: the zero-padded parity of SURVEY.md Appendix A, for output slots
// that have the room -- the write-granularity probe of round 6); 4 = no tail
// logic (every window XORed whole, in place: the VALU probe of round 6, not
// exact); 8 = parity stores through the caches (not nontemporal); 16 = payload
// loads through the caches (both exact: the cache-policy probe of round 6);
// bits 5-7 = P != 0: parity stores with explicit policy st16pol<P> (exact).
template <bool RECOVER, int WAVES, int GPB, int U = 2, bool PF = true, bool AL = true, int DIAG = 0>
__device__ __forceinline__ void ragged_block_body(const RaggedArgs& a) {
  static_assert(GPB >= 2 && GPB <= 64, "group slots are lanes of wave 0");
  constexpr uint32_t NT = 64u * WAVES;
  constexpr uint32_t NBLK = NT;        // 64-window blocks: CAPW = 64 NT windows
  constexpr uint32_t CAPW = 64u * NBLK;
  // per-wave fallback scratch (ragged_group): accumulator, start mask, table
  constexpr uint32_t kFbWords = 4u * kParWin + 2u * kParWin + 4u * 64u;
  constexpr uint32_t kMainWords = GPB * kAccWords + 4u * NT;  // accumulators + packet table
  constexpr uint32_t kRawWords = kMainWords > WAVES * kFbWords ? kMainWords : WAVES * kFbWords;
  __shared__ uint32_t s_raw[kRawWords];
  __shared__ uint64_t s_head[NBLK];
  __shared__ uint32_t s_cnt[NBLK];
  __shared__ uint32_t s_rb[GPB + 1], s_kb[GPB], s_m[GPB], s_pl[GPB], s_ob[GPB + 1];
  __shared__ uint64_t s_doff[GPB], s_poff[GPB];
  __shared__ uint32_t s_w[WAVES], s_fit;
  uint32_t* acc = s_raw;
  u32x4* pk = reinterpret_cast<u32x4*>(s_raw + GPB * kAccWords);
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t g0 = (uint64_t)blockIdx.x * GPB;
  if (g0 >= a.n_groups) return;  // block-uniform
  const uint32_t ng = (uint32_t)min<uint64_t>((uint64_t)GPB, a.n_groups - g0);
  s_head[tid] = 0ull;  // NBLK == NT
  // ---- 1. group scalars (wave 0, lane j = group slot j)
  if (wv == 0u) {
    uint32_t k = 0, m = 0xFFFFFFFFu, pl = 0, r = 0, p0 = 0;
    uint64_t d = 0, po = 0;
    bool ok = true;
    if (lane < ng) {
      p0 = a.grp_ptr[g0 + lane];
      k = a.grp_ptr[g0 + lane + 1] - p0;
      if constexpr (RECOVER) {
        m = a.missing[g0 + lane];
        pl = a.parity_len[g0 + lane];
        d = a.out_off[g0 + lane];
        po = a.parity_off[g0 + lane];
        ok = m < k && pl >= 16u && pl <= kMaxPacket;
      } else {
        d = a.parity_off[g0 + lane];
      }
      ok = ok && k >= 1u && k <= 255u;
      r = ok ? (RECOVER ? k - 1u : k) : 0u;
    }
    const uint32_t incl = wave_incl_scan(r, lane);
    const uint32_t R = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (lane < (uint32_t)GPB) {
      s_rb[lane] = incl - r;
      s_kb[lane] = p0;
      s_m[lane] = m;
      s_pl[lane] = pl;
      s_doff[lane] = d;
      s_poff[lane] = po;
    }
    const bool all_ok = !wave_any(lane < ng && !ok);  // every lane of wave 0
    if (lane == 0u) {
      s_rb[GPB] = R;
      s_fit = (all_ok && R <= NT) ? 1u : 0u;
    }
  }
  __syncthreads();
  const uint32_t R = s_rb[GPB];
  bool fit = s_fit != 0u;
  // ---- 2. one received packet per lane
  if (RECOVER && PF && fit) {
    for (uint32_t q = tid; q < GPB * (uint32_t)kParWin; q += NT) {
      const uint32_t jq = q / (uint32_t)kParWin, t = q - jq * (uint32_t)kParWin;
      u32x4 w = {0u, 0u, 0u, 0u};
      if (jq < ng) w = parity_window_bf<true>(a.parity + s_poff[jq], s_pl[jq], t);
      lds_put16<1>(acc + jq * kAccWords, t, w);
    }
  }
  uint32_t len = 0, offlo = 0, offhi = 0, j = 0;
  if (fit && tid < R) {
#pragma unroll
    for (int q = 1; q < GPB; ++q) j += tid >= s_rb[q] ? 1u : 0u;
    const uint32_t i = tid - s_rb[j];
    const uint32_t p = s_kb[j] + i + (RECOVER && i >= s_m[j] ? 1u : 0u);
    len = a.pkt_len[p];
    const uint64_t o = a.pkt_off[p];
    offlo = (uint32_t)o;
    offhi = (uint32_t)(o >> 32);
    const uint32_t lim = RECOVER ? s_pl[j] : kMaxPacket;
    if (len < 16u || len > lim) s_fit = 0u;  // benign race: every writer stores 0
    if (!RECOVER) atomicMax(&s_pl[j], len);
  }
  const uint32_t n = (len + 15u) >> 4;
  uint32_t W;
  const uint32_t S = block_excl_scan<WAVES>(n, lane, wv, s_w, W);  // (barriers publish s_fit)
  fit = fit && s_fit != 0u && W <= CAPW;
  if (!fit) {
    // per-group body, one wave per group (exact outputs and error bits)
    uint32_t* fb = s_raw + wv * kFbWords;
    for (uint32_t jj = wv; jj < ng; jj += WAVES) {
      GroupPrefetch f;
      group_scalars<RECOVER>(a, g0 + jj, f);
      group_vectors<RECOVER, true>(a, g0 + jj, lane, f);
      wave_lds_order();
      ragged_group<RECOVER, true, 2, 1>(a, g0 + jj, lane, f, fb,
                                        reinterpret_cast<uint64_t*>(fb + 4u * kParWin),
                                        reinterpret_cast<u32x4*>(fb + 6u * kParWin));
      wave_lds_order();
    }
    return;
  }
  if (tid < R) {
    pk[tid] = u32x4{offlo, offhi, len | (j << 16), S};
    __hip_atomic_fetch_or(&s_head[S >> 6], 1ull << (S & 63u), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  // accumulators: the parity rows (recover) or zero (encode), windows of all groups
  if (!(RECOVER && PF)) {
    for (uint32_t q = tid; q < GPB * (uint32_t)kParWin; q += NT) {
      const uint32_t jq = q / (uint32_t)kParWin, t = q - jq * (uint32_t)kParWin;
      u32x4 w = {0u, 0u, 0u, 0u};
      if constexpr (RECOVER) {
        if (jq < ng) w = parity_window_bf<true>(a.parity + s_poff[jq], s_pl[jq], t);
      }
      lds_put16<1>(acc + jq * kAccWords, t, w);
    }
  }
  __syncthreads();  // packet table, start mask, accumulators, parity lengths
  const uint32_t nblk = (W + 63u) >> 6;
  uint32_t tot;
  const uint32_t c = block_excl_scan<WAVES>(tid < nblk ? (uint32_t)__popcll(s_head[tid]) : 0u,
                                            lane, wv, s_w, tot);
  s_cnt[tid] = c;
  if (wv == 0u) {  // output windows per group (encode: the max lengths are final)
    uint32_t nw = lane < ng ? (s_pl[lane] + 15u) >> 4 : 0u;
    if (DIAG & 2) nw = lane < ng ? ((s_pl[lane] + 127u) >> 7) << 3 : 0u;
    const uint32_t incl = wave_incl_scan(nw, lane);
    if (lane < (uint32_t)GPB) s_ob[lane] = incl - nw;
    if (lane == 0u) s_ob[GPB] = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (!RECOVER && lane < ng) a.parity_len_out[g0 + lane] = (uint16_t)s_pl[lane];
  }
  __syncthreads();
  // ---- 3. the flat windows, U iterations' loads in flight
  const uint64_t below = lane == 63u ? ~0ull : ((2ull << lane) - 1ull);
  const uint32_t nit = (W + NT - 1u) / NT;
  for (uint32_t it = 0; it < nit; it += U) {
    u32x4 md[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t f = (it + (uint32_t)u) * NT + tid;
      const uint32_t b = min(f >> 6, nblk - 1u);
      const uint64_t M = s_head[b];
      const uint32_t pi = min(s_cnt[b] + (uint32_t)__popcll(M & below) - 1u, R - 1u);
      md[u] = pk[pi];
    }
    u32x4 v[U];
    uint32_t tt[U], sh[U];
    bool inp[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t f = (it + (uint32_t)u) * NT + tid;
      const uint32_t ln = md[u].z & 0xFFFFu;
      const uint32_t win = 16u * (f - md[u].w);
      const bool full = win + 16u <= ln;
      const uint64_t at = (((uint64_t)md[u].y << 32) | md[u].x) + win;
      // AL: a last window whose start is 16-B aligned (payloads on 16-B
      // boundaries, the payload arena's layout) is loaded in place and its
      // bytes past the packet masked: an aligned 16-B load holding one packet
      // byte cannot leave that byte's page.  Otherwise the 16 bytes ending at
      // the packet end, shifted down.
      inp[u] = full || (AL && win < ln && (at & 15u) == 0u) || (DIAG & 4);
      v[u] = ld16t<(DIAG & 16) == 0>(a.bytes + (inp[u] ? at : at - win + ln - 16u));
      sh[u] = full ? 0u : min(win + 16u - ln, 15u);
      tt[u] = f < W ? (md[u].z >> 16) * kAccWords + (f - md[u].w) : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (tt[u] != 0xFFFFFFFFu) {
        u32x4 w;
        if constexpr ((DIAG & 4) != 0) {
          w = v[u];
        } else if constexpr (AL) {
          // in place: v & (ones >> sh); shifted: v >> sh (sh = 0 when full)
          const u32x4 ones = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
          const u32x4 m = shr_bytes_bf(inp[u] ? ones : v[u], sh[u]);
          w = inp[u] ? (m & v[u]) : m;
        } else {
          w = shr_bytes_bf(v[u], sh[u]);
        }
        lds_xor16<1, __HIP_MEMORY_SCOPE_WORKGROUP>(acc, tt[u], w);
      }
  }
  __syncthreads();  // every lane's XORs done
  // ---- 4. stores, flattened over the groups' output windows
  const uint32_t NW = s_ob[GPB];
  for (uint32_t q = tid; q < NW; q += NT) {
    uint32_t jq = 0;
#pragma unroll
    for (int i = 1; i < GPB; ++i) jq += q >= s_ob[i] ? 1u : 0u;
    const uint32_t t = q - s_ob[jq];
    const uint32_t plen = s_pl[jq];
    uint8_t* dst = a.out + s_doff[jq];
    const uint32_t* ac = acc + jq * kAccWords;
    if ((DIAG & 1) && plen != 0xFFFFFu) continue;  // never a real length: no stores
    if (DIAG & 2) {  // whole lines: the accumulator is zero past plen
      const u32x4 z = {0u, 0u, 0u, 0u};
      st16t<(DIAG & 8) == 0>(dst + 16u * t, t < (uint32_t)kParWin ? lds_get16<1>(ac, t) : z);
      continue;
    }
    if (16u * t + 16u <= plen) {
      if constexpr ((DIAG >> 5) != 0)
        st16pol<(DIAG >> 5)>(dst + 16u * t, lds_get16<1>(ac, t));
      else
        st16t<(DIAG & 8) == 0>(dst + 16u * t, lds_get16<1>(ac, t));
    } else {
      const uint32_t o = plen - 16u * t;  // 1..15
      const u32x4 x = bytes16_at(lds_get16<1>(ac, t - 1u), lds_get16<1>(ac, t), o);
      if constexpr ((DIAG >> 5) != 0)
        st16pol<(DIAG >> 5)>(dst + plen - 16u, x);
      else
        st16t<(DIAG & 8) == 0>(dst + plen - 16u, x);
    }
  }
}


// Completion signal for a host that spins on mapped memory instead of
// waiting on an event (~6 us less per flush, tools/tune/tune_latency): every
// thread's stores (outputs in mapped host memory) are made visible
// system-wide, the block is counted, and the last block to finish resets the
// counter and stores the token into the host-mapped flag.  Block-uniform
// call, after the block's work.
__device__ __forceinline__ void ragged_signal_done(const RaggedArgs& a) {
  if (a.done_flag == nullptr) return;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(a.done_count, 1u, __ATOMIC_ACQ_REL,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1u) {
      __hip_atomic_store(a.done_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(a.done_flag, a.done_token, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// The block kernel; with done_flag set (mapped batches of any size, round 4)
// it signals completion like the small-batch kernel, so the host neither
// stages the tables nor waits on an event.
template <bool RECOVER, int WAVES, int GPB, int U = 2, bool PF = true, bool AL = true, int DIAG = 0>
__global__ __launch_bounds__(64 * WAVES) void ragged_block_kernel(RaggedArgs a) {
  ragged_block_body<RECOVER, WAVES, GPB, U, PF, AL, DIAG>(a);
  ragged_signal_done(a);
}


// Two groups per wave (round 2's product kernel; since round 6 the kernel of
// large batches whose groups are small -- launch_ragged's shape-aware choice,
// below): GPW consecutive groups in
// ONE flat window space — their received packets fill the 64-lane packet
// table together — so the per-group load chain (group pointer -> packet table
// -> packet bytes), which parks the one-group waves for 70% of their cycles
// (SQ_WAIT_ANY, profiles/round1/sq_stalls_fec_pq.txt), and the partially idle
// last iteration are paid once per GPW groups.  Groups that do not fit (more
// than 64 received packets together, a packet below 16 B, any invalid field)
// run the per-group body above with its exact error semantics.  Measured
// +1.0-1.6% encode and recover over one group per wave in three interleaved
// A/B runs (tune_multi_t2.txt, ragged_slots_p*.txt, tune_multi_sp.txt);
// three groups per wave overflow the table too often (-10%).  tools/tune runs
// it with GPW = 2.

template <int N, typename T>
__device__ __forceinline__ T sel_n(const T (&v)[N], uint32_t j) {
  T r = v[0];
#pragma unroll
  for (int i = 1; i < N; ++i) r = j == (uint32_t)i ? v[i] : r;
  return r;
}

// GPW groups g0 .. g0+ng-1 of one wave, up to their XOR into the LDS
// accumulators `par` (GPW x kAccWords).  Returns false when the groups took
// the per-group body (odd packets, invalid fields, > 64 received packets):
// then their outputs are already stored; true: ragged_pair_store writes them
// from `par` with lengths pl[] at offsets doff[].

template <bool RECOVER, bool NT, int GPW, int U, bool BF, bool PBF = true>
__device__ __forceinline__ bool ragged_pair_xor(const RaggedArgs& a, uint64_t g0, uint32_t ng,
                                                uint32_t lane, uint32_t* par, uint64_t* head,
                                                u32x4* meta, uint32_t (&pl)[GPW],
                                                uint64_t (&doff)[GPW]) {
  constexpr int ACC = 1;
  // wave-uniform group scalars
  uint32_t kb[GPW + 1], rb[GPW + 1], mm[GPW];
  const uint32_t P0 = a.grp_ptr[g0];
  bool ok = true;
  kb[0] = rb[0] = 0;
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    uint32_t k = 0, m = 0xFFFFFFFFu, p = 0;
    uint64_t d = 0;
    if ((uint32_t)j < ng) {
      k = a.grp_ptr[g0 + j + 1] - P0 - kb[j];
      if constexpr (RECOVER) {
        m = a.missing[g0 + j];
        p = a.parity_len[g0 + j];
        d = a.out_off[g0 + j];
        ok = ok && m < k && p >= 16u && p <= kMaxPacket;
      } else {
        d = a.parity_off[g0 + j];
      }
      ok = ok && k >= 1u && k <= 255u;
    }
    kb[j + 1] = kb[j] + k;
    rb[j + 1] = rb[j] + (RECOVER && k ? k - 1u : k);
    mm[j] = m;
    pl[j] = p;
    doff[j] = d;
  }
  const uint32_t R = rb[GPW];
  ok = ok && R <= 64u;

  // lane r: received packet r of the wave's groups
  uint32_t jl = 0, base = 0, kbase = 0, ml = 0xFFFFFFFFu, lim = kMaxPacket;
#pragma unroll
  for (int j = 1; j < GPW; ++j) {
    const bool in = lane >= rb[j];
    jl += in ? 1u : 0u;
    base = in ? rb[j] : base;
    kbase = in ? kb[j] : kbase;
  }
  ml = sel_n<GPW>(mm, jl);
  if constexpr (RECOVER) lim = sel_n<GPW>(pl, jl);
  uint32_t len = 0, offlo = 0, offhi = 0;
  if (ok && lane < R) {
    const uint32_t i = lane - base;
    const uint32_t p = P0 + kbase + i + (RECOVER && i >= ml ? 1u : 0u);
    len = a.pkt_len[p];
    const uint64_t o = a.pkt_off[p];
    offlo = (uint32_t)o;
    offhi = (uint32_t)(o >> 32);
  }
  // accumulators: the parity rows (recover) or zero (encode)
  if (ok) {
#pragma unroll
    for (int j = 0; j < GPW; ++j) {
      uint32_t* acc = par + j * kAccWords;
      if constexpr (RECOVER) {
        const uint8_t* prow = a.parity + ((uint32_t)j < ng ? a.parity_off[g0 + j] : 0ull);
        const uint32_t plj = (uint32_t)j < ng ? pl[j] : 0u;
        // branch-free parity windows: every lane loads a window inside the
        // row (lanes past plj re-read its last 16 bytes and keep zero), so
        // neither load runs with lanes masked off.  plj >= 16 whenever the
        // pair takes this path (ok); the branch is wave-uniform.
        const u32x4 zero = {0u, 0u, 0u, 0u};
        u32x4 w0 = zero, w1 = zero;
        if (!PBF) {  // the round-2 form (A/B reference, tools/tune/ragged_exp.inc)
          if (16u * lane < plj) w0 = packet_window<NT>(prow, plj, lane);
          if (16u * (lane + 64u) < plj) w1 = packet_window<NT>(prow, plj, lane + 64u);
        } else if (plj >= 16u) {
          w0 = parity_window_bf<NT>(prow, plj, lane);
          w1 = parity_window_bf<NT>(prow, plj, lane + 64u);
        }
        lds_put16<ACC>(acc, lane, w0);
        if (lane + 64u < kParWin) lds_put16<ACC>(acc, lane + 64u, w1);
      } else {
        const u32x4 zero = {0u, 0u, 0u, 0u};
        for (uint32_t t = lane; t < kParWin; t += 64u) lds_put16<ACC>(acc, t, zero);
      }
    }
  }
  const bool odd = lane < R && (len < 16u || len > lim);
  if (!ok || wave_any(odd)) {
    // per-group body (exact error semantics of the one-group kernel)
    for (uint32_t j = 0; j < ng; ++j) {
      GroupPrefetch f;
      group_scalars<RECOVER>(a, g0 + j, f);
      group_vectors<RECOVER, NT>(a, g0 + j, lane, f);
      wave_lds_order();
      ragged_group<RECOVER, NT, U, ACC, BF>(a, g0 + j, lane, f, par, head, meta);
      wave_lds_order();
    }
    return false;
  }
  const uint32_t n = (len + 15u) >> 4;
  const uint32_t incl = wave_incl_scan(n, lane);
  const uint32_t S = incl - n;
  const uint32_t W = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  const uint32_t nit = (W + 63u) >> 6;  // W <= 64 x 91
  for (uint32_t q = lane; q < nit; q += 64u) head[q] = 0ull;
  wave_lds_order();
  if (lane < R) {
    meta[lane] = u32x4{offlo, offhi, len | (jl << 16), S};
    __hip_atomic_fetch_or(&head[S >> 6], 1ull << (S & 63u), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  wave_lds_order();  // accumulators, packet table and start mask complete
  const uint64_t below = lane == 63u ? ~0ull : ((2ull << lane) - 1ull);
  const uint32_t last = R - 1u;
  uint32_t before = 0;
  for (uint32_t it = 0; it < nit; it += U) {
    uint64_t M[U];
#pragma unroll
    for (int u = 0; u < U; ++u) M[u] = it + u < nit ? head[it + u] : 0ull;
    u32x4 md[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t pi = min(before + (uint32_t)__popcll(M[u] & below) - 1u, last);
      before += (uint32_t)__popcll(M[u]);
      md[u] = meta[pi];
    }
    u32x4 v[U];
    uint32_t tt[U], sh[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t fl = 64u * (it + u) + lane;
      const uint32_t ln = md[u].z & 0xFFFFu;
      const uint32_t win = 16u * (fl - md[u].w);
      const bool full = win + 16u <= ln;
      v[u] = ld16t<NT>(a.bytes + (((uint64_t)md[u].y << 32) | md[u].x) + (full ? win : ln - 16u));
      sh[u] = full ? 0u : min(win + 16u - ln, 15u);
      tt[u] = fl < W ? (md[u].z >> 16) * kAccWords + (fl - md[u].w) : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (BF) {
        // branch-free: a lane past W XORs ZERO into window `lane` of the first
        // accumulator (a no-op, conflict-free), so no load or LDS atomic sits
        // in an exec-masked block
        uint32_t keep = tt[u] != 0xFFFFFFFFu ? 0xFFFFFFFFu : 0u;
        __asm__ volatile("" : "+v"(keep));
        lds_xor16<ACC>(par, tt[u] != 0xFFFFFFFFu ? tt[u] : lane, shr_bytes_bf(v[u], sh[u]) & keep);
      } else if (tt[u] != 0xFFFFFFFFu) {
        lds_xor16<ACC>(par, tt[u], shr_bytes_bf(v[u], sh[u]));
      }
    }
  }
  if constexpr (!RECOVER) {
#pragma unroll
    for (int j = 0; j < GPW; ++j) {
      pl[j] = wave_max11(lane < R && jl == (uint32_t)j ? len : 0u);
      if (lane == 0 && (uint32_t)j < ng) a.parity_len_out[g0 + j] = (uint16_t)pl[j];
    }
  }
  return true;
}

template <bool NT, int GPW>
__device__ __forceinline__ void ragged_pair_store(const RaggedArgs& a, uint32_t ng, uint32_t lane,
                                                  const uint32_t* par, const uint32_t (&pl)[GPW],
                                                  const uint64_t (&doff)[GPW]) {
  constexpr int ACC = 1;
  wave_lds_order();  // every lane's XORs done
  // write-out, flattened over the groups' output windows
  uint32_t ob[GPW + 1];
  ob[0] = 0;
#pragma unroll
  for (int j = 0; j < GPW; ++j) ob[j + 1] = ob[j] + ((uint32_t)j < ng ? (pl[j] + 15u) >> 4 : 0u);
  const uint32_t NW = ob[GPW];
  for (uint32_t q = lane; q < NW; q += 64u) {
    uint32_t jq = 0, qb = 0;
#pragma unroll
    for (int j = 1; j < GPW; ++j) {
      const bool in = q >= ob[j];
      jq += in ? 1u : 0u;
      qb = in ? ob[j] : qb;
    }
    const uint32_t t = q - qb;
    const uint32_t plen = sel_n<GPW>(pl, jq);
    uint8_t* dst = a.out + sel_n<GPW>(doff, jq);
    const uint32_t* acc = par + jq * kAccWords;
    if (16u * t + 16u <= plen) {
      st16t<NT>(dst + 16u * t, lds_get16<ACC>(acc, t));
    } else {
      const uint32_t o = plen - 16u * t;  // 1..15
      const u32x4 lo = lds_get16<ACC>(acc, t - 1u), hi = lds_get16<ACC>(acc, t);
      st16t<NT>(dst + plen - 16u, bytes16_at(lo, hi, o));
    }
  }
}

// (with done_flag set -- a direct mapped batch -- it signals completion like
// the block kernel: every wave reaches ragged_signal_done)
template <bool RECOVER, bool NT, int GPW, int U = 2, int WAVES = kFlatWaves, bool BF = false>
__global__ __launch_bounds__(64 * WAVES) void ragged_multi_kernel(RaggedArgs a) {
  __shared__ uint32_t s_par[WAVES][GPW * kAccWords];
  __shared__ uint64_t s_head[WAVES][kParWin];
  __shared__ u32x4 s_meta[WAVES][64];
  const uint32_t lane = lane_id();
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t g0 = ((uint64_t)blockIdx.x * WAVES + wv) * GPW;
  if (g0 < a.n_groups) {  // wave-uniform
    const uint32_t ng = (uint32_t)min<uint64_t>((uint64_t)GPW, a.n_groups - g0);
    uint32_t pl[GPW];
    uint64_t doff[GPW];
    if (ragged_pair_xor<RECOVER, NT, GPW, U, BF>(a, g0, ng, lane, s_par[wv], s_head[wv],
                                                  s_meta[wv], pl, doff))
      ragged_pair_store<NT, GPW>(a, ng, lane, s_par[wv], pl, doff);
  }
  ragged_signal_done(a);
}


// Ragged CSR, parity-window form — the SMALL-BATCH (latency) kernel: the
// mapped host path runs a batch of <= kDirectGroups groups with it
// (qfec_capi.cpp ragged_mapped), where the payloads are read over PCIe and a
// group's time is its count of dependent round trips, not bandwidth.  (On
// large device-resident batches it is 0.77x ragged_multi_kernel: the
// texture-address unit costs ~64 cycles per 64-lane load whatever its useful
// lanes; tools/tune/tune_rw.hip)
// One wave per group, lane l owns the parity
// windows at bytes w0 = min(16l, plen-16) and w1 = min(16(l+64), plen-16) —
// the fixed-shape kernel's mapping (the last window ends exactly at plen and
// overlaps its neighbour with identical bytes), so there is no accumulator in
// LDS, no atomics and no packet search.  The group's packet table is one
// coalesced vector load (lane r = received packet r); packet r's offset and
// length are then wave-uniform (v_readlane), and every lane loads the 16 bytes
// of packet r under its window (a window crossing the packet end loads the 16
// bytes ending at the packet end and shifts them down; a window past it loads
// them too — the same lines as the lane that needs them — and XORs zero).
// Load slots: window w0 of every received packet, then window w1 of the
// packets that reach one (found by a ballot, walked with s_ff1); PB slots'
// loads are in flight before the first XOR, independent of one another, so a
// group costs three dependent round trips (group scalars -> packet table ->
// all packet bytes) instead of one per 2 KiB (ragged_multi_kernel's flat
// windows: profiles/round1/sq_stalls_fec_pq.txt, parked 68-78% of cycles).
// Groups outside the form (more than 64 received packets, a packet < 16 B,
// any invalid field) run the exact per-group body (ragged_group).
// a value every lane holds alike, moved to an SGPR
__device__ __forceinline__ uint32_t uni32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni32((uint32_t)(v >> 32)) << 32) | uni32((uint32_t)v);
}

// NP > 1: one group on NP waves (the service's one-group job).  Wave `part`
// takes every NP-th slot and leaves its partial windows in red0 / red1
// [part * 64 + lane]; the caller XORs the NP partials after a barrier and
// stores them where the returned WinOut says (red); a group out of the fast
// form is finished by part 0 alone (!red).  Only part 0 stores the encode length and
// folds in the recover parity.
struct WinOut {
  uint8_t* dst;
  uint32_t w0, w1, nwin;
  bool red;  // partials left in red0 / red1 (false: finished, or NP == 1)
};

template <bool RECOVER, bool NT, int PB, int NP = 1>
__device__ __forceinline__ WinOut window_group(const RaggedArgs& a, uint64_t g, uint32_t lane,
                                               uint32_t* s_par, uint64_t* s_head, u32x4* s_meta,
                                               uint32_t part = 0, u32x4* red0 = nullptr,
                                               u32x4* red1 = nullptr) {
  static_assert(PB % NP == 0, "slots split evenly over the waves");
  constexpr int PW = PB / NP;                     // loads per wave per chunk
  const uint32_t pt = NP == 1 ? 0u : part;        // (NP == 1: constant slot numbers)
  // trip 1: the group's scalars (s_load; the service's tables sit in LDS
  // behind generic pointers: flat loads into VGPRs, which the compiler takes
  // for per-lane values -- every slot below then became a waterfall loop
  // around its load, ~3 us of issue for one group -- so the scalars are
  // moved to SGPRs explicitly)
  const uint32_t p0 = uni32(a.grp_ptr[g]);
  const uint32_t k = uni32(a.grp_ptr[g + 1]) - p0;
  uint32_t m = 0xFFFFFFFFu, plen = 0;
  uint64_t dst_off, par_off = 0;
  if constexpr (RECOVER) {
    m = uni32(a.missing[g]);
    plen = uni32(a.parity_len[g]);
    dst_off = uni64(a.out_off[g]);
    par_off = uni64(a.parity_off[g]);
  } else {
    dst_off = uni64(a.parity_off[g]);
  }
  const uint32_t kr = RECOVER ? k - 1u : k;  // received packets
  const bool form = k >= 1u && k <= 255u && kr <= 64u &&
                    (!RECOVER || (m < k && plen >= 16u && plen <= kMaxPacket));
  // trip 2: the packet table (lane r = received packet r) and, for recover,
  // the parity windows (they need only the scalars)
  uint32_t len = 0, offlo = 0, offhi = 0;
  if (form && lane < kr) {
    const uint32_t p = p0 + lane + (RECOVER && lane >= m ? 1u : 0u);
    len = a.pkt_len[p];
    const uint64_t o = a.pkt_off[p];
    offlo = (uint32_t)o;
    offhi = (uint32_t)(o >> 32);
  }
  u32x4 acc0 = {0u, 0u, 0u, 0u}, acc1 = {0u, 0u, 0u, 0u};
  uint32_t w0 = 0, w1 = 0;
  if (RECOVER && form) {
    w0 = min(16u * lane, plen - 16u);
    w1 = min(16u * (lane + 64u), plen - 16u);
    if (pt == 0u) {
      const uint8_t* prow = a.parity + par_off;
      acc0 = ld16t<NT>(prow + w0);
      if (plen > 1024u) acc1 = ld16t<NT>(prow + w1);
    }
  }
  const uint32_t lim = RECOVER ? plen : kMaxPacket;
  if (!form || wave_any(lane < kr && (len < 16u || len > lim))) {
    if (pt == 0u) {
      GroupPrefetch f;
      group_scalars<RECOVER>(a, g, f);
      group_vectors<RECOVER, NT>(a, g, lane, f);
      ragged_group<RECOVER, NT, 2, 1>(a, g, lane, f, s_par, s_head, s_meta);
    }
    return WinOut{nullptr, 0u, 0u, 0u, false};
  }
  if constexpr (!RECOVER) {
    plen = wave_max11(len);
    if (lane == 0 && pt == 0u) a.parity_len_out[g] = (uint16_t)plen;
    w0 = min(16u * lane, plen - 16u);
    w1 = min(16u * (lane + 64u), plen - 16u);
  }
  // second windows: lanes' w1 >= min(1024, plen - 16), so exactly the packets
  // longer than that reach one
  const uint64_t longm = plen > 1024u ? __ballot(lane < kr && len > min(1024u, plen - 16u)) : 0ull;
  const uint32_t ns = kr + (uint32_t)__popcll(longm);
  // slot tables, lane t describing slots t and t + 64: slot j < kr is packet
  // j's first window, slot kr + n the second window of the n-th long packet
  // (the n-th set bit of longm, found by halving), a slot at or past ns none
  // (length 0).  A slot's load then costs three readlanes and its descriptor.
  // (One wave issues an instruction every few cycles: the per-slot search
  // for the next long packet, ~35 instructions a slot, spread a group's 20
  // loads over ~1.5 us of the service's one-group latency.)
  auto slot_packet = [&](uint32_t j) -> uint32_t {
    uint32_t n = j - kr, pos = 0u, w = (uint32_t)longm;
    const uint32_t clo = (uint32_t)__popc((uint32_t)longm);
    const bool up = n >= clo;
    n = up ? n - clo : n;
    pos = up ? 32u : 0u;
    w = up ? (uint32_t)(longm >> 32) : w;
#pragma unroll
    for (uint32_t b = 16u; b >= 1u; b >>= 1) {
      const uint32_t c = (uint32_t)__popc(w & ((1u << b) - 1u));
      const bool ge = n >= c;
      n = ge ? n - c : n;
      pos = ge ? pos + b : pos;
      w = ge ? w >> b : w;
    }
    return j < kr ? j : pos;  // (pos <= 63 for any j: a valid shuffle lane)
  };
  const uint32_t rA = slot_packet(lane), rB = slot_packet(lane + 64u);
  // (every shuffle with the whole wave active: a lane that reads an inactive
  // lane's value gets 0, so none sits under the `< ns` condition)
  const uint32_t shA = lane_read(len, rA);
  const uint32_t shB = lane_read(len, rB);
  const uint32_t lenA = lane < ns ? shA : 0u;
  const uint32_t lenB = lane + 64u < ns ? shB : 0u;
  const uint32_t olA = lane_read(offlo, rA);
  const uint32_t ohA = lane_read(offhi, rA);
  const uint32_t olB = lane_read(offlo, rB);
  const uint32_t ohB = lane_read(offhi, rB);
  // trip 3: every slot's bytes, PB loads in flight per lane.  Branch-free: a
  // slot past the end loads through a descriptor of 0 bytes (its length: the
  // bounds check returns zeros, no memory access; a real slot's load ends
  // inside its packet), so no load sits in a branch and the wait counts stay
  // exact (branches made the compiler drain vmcnt before every load).  A
  // chunk of PB slots reads ONE table (slots base .. base + 63; slots at or
  // past lim none), this wave's PW of them (slot s + pt + NP u).  The first
  // PB slots (every group of up to 12 full-size packets) with the loads
  // issued before any use.
  auto chunk = [&](uint32_t s, uint32_t base, uint32_t lim, uint32_t lenT, uint32_t olT, uint32_t ohT,
                   auto first) __attribute__((always_inline)) {
    u32x4 v[PW];
    uint32_t li[PW];
#pragma unroll
    for (int u = 0; u < PW; ++u) {
      const uint32_t j = s + pt + (uint32_t)(NP * u);
      const int t = (int)min(j - base, 63u);  // (slots past the table: li = 0)
      li[u] = (uint32_t)__builtin_amdgcn_readlane((int)lenT, t);
      // (the first chunk's slots are below 64, where the table is 0 past ns)
      if constexpr (!decltype(first)::value) li[u] = j < lim ? li[u] : 0u;
      const uint64_t o = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)ohT, t) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)olT, t);
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(a.bytes + o), 0, (int)li[u], 0x00020000);
      const uint32_t w = j >= kr ? w1 : w0;
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)min(w, li[u] - 16u), 0, NT ? 2 : 0);
      // the first chunk in source order: each slot's descriptor right before
      // its load (hoisting them all holds 4 SGPRs a slot: spills) and every
      // load before any use (the scheduler otherwise interleaves the uses and
      // waits on the first loads before issuing the last)
      if constexpr (decltype(first)::value) __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int u = 0; u < PW; ++u) {
      const bool second = s + pt + (uint32_t)(NP * u) >= kr;
      const uint32_t w = second ? w1 : w0;
      const uint32_t keep = w < li[u] ? 0xFFFFFFFFu : 0u;
      const uint32_t sh = w + 16u > li[u] ? min(w + 16u - li[u], 15u) : 0u;
      const u32x4 x = shr_bytes_bf(v[u], sh) & keep;
      const u32x4 zero = {0u, 0u, 0u, 0u};
      acc0 ^= second ? zero : x;
      acc1 ^= second ? x : zero;
    }
  };
  const uint32_t limA = min(ns, 64u);
  chunk(0u, 0u, limA, lenA, olA, ohA, std::true_type{});
  for (uint32_t s = PB; s < limA; s += PB) chunk(s, 0u, limA, lenA, olA, ohA, std::false_type{});
  for (uint32_t s = 64u; s < ns; s += PB) chunk(s, 64u, ns, lenB, olB, ohB, std::false_type{});
  uint8_t* dst = a.out + dst_off;
  const uint32_t nwin = (plen + 15u) >> 4;
  if constexpr (NP > 1) {
    red0[pt * 64u + lane] = acc0;
    red1[pt * 64u + lane] = acc1;
    return WinOut{dst, w0, w1, nwin, true};
  }
  if (lane < nwin) st16t<NT>(dst + w0, acc0);
  if (lane + 64u < nwin) st16t<NT>(dst + w1, acc1);
  return WinOut{nullptr, 0u, 0u, 0u, false};
}

// (one workgroup per 4 groups of a small batch: occupancy is no object; the
// default 4-waves-per-SIMD target left the recover body 128 VGPRs and spilled)
template <bool RECOVER, bool NT, int PB>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 2))) void ragged_window_kernel(
    RaggedArgs a) {
  __shared__ uint32_t s_par[kFlatWaves][4 * kParWin];
  __shared__ uint64_t s_head[kFlatWaves][kParWin];
  __shared__ u32x4 s_meta[kFlatWaves][64];
  const uint32_t lane = lane_id();
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t g = (uint64_t)blockIdx.x * kFlatWaves + wv;
  if (g < a.n_groups) window_group<RECOVER, NT, PB>(a, g, lane, s_par[wv], s_head[wv], s_meta[wv]);
  ragged_signal_done(a);
}

// The small-batch service worker (qfec_internal.h SvcJob / SvcShared /
// SvcDev): kSvcWgs workgroups of kSvcWaves waves, resident while batches keep
// coming.  The leader's thread 0 polls the host-mapped pub_end and hands the
// turn's end to the followers through device memory; for every published job
// each workgroup copies the job's ring entry -- its header AND its index
// tables, which the host writes inline -- into LDS in one PCIe round trip,
// and each group is then taken by one wave (window_group, as the small-batch
// kernel) with its tables read from LDS: a group costs one dependent PCIe
// round trip (its payload bytes) instead of three (group scalars -> packet
// table -> bytes, round 4).  A job of at most kSvcWaves groups is the
// leader's alone; a larger one is spread over all kSvcWgs x kSvcWaves waves
// (one round of groups for up to 64), each workgroup making its outputs
// visible system-wide before it adds itself to the entry's done counter, and
// the last one stores the token.  Host memory is read after a system-scope
// acquire following each poll (a resident kernel gets no cache invalidation
// from a dispatch).  Exit: idle_ticks without work, or quit (the leader
// decides; the followers leave on its word).  All control stores are vector
// stores.
constexpr int kSvcWaves = 8;
// the leader's poll reads the next job's head with pub_end for this long after
// its last job (100-MHz ticks: 50 us, half the idle time), then pub_end alone
// 
constexpr uint64_t kSvcQuietTicks = 5000;
// Load slots per trip of a group's bytes.  A one-group job (all eight waves,
// three slots each): 24 = every window of a group of up to 12 packets longer
// than 1024 B in ONE PCIe round trip.  A job of several groups (a wave per
// group): 20 = the 10 x 1350 B group (kDefaultMaxPacketsPerFecGroup) in one
// trip (16 made it two; 24 beside the one-group form spilled at 2 waves/SIMD)
constexpr int kSvcPB = 24;
constexpr int kSvcPBw = 20;

__device__ __forceinline__ uint64_t svc_load64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t svc_load32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The ring entry's first `bytes` bytes (a multiple of 16) into LDS, every
// thread 16 B per pass (the tables follow the header: one round trip).
__device__ __forceinline__ void svc_copy_entry(const SvcJob* e, uint8_t* dst, uint32_t from,
                                               uint32_t bytes, uint32_t tid) {
  const uint8_t* src = reinterpret_cast<const uint8_t*>(e);
  for (uint32_t o = from + 16u * tid; o < bytes; o += 16u * 64u * kSvcWaves)
    *reinterpret_cast<u32x4*>(dst + o) = ld16(src + o);
}

__global__ __launch_bounds__(64 * kSvcWaves) void ragged_service_kernel(
    SvcShared* sh, SvcDev* dv, const SvcJob* ring, uint32_t* flags, uint64_t idle_ticks,
    uint32_t epoch) {
  __shared__ uint32_t s_par[kSvcWaves][4 * kParWin];
  __shared__ uint64_t s_head[kSvcWaves][kParWin];
  __shared__ u32x4 s_meta[kSvcWaves][64];
  __shared__ u32x4 s_red[2][kSvcWaves * 64];  // a one-group job's partial windows
  __shared__ __attribute__((aligned(16))) uint8_t s_ent[sizeof(SvcJob)];
  __shared__ uint64_t s_from, s_to;
  // the leader: split jobs it has announced; a follower: the next announcement it takes
  __shared__ uint64_t s_split;
  __shared__ uint32_t s_job, s_exit, s_stamp;
  // the job whose entry size is known (s_need bytes; the leader: s_have of
  // them already in LDS from its poll), else no job
  __shared__ uint32_t s_entjob, s_have, s_need;
  static_assert(sizeof(SvcJob) % 16u == 0u, "entry copied in 16-B pieces");
  static_assert(kSvcRing > 3u, "announcement ring: more entries than outstanding jobs");
  constexpr uint32_t kHead = (uint32_t)offsetof(SvcJob, tab);
  constexpr uint32_t kFirst = 4096u;  // first pass: the header and the first tables
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t wg = blockIdx.x;
  const bool lead = wg == 0u;
  const SvcJob& J = *reinterpret_cast<const SvcJob*>(s_ent);
  __shared__ uint64_t st[6];  // measurement hook (sh->stamp_on): the leader's stamps of a job (thread 0; LDS, not 12 VGPRs live through the job)

  // This workgroup's share of job jj, whose entry is in LDS: a split job's
  // group g on wave g / kSvcWgs of workgroup g % kSvcWgs (a 9..64-group job is
  // one round, spread over the workgroups), a smaller one the leader's alone.
  // Then its outputs visible, its count (split) and the token from the last.
  auto run_job = [&](uint32_t jj, bool split) __attribute__((always_inline)) {
    if (tid == 0) st[1] = wall_clock64();
    // the job's tables live in LDS (generic pointers: flat loads)
    RaggedArgs a = J.a;
    a.pkt_off = reinterpret_cast<const uint64_t*>(J.tab + J.t_off);
    a.pkt_len = reinterpret_cast<const uint16_t*>(J.tab + J.t_len);
    a.grp_ptr = reinterpret_cast<const uint32_t*>(J.tab + J.t_ptr);
    a.parity_off = reinterpret_cast<const uint64_t*>(J.tab + J.t_poff);
    if (J.recover) {
      a.parity_len = reinterpret_cast<const uint16_t*>(J.tab + J.t_plen);
      a.missing = J.tab + J.t_miss;
      a.out_off = reinterpret_cast<const uint64_t*>(J.tab + J.t_ooff);
    }
    const uint64_t n = J.a.n_groups;
    const uint64_t step = split ? (uint64_t)kSvcWaves * kSvcWgs : (uint64_t)kSvcWaves;
    if (n <= 2u) {
      // one or two groups: each on 8 / n waves of the leader -- its slots
      // dealt round its waves (a
      // wave issues an instruction every few cycles: one group alone on one
      // wave took ~7.5 us from its entry to its stores, on all 8 waves 3.9,
      // profiles/round6/svc_trace_n_r6t.txt), each group's partial windows
      // XORed out of LDS by two of its waves
      const uint32_t NPn = n == 1u ? (uint32_t)kSvcWaves : 4u;
      const uint32_t q = wv / NPn, part = wv - q * NPn;
      u32x4* const r0 = s_red[0] + q * NPn * 64u;
      u32x4* const r1 = s_red[1] + q * NPn * 64u;
      WinOut o{nullptr, 0u, 0u, 0u, false};
      if (q < n) {
        if (n == 1u)
          o = J.recover ? window_group<true, true, kSvcPB, kSvcWaves>(
                              a, 0, lane, s_par[wv], s_head[wv], s_meta[wv], part, r0, r1)
                        : window_group<false, true, kSvcPB, kSvcWaves>(
                              a, 0, lane, s_par[wv], s_head[wv], s_meta[wv], part, r0, r1);
        else
          o = J.recover ? window_group<true, true, kSvcPB, 4>(
                              a, q, lane, s_par[wv], s_head[wv], s_meta[wv], part, r0, r1)
                        : window_group<false, true, kSvcPB, 4>(
                              a, q, lane, s_par[wv], s_head[wv], s_meta[wv], part, r0, r1);
      }
      __syncthreads();
      if (q < n && o.red && part < 2u) {
        const u32x4* r = part == 0u ? r0 : r1;
        u32x4 x = r[lane];
        for (uint32_t p = 1; p < NPn; ++p) x ^= r[p * 64u + lane];
        if (lane + 64u * part < o.nwin) st16t<true>(o.dst + (part == 0u ? o.w0 : o.w1), x);
      }
      if (tid == 0) st[2] = wall_clock64();
    } else {
      for (uint64_t g = split ? (uint64_t)wv * kSvcWgs + wg : wv; g < n; g += step) {
        if (J.recover)
          window_group<true, true, kSvcPBw>(a, g, lane, s_par[wv], s_head[wv], s_meta[wv]);
        else
          window_group<false, true, kSvcPBw>(a, g, lane, s_par[wv], s_head[wv], s_meta[wv]);
        if (tid == 0 && g == 0) st[2] = wall_clock64();
      }
    }
    // every wave's output stores acknowledged, then ONE system-scope
    // release (thread 0's: its L2 write-back covers the workgroup) before
    // the count / token -- not one per thread
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      st[3] = wall_clock64();
      __threadfence_system();  // this workgroup's outputs visible before its count
      st[4] = wall_clock64();
      bool last = true;
      if (split) {
        // every workgroup takes every split job (announced to the followers,
        // below), so the count reaches kSvcWgs exactly once per job; the
        // last resets it for the entry's next split job (which the host
        // publishes only after this job's token, stored after the reset)
        last = __hip_atomic_fetch_add(&dv->done[jj % kSvcRing], 1u, __ATOMIC_ACQ_REL,
                                      __HIP_MEMORY_SCOPE_SYSTEM) +
                   1u ==
               kSvcWgs;
        if (last)
          __hip_atomic_store(&dv->done[jj % kSvcRing], 0u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      if (last)
        __hip_atomic_store(flags + J.flag_slot, J.token, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      if (s_stamp) {
        st[5] = wall_clock64();
        if (lead)
          for (int q = 0; q < 6; ++q)
            __hip_atomic_store(&sh->stamps[q], st[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t row[4] = {st[1], st[3], st[4], st[5]};
        for (int q = 0; q < 4; ++q)
          __hip_atomic_store(&sh->wg_stamps[wg][q], row[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (last) {
          __hip_atomic_store(&sh->stamps[6], st[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(&sh->stamps[7], (uint64_t)wg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  };

  // One loop for both roles and one run_job site, round 5's loop nest (a
  // second site, or one job per turn of the outer loop, spilled 72-168 B of
  // scratch at 256 VGPRs): each turn the leader polls and walks the jobs
  // published so far; a follower takes one announcement of a split job.
  // (round 5's followers walked the ring themselves from the
  // host's `consumed`, read at their own start; a follower dispatched late
  // -- the CUs held by another kernel -- started past a split job the leader
  // had already counted and never did its share, so that job's token never
  // came.  Now a follower starts at its own count of announcements taken,
  // kept in device memory across launches, and reads only the entries of
  // split jobs, whose tokens wait for it.)
  if (tid == 0) {
    if (lead) {
      // where the previous worker stopped (stable: it has left): jobs are
      // finished whole and in order, so the next job's number is the count
      s_from = svc_load64(&sh->consumed);
      s_to = s_from;
      s_job = (uint32_t)svc_load64(&sh->jobs);
      s_stamp = svc_load32(&sh->stamp_on);
      s_split = __hip_atomic_load(&dv->nsplit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // running: a worker queued behind one that cleared `alive` on its way
      // out says so itself (the host then stops it before a phased
      // launch)
      __hip_atomic_store(&sh->alive, 1u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      // test hook: a follower dispatched late (the hold released)
      while (svc_load32(&sh->hold) != 0u) __builtin_amdgcn_s_sleep(8);
      s_split = __hip_atomic_load(&dv->taken[wg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_stamp = svc_load32(&sh->stamp_on);  // (its own row of wg_stamps)
    }
  }
  __syncthreads();
  // the leader announces split job jj (entry bytes `need`) to the followers (thread 0)
  auto announce = [&](uint32_t jj, uint32_t need) {
    const uint64_t i = s_split;
    __hip_atomic_store(&dv->split[i % kSvcRing], ((uint64_t)jj << 32) | (need >> 4),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&dv->nsplit, i + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    s_split = i + 1u;
  };
  bool miss = false;
  for (;;) {
    // tid and lane redefined (opaquely) every turn of the worker's loop:
    // nothing derived from them is hoisted out of it -- shuffle addresses,
    // head-hash multipliers, slot masks were, live through the whole job
    // body, and spilled to scratch at 256 VGPRs
    if (lead) {
      if (wv == 0u) {
        // Wave 0 polls.  Every look
        // reads pub_end AND the next job's first kSvcHead bytes (16 per lane,
        // relaxed system-scope loads, all in flight together: one PCIe round
        // trip); when the look that sees the job holds it whole -- its head
        // hash, seq and start agree -- the entry copy below is skipped (round
        // 5: one round trip less per job).
        const uint64_t from = s_from;
        const uint32_t job0 = s_job;
        const uint32_t lane2 = 2u * lane;
        const uint64_t* hp = reinterpret_cast<const uint64_t*>(ring + (job0 % kSvcRing)) + lane2;
        uint64_t h0 = 0, h1 = 0;
        uint32_t rot = 0;  // the rotate word, read with every look (same round trip)
        uint32_t wm = 0;   // the host's warm count, likewise
        auto look = [&]() -> uint64_t {
          const uint64_t t = __hip_atomic_load(&sh->pub_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          rot = __hip_atomic_load(&sh->rotate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          wm = __hip_atomic_load(&sh->warm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          h0 = __hip_atomic_load(hp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          h1 = __hip_atomic_load(hp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return t;
        };
        // rotated out (wrap-safe epoch compare): leave between turns, the
        // published jobs to the successor queued behind (it starts at consumed)
        auto rotated = [&]() { return (int32_t)(rot - epoch) >= 0; };
        uint64_t to = look();
        uint32_t ex = 0;
        uint64_t t0 = wall_clock64();
        uint32_t warm_seen = wm;
        while (to == from) {
          if (svc_load32(&sh->quit) != 0u) {
            ex = 1;
            break;
          }
          if (wall_clock64() - t0 > idle_ticks) {
            // leaving: say so, then look once more (the host publishes, then
            // reads alive: one of the two sees the other's store)
            __hip_atomic_store(&sh->alive, 0u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            to = look();
            if (to == from) {
              ex = 1;
              break;
            }
            __hip_atomic_store(&sh->alive, 1u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
          if (wall_clock64() - t0 > kSvcQuietTicks) {
            // a quiet stretch: pub_end alone, less often (one 8-B
            // read instead of 1 KiB over the link every look); a job seen
            // this way costs one more round trip for its head
            __builtin_amdgcn_s_sleep(16);
            to = __hip_atomic_load(&sh->pub_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            wm = __hip_atomic_load(&sh->warm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (to != from) to = look();
          } else {
            __builtin_amdgcn_s_sleep(2);
            to = look();
          }
          // a warm call (a batch is coming this loop turn): the idle time
          // restarts, so a turn whose batch takes most of it to assemble
          // still finds the worker resident (round 6)
          if (wm != warm_seen) {
            warm_seen = wm;
            t0 = wall_clock64();
          }
        }
        if (!ex && rotated()) ex = 1;
        // the head found whole (its hash, seq and start agree): the entry's
        // size is known -- a small job is all in LDS already, a larger one's
        // header is, and the rest is copied in one pass
        uint32_t have = 0, need = 0;
        if (!ex) {
          uint64_t* sw = reinterpret_cast<uint64_t*>(s_ent);
          sw[lane2] = h0;
          sw[lane2 + 1u] = h1;
          wave_lds_order();
          const uint32_t tbb = J.tab_bytes;
          const uint32_t full = min((kHead + min(tbb, kSvcTab) + 15u) & ~15u, (uint32_t)sizeof(SvcJob));
          const uint32_t nb = min(full, kSvcHead);
          uint64_t part = 0;
          if (lane2 < nb / 8u && lane2 != kSvcHeadSumWord) part += svc_head_word(h0, lane2);
          if (lane2 + 1u < nb / 8u && lane2 + 1u != kSvcHeadSumWord)
            part += svc_head_word(h1, lane2 + 1u);
#pragma unroll
          for (uint32_t d = 32; d > 0; d >>= 1)
            part += ((uint64_t)lane_read((uint32_t)(part >> 32), lane ^ d) << 32) |
                    lane_read((uint32_t)part, lane ^ d);
          const bool whole = (part | 1ull) == J.head_sum && J.seq == job0 && J.start == from &&
                             tbb <= kSvcTab;
          have = whole ? nb : 0u;
          need = whole ? full : 0u;
        }
        if (lane == 0u) {
          st[0] = wall_clock64();
          s_to = to;
          s_exit = ex;
          s_entjob = need != 0u ? job0 : 0xFFFFFFFFu;
          s_have = have;
          s_need = need;
        }
      }
    } else if (tid == 0) {
      // follower: the next announcement, or the leader's exit
      const uint64_t mine = s_split;
      uint64_t ann = 0;
      uint32_t ex = 0;
      for (;;) {
        // the exit word first: the leader stores it after its last
        // announcement, so an exit seen here means nsplit is final
        const uint32_t e = __hip_atomic_load(&dv->exit, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_load(&dv->nsplit, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) > mine) {
          ann = __hip_atomic_load(&dv->split[mine % kSvcRing], __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        if (e == epoch) {
          ex = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s_exit = ex;
      s_entjob = (uint32_t)(ann >> 32);
      s_have = 0u;
      s_need = (uint32_t)(ann & 0xFFFFu) << 4;
    }
    __syncthreads();
    if (s_exit) break;
    // every thread: drop cached copies of host memory (ring entries, payloads)
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    // the leader: the published jobs, in order (pub_end moves by whole
    // jobs); a follower: the one announced
    const uint64_t to = s_to;
    uint64_t gi = s_from;
    uint32_t jj = lead ? s_job : s_entjob;
    bool once = true;
    while (lead ? gi < to : once) {
      once = false;
      const SvcJob* e = ring + (jj % kSvcRing);
      // a job of known size in one pass (the leader's poll holds its header
      // and maybe all of it), else the header and first tables, then the rest
      const uint32_t have = jj == s_entjob ? s_have : 0u;
      const uint32_t need = jj == s_entjob ? s_need : 0u;
      // a split job whose header the poll holds: announced before the copy,
      // so the followers' entry copies overlap the leader's
      if (lead && need != 0u && tid == 0 && J.a.n_groups > (uint64_t)kSvcWaves) announce(jj, need);
      if (need == 0u)
        svc_copy_entry(e, s_ent, 0u, min(kFirst, (uint32_t)sizeof(SvcJob)), tid);
      else if (have < need)
        svc_copy_entry(e, s_ent, have, min(need, (uint32_t)sizeof(SvcJob)), tid);
      __syncthreads();
      if (lead && (J.seq != jj || gi != J.start || J.tab_bytes > kSvcTab)) {
        // a malformed ring: nothing of this turn is done
        // (and no announcement of it)
        miss = true;
        break;
      }
      const uint64_t n = J.a.n_groups;
      const bool split = n > (uint64_t)kSvcWaves;
      if (lead && need == 0u) {
        const uint32_t full = (kHead + J.tab_bytes + 15u) & ~15u;
        if (split && tid == 0) announce(jj, full);
        if (full > kFirst) {  // a large job's tables: a second pass
          svc_copy_entry(e, s_ent, kFirst, full, tid);
          __syncthreads();
        }
      }
      // (a follower's entry cannot be wrong while the host keeps its ring:
      // the entry of a split job is reused only after its token, which waits
      // for this workgroup)
      const bool ok = lead || (J.seq == jj && split && J.tab_bytes <= kSvcTab &&
                               kHead + J.tab_bytes <= need);
      if (ok) run_job(jj, split);
      // no share, so no token: the host's wait sees the fault once the
      // worker has left, and fails the job instead of reporting stale output
      if (!ok && tid == 0) __hip_atomic_store(&sh->fault, 1u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
      gi = J.start + n;
      ++jj;
      __syncthreads();  // s_ent is the next job's
    }
    if (miss) break;
    if (tid == 0) {
      if (lead) {
        s_job = jj;
        s_from = to;
        __hip_atomic_store(&sh->consumed, to, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&sh->jobs, (uint64_t)jj, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        s_split = s_split + 1u;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    if (lead) {
      // latch a malformed ring's fault and leave WITHOUT the job's token --
      // the host's wait sees the stream drained and the fault word and fails
      // the job instead of reporting stale output as finished
      if (miss) __hip_atomic_store(&sh->fault, 1u, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
      // the followers leave once they have taken every announcement (this
      // store is after the last one: release)
      __hip_atomic_store(&dv->exit, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(&dv->taken[wg], s_split, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // (no store to `alive` here: an idle exit cleared it before its last look,
  // and a late store could clobber the 1 the host wrote for a worker it has
  // already queued behind this one; stop_service clears it after a quit)
}

// ---------------------------------------------------------------------------
// out ^= in (XorBuffers).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void xor_into_kernel(const uint8_t* in, uint64_t n,
                                                          uint8_t* out) {
  const uint64_t nwin = n / 16u;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < nwin; w += stride) {
    st16(out + 16u * w, ld16(out + 16u * w) ^ ld16(in + 16u * w));
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 15u)) {
    const uint64_t j = 16u * nwin + threadIdx.x;
    out[j] ^= in[j];
  }
}

// ---------------------------------------------------------------------------
// Bandwidth probes (bench.py's measured ceilings): streaming
// read (nt 16-B loads, 8 in flight per lane, XOR-folded) and copy (nt load +
// nt store), grid-stride over n bytes (n a multiple of 16).
// ---------------------------------------------------------------------------
template <bool COPY>
__global__ __launch_bounds__(kBlock) void stream_probe_kernel(const uint8_t* src, uint64_t n,
                                                              uint8_t* dst) {
  constexpr uint32_t U = 8;
  const uint64_t nwin = n / 16u;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  u32x4 acc = {0u, 0u, 0u, 0u};
  uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  for (; w + (U - 1) * stride < nwin; w += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) v[u] = ld16t<true>(src + 16u * (w + u * stride));
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      if constexpr (COPY) st16t<true>(dst + 16u * (w + u * stride), v[u]);
      else acc ^= v[u];
    }
  }
  for (; w < nwin; w += stride) {
    const u32x4 v = ld16t<true>(src + 16u * w);
    if constexpr (COPY) st16t<true>(dst + 16u * w, v);
    else acc ^= v;
  }
  if constexpr (!COPY) {
    if ((acc.x & acc.y & acc.z & acc.w) == 0xFFFFFFFFu) st16(dst, acc);  // keeps the loads
  }
}

// ---------------------------------------------------------------------------
// Synthetic inputs (counter-based splitmix64).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ void synth_word(uint8_t* row, uint64_t key, uint32_t w, uint32_t len) {
  const uint64_t v = splitmix64(key ^ (uint64_t)w);
  const uint32_t j = w * 8u;
  if (j + 8u <= len) {
    __builtin_memcpy(row + j, &v, 8);
  } else {
    for (uint32_t b = 0; j + b < len; ++b) row[j + b] = (uint8_t)(v >> (8u * b));
  }
}

// One workgroup per row (blockIdx.x = row within the launch), lanes = words.
__global__ __launch_bounds__(kBlock) void synth_fixed_kernel(uint8_t* rows, uint32_t k,
                                                             uint32_t L, uint64_t row_stride,
                                                             uint64_t group_stride, uint64_t g0,
                                                             uint64_t row0, uint64_t seed) {
  const uint64_t r = row0 + blockIdx.x;
  const uint64_t g = r / k;
  const uint32_t i = (uint32_t)(r - g * k);
  const uint64_t key = seed ^ (((g0 + g) * 256u + i) << 32);
  uint8_t* row = rows + g * group_stride + i * row_stride;
  const uint32_t words = (L + 7u) / 8u;
  for (uint32_t w = threadIdx.x; w < words; w += kBlock) synth_word(row, key, w, L);
}

// One workgroup per group.
__global__ __launch_bounds__(kBlock) void synth_ragged_kernel(uint8_t* bytes,
                                                              const uint64_t* pkt_off,
                                                              const uint16_t* pkt_len,
                                                              const uint32_t* grp_ptr,
                                                              uint64_t g0, uint64_t gbase,
                                                              uint64_t seed) {
  const uint64_t g = gbase + blockIdx.x;
  const uint32_t p0 = grp_ptr[g], p1 = grp_ptr[g + 1];
  for (uint32_t i = 0; i < p1 - p0; ++i) {
    const uint32_t len = pkt_len[p0 + i];
    const uint64_t key = seed ^ (((g0 + g) * 256u + i) << 32);
    uint8_t* row = bytes + pkt_off[p0 + i];
    const uint32_t words = (len + 7u) / 8u;
    for (uint32_t w = threadIdx.x; w < words; w += kBlock) synth_word(row, key, w, len);
  }
}

// Every group size up to 16 is templated (round 5; round 4 had 2, 4, 5, 8,
// 10, 16 and ran the others through the runtime-k bodies).
#define QFEC_K_ALL(X) \
  X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)

template <bool RECOVER, bool NT, bool SM, bool INPL = false>
hipError_t launch_fixed_k(const FixedArgs& a, uint32_t C, uint32_t gpb, uint64_t blocks,
                          hipStream_t s) {
  switch (a.k) {
#define QFEC_K_CASE(KV)                                                                       \
  case KV:                                                                                     \
    hipLaunchKernelGGL((fixed_xor_kernel<KV, RECOVER, NT, SM, false, INPL>),                   \
                       dim3((uint32_t)blocks), dim3(kBlock), 0, s, a, C, gpb);                 \
    break;
    QFEC_K_ALL(QFEC_K_CASE)
#undef QFEC_K_CASE
    default:
      hipLaunchKernelGGL((fixed_xor_kernel<0, RECOVER, NT, SM, false, INPL>),
                         dim3((uint32_t)blocks), dim3(kBlock), 0, s, a, C, gpb);
  }
  return hipGetLastError();
}

// Register-held steps per phase for a templated group size (0: none): every
// templated k takes kPhRegSteps (round 4; round 3 had
// them for k = 10 only; round 5 templates every k up to 16).  Larger k run
// the runtime-k body with the LDS steps alone.
// Round 6: the phased RECOVER of group sizes 17-25 is templated too (its
// register steps, parity rows first and compact received rows, as k <= 16):
// recover 0.709 / 0.731 / 0.759 (runtime body) -> 0.779 / 0.785 / 0.797 at
// k = 17 / 20 / 24, where the templated encode is no faster than the runtime
// body's batches of 16 (k = 20: 0.804 vs 0.809); from k = 26 the templated
// recover spills (528 B of scratch) and loses (0.70-0.71 against the
// runtime body's 0.76-0.77) (profiles/round6/phase_k_table_r6{i,j}.txt).  So
// encode, the in-place form, recover above 25 and the one-pass kernel keep
// the runtime body above 16.
#define QFEC_K_PHASE_RECOVER(X) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25)
__host__ __device__ constexpr bool phase_k_templated(bool recover, uint32_t k) {
  return (k >= 2u && k <= 16u) || (recover && k >= 17u && k <= 25u);
}
__host__ __device__ constexpr uint32_t phase_reg_steps(bool recover, uint32_t k) {
  return phase_k_templated(recover, k) ? (uint32_t)kPhRegSteps : 0u;
}

// The runtime-k phased body's load batch (k > 16) by operation and group
// size, from the round-6 per-k table (tools/phase_k_table.py, 2^20 groups up
// to k = 32, 2^18 above; batch 16 / 32, fraction of 8 TB/s,
// profiles/round6/phase_k_table_r6b.txt, r6c.txt): encode 16 at every k
// (k = 20: 0.796 / 0.764, k = 255: 0.804 / 0.780); recover 32 up to k = 32
// (k = 20: 0.679 / 0.720), 16 above (k = 64: 0.765 / 0.725).
__host__ __device__ constexpr uint32_t phase_rt_batch(bool recover, uint32_t k) {
  return recover && k <= 32u ? 32u : 16u;
}

template <bool RECOVER, bool INPL = false>
hipError_t launch_phase_k(const FixedArgs& a, uint32_t C, uint32_t gpb, uint32_t grid,
                          uint32_t nphase, hipStream_t s) {
  const bool rs = a.no_regsteps == 0u;
  // (test hook rt_batch: the runtime-k body even where k is templated)
  switch (a.rt_batch != 0u && a.k > 16u ? 0u : a.k) {
    // templated k: kPhRegSteps more steps per phase held in registers after
    // the LDS steps (recover: their parity rows first, RPF), or without them
    // (test hook; not for the in-place form)
#define QFEC_K_CASE(KV)                                                                        \
  case KV:                                                                                      \
    if (rs || INPL)                                                                             \
      hipLaunchKernelGGL((phase_xor_kernel<KV, RECOVER, false, false, kPhUDefault, kPhSteps,    \
                                           kBlock, false, true, true, false, true, kPhRegSteps, \
                                           true, false, INPL>),                                 \
                         dim3(grid), dim3(kBlock), 0, s, a, C, gpb, nphase);                    \
    else                                                                                        \
      hipLaunchKernelGGL((phase_xor_kernel<KV, RECOVER>), dim3(grid), dim3(kBlock), 0, s, a, C, \
                         gpb, nphase);                                                          \
    break;
    QFEC_K_ALL(QFEC_K_CASE)
    default:
      if constexpr (RECOVER) {
        switch (a.rt_batch != 0u ? 0u : a.k) {
          QFEC_K_PHASE_RECOVER(QFEC_K_CASE)
          default:
            break;
        }
        if (a.rt_batch == 0u && phase_k_templated(true, a.k)) break;
      }
      // runtime k: batches of up to 16 or 32 loads, by the measured table
      // (phase_rt_batch; test hook rt_batch: either, the A/B of
      // tools/phase_k_table.py)
      if ((a.rt_batch ? a.rt_batch : phase_rt_batch(RECOVER, a.k)) == 16u)
        hipLaunchKernelGGL((phase_xor_kernel<0, RECOVER, false, false, kPhUDefault, kPhSteps, kBlock,
                                             false, true, true, false, true, 0, false, false, INPL,
                                             16>),
                           dim3(grid), dim3(kBlock), 0, s, a, C, gpb, nphase);
      else
        hipLaunchKernelGGL((phase_xor_kernel<0, RECOVER, false, false, kPhUDefault, kPhSteps, kBlock,
                                             false, true, true, false, true, 0, false, false, INPL,
                                             32>),
                           dim3(grid), dim3(kBlock), 0, s, a, C, gpb, nphase);
  }
#undef QFEC_K_CASE
  return hipGetLastError();
}

// The phased kernel for a batch of at least kPhMinPhases phases (about 184K
// groups at L = 1350 on 256 CUs): the two meetings per phase cost ~2-3 us
// each, and below that the one-pass kernel's placement luck matters less
// than they do.  Measured crossover (tools/phase_band.py,
// profiles/round3/phase/phase_band_r3d.txt): one-pass 0.77 vs phased 0.73 of
// 8 TB/s at 131K groups, 0.75 vs 0.76 at 196K, 0.74 vs 0.78 at 262K.
// Returns false when it does not apply.
constexpr uint32_t kPhMinPhases = 6;

// The CU count comes cached from the context (FixedArgs::ncu); the test hook
// phase_extra (tests/test_hip_phase.py) adds workgroups beyond one per CU,
// which cannot all be resident, so the first meeting times out — the abandon
// path.
// Group sizes the phased kernel loses at (round 4, tools/phase_k_table.py,
// profiles/round4/phase_k_table_r4a.txt, 2^20 groups of 1350 B, fraction of
// 8 TB/s phased / one-pass): encode k = 2 0.47 / 0.77, k = 4 0.64 / 0.74,
// k = 5 0.73 / 0.71, k = 8 0.79 / 0.72; recover k = 4 0.54 / 0.72, k = 5
// 0.62 / 0.67, k = 8 0.745 / 0.740, k = 10 0.76 / 0.72 -- a phase of few
// rows per group reads too little between its meetings.  So encode phases
// from k = 5, recover from k = 8.  Round 4 phased only the templated k: the
// runtime-k phased body then loaded the rows past the last batch of 8 one at
// a time (profiles/round4/phase_k_table_nontemplated_r4o.txt: k = 6 0.27 vs
// 0.69 one-pass); round 5 templates every k up to 16 and gives the runtime
// body (k > 16) batches of 16 with a one-batch remainder (xor_rows_rt), so
// the rule is by k alone again (tools/phase_k_table.py); its
// round-5 table moved recover's threshold to k = 7 (phased 0.719 vs one-pass
// 0.697; k = 6 0.684 vs 0.720: profiles/round5/phase_k_table_r5b.txt).  An
// explicit phase_min (test hook) keeps the phase-count rule alone.
constexpr uint32_t kPhMinKEncode = 5, kPhMinKRecover = 7;

bool phase_plan(const FixedArgs& a, uint32_t gpb, uint32_t* grid, uint32_t* nphase) {
  if (a.ncu == 0) return false;
  if (a.phase_min == 0 &&
      a.k < (a.parity != nullptr ? kPhMinKRecover : kPhMinKEncode))
    return false;
  // resident service workers of other contexts hold svc_cus CUs' LDS: the
  // grid leaves them, so every workgroup is resident and the meetings hold
  // (round 6); more than a quarter of the device so held: one-pass
  if (a.svc_cus > a.ncu / 4u) return false;
  // (the test hook phase_extra: that many workgroups beyond one per CU, the
  // other contexts' workers ignored)
  const uint32_t wg =
      a.phase_extra ? a.ncu + std::min<uint32_t>(a.phase_extra, 64u) : a.ncu - a.svc_cus;
  // the threshold counts phases of the LDS steps alone (the measured band);
  // the launch's phases hold the register steps too (k = 10)
  const uint64_t per = (uint64_t)wg * kPhSteps * gpb;
  const uint64_t np = (a.n_groups + per - 1) / per;
  if (np < (a.phase_min ? a.phase_min : kPhMinPhases) || np > 0xFFFFFFFFull) return false;
  const uint64_t per_l =
      (uint64_t)wg *
      (kPhSteps + ((a.no_regsteps && !a.inplace_missing) || (a.rt_batch != 0u && a.k > 16u)
                       ? 0u
                       : phase_reg_steps(a.parity != nullptr && !a.inplace_missing, a.k))) *
      gpb;
  *grid = wg;
  *nphase = (uint32_t)((a.n_groups + per_l - 1) / per_l);
  return true;
}

// Steps per phase that spread n_groups evenly over nphase phases (a 393K-group
// batch: 8 phases of 64 steps instead of 7 of 72 and one of 7).
uint32_t phase_steps_for(const FixedArgs& a, uint32_t gpb, uint32_t grid, uint32_t nphase) {
  const uint64_t per_step = (uint64_t)grid * gpb * nphase;
  return (uint32_t)((a.n_groups + per_step - 1) / per_step);
}

}  // namespace

bool fixed_uses_phases(const FixedArgs& a, bool nontemporal, uint32_t* grid) {
  if (!a.phase_sync || !nontemporal || a.L < 16u || a.n_groups == 0) return false;
  uint32_t g = 0, nphase = 0;
  const bool on = phase_plan(a, kBlock / ((a.L + 15u) / 16u), &g, &nphase);
  if (grid) *grid = on ? g : 0u;
  return on;
}

hipError_t launch_fixed(const FixedArgs& a0, bool nontemporal, hipStream_t s) {
  const bool recover = a0.parity != nullptr;
  if (a0.n_groups == 0) return hipSuccess;
  if (a0.L < 16u) {
    const uint64_t maxg = kMaxBlocks256 * kBlock / a0.L;  // one lane per output byte
    for (uint64_t g = 0; g < a0.n_groups; g += maxg) {
      FixedArgs a = a0;
      a.n_groups = std::min<uint64_t>(maxg, a0.n_groups - g);
      a.rows = a0.rows + g * a0.group_stride;
      if (recover) {
        a.parity = a0.parity + g * a0.parity_stride;
        a.missing = a0.missing + g;
      }
      a.out = a0.out + g * a0.out_stride;
      if (a0.inplace_missing) a.inplace_missing = a0.inplace_missing + g;
      const uint64_t blocks = (a.n_groups * a.L + kBlock - 1) / kBlock;
      if (recover)
        hipLaunchKernelGGL(fixed_small_kernel<true>, dim3((uint32_t)blocks), dim3(kBlock), 0, s, a);
      else
        hipLaunchKernelGGL(fixed_small_kernel<false>, dim3((uint32_t)blocks), dim3(kBlock), 0, s, a);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  const uint32_t C = (a0.L + 15u) / 16u;  // <= 91 for L <= 1452
  const uint32_t gpb = kBlock / C;         // whole groups per workgroup (>= 2)
  uint32_t grid = 0, nphase = 0;
  if (a0.phase_sync && nontemporal && phase_plan(a0, gpb, &grid, &nphase)) {
    FixedArgs a = a0;
    a.phase_steps = phase_steps_for(a0, gpb, grid, nphase);
    if (a.inplace_missing) return launch_phase_k<false, true>(a, C, gpb, grid, nphase, s);
    return recover ? launch_phase_k<true>(a, C, gpb, grid, nphase, s)
                   : launch_phase_k<false>(a, C, gpb, grid, nphase, s);
  }
  const uint64_t maxg = kMaxBlocks256 * gpb;
  for (uint64_t g = 0; g < a0.n_groups; g += maxg) {
    FixedArgs a = a0;
    a.n_groups = std::min<uint64_t>(maxg, a0.n_groups - g);
    a.rows = a0.rows + g * a0.group_stride;
    if (recover) {
      a.parity = a0.parity + g * a0.parity_stride;
      a.missing = a0.missing + g;
    }
    a.out = a0.out + g * a0.out_stride;
    if (a0.inplace_missing) a.inplace_missing = a0.inplace_missing + g;
    const uint64_t blocks = (a.n_groups + gpb - 1) / gpb;
    hipError_t e;
    if (a.inplace_missing)
      e = launch_fixed_k<false, true, false, true>(a, C, gpb, blocks, s);
    else if (recover && gpb <= 8u)
      e = nontemporal ? launch_fixed_k<true, true, true>(a, C, gpb, blocks, s)
                      : launch_fixed_k<true, false, true>(a, C, gpb, blocks, s);
    else if (recover)
      e = nontemporal ? launch_fixed_k<true, true, false>(a, C, gpb, blocks, s)
                      : launch_fixed_k<true, false, false>(a, C, gpb, blocks, s);
    else
      e = nontemporal ? launch_fixed_k<false, true, false>(a, C, gpb, blocks, s)
                      : launch_fixed_k<false, false, false>(a, C, gpb, blocks, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

constexpr int kRaggedBlockWaves = 4, kRaggedBlockGroups = 8;  // ragged_block_kernel shape

hipError_t launch_ragged(const RaggedArgs& a0, bool recover, hipStream_t s, bool small_groups) {
  if (a0.n_groups == 0) return hipSuccess;
  const uint64_t gpb = kRaggedBlockGroups;
  const uint64_t maxg = kMaxBlocks256 * gpb;
  for (uint64_t g = 0; g < a0.n_groups; g += maxg) {
    RaggedArgs a = a0;
    a.n_groups = std::min<uint64_t>(maxg, a0.n_groups - g);
    a.grp_ptr = a0.grp_ptr + g;
    if (recover) {
      a.parity_len = a0.parity_len + g;
      a.missing = a0.missing + g;
      a.out_off = a0.out_off + g;
      a.parity_off = a0.parity_off + g;
    } else {
      a.parity_off = a0.parity_off + g;
      a.parity_len_out = a0.parity_len_out + g;
    }
    const uint64_t blocks = (a.n_groups + gpb - 1) / gpb;
    // (two groups per wave x 4 waves: the block kernel's 8 groups per block)
    static_assert(2 * kFlatWaves == kRaggedBlockGroups, "one grid for both kernels");
    if (small_groups) {
      if (recover)
        hipLaunchKernelGGL((ragged_multi_kernel<true, true, 2>), dim3((uint32_t)blocks),
                           dim3(kBlock), 0, s, a);
      else
        hipLaunchKernelGGL((ragged_multi_kernel<false, true, 2>), dim3((uint32_t)blocks),
                           dim3(kBlock), 0, s, a);
    } else if (recover) {
      hipLaunchKernelGGL((ragged_block_kernel<true, kRaggedBlockWaves, kRaggedBlockGroups>),
                         dim3((uint32_t)blocks), dim3(64 * kRaggedBlockWaves), 0, s, a);
    } else {
      hipLaunchKernelGGL((ragged_block_kernel<false, kRaggedBlockWaves, kRaggedBlockGroups>),
                         dim3((uint32_t)blocks), dim3(64 * kRaggedBlockWaves), 0, s, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_ragged_latency(const RaggedArgs& a, bool recover, hipStream_t s) {
  if (a.n_groups == 0) return hipSuccess;
  if (a.n_groups > kMaxBlocks256) return hipErrorInvalidValue;  // small batches only
  const uint64_t blocks = (a.n_groups + kFlatWaves - 1) / kFlatWaves;
  // all of a group's loads in flight at once: 16 load slots per lane covers
  // up to 16 received packets (+ their second windows) in one round trip
  if (recover)
    hipLaunchKernelGGL((ragged_window_kernel<true, true, 16>), dim3((uint32_t)blocks),
                       dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((ragged_window_kernel<false, true, 16>), dim3((uint32_t)blocks),
                       dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_ragged_service(SvcShared* sh, SvcDev* dv, const SvcJob* ring, uint32_t* flags,
                                 uint64_t idle_ticks, uint32_t epoch, hipStream_t s) {
  hipLaunchKernelGGL(ragged_service_kernel, dim3(kSvcWgs), dim3(64 * kSvcWaves), 0, s, sh, dv,
                     ring, flags, idle_ticks, epoch);
  return hipGetLastError();
}

hipError_t launch_xor_into(const uint8_t* in, uint64_t n, uint8_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n / 16u + kBlock - 1) / kBlock;
  if (blocks < 1) blocks = 1;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(xor_into_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, s, in, n, out);
  return hipGetLastError();
}

hipError_t launch_stream_probe(const uint8_t* src, uint64_t n, uint8_t* dst, bool copy,
                               hipStream_t s) {
  if (n < 16) return hipSuccess;
  const dim3 grid(8192), blk(kBlock);
  if (copy)
    hipLaunchKernelGGL(stream_probe_kernel<true>, grid, blk, 0, s, src, n & ~15ull, dst);
  else
    hipLaunchKernelGGL(stream_probe_kernel<false>, grid, blk, 0, s, src, n & ~15ull, dst);
  return hipGetLastError();
}

hipError_t launch_synth_fixed(uint8_t* rows, uint32_t k, uint32_t L, uint64_t row_stride,
                              uint64_t group_stride, uint64_t g0, uint64_t n, uint64_t seed,
                              hipStream_t s) {
  const uint64_t total_rows = n * k;
  const uint64_t chunk = kMaxBlocks256;  // rows per launch (one workgroup each)
  for (uint64_t r = 0; r < total_rows; r += chunk) {
    const uint64_t cnt = std::min<uint64_t>(chunk, total_rows - r);
    hipLaunchKernelGGL(synth_fixed_kernel, dim3((uint32_t)cnt), dim3(kBlock), 0, s, rows, k, L,
                       row_stride, group_stride, g0, r, seed);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_synth_ragged(uint8_t* bytes, const uint64_t* pkt_off, const uint16_t* pkt_len,
                               const uint32_t* grp_ptr, uint64_t g0, uint64_t n, uint64_t seed,
                               hipStream_t s) {
  const uint64_t chunk = kMaxBlocks256;  // groups per launch (one workgroup each)
  for (uint64_t g = 0; g < n; g += chunk) {
    const uint64_t cnt = std::min<uint64_t>(chunk, n - g);
    hipLaunchKernelGGL(synth_ragged_kernel, dim3((uint32_t)cnt), dim3(kBlock), 0, s, bytes,
                       pkt_off, pkt_len, grp_ptr, g0, g, seed);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace qfec
