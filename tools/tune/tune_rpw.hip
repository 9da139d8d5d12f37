// tune_rpw.hip — VERDICT r4 item 1, second form: a grid-phased ragged kernel
// with a STATIC lane -> parity-window mapping and no input staging.
//
// ragged_rpw_kernel (below): a persistent grid of one NW-wave workgroup per CU
// walks the batch in phases.  Phase p of CU c is segment s = p * ncu + c of the
// batch, a contiguous group range holding ~1/(nphase ncu) of its PACKETS
// (rw_bounds_kernel, a binary search over grp_ptr: segments balanced by packet
// count, not by group count).  Inside the segment the CU's waves take groups
// one at a time from an LDS ticket.  A wave reduces its group in registers:
// lane t owns parity window t (bytes 16t..16t+15, set 0) and, for windows
// 64..90, lane t & 31 of the half-wave (set 1: lanes 0-31 take the even inputs'
// windows, lanes 32-63 the odd ones', one load instruction for two inputs; the
// halves are XORed together at the end).  Every load is an in-packet 16-B
// load: with 16-B aligned inputs (the payload arena) the window is loaded in
// place and the bytes past the packet masked; otherwise the window crossing
// the end is the 16 bytes ending there, shifted.  The finished parity row is
// put into an LDS hold area (~150 KiB per CU); the grid meets, then every CU
// stores its held rows.  The HBM sees read phases and write phases, as with
// the fixed kernel's phase_xor_kernel.  Groups whose row does not fit in the
// hold area are stored directly (exact either way).
//
//   tune_rpw [reps=5] [rounds=3] [palign=16] [slot=1536]
// Outputs byte-compared with ragged_block_kernel (the product) first.
#include "../../libquic_amd/csrc/qfec_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

namespace qfec {
namespace {

__device__ uint64_t* g_stamps;  // DIAG 2: per wave cycle counts

// RW_GUARD builds (tune_rpw_guard): every global access is checked against the
// batch's buffers first; the first bad one is recorded and replaced by a safe
// address (finding a fault without faulting the card).
struct RwDbg {
  uint64_t lo[4], hi[4];  // bytes, parity, out, aux
  uint32_t bad, where, g, lane;
  uint64_t addr;
};
__device__ RwDbg* g_dbg;
__device__ uint32_t g_dbg_g;
#ifdef RW_GUARD
__device__ __forceinline__ const uint8_t* rw_chk(const uint8_t* p, uint32_t n, uint32_t where) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  RwDbg* d = g_dbg;
  for (int i = 0; i < 4; ++i)
    if (a >= d->lo[i] && a + n <= d->hi[i]) return p;
  if (atomicCAS(&d->bad, 0u, 1u) == 0u) {
    d->where = where;
    d->addr = a;
    d->lane = threadIdx.x;
    d->g = g_dbg_g;
  }
  return reinterpret_cast<const uint8_t*>(d->lo[0]);
}
#define RWCHK(p, n, w) rw_chk((p), (n), (w))
#else
#define RWCHK(p, n, w) (p)
#endif

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t rdl(uint32_t x, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
}

// keep the first n (0..16) bytes of a 16-byte window: dword d's mask
__device__ __forceinline__ uint32_t keep_dw(uint32_t n, uint32_t d) {
  const int r = (int)n - 4 * (int)d;
  return r >= 4 ? 0xFFFFFFFFu : (r <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * r)));
}

// Window [win, win+16) of a zero-padded input of len bytes (any lane, any
// win).  AL: the input starts on a 16-B boundary -- the window is loaded in
// place (an aligned 16-B load holding one input byte cannot leave that byte's
// page) and its bytes past len masked; a window past the end loads the
// input's first 16 bytes and keeps none.  !AL (len >= 16): window16.
template <bool AL>
__device__ __forceinline__ u32x4 rw_window(const uint8_t* base, uint32_t len, uint32_t win) {
  if constexpr (AL) {
    const bool in = win < len;
    u32x4 v = ld16t<true>(RWCHK(base + (in ? win : 0u), 16u, 1u));
    const uint32_t rem = in ? min(len - win, 16u) : 0u;
    v.x &= keep_dw(rem, 0);
    v.y &= keep_dw(rem, 1);
    v.z &= keep_dw(rem, 2);
    v.w &= keep_dw(rem, 3);
    return v;
  } else {
    return window16<true>(base, len, win);
  }
}

// Inputs j0 .. j0+N-1 of the group (table lanes: address lo / hi, length),
// every load in flight before the first XOR.  S1: the group has an input
// longer than 1024 B (set-1 windows 64..), two inputs per load instruction.
template <int N, bool AL, bool S1>
__device__ __forceinline__ void rw_batch(u32x4& a0, u32x4& a1, uint32_t lane, uint32_t j0,
                                         uint32_t tlo, uint32_t thi, uint32_t tlen) {
  u32x4 v[N];
  constexpr int N1 = S1 ? (N + 1) / 2 : 1;
  u32x4 w[N1];
  const uint32_t win0 = 16u * lane;
  const uint32_t win1 = 16u * (64u + (lane & 31u));
  const bool hi_half = lane >= 32u;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const uint32_t len = rdl(tlen, j0 + j);
    const uint64_t b = ((uint64_t)rdl(thi, j0 + j) << 32) | rdl(tlo, j0 + j);
    v[j] = rw_window<AL>(reinterpret_cast<const uint8_t*>(b), len, win0);
  }
  if constexpr (S1) {
#pragma unroll
    for (int j = 0; j < N; j += 2) {
      const uint32_t le = rdl(tlen, j0 + j);
      const uint64_t be = ((uint64_t)rdl(thi, j0 + j) << 32) | rdl(tlo, j0 + j);
      uint32_t lo_ = le;
      uint64_t bo = be;
      if (j + 1 < N) {
        lo_ = rdl(tlen, j0 + j + 1);
        bo = ((uint64_t)rdl(thi, j0 + j + 1) << 32) | rdl(tlo, j0 + j + 1);
      }
      // the odd half of an odd batch's last pair XORs nothing (len 0: AL keeps
      // no byte; !AL: window16 past the end is zero)
      const uint32_t len = hi_half ? (j + 1 < N ? lo_ : 0u) : le;
      const uint64_t b = hi_half ? bo : be;
      if constexpr (AL) {
        w[j / 2] = rw_window<true>(reinterpret_cast<const uint8_t*>(b), len, win1);
      } else {
        // window16 needs len >= 16 to place its load: a zero-length half
        // loads the even input's window and is masked
        const uint32_t l2 = len == 0u ? le : len;
        const u32x4 x = window16<true>(reinterpret_cast<const uint8_t*>(b), l2, win1);
        const uint32_t keep = len == 0u ? 0u : 0xFFFFFFFFu;
        w[j / 2] = u32x4{x.x & keep, x.y & keep, x.z & keep, x.w & keep};
      }
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) a0 ^= v[j];
  if constexpr (S1) {
#pragma unroll
    for (int j = 0; j < N1; ++j) a1 ^= w[j];
  }
}

template <bool AL, bool S1, int B = 16>
__device__ __forceinline__ void rw_batch_n(uint32_t n, u32x4& a0, u32x4& a1, uint32_t lane,
                                           uint32_t j0, uint32_t tlo, uint32_t thi, uint32_t tlen) {
  switch (n) {
#define RWB(N) \
  case N: rw_batch<N, AL, S1>(a0, a1, lane, j0, tlo, thi, tlen); break;
    RWB(1) RWB(2) RWB(3) RWB(4) RWB(5) RWB(6) RWB(7) RWB(8)
    default:
      if constexpr (B > 8) {
        switch (n) {
          RWB(9) RWB(10) RWB(11) RWB(12) RWB(13) RWB(14) RWB(15) RWB(16)
          default: break;
        }
      }
      break;
#undef RWB
  }
}

// window t (wave-uniform) of the row held in a0 (t < 64) / a1 (lanes 0-31: 64..95)
__device__ __forceinline__ u32x4 rw_win_at(const u32x4& a0, const u32x4& a1, uint32_t t) {
  const bool s0 = t < 64u;
  const uint32_t l = s0 ? t : t - 64u;
  const u32x4 r = s0 ? a0 : a1;  // (uniform select)
  return u32x4{rdl(r.x, l), rdl(r.y, l), rdl(r.z, l), rdl(r.w, l)};
}

// Store a row of plen bytes held in registers (the ragged_group store: full
// windows in place, a partial last window as the 16 bytes ending at plen).
__device__ __forceinline__ void rw_store(uint8_t* dst, uint32_t plen, const u32x4& a0,
                                         const u32x4& a1, uint32_t lane) {
  if (plen >= 16u) {
    const uint32_t nw = (plen + 15u) >> 4, o = plen - 16u * (nw - 1u);
    const uint32_t nfull = o == 16u ? nw : nw - 1u;
    if (lane < nfull) st16t<true>(const_cast<uint8_t*>(RWCHK(dst + 16u * lane, 16u, 2u)), a0);
    if (lane < 32u && 64u + lane < nfull) st16t<true>(const_cast<uint8_t*>(RWCHK(dst + 16u * (64u + lane), 16u, 3u)), a1);
    if (o != 16u) {
      const u32x4 lo = rw_win_at(a0, a1, nw - 2u), hi = rw_win_at(a0, a1, nw - 1u);
      if (lane == 0u) st16t<true>(const_cast<uint8_t*>(RWCHK(dst + plen - 16u, 16u, 4u)), bytes16_at(lo, hi, o));
    }
  } else {
    const uint32_t d = lane >> 2;
    const uint32_t w = rdl(a0.x, 0) * (d == 0u) | rdl(a0.y, 0) * (d == 1u) |
                       rdl(a0.z, 0) * (d == 2u) | rdl(a0.w, 0) * (d == 3u);
    if (lane < plen) dst[lane] = (uint8_t)(w >> (8u * (lane & 3u)));
  }
}

// LDS hold area: rows at 16-B granularity, entries {dst lo, dst hi, group, plen | row << 16}
constexpr uint32_t kRwHoldW = 9600;  // 150 KiB
constexpr uint32_t kRwEnt = 192;

// One group: reduce into (a0, a1); returns plen, or 0xFFFFFFFF on an error
// (error bit set, nothing to store).
template <bool RECOVER, int B = 16>
__device__ __forceinline__ uint32_t rw_group(const RaggedArgs& a, uint64_t g, uint32_t lane,
                                             u32x4& a0, u32x4& a1, uint64_t& dst_off) {
  const u32x4 zero = {0u, 0u, 0u, 0u};
  a0 = zero;
  a1 = zero;
#ifdef RW_GUARD
  if (g >= a.n_groups) {
    RWCHK(reinterpret_cast<const uint8_t*>(0x10), 1u, 100u);
    return 0xFFFFFFFFu;
  }
  if (lane == 0u) g_dbg_g = (uint32_t)g;
#endif
  const uint32_t p0 = rfl(a.grp_ptr[g]);
  const uint32_t k = rfl(a.grp_ptr[g + 1]) - p0;
  if (k == 0u || k > 255u) {
    if (lane == 0u) atomicOr(a.err, kErrGroupSize);
    return 0xFFFFFFFFu;
  }
  uint32_t m = 0xFFFFFFFFu, plen = 0;
  const uint8_t* prow = nullptr;
  if constexpr (RECOVER) {
    m = rfl(a.missing[g]);
    plen = rfl(a.parity_len[g]);
    dst_off = a.out_off[g];
    if (m >= k) {
      if (lane == 0u) atomicOr(a.err, kErrMissingIndex);
      return 0xFFFFFFFFu;
    }
    if (plen == 0u || plen > kMaxPacket) {
      if (lane == 0u) atomicOr(a.err, kErrParityLength);
      return 0xFFFFFFFFu;
    }
    prow = a.parity + a.parity_off[g];
  } else {
    dst_off = a.parity_off[g];
  }
  const uint32_t nin = k;  // encode: k packets; recover: k-1 received + the parity row
  const uint32_t lim = RECOVER ? plen : kMaxPacket;
  uint32_t mx = 0;
  for (uint32_t c0 = 0; c0 < nin; c0 += 64u) {
    const uint32_t r = c0 + lane;
    uint32_t len = 0, tlo = 0, thi = 0;
    if (r < nin) {
      uint64_t ad;
      if (RECOVER && r == nin - 1u) {
        ad = (uint64_t)(uintptr_t)prow;
        len = plen;
      } else {
        const uint32_t p = p0 + r + (RECOVER && r >= m ? 1u : 0u);
#ifdef RW_GUARD
        if (p >= a.grp_ptr[a.n_groups]) RWCHK(reinterpret_cast<const uint8_t*>(0x20), 1u, 101u);
#endif
        len = a.pkt_len[p];
        ad = (uint64_t)(uintptr_t)a.bytes + a.pkt_off[p];
      }
      tlo = (uint32_t)ad;
      thi = (uint32_t)(ad >> 32);
    }
    if (wave_any(r < nin && (len == 0u || len > lim))) {
      if (lane == 0u) atomicOr(a.err, kErrPacketLength);
      return 0xFFFFFFFFu;
    }
    mx = max(mx, len);
    const uint32_t cn = min(nin - c0, 64u);
    const bool al = !wave_any(r < nin && (tlo & 15u) != 0u);
    const bool s1 = wave_any(r < nin && len > 1024u);
    const bool small = wave_any(r < nin && len < 16u);
    if (!al && small) {
      // an unaligned input below 16 B (rare): input by input, exact windows
      for (uint32_t j = 0; j < cn; ++j) {
        const uint32_t ln = rdl(len, j);
        const uint8_t* b = reinterpret_cast<const uint8_t*>(((uint64_t)rdl(thi, j) << 32) | rdl(tlo, j));
        if (16u * lane < ln) a0 ^= packet_window<true>(b, ln, lane);
        if (lane < 32u && 16u * (64u + lane) < ln) a1 ^= packet_window<true>(b, ln, 64u + lane);
      }
      continue;
    }
    // batches of <= B inputs, sizes as even as possible
    const uint32_t nb = (cn + (uint32_t)B - 1u) / (uint32_t)B;
    const uint32_t base = cn / nb, extra = cn - base * nb;
    uint32_t j0 = 0;
    for (uint32_t b = 0; b < nb; ++b) {
      const uint32_t n = base + (b < extra ? 1u : 0u);
      if (al) {
        if (s1) rw_batch_n<true, true, B>(n, a0, a1, lane, j0, tlo, thi, len);
        else rw_batch_n<true, false, B>(n, a0, a1, lane, j0, tlo, thi, len);
      } else {
        if (s1) rw_batch_n<false, true, B>(n, a0, a1, lane, j0, tlo, thi, len);
        else rw_batch_n<false, false, B>(n, a0, a1, lane, j0, tlo, thi, len);
      }
      j0 += n;
    }
  }
  // set 1: lanes 32-63 held the odd inputs' windows
  a1.x ^= (uint32_t)__shfl_xor((int)a1.x, 32, 64);
  a1.y ^= (uint32_t)__shfl_xor((int)a1.y, 32, 64);
  a1.z ^= (uint32_t)__shfl_xor((int)a1.z, 32, 64);
  a1.w ^= (uint32_t)__shfl_xor((int)a1.w, 32, 64);
  if constexpr (!RECOVER) plen = wave_max11(mx);
  return rfl(plen);
}

// Segment bounds: bnd[s] = the first group whose packets start at or after
// packet floor(s P / nseg) (P = grp_ptr[G]); bnd[0] = 0, bnd[nseg] = G.  Any
// grp_ptr gives a cover of [0, G) (the kernel takes [bnd[s], max(bnd[s+1],
// bnd[s]))); a monotone one, a partition.
__global__ __launch_bounds__(256) void rw_bounds_kernel(const uint32_t* grp_ptr, uint64_t G,
                                                        uint32_t nseg, uint32_t* bnd) {
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  if (s > nseg) return;
  if (s == 0u || s == nseg) {
    bnd[s] = s == 0u ? 0u : (uint32_t)G;
    return;
  }
  const uint64_t P = grp_ptr[G];
  const uint64_t t = P * s / nseg;
  uint64_t lo = 0, hi = G;  // first g in [0, G] with grp_ptr[g] >= t
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (grp_ptr[mid] < t) lo = mid + 1;
    else hi = mid;
  }
  bnd[s] = (uint32_t)lo;
}

template <bool RECOVER, int NW, int DIAG = 0, int B = (NW > 8 ? 8 : 16)>
__global__ __launch_bounds__(64 * NW) void ragged_rpw_kernel(RaggedArgs a, const uint32_t* bnd,
                                                             uint32_t nphase, uint32_t* phase_sync) {
  __shared__ u32x4 s_hold[kRwHoldW];
  __shared__ u32x4 s_ent[kRwEnt];
  __shared__ uint32_t s_next, s_alloc, s_nent;
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wv = rfl(tid >> 6);
  const uint32_t ncu = gridDim.x, cu = blockIdx.x;
  uint64_t c_work = 0, c_meet = 0, c_store = 0, c_idle = 0;
  u32x4 sink = {0u, 0u, 0u, 0u};
  auto stamp = [&]() -> uint64_t { return DIAG == 2 ? __builtin_amdgcn_s_memtime() : 0ull; };
  if (tid == 0u) {
    s_alloc = 0u;
    s_nent = 0u;
  }
  for (uint32_t p = 0; p < nphase; ++p) {
    const uint32_t seg = p * ncu + cu;
    const uint32_t gs = rfl(bnd[seg]);
    const uint32_t ge = max(rfl(bnd[seg + 1]), gs);
    if (tid == 0u) s_next = 0u;
    __syncthreads();
    uint64_t t0 = stamp();
    for (;;) {
      // every lane of the (full) wave adds the same value: one ds_add of 64x
      // the value, lane 0 reading the old sum -- the counters count in units
      // of 64.  (A lane-0-only atomic feeding the readfirstlane compiled to a
      // loop whose later iterations read another lane's zero, round 5; a
      // per-lane value, to the atomic optimizer's 64-step scan loop.)
      const uint32_t g = gs + rfl(atomicAdd(&s_next, 1u)) / 64u;
      if (g >= ge) break;
      u32x4 a0, a1;
      uint64_t doff = 0;
      const uint32_t plen = rw_group<RECOVER, B>(a, g, lane, a0, a1, doff);
      if (plen == 0xFFFFFFFFu) continue;
      const uint32_t nw = (plen + 15u) >> 4;
      const uint32_t e = rfl(atomicAdd(&s_nent, 1u)) / 64u;
      const uint32_t h = rfl(atomicAdd(&s_alloc, nw)) / 64u;
      if (e < kRwEnt && h + nw <= kRwHoldW) {
        if (lane < nw) s_hold[h + lane] = a0;
        if (lane < 32u && 64u + lane < nw) s_hold[h + 64u + lane] = a1;
        const uint64_t d = (uint64_t)(uintptr_t)a.out + doff;
        if (lane == 0u) s_ent[e] = u32x4{(uint32_t)d, (uint32_t)(d >> 32), g, plen | (h << 16)};
      } else {
        if (lane == 0u && e < kRwEnt) s_ent[e] = u32x4{0u, 0u, 0u, 0xFFFFFFFFu};  // no row held
        rw_store(a.out + doff, plen, a0, a1, lane);
        if (!RECOVER && lane == 0u) a.parity_len_out[g] = (uint16_t)plen;
      }
    }
    uint64_t t1 = stamp();
    if constexpr (DIAG == 2) c_work += t1 - t0;
    phase_meet(phase_sync, p + 1u);  // (its barrier also publishes the hold area)
    uint64_t t2 = stamp();
    if constexpr (DIAG == 2) c_meet += t2 - t1;
    const uint32_t ne = min(s_nent / 64u, kRwEnt);
    for (uint32_t e = wv; e < ne; e += NW) {
      const u32x4 en = s_ent[e];
      const uint32_t w3 = rfl(en.w);
      if (w3 == 0xFFFFFFFFu) continue;
      const uint32_t plen = w3 & 0xFFFFu, h = w3 >> 16, nw = (plen + 15u) >> 4;
      const u32x4 zero = {0u, 0u, 0u, 0u};
      const u32x4 a0 = lane < nw ? s_hold[h + lane] : zero;
      const u32x4 a1 = (lane < 32u && 64u + lane < nw) ? s_hold[h + 64u + lane] : zero;
      uint8_t* dst = reinterpret_cast<uint8_t*>(((uint64_t)rfl(en.y) << 32) | rfl(en.x));
      if constexpr (DIAG != 1) {
        rw_store(dst, plen, a0, a1, lane);
        if (!RECOVER && lane == 0u) a.parity_len_out[rfl(en.z)] = (uint16_t)plen;
      } else {
        sink ^= a0 ^ a1;  // keeps the reduce alive without the stores
      }
    }
    __syncthreads();  // hold area read
    if (tid == 0u) {
      s_alloc = 0u;
      s_nent = 0u;
    }
    uint64_t t3 = stamp();
    if constexpr (DIAG == 2) c_store += t3 - t2;
  }
  if constexpr (DIAG == 2) {
    if (lane == 0u) {
      uint64_t* o = g_stamps + ((uint64_t)blockIdx.x * NW + wv) * 8u;
      o[0] = c_work; o[1] = c_meet; o[2] = c_store; o[3] = c_idle;
    }
  }
  if constexpr (DIAG == 1) {
    if ((sink.x ^ sink.y ^ sink.z ^ sink.w) == 0x9E3779B9u) atomicOr(a.err, 0x80000000u);
  }
  phase_exit(phase_sync, nullptr);
}


// ---------------------------------------------------------------------------
// v2: the same reduce, software-pipelined across a wave's groups.  A group's
// three dependent round trips (group scalars -> packet table -> payloads)
// were each exposed in v1 (work 78-80% of the time at 0.26-0.44 of 8 TB/s).
// Here, in the iteration that XORs group i, the wave has already issued the
// packet table of group i+1 (vector loads, ahead of group i's payload loads,
// so waiting for those implies them) and the scalars of group i+2 (scalar
// loads through the constant address space: s_load into SGPRs, counted by
// lgkmcnt, waited at the deposit's LDS atomics a payload round trip later).
// Payloads are loaded through global (not flat) pointers, so no LDS wait
// drains them.
typedef const __attribute__((address_space(4))) uint32_t* cptr32;
typedef const __attribute__((address_space(4))) uint64_t* cptr64;
typedef const __attribute__((address_space(1))) u32x4* gptr16;
typedef __attribute__((address_space(1))) u32x4* gptr16w;

__device__ __forceinline__ u32x4 ldg16(uint64_t ad) {
#ifdef RW_GUARD
  ad = (uint64_t)(uintptr_t)rw_chk(reinterpret_cast<const uint8_t*>(ad), 16u, 11u);
#endif
  return __builtin_nontemporal_load((gptr16)ad);
}
__device__ __forceinline__ void stg16(uint64_t ad, u32x4 v) {
#ifdef RW_GUARD
  ad = (uint64_t)(uintptr_t)rw_chk(reinterpret_cast<const uint8_t*>(ad), 16u, 12u);
#endif
  __builtin_nontemporal_store(v, (gptr16w)ad);
}
// a scalar load of the dword holding byte address ad (constant address space)
__device__ __forceinline__ uint32_t sld_dw(uint64_t ad) { return *(cptr32)(ad & ~3ull); }
__device__ __forceinline__ uint32_t sld32(const uint32_t* p) { return *(cptr32)(uintptr_t)p; }
__device__ __forceinline__ uint64_t sld64(const uint64_t* p) { return *(cptr64)(uintptr_t)p; }

template <bool AL>
__device__ __forceinline__ u32x4 rw2_window(uint64_t base, uint32_t len, uint32_t win) {
  if constexpr (AL) {
    const bool in = win < len;
    u32x4 v = ldg16(base + (in ? win : 0u));
    const uint32_t rem = in ? min(len - win, 16u) : 0u;
    v.x &= keep_dw(rem, 0);
    v.y &= keep_dw(rem, 1);
    v.z &= keep_dw(rem, 2);
    v.w &= keep_dw(rem, 3);
    return v;
  } else {
    const bool full = win + 16u <= len;
    const u32x4 v = ldg16(base + (full ? win : len - 16u));
    const uint32_t sh = full ? 0u : min(win + 16u - len, 15u);
    const uint32_t keep = win < len ? 0xFFFFFFFFu : 0u;
    return shr_bytes_bf(v, sh) & keep;
  }
}

template <int N, bool AL, bool S1>
__device__ __forceinline__ void rw2_batch(u32x4& a0, u32x4& a1, uint32_t lane, uint32_t j0,
                                          uint32_t tlo, uint32_t thi, uint32_t tlen) {
  u32x4 v[N];
  constexpr int N1 = S1 ? (N + 1) / 2 : 1;
  u32x4 w[N1];
  const uint32_t win0 = 16u * lane;
  const uint32_t win1 = 16u * (64u + (lane & 31u));
  const bool hi_half = lane >= 32u;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const uint32_t len = rdl(tlen, j0 + j);
    const uint64_t b = ((uint64_t)rdl(thi, j0 + j) << 32) | rdl(tlo, j0 + j);
    v[j] = rw2_window<AL>(b, len, win0);
  }
  if constexpr (S1) {
#pragma unroll
    for (int j = 0; j < N; j += 2) {
      const uint32_t le = rdl(tlen, j0 + j);
      const uint64_t be = ((uint64_t)rdl(thi, j0 + j) << 32) | rdl(tlo, j0 + j);
      uint32_t lo_ = le;
      uint64_t bo = be;
      if (j + 1 < N) {
        lo_ = rdl(tlen, j0 + j + 1);
        bo = ((uint64_t)rdl(thi, j0 + j + 1) << 32) | rdl(tlo, j0 + j + 1);
      }
      const uint32_t len = hi_half ? (j + 1 < N ? lo_ : 0u) : le;
      const uint64_t b = hi_half ? bo : be;
      if constexpr (AL) {
        w[j / 2] = rw2_window<true>(b, len, win1);
      } else {
        const uint32_t l2 = len == 0u ? le : len;
        const u32x4 x = rw2_window<false>(b, l2, win1);
        const uint32_t keep = len == 0u ? 0u : 0xFFFFFFFFu;
        w[j / 2] = u32x4{x.x & keep, x.y & keep, x.z & keep, x.w & keep};
      }
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) a0 ^= v[j];
  if constexpr (S1) {
#pragma unroll
    for (int j = 0; j < N1; ++j) a1 ^= w[j];
  }
}

template <bool AL, bool S1, int B>
__device__ __forceinline__ void rw2_batch_n(uint32_t n, u32x4& a0, u32x4& a1, uint32_t lane,
                                            uint32_t j0, uint32_t tlo, uint32_t thi, uint32_t tlen) {
  switch (n) {
#define RWB(N) \
  case N: rw2_batch<N, AL, S1>(a0, a1, lane, j0, tlo, thi, tlen); break;
    RWB(1) RWB(2) RWB(3) RWB(4) RWB(5) RWB(6) RWB(7) RWB(8)
    default:
      if constexpr (B > 8) {
        switch (n) {
          RWB(9) RWB(10) RWB(11) RWB(12) RWB(13) RWB(14) RWB(15) RWB(16)
          default: break;
        }
      }
      break;
#undef RWB
  }
}

// the group's scalars (wave-uniform, scalar loads)
struct RwS {
  uint32_t g, p0, k, m, plen;
  uint64_t doff, poff;
};

template <bool RECOVER>
__device__ __forceinline__ void rw2_scalars(const RaggedArgs& a, uint32_t g, RwS& s) {
#ifdef RW_GUARD
  if (g >= a.n_groups) {
    rw_chk(reinterpret_cast<const uint8_t*>(0x30), 1u, 110u);
    g = 0;
  }
#endif
  s.g = g;
  s.p0 = sld32(a.grp_ptr + g);
  s.k = sld32(a.grp_ptr + g + 1) - s.p0;
  if constexpr (RECOVER) {
    const uint64_t ma = (uint64_t)(uintptr_t)(a.missing + g);
    s.m = (sld_dw(ma) >> (8u * (uint32_t)(ma & 3u))) & 0xFFu;
    const uint64_t la = (uint64_t)(uintptr_t)(a.parity_len + g);
    s.plen = (sld_dw(la) >> (8u * (uint32_t)(la & 3u))) & 0xFFFFu;
    s.doff = sld64(a.out_off + g);
    s.poff = sld64(a.parity_off + g);
  } else {
    s.m = 0xFFFFFFFFu;
    s.plen = 0;
    s.doff = sld64(a.parity_off + g);
    s.poff = 0;
  }
}

// lane r: input r of the group's first 64 (address lo / hi, length); nothing
// for a group the reduce will refuse (its table is never read)
template <bool RECOVER>
__device__ __forceinline__ void rw2_table(const RaggedArgs& a, const RwS& s, uint32_t lane,
                                          uint32_t c0, uint32_t& tlo, uint32_t& thi, uint32_t& tlen) {
  tlo = thi = tlen = 0;
  const bool ok = s.k >= 1u && s.k <= 255u &&
                  (!RECOVER || (s.m < s.k && s.plen >= 1u && s.plen <= kMaxPacket));
  if (!ok) return;
  const uint32_t r = c0 + lane;
  if (r >= s.k) return;
  uint64_t ad;
  if (RECOVER && r == s.k - 1u) {
    ad = (uint64_t)(uintptr_t)a.parity + s.poff;
    tlen = s.plen;
  } else {
    uint32_t p = s.p0 + r + (RECOVER && r >= s.m ? 1u : 0u);
#ifdef RW_GUARD
    if (p >= a.grp_ptr[a.n_groups]) {
      rw_chk(reinterpret_cast<const uint8_t*>(0x40), 1u, 111u);
      p = 0;
    }
#endif
    tlen = a.pkt_len[p];
    ad = (uint64_t)(uintptr_t)a.bytes + a.pkt_off[p];
  }
  tlo = (uint32_t)ad;
  thi = (uint32_t)(ad >> 32);
}

// Reduce one group (its scalars s, its first table chunk t*); returns plen or
// 0xFFFFFFFF on an error (bit set, nothing to store).
template <bool RECOVER, int B>
__device__ __forceinline__ uint32_t rw2_reduce(const RaggedArgs& a, const RwS& s, uint32_t lane,
                                               uint32_t tlo, uint32_t thi, uint32_t tlen,
                                               u32x4& a0, u32x4& a1) {
  const u32x4 zero = {0u, 0u, 0u, 0u};
  a0 = zero;
  a1 = zero;
  const uint32_t k = s.k;
  if (k == 0u || k > 255u) {
    if (lane == 0u) atomicOr(a.err, kErrGroupSize);
    return 0xFFFFFFFFu;
  }
  if constexpr (RECOVER) {
    if (s.m >= k) {
      if (lane == 0u) atomicOr(a.err, kErrMissingIndex);
      return 0xFFFFFFFFu;
    }
    if (s.plen == 0u || s.plen > kMaxPacket) {
      if (lane == 0u) atomicOr(a.err, kErrParityLength);
      return 0xFFFFFFFFu;
    }
  }
  const uint32_t nin = k;
  const uint32_t lim = RECOVER ? s.plen : kMaxPacket;
  uint32_t mx = 0;
  for (uint32_t c0 = 0; c0 < nin; c0 += 64u) {
    const uint32_t r = c0 + lane;
    if (c0 > 0u) rw2_table<RECOVER>(a, s, lane, c0, tlo, thi, tlen);
    if (wave_any(r < nin && (tlen == 0u || tlen > lim))) {
      if (lane == 0u) atomicOr(a.err, kErrPacketLength);
      return 0xFFFFFFFFu;
    }
    mx = max(mx, tlen);
    const uint32_t cn = min(nin - c0, 64u);
    const bool al = !wave_any(r < nin && (tlo & 15u) != 0u);
    const bool s1 = wave_any(r < nin && tlen > 1024u);
    const bool small = wave_any(r < nin && tlen < 16u);
    if (!al && small) {
      for (uint32_t j = 0; j < cn; ++j) {
        const uint32_t ln = rdl(tlen, j);
        const uint8_t* b = reinterpret_cast<const uint8_t*>(((uint64_t)rdl(thi, j) << 32) | rdl(tlo, j));
        if (16u * lane < ln) a0 ^= packet_window<true>(b, ln, lane);
        if (lane < 32u && 16u * (64u + lane) < ln) a1 ^= packet_window<true>(b, ln, 64u + lane);
      }
      continue;
    }
    const uint32_t nb = (cn + (uint32_t)B - 1u) / (uint32_t)B;
    const uint32_t base = cn / nb, extra = cn - base * nb;
    uint32_t j0 = 0;
    for (uint32_t b = 0; b < nb; ++b) {
      const uint32_t n = base + (b < extra ? 1u : 0u);
      if (al) {
        if (s1) rw2_batch_n<true, true, B>(n, a0, a1, lane, j0, tlo, thi, tlen);
        else rw2_batch_n<true, false, B>(n, a0, a1, lane, j0, tlo, thi, tlen);
      } else {
        if (s1) rw2_batch_n<false, true, B>(n, a0, a1, lane, j0, tlo, thi, tlen);
        else rw2_batch_n<false, false, B>(n, a0, a1, lane, j0, tlo, thi, tlen);
      }
      j0 += n;
    }
  }
  a1.x ^= (uint32_t)__shfl_xor((int)a1.x, 32, 64);
  a1.y ^= (uint32_t)__shfl_xor((int)a1.y, 32, 64);
  a1.z ^= (uint32_t)__shfl_xor((int)a1.z, 32, 64);
  a1.w ^= (uint32_t)__shfl_xor((int)a1.w, 32, 64);
  return RECOVER ? s.plen : rfl(wave_max11(mx));
}

// Store a held row (global stores; the ragged_group store's windows).
__device__ __forceinline__ void rw2_store(uint64_t dst, uint32_t plen, const u32x4& a0,
                                          const u32x4& a1, uint32_t lane) {
  if (plen >= 16u) {
    const uint32_t nw = (plen + 15u) >> 4, o = plen - 16u * (nw - 1u);
    const uint32_t nfull = o == 16u ? nw : nw - 1u;
    if (lane < nfull) stg16(dst + 16u * lane, a0);
    if (lane < 32u && 64u + lane < nfull) stg16(dst + 16u * (64u + lane), a1);
    if (o != 16u) {
      const u32x4 lo = rw_win_at(a0, a1, nw - 2u), hi = rw_win_at(a0, a1, nw - 1u);
      if (lane == 0u) stg16(dst + plen - 16u, bytes16_at(lo, hi, o));
    }
  } else {
    rw_store(reinterpret_cast<uint8_t*>(dst), plen, a0, a1, lane);
  }
}

template <bool RECOVER, int NW, int DIAG = 0, int B = (NW > 8 ? 8 : 16)>
__global__ __launch_bounds__(64 * NW) void ragged_rpw2_kernel(RaggedArgs a, const uint32_t* bnd,
                                                              uint32_t nphase, uint32_t* phase_sync) {
  __shared__ u32x4 s_hold[kRwHoldW];
  __shared__ u32x4 s_ent[kRwEnt];
  __shared__ uint32_t s_next, s_alloc, s_nent;
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wv = rfl(tid >> 6);
  const uint32_t ncu = gridDim.x, cu = blockIdx.x;
  uint64_t c_work = 0, c_meet = 0, c_store = 0, c_idle = 0;
  u32x4 sink = {0u, 0u, 0u, 0u};
  auto stamp = [&]() -> uint64_t { return DIAG == 2 ? __builtin_amdgcn_s_memtime() : 0ull; };
  if (tid == 0u) {
    s_alloc = 0u;
    s_nent = 0u;
  }
  for (uint32_t p = 0; p < nphase; ++p) {
    const uint32_t seg = p * ncu + cu;
    const uint32_t gs = rfl(bnd[seg]);
    const uint32_t ge = max(rfl(bnd[seg + 1]), gs);
    if (tid == 0u) s_next = 0u;
    __syncthreads();
    uint64_t t0 = stamp();
    // (tickets: every lane adds 1, lane 0 reads the old sum: units of 64)
    auto ticket = [&]() -> uint32_t { return gs + rfl(atomicAdd(&s_next, 1u)) / 64u; };
    RwS s0, s1, s2;
    uint32_t g0 = ticket();
    if (g0 < ge) rw2_scalars<RECOVER>(a, g0, s0);
    uint32_t g1 = ticket();
    if (g1 < ge) rw2_scalars<RECOVER>(a, g1, s1);
    uint32_t tlo0 = 0, thi0 = 0, tlen0 = 0;
    if (g0 < ge) rw2_table<RECOVER>(a, s0, lane, 0u, tlo0, thi0, tlen0);
    while (g0 < ge) {
      // 1. the next-but-one ticket; 2. group i+1's table (its scalars came a
      // round trip ago); 3. group i+2's scalars; 4. group i's payloads
      const uint32_t g2 = ticket();
      uint32_t tlo1 = 0, thi1 = 0, tlen1 = 0;
      if (g1 < ge) rw2_table<RECOVER>(a, s1, lane, 0u, tlo1, thi1, tlen1);
      __builtin_amdgcn_sched_barrier(0);
      if (g2 < ge) rw2_scalars<RECOVER>(a, g2, s2);
      __builtin_amdgcn_sched_barrier(0);
      u32x4 a0, a1;
      const uint32_t plen = rw2_reduce<RECOVER, B>(a, s0, lane, tlo0, thi0, tlen0, a0, a1);
      if (plen != 0xFFFFFFFFu) {
        const uint32_t nw = (plen + 15u) >> 4;
        const uint32_t e = rfl(atomicAdd(&s_nent, 1u)) / 64u;
        const uint32_t h = rfl(atomicAdd(&s_alloc, nw)) / 64u;
        const uint64_t d = (uint64_t)(uintptr_t)a.out + s0.doff;
        if (e < kRwEnt && h + nw <= kRwHoldW) {
          if (lane < nw) s_hold[h + lane] = a0;
          if (lane < 32u && 64u + lane < nw) s_hold[h + 64u + lane] = a1;
          if (lane == 0u) s_ent[e] = u32x4{(uint32_t)d, (uint32_t)(d >> 32), g0, plen | (h << 16)};
        } else {
          if (lane == 0u && e < kRwEnt) s_ent[e] = u32x4{0u, 0u, 0u, 0xFFFFFFFFu};
          rw2_store(d, plen, a0, a1, lane);
          if (!RECOVER && lane == 0u) a.parity_len_out[g0] = (uint16_t)plen;
        }
      }
      g0 = g1;
      s0 = s1;
      tlo0 = tlo1;
      thi0 = thi1;
      tlen0 = tlen1;
      g1 = g2;
      s1 = s2;
    }
    uint64_t t1 = stamp();
    if constexpr (DIAG == 2) c_work += t1 - t0;
    phase_meet(phase_sync, p + 1u);
    uint64_t t2 = stamp();
    if constexpr (DIAG == 2) c_meet += t2 - t1;
    const uint32_t ne = min(s_nent / 64u, kRwEnt);
    for (uint32_t e = wv; e < ne; e += NW) {
      const u32x4 en = s_ent[e];
      const uint32_t w3 = rfl(en.w);
      if (w3 == 0xFFFFFFFFu) continue;
      const uint32_t plen = w3 & 0xFFFFu, h = w3 >> 16, nw = (plen + 15u) >> 4;
      const u32x4 zero = {0u, 0u, 0u, 0u};
      const u32x4 a0 = lane < nw ? s_hold[h + lane] : zero;
      const u32x4 a1 = (lane < 32u && 64u + lane < nw) ? s_hold[h + 64u + lane] : zero;
      const uint64_t dst = ((uint64_t)rfl(en.y) << 32) | rfl(en.x);
      if constexpr (DIAG != 1) {
        rw2_store(dst, plen, a0, a1, lane);
        if (!RECOVER && lane == 0u) a.parity_len_out[rfl(en.z)] = (uint16_t)plen;
      } else {
        sink ^= a0 ^ a1;
      }
    }
    __syncthreads();
    if (tid == 0u) {
      s_alloc = 0u;
      s_nent = 0u;
    }
    uint64_t t3 = stamp();
    if constexpr (DIAG == 2) c_store += t3 - t2;
  }
  if constexpr (DIAG == 2) {
    if (lane == 0u) {
      uint64_t* o = g_stamps + ((uint64_t)blockIdx.x * NW + wv) * 8u;
      o[0] = c_work; o[1] = c_meet; o[2] = c_store; o[3] = c_idle;
    }
  }
  if constexpr (DIAG == 1) {
    if ((sink.x ^ sink.y ^ sink.z ^ sink.w) == 0x9E3779B9u) atomicOr(a.err, 0x80000000u);
  }
  phase_exit(phase_sync, nullptr);
}


// ---------------------------------------------------------------------------
// v3: v2's pipeline with the FULL windows of each input loaded through a
// buffer descriptor whose record count is the input's length rounded down to
// 16 B: the hardware range check returns zero for every lane past them, so a
// window load is one instruction and no VALU (v1/v2 spent ~30 VALU per load on
// the address select and the byte mask: VALU-bound, stamps r5).  The partial
// last window of each input (len % 16 bytes) is loaded by ONE lane per input
// in a separate instruction, masked, and XORed into the held row through LDS
// atomics (or, for a row not held, broadcast into the registers).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rw3_rsrc(uint64_t base, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(base), 0, (int)nbytes, 0x00020000);
}
__device__ __forceinline__ u32x4 rw3_ld(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 2);  // nt
}

struct Acc2 {
  u32x4 a0, a1;
};

template <int N, bool S1>
__device__ __forceinline__ Acc2 rw3_batch(Acc2 acc, uint32_t lane, uint32_t j0, uint32_t tlo,
                                          uint32_t thi, uint32_t tlen) {
  // S1: set-1 windows (64..) of every input too, unconditionally (the range
  // check zeroes the inputs that have none; a branch per input made the
  // compiler wait on each load)
  u32x4 v[N], w[S1 ? N : 1];
  const uint32_t vo0 = 16u * lane, vo1 = 16u * (64u + lane);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const uint32_t len = rdl(tlen, j0 + j);
    const uint64_t b = ((uint64_t)rdl(thi, j0 + j) << 32) | rdl(tlo, j0 + j);
#ifdef RW_GUARD
    const uint64_t bb = (len & ~15u) ? (uint64_t)(uintptr_t)rw_chk(reinterpret_cast<const uint8_t*>(b), len & ~15u, 13u) : b;
    const __amdgpu_buffer_rsrc_t r = rw3_rsrc(bb, len & ~15u);
#else
    const __amdgpu_buffer_rsrc_t r = rw3_rsrc(b, len & ~15u);
#endif
    v[j] = rw3_ld(r, vo0);
    if constexpr (S1) w[j] = rw3_ld(r, vo1);
  }
  // every load of the batch issued before the first XOR (the scheduler,
  // near the register limit, interleaved them with vmcnt(0..3) waits)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < N; ++j) acc.a0 ^= v[j];
  if constexpr (S1) {
#pragma unroll
    for (int j = 0; j < N; ++j) acc.a1 ^= w[j];
  }
  return acc;
}

template <bool S1, int B>
__device__ __forceinline__ Acc2 rw3_batch_n(uint32_t n, Acc2 acc, uint32_t lane, uint32_t j0,
                                            uint32_t tlo, uint32_t thi, uint32_t tlen) {
  switch (n) {
#define RWB(N) \
  case N: return rw3_batch<N, S1>(acc, lane, j0, tlo, thi, tlen);
    RWB(1) RWB(2) RWB(3) RWB(4) RWB(5) RWB(6) RWB(7) RWB(8)
    default:
      if constexpr (B > 8) {
        switch (n) {
          RWB(9) RWB(10) RWB(11) RWB(12) RWB(13) RWB(14) RWB(15) RWB(16)
          default: break;
        }
      }
      break;
#undef RWB
  }
  return acc;
}

// Lane j's input (address, len): its partial last window (bytes 16*(len>>4)
// .. len-1 at positions 0 .. len%16-1, zero above); zero when len % 16 == 0.
// Issued without a branch (a per-lane branch around the load made the
// compiler wait for it right there: a round trip per group) and finished
// later: in place when the window starts on a 16-B boundary (cannot leave
// the page of the input's byte there), else the 16 bytes ending at len
// (len >= 16: the caller sends groups with an unaligned input below 16 B
// down the exact input-by-input path).
__device__ __forceinline__ u32x4 rw3_partial_issue(uint64_t base, uint32_t len, bool on,
                                                   uint64_t any) {
  // (a lane without an input loads the first input's first bytes: `any`)
  const uint64_t pa = base + (len & ~15u);
  const bool inpl = (pa & 15u) == 0u;
  const uint64_t at = !on ? any : (inpl ? pa : base + len - 16u);
  return ldg16(at);
}
__device__ __forceinline__ u32x4 rw3_partial_finish(u32x4 v, uint64_t base, uint32_t len, bool on) {
  const uint32_t rem = len & 15u;
  const bool inpl = ((base + (len & ~15u)) & 15u) == 0u;
  const u32x4 sh = shr_bytes_bf(v, (16u - rem) & 15u);
  const uint32_t k0 = keep_dw(rem, 0), k1 = keep_dw(rem, 1), k2 = keep_dw(rem, 2), k3 = keep_dw(rem, 3);
  u32x4 r = inpl ? u32x4{v.x & k0, v.y & k1, v.z & k2, v.w & k3} : sh;
  const uint32_t z = (on && rem != 0u) ? 0xFFFFFFFFu : 0u;
  return u32x4{r.x & z, r.y & z, r.z & z, r.w & z};
}

// XOR the table lanes' partial windows into the row in registers (a row not
// held, or a chunk of a group of more than 64 inputs): lane t takes the
// partials of the inputs whose last window is t.
__device__ __forceinline__ void rw3_partials_regs(u32x4& a0, u32x4& a1, uint32_t lane, uint32_t cn,
                                                  uint32_t tlen, const u32x4& pw) {
  for (uint32_t j = 0; j < cn; ++j) {
    const uint32_t len = rdl(tlen, j);
    if ((len & 15u) == 0u) continue;
    const uint32_t t = len >> 4;
    const u32x4 x = {rdl(pw.x, j), rdl(pw.y, j), rdl(pw.z, j), rdl(pw.w, j)};
    const u32x4 zero = {0u, 0u, 0u, 0u};
    // (selects, not a branch per set: a branch became a pointer phi between
    // the two accumulators and put both in scratch memory)
    a0 ^= lane == t ? x : zero;
    a1 ^= lane + 64u == t ? x : zero;
  }
}

// v4: set-1 loads (full windows 64..) only for the inputs that have one
// (len >= 1040, ~1 in 4 of configs[3]'s): table lanes from a ballot mask,
// at most 4 issued ahead of the set-0 batch, so a group of <= 16 inputs is
// ONE round trip with 16-B batches of set-0 loads (v3: batches of 8, every
// input's set-1 load, two round trips for k > 8).
template <int N1>
__device__ __forceinline__ void rw4_s1(u32x4 (&w)[4], uint64_t& mask1, uint32_t tlo, uint32_t thi,
                                       uint32_t tlen, uint32_t vo1) {
#pragma unroll
  for (int j = 0; j < N1; ++j) {
    const uint32_t idx = (uint32_t)__builtin_ctzll(mask1);
    mask1 &= mask1 - 1ull;
    const uint32_t len = rdl(tlen, idx);
    const uint64_t b = ((uint64_t)rdl(thi, idx) << 32) | rdl(tlo, idx);
    w[j] = rw3_ld(rw3_rsrc(b, len & ~15u), vo1);
  }
}
__device__ __forceinline__ void rw4_s1_n(uint32_t n, u32x4 (&w)[4], uint64_t& mask1, uint32_t tlo,
                                         uint32_t thi, uint32_t tlen, uint32_t vo1) {
  switch (n) {
    case 1: rw4_s1<1>(w, mask1, tlo, thi, tlen, vo1); break;
    case 2: rw4_s1<2>(w, mask1, tlo, thi, tlen, vo1); break;
    case 3: rw4_s1<3>(w, mask1, tlo, thi, tlen, vo1); break;
    case 4: rw4_s1<4>(w, mask1, tlo, thi, tlen, vo1); break;
    default: break;
  }
}

// Reduce; hold = the LDS row (16-B units) the partials go to, or ~0: registers.
template <bool RECOVER, int B, bool V4 = false>
__device__ __forceinline__ uint32_t rw3_reduce(const RaggedArgs& a, const RwS& s, uint32_t lane,
                                               uint32_t tlo, uint32_t thi, uint32_t tlen,
                                               u32x4& a0, u32x4& a1, u32x4& pw, bool& deferred) {
  const u32x4 zero = {0u, 0u, 0u, 0u};
  a0 = zero;
  a1 = zero;
  pw = zero;
  deferred = false;
  const uint32_t k = s.k;
  if (k == 0u || k > 255u) {
    if (lane == 0u) atomicOr(a.err, kErrGroupSize);
    return 0xFFFFFFFFu;
  }
  if constexpr (RECOVER) {
    if (s.m >= k) {
      if (lane == 0u) atomicOr(a.err, kErrMissingIndex);
      return 0xFFFFFFFFu;
    }
    if (s.plen == 0u || s.plen > kMaxPacket) {
      if (lane == 0u) atomicOr(a.err, kErrParityLength);
      return 0xFFFFFFFFu;
    }
  }
  const uint32_t nin = k;
  const uint32_t lim = RECOVER ? s.plen : kMaxPacket;
  uint32_t mx = 0;
  for (uint32_t c0 = 0; c0 < nin; c0 += 64u) {
    const uint32_t r = c0 + lane;
    if (c0 > 0u) rw2_table<RECOVER>(a, s, lane, c0, tlo, thi, tlen);
    if (wave_any(r < nin && (tlen == 0u || tlen > lim))) {
      if (lane == 0u) atomicOr(a.err, kErrPacketLength);
      return 0xFFFFFFFFu;
    }
    mx = max(mx, tlen);
    const uint32_t cn = min(nin - c0, 64u);
    const bool s1 = wave_any(r < nin && tlen >= 1040u);  // a full window 64 (bytes 1024..1039)
    // this chunk's partial windows: one load per lane, finished after the XORs
    const uint64_t tb = ((uint64_t)thi << 32) | tlo;
    const bool small = wave_any(r < nin && tlen < 16u && (tlo & 15u) != 0u);
    if (small) {
      // an unaligned input below 16 B (rare): input by input, exact windows
      for (uint32_t j = 0; j < cn; ++j) {
        const uint32_t ln = rdl(tlen, j);
        const uint8_t* bp = reinterpret_cast<const uint8_t*>(((uint64_t)rdl(thi, j) << 32) | rdl(tlo, j));
        if (16u * lane < ln) a0 ^= packet_window<true>(bp, ln, lane);
        if (16u * (64u + lane) < ln) a1 ^= packet_window<true>(bp, ln, 64u + lane);
      }
      if (nin > 64u) continue;
      pw = zero;
      deferred = true;
      continue;
    }
    const u32x4 praw = rw3_partial_issue(tb, tlen, r < nin, ((uint64_t)rdl(thi, 0u) << 32) | rdl(tlo, 0u));
    const uint32_t nb = (cn + (uint32_t)B - 1u) / (uint32_t)B;
    const uint32_t base = cn / nb, extra = cn - base * nb;
    uint32_t j0 = 0;
    if constexpr (V4) {
      const uint32_t vo1 = 16u * (64u + lane);
      uint64_t mask1 = __ballot(r < nin && tlen >= 1040u);
      u32x4 w[4] = {zero, zero, zero, zero};
      rw4_s1_n(min((uint32_t)__popcll(mask1), 4u), w, mask1, tlo, thi, tlen, vo1);
      for (uint32_t b = 0; b < nb; ++b) {
        const uint32_t n = base + (b < extra ? 1u : 0u);
        Acc2 acc{a0, a1};
        acc = rw3_batch_n<false, B>(n, acc, lane, j0, tlo, thi, tlen);
        a0 = acc.a0;
        j0 += n;
      }
      a1 ^= w[0] ^ w[1] ^ w[2] ^ w[3];
      while (mask1 != 0ull) {  // more than 4 long inputs (rare)
        u32x4 x[4] = {zero, zero, zero, zero};
        rw4_s1_n(min((uint32_t)__popcll(mask1), 4u), x, mask1, tlo, thi, tlen, vo1);
        a1 ^= x[0] ^ x[1] ^ x[2] ^ x[3];
      }
    } else {
      for (uint32_t b = 0; b < nb; ++b) {
        const uint32_t n = base + (b < extra ? 1u : 0u);
        Acc2 acc{a0, a1};
        acc = s1 ? rw3_batch_n<true, B>(n, acc, lane, j0, tlo, thi, tlen)
                 : rw3_batch_n<false, B>(n, acc, lane, j0, tlo, thi, tlen);
        a0 = acc.a0;
        a1 = acc.a1;
        j0 += n;
      }
    }
    pw = rw3_partial_finish(praw, tb, tlen, r < nin);
    if (nin <= 64u) {
      deferred = true;  // the caller XORs pw into the held row, or into registers
    } else {
      rw3_partials_regs(a0, a1, lane, cn, tlen, pw);
    }
  }
  return RECOVER ? s.plen : rfl(wave_max11(mx));
}

template <bool RECOVER, int NW, int DIAG = 0, int B = (NW > 8 ? 8 : 16), bool V4 = false>
__global__ __launch_bounds__(64 * NW) void ragged_rpw3_kernel(RaggedArgs a, const uint32_t* bnd,
                                                              uint32_t nphase, uint32_t* phase_sync) {
  __shared__ u32x4 s_hold[kRwHoldW];
  __shared__ u32x4 s_ent[kRwEnt];
  __shared__ uint32_t s_next, s_alloc, s_nent;
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wv = rfl(tid >> 6);
  const uint32_t ncu = gridDim.x, cu = blockIdx.x;
  uint64_t c_work = 0, c_meet = 0, c_store = 0, c_idle = 0;
  u32x4 sink = {0u, 0u, 0u, 0u};
  auto stamp = [&]() -> uint64_t { return DIAG == 2 ? __builtin_amdgcn_s_memtime() : 0ull; };
  uint32_t* hold32 = reinterpret_cast<uint32_t*>(s_hold);
  if (tid == 0u) {
    s_alloc = 0u;
    s_nent = 0u;
  }
  for (uint32_t p = 0; p < nphase; ++p) {
    const uint32_t seg = p * ncu + cu;
    const uint32_t gs = rfl(bnd[seg]);
    const uint32_t ge = max(rfl(bnd[seg + 1]), gs);
    if (tid == 0u) s_next = 0u;
    __syncthreads();
    uint64_t t0 = stamp();
    auto ticket = [&]() -> uint32_t { return gs + rfl(atomicAdd(&s_next, 1u)) / 64u; };
    RwS s0, s1, s2;
    uint32_t g0 = ticket();
    if (g0 < ge) rw2_scalars<RECOVER>(a, g0, s0);
    uint32_t g1 = ticket();
    if (g1 < ge) rw2_scalars<RECOVER>(a, g1, s1);
    uint32_t tlo0 = 0, thi0 = 0, tlen0 = 0;
    if (g0 < ge) rw2_table<RECOVER>(a, s0, lane, 0u, tlo0, thi0, tlen0);
    while (g0 < ge) {
      const uint32_t g2 = ticket();
      uint32_t tlo1 = 0, thi1 = 0, tlen1 = 0;
      if (g1 < ge) rw2_table<RECOVER>(a, s1, lane, 0u, tlo1, thi1, tlen1);
      __builtin_amdgcn_sched_barrier(0);
      if (g2 < ge) rw2_scalars<RECOVER>(a, g2, s2);
      __builtin_amdgcn_sched_barrier(0);
      u32x4 a0, a1, pw;
      bool deferred;
      const uint32_t plen = rw3_reduce<RECOVER, B, V4>(a, s0, lane, tlo0, thi0, tlen0, a0, a1, pw, deferred);
      if (plen != 0xFFFFFFFFu) {
        const uint32_t nw = (plen + 15u) >> 4;
        const uint32_t e = rfl(atomicAdd(&s_nent, 1u)) / 64u;
        // lane 0 adds nw, the others 0: lane 0's old value is the row whatever
        // order the LDS takes the lanes in (x64 units assumed lane 0 first)
        const uint32_t h = rdl(atomicAdd(&s_alloc, lane == 0u ? nw : 0u), 0u);
        const uint64_t d = (uint64_t)(uintptr_t)a.out + s0.doff;
        if (e < kRwEnt && h + nw <= kRwHoldW) {
          if (lane < nw) s_hold[h + lane] = a0;
          if (lane < 32u && 64u + lane < nw) s_hold[h + 64u + lane] = a1;
          if (deferred) {
            wave_lds_order();
            // lane j: input j's partial window into row window len_j >> 4
            const uint32_t t = tlen0 >> 4;
            if (lane < s0.k && (tlen0 & 15u) != 0u) {
              uint32_t* w = hold32 + 4u * (h + t);
              __hip_atomic_fetch_xor(w, pw.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
              __hip_atomic_fetch_xor(w + 1, pw.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
              __hip_atomic_fetch_xor(w + 2, pw.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
              __hip_atomic_fetch_xor(w + 3, pw.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
          }
          if (lane == 0u) s_ent[e] = u32x4{(uint32_t)d, (uint32_t)(d >> 32), g0, plen | (h << 16)};
        } else {
          if (lane == 0u && e < kRwEnt) s_ent[e] = u32x4{0u, 0u, 0u, 0xFFFFFFFFu};
          if (deferred) rw3_partials_regs(a0, a1, lane, s0.k, tlen0, pw);
          rw2_store(d, plen, a0, a1, lane);
          if (!RECOVER && lane == 0u) a.parity_len_out[g0] = (uint16_t)plen;
        }
      }
      g0 = g1;
      s0 = s1;
      tlo0 = tlo1;
      thi0 = thi1;
      tlen0 = tlen1;
      g1 = g2;
      s1 = s2;
    }
    uint64_t t1 = stamp();
    if constexpr (DIAG == 2) c_work += t1 - t0;
    phase_meet(phase_sync, p + 1u);
    uint64_t t2 = stamp();
    if constexpr (DIAG == 2) c_meet += t2 - t1;
    const uint32_t ne = min(s_nent / 64u, kRwEnt);
    for (uint32_t e = wv; e < ne; e += NW) {
      const u32x4 en = s_ent[e];
      const uint32_t w3 = rfl(en.w);
      if (w3 == 0xFFFFFFFFu) continue;
      const uint32_t plen = w3 & 0xFFFFu, h = w3 >> 16, nw = (plen + 15u) >> 4;
      const u32x4 zero = {0u, 0u, 0u, 0u};
      const u32x4 a0 = lane < nw ? s_hold[h + lane] : zero;
      const u32x4 a1 = (lane < 32u && 64u + lane < nw) ? s_hold[h + 64u + lane] : zero;
      const uint64_t dst = ((uint64_t)rfl(en.y) << 32) | rfl(en.x);
      if constexpr (DIAG != 1) {
        rw2_store(dst, plen, a0, a1, lane);
        if (!RECOVER && lane == 0u) a.parity_len_out[rfl(en.z)] = (uint16_t)plen;
      } else {
        sink ^= a0 ^ a1;
      }
    }
    __syncthreads();
    if (tid == 0u) {
      s_alloc = 0u;
      s_nent = 0u;
    }
    uint64_t t3 = stamp();
    if constexpr (DIAG == 2) c_store += t3 - t2;
  }
  if constexpr (DIAG == 2) {
    if (lane == 0u) {
      uint64_t* o = g_stamps + ((uint64_t)blockIdx.x * NW + wv) * 8u;
      o[0] = c_work; o[1] = c_meet; o[2] = c_store; o[3] = c_idle;
    }
  }
  if constexpr (DIAG == 1) {
    if ((sink.x ^ sink.y ^ sink.z ^ sink.w) == 0x9E3779B9u) atomicOr(a.err, 0x80000000u);
  }
  phase_exit(phase_sync, nullptr);
}

}  // namespace
}  // namespace qfec

using qfec::RaggedArgs;

static uint64_t sm64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <typename T>
static T* up(const std::vector<T>& v) {
  T* d;
  CK(hipMalloc(&d, v.size() * sizeof(T)));
  CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

struct V {
  std::string name;
  bool rec;
  std::function<void(const RaggedArgs&)> run;
};

static uint32_t* g_bnd = nullptr;
static uint32_t* g_sync = nullptr;
static int g_ncu = 256;
static uint64_t g_total_pk = 0;

#define BLK(REC)                                                                           \
  [=](const RaggedArgs& a) {                                                               \
    hipLaunchKernelGGL((qfec::ragged_block_kernel<REC, 4, 8, 2, true, true, 0>),          \
                       dim3((uint32_t)((a.n_groups + 7) / 8)), dim3(256), 0, 0, a);        \
  }

// phases: packets per CU per phase ~ PPC
template <bool REC, int NW, int DIAG = 0>
static void run_rpw_n(const RaggedArgs& a, uint32_t ppc, bool bounds = true) {
  const uint32_t nphase = (uint32_t)std::max<uint64_t>(1, (g_total_pk + (uint64_t)ppc * g_ncu - 1) / ((uint64_t)ppc * g_ncu));
  const uint32_t nseg = nphase * g_ncu;
  if (bounds)
    hipLaunchKernelGGL(qfec::rw_bounds_kernel, dim3((nseg + 256) / 256), dim3(256), 0, 0, a.grp_ptr,
                       a.n_groups, nseg, g_bnd);
  hipLaunchKernelGGL((qfec::ragged_rpw_kernel<REC, NW, DIAG>), dim3(g_ncu), dim3(64 * NW), 0, 0, a,
                     (const uint32_t*)g_bnd, nphase, g_sync);
}

template <bool REC, int NW, int DIAG = 0>
static void run_rpw2_n(const RaggedArgs& a, uint32_t ppc, bool bounds = true) {
  const uint32_t nphase = (uint32_t)std::max<uint64_t>(1, (g_total_pk + (uint64_t)ppc * g_ncu - 1) / ((uint64_t)ppc * g_ncu));
  const uint32_t nseg = nphase * g_ncu;
  if (bounds)
    hipLaunchKernelGGL(qfec::rw_bounds_kernel, dim3((nseg + 256) / 256), dim3(256), 0, 0, a.grp_ptr,
                       a.n_groups, nseg, g_bnd);
  hipLaunchKernelGGL((qfec::ragged_rpw2_kernel<REC, NW, DIAG>), dim3(g_ncu), dim3(64 * NW), 0, 0, a,
                     (const uint32_t*)g_bnd, nphase, g_sync);
}

template <bool REC, int NW, int DIAG = 0, int B = (NW > 8 ? 8 : 16), bool V4 = false>
static void run_rpw3_n(const RaggedArgs& a, uint32_t ppc, bool bounds = true) {
  const uint32_t nphase = (uint32_t)std::max<uint64_t>(1, (g_total_pk + (uint64_t)ppc * g_ncu - 1) / ((uint64_t)ppc * g_ncu));
  const uint32_t nseg = nphase * g_ncu;
  if (bounds)
    hipLaunchKernelGGL(qfec::rw_bounds_kernel, dim3((nseg + 256) / 256), dim3(256), 0, 0, a.grp_ptr,
                       a.n_groups, nseg, g_bnd);
  hipLaunchKernelGGL((qfec::ragged_rpw3_kernel<REC, NW, DIAG, B, V4>), dim3(g_ncu), dim3(64 * NW), 0, 0, a,
                     (const uint32_t*)g_bnd, nphase, g_sync);
}

static uint64_t* g_stamps_d = nullptr;
template <bool REC, int NW>
static void stamps_report(const RaggedArgs& a, uint32_t ppc, const char* tag) {
  const size_t nw = (size_t)g_ncu * NW;
  if (!g_stamps_d) {
    CK(hipMalloc(&g_stamps_d, (size_t)g_ncu * 16 * 8 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(qfec::g_stamps), &g_stamps_d, sizeof(g_stamps_d)));
  }
  CK(hipMemset(g_stamps_d, 0, nw * 8 * 8));
  run_rpw3_n<REC, NW, 0, 16, true>(a, ppc);  // bounds
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  run_rpw3_n<REC, NW, 2, 16, true>(a, ppc, false);
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<uint64_t> h(nw * 8);
  CK(hipMemcpy(h.data(), g_stamps_d, nw * 64, hipMemcpyDeviceToHost));
  double sum[4] = {0};
  for (size_t w = 0; w < nw; ++w)
    for (int i = 0; i < 4; ++i) sum[i] += (double)h[w * 8 + i];
  double tot = 0;
  for (int i = 0; i < 3; ++i) tot += sum[i];
  const char* nm[3] = {"work", "meet", "store"};
  std::printf("stamps %s (NW%d PPC%u, %.1f us): per wave mean s_memtime ticks:", tag, NW, ppc,
              ms * 1e3);
  for (int i = 0; i < 3; ++i) std::printf(" %s %.0f (%.1f%%)", nm[i], sum[i] / nw, 100.0 * sum[i] / tot);
  std::printf("\n");
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const bool guard = argc > 5 && std::strcmp(argv[5], "guard") == 0;
  const uint64_t G = argc > 6 ? (uint64_t)atoll(argv[6]) : (1u << 20);
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  const uint64_t palign = argc > 3 ? (uint64_t)atoi(argv[3]) : 16u;
  const uint64_t slot = argc > 4 ? (uint64_t)atoi(argv[4]) : 1536u;
  const uint64_t seed = 0x51554944;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  g_ncu = prop.multiProcessorCount;
  std::vector<uint32_t> ptr{0};
  std::vector<uint16_t> len;
  std::vector<uint64_t> off, poff(G);
  std::vector<uint8_t> miss(G);
  uint64_t bytes = 0;
  double enc_alg = 0, rec_alg = 0;
  for (uint64_t g = 0; g < G; ++g) {
    const uint32_t k = 5 + (uint32_t)(sm64(seed ^ (0x6Bull << 56) ^ g) % 11);
    miss[g] = (uint8_t)(sm64(seed ^ (0x4Dull << 56) ^ g) % k);
    uint32_t mx = 0;
    double s = 0, sm = 0;
    for (uint32_t i = 0; i < k; ++i) {
      const uint32_t ln = 64 + (uint32_t)(sm64(seed ^ (0x4Cull << 56) ^ (g * 256 + i)) % 1287);
      len.push_back((uint16_t)ln);
      off.push_back(bytes);
      bytes += (ln + palign - 1) / palign * palign;
      s += ln;
      if (i != miss[g]) sm += ln;
      mx = std::max(mx, ln);
    }
    enc_alg += s + mx;
    rec_alg += sm + 2.0 * mx;
    ptr.push_back((uint32_t)len.size());
    poff[g] = g * slot;
  }
  g_total_pk = len.size();
  uint8_t* data;
  CK(hipMalloc(&data, bytes + 4096));
  CK(hipMemset(data, 0x77, bytes + 4096));  // gaps between aligned payloads: not zero
  uint64_t* d_off = up(off);
  uint16_t* d_len = up(len);
  uint32_t* d_ptr = up(ptr);
  uint64_t* d_poff = up(poff);
  uint8_t* d_miss = up(miss);
  CK(qfec::launch_synth_ragged(data, d_off, d_len, d_ptr, 0, G, seed, 0));
  const uint64_t OB = G * slot;
  uint8_t *par_ref, *out_ref, *buf;
  uint16_t *plen_ref, *plen_v;
  uint32_t* err;
  CK(hipMalloc(&par_ref, OB));
  CK(hipMalloc(&out_ref, OB));
  CK(hipMalloc(&buf, OB));
  CK(hipMalloc(&plen_ref, G * 2));
  CK(hipMalloc(&plen_v, G * 2));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&g_bnd, (size_t)4 * (G + 2)));
  CK(hipMalloc(&g_sync, 20 * 256));
  CK(hipMemset(g_sync, 0, 20 * 256));
  CK(hipMemset(err, 0, 4));
  CK(hipMemset(par_ref, 0xA5, OB));
  CK(hipMemset(out_ref, 0xA5, OB));

  RaggedArgs e{};
  e.bytes = data;
  e.pkt_off = d_off;
  e.pkt_len = d_len;
  e.grp_ptr = d_ptr;
  e.parity_off = d_poff;
  e.parity_len_out = plen_ref;
  e.out = par_ref;
  e.n_groups = G;
  e.err = err;
  RaggedArgs r = e;
  r.parity = par_ref;
  r.parity_len = plen_ref;
  r.missing = d_miss;
  r.out_off = d_poff;
  r.parity_len_out = nullptr;
  r.out = out_ref;
  BLK(false)(e);
  BLK(true)(r);
  CK(hipDeviceSynchronize());
  RaggedArgs ev = e, rv = r;
  ev.out = buf;
  ev.parity_len_out = plen_v;
  rv.out = buf;

  if (guard) {
#ifndef RW_GUARD
    std::printf("guard mode needs the RW_GUARD build\n");
    return 3;
#else
    qfec::RwDbg hd{};
    hd.lo[0] = (uint64_t)(uintptr_t)data; hd.hi[0] = hd.lo[0] + bytes + 4096;
    hd.lo[1] = (uint64_t)(uintptr_t)par_ref; hd.hi[1] = hd.lo[1] + OB;
    hd.lo[2] = (uint64_t)(uintptr_t)buf; hd.hi[2] = hd.lo[2] + OB;
    hd.lo[3] = (uint64_t)(uintptr_t)out_ref; hd.hi[3] = hd.lo[3] + OB;
    qfec::RwDbg* dd;
    CK(hipMalloc(&dd, sizeof(hd)));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(qfec::g_dbg), &dd, sizeof(dd)));
    for (int rec = 0; rec < 2; ++rec) {
      CK(hipMemcpy(dd, &hd, sizeof(hd), hipMemcpyHostToDevice));
      CK(hipMemset(buf, 0xA5, OB));
      CK(hipMemset(err, 0, 4));
      const RaggedArgs& a = rec ? rv : ev;
      const uint32_t ppc = 1000;
      const uint32_t nphase = (uint32_t)std::max<uint64_t>(1, (g_total_pk + (uint64_t)ppc * g_ncu - 1) / ((uint64_t)ppc * g_ncu));
      const uint32_t nseg = nphase * g_ncu;
      hipLaunchKernelGGL(qfec::rw_bounds_kernel, dim3((nseg + 256) / 256), dim3(256), 0, 0, a.grp_ptr,
                         a.n_groups, nseg, g_bnd);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      std::vector<uint32_t> hb(nseg + 1);
      CK(hipMemcpy(hb.data(), g_bnd, 4 * (nseg + 1), hipMemcpyDeviceToHost));
      bool mono = hb[0] == 0 && hb[nseg] == G;
      size_t mx = 0;
      for (uint32_t q = 0; q < nseg; ++q) {
        mono = mono && hb[q] <= hb[q + 1];
        mx = std::max<size_t>(mx, hb[q + 1] - hb[q]);
      }
      std::printf("guard %s: nphase %u nseg %u bounds monotone %d, max groups per segment %zu\n",
                  rec ? "recover" : "encode", nphase, nseg, (int)mono, mx);
      if (!mono) return 4;
      if (rec) hipLaunchKernelGGL((qfec::ragged_rpw3_kernel<true, 16, 0, 16, true>), dim3(g_ncu), dim3(1024), 0, 0, a,
                                  (const uint32_t*)g_bnd, nphase, g_sync);
      else hipLaunchKernelGGL((qfec::ragged_rpw3_kernel<false, 16, 0, 16, true>), dim3(g_ncu), dim3(1024), 0, 0, a,
                              (const uint32_t*)g_bnd, nphase, g_sync);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      qfec::RwDbg r_{};
      CK(hipMemcpy(&r_, dd, sizeof(r_), hipMemcpyDeviceToHost));
      uint32_t e_h = 0;
      CK(hipMemcpy(&e_h, err, 4, hipMemcpyDeviceToHost));
      std::vector<uint8_t> h_ref(OB), h_v(OB);
      CK(hipMemcpy(h_ref.data(), rec ? out_ref : par_ref, OB, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h_v.data(), buf, OB, hipMemcpyDeviceToHost));
      size_t badb = 0;
      for (size_t i = 0; i < OB; ++i) badb += h_ref[i] != h_v[i];
      std::printf("guard %s: bad access %u (where %u, addr 0x%llx, thread %u, group %u); err %u; %zu bad bytes\n",
                  rec ? "recover" : "encode", r_.bad, r_.where, (unsigned long long)r_.addr, r_.lane, r_.g,
                  e_h, badb);
    }
    return 0;
#endif
  }
  std::vector<V> vs;
  vs.push_back({"product block encode", false, BLK(false)});
  vs.push_back({"rpw3 NW16 P1000 encode", false, [](const RaggedArgs& a) { run_rpw3_n<false, 16>(a, 1000); }});
  vs.push_back({"rpw4 NW16 B16 encode", false, [](const RaggedArgs& a) { run_rpw3_n<false, 16, 0, 16, true>(a, 1000); }});
  vs.push_back({"rpw4 NW12 B16 encode", false, [](const RaggedArgs& a) { run_rpw3_n<false, 12, 0, 16, true>(a, 1000); }});
  vs.push_back({"rpw4 NW16 B8 encode", false, [](const RaggedArgs& a) { run_rpw3_n<false, 16, 0, 8, true>(a, 1000); }});
  vs.push_back({"product block recover", true, BLK(true)});
  vs.push_back({"rpw4 NW16 B16 recover", true, [](const RaggedArgs& a) { run_rpw3_n<true, 16, 0, 16, true>(a, 1000); }});
  vs.push_back({"rpw4 NW12 B16 recover", true, [](const RaggedArgs& a) { run_rpw3_n<true, 12, 0, 16, true>(a, 1000); }});
  std::vector<V> diag;
  diag.push_back({"rpw4 NW16 B16 enc, no stores", false,
                  [](const RaggedArgs& a) { run_rpw3_n<false, 16, 1, 16, true>(a, 1000); }});
  std::vector<uint8_t> h_ref(OB), h_v(OB);
  std::vector<uint16_t> hp_ref(G), hp_v(G);
  CK(hipMemcpy(hp_ref.data(), plen_ref, G * 2, hipMemcpyDeviceToHost));
  bool all_ok = true;
  for (const V& v : vs) {
    CK(hipMemset(buf, 0xA5, OB));
    CK(hipMemset(plen_v, 0, G * 2));
    CK(hipMemset(err, 0, 4));
    v.run(v.rec ? rv : ev);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h_ref.data(), v.rec ? out_ref : par_ref, OB, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h_v.data(), buf, OB, hipMemcpyDeviceToHost));
    uint32_t e_h = 0;
    CK(hipMemcpy(&e_h, err, 4, hipMemcpyDeviceToHost));
    size_t bad = 0, first = (size_t)-1;
    for (size_t i = 0; i < OB; ++i)
      if (h_ref[i] != h_v[i]) {
        if (first == (size_t)-1) first = i;
        ++bad;
      }
    bool ok = bad == 0 && e_h == 0;
    if (!v.rec) {
      CK(hipMemcpy(hp_v.data(), plen_v, G * 2, hipMemcpyDeviceToHost));
      ok = ok && hp_ref == hp_v;
    }
    std::printf("check %-30s == product: %s (err %u, %zu bad bytes, first at %zd = group %zd)\n",
                v.name.c_str(), ok ? "yes" : "NO", e_h, bad, (ssize_t)first,
                first == (size_t)-1 ? (ssize_t)-1 : (ssize_t)(first / slot));
    all_ok = all_ok && ok;
  }
  if (!all_ok) return 2;
  stamps_report<false, 16>(ev, 1000, "encode");
  stamps_report<true, 16>(rv, 1000, "recover");
  for (const V& v : diag) vs.push_back(v);

  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  std::vector<std::vector<float>> ms(vs.size());
  for (int rd = 0; rd < rounds; ++rd) {
    for (size_t i = 0; i < vs.size(); ++i) {
      const V& v = vs[i];
      v.run(v.rec ? rv : ev);  // warm
      CK(hipEventRecord(t0, 0));
      for (int q = 0; q < reps; ++q) v.run(v.rec ? rv : ev);
      CK(hipEventRecord(t1, 0));
      CK(hipEventSynchronize(t1));
      float m = 0;
      CK(hipEventElapsedTime(&m, t0, t1));
      ms[i].push_back(m / reps);
    }
  }
  std::printf("\nconfigs[3]: %llu groups, k 5-15, len 64-1350, palign %llu, slot %llu, %d CUs; "
              "algorithmic GB: encode %.3f, recover %.3f\n",
              (unsigned long long)G, (unsigned long long)palign, (unsigned long long)slot, g_ncu,
              enc_alg / 1e9, rec_alg / 1e9);
  for (size_t i = 0; i < vs.size(); ++i) {
    std::vector<float> s = ms[i];
    std::sort(s.begin(), s.end());
    const double med = s[s.size() / 2] * 1e-3;
    const double gbs = (vs[i].rec ? rec_alg : enc_alg) / med / 1e9;
    std::printf("%-32s median %8.1f us  min %8.1f us  %7.1f GB/s  %.4f of 8 TB/s\n",
                vs[i].name.c_str(), med * 1e6, s[0] * 1e3, gbs, gbs / 8000.0);
  }
  return 0;
}
