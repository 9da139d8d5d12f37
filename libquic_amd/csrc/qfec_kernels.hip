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
//  * Ragged CSR batches: one wave per group, lanes own 16-byte windows of the
//    parity; a packet shorter than the window is loaded as the 16 bytes that
//    end at its last byte and shifted down (zero fill), so again no load leaves
//    the packet.
#include "qfec_internal.h"

#include <algorithm>

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

// ---------------------------------------------------------------------------
// Fixed shape, L >= 16.
// ---------------------------------------------------------------------------
// SM (recover, gpb <= 8): lost-slot indices by scalar loads, see below.
template <int KC, bool RECOVER, bool NT, bool SM>
__global__ __launch_bounds__(kBlock) void fixed_xor_kernel(FixedArgs a, uint32_t C,
                                                           uint32_t gpb) {
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;  // group within the workgroup
  const uint32_t t = tid - gl * C;
  const uint64_t gb = (uint64_t)blockIdx.x * gpb;
  const uint64_t g = gb + gl;
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
      uint32_t i = 0;
      for (; i + 8 <= k; i += 8) {
        u32x4 v[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
          const uint8_t* p = (i + u == m) ? par : src + (i + u) * a.row_stride;
          v[u] = ld16t<NT>(p);
        }
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) acc ^= v[u];
      }
      for (; i < k; ++i) {
        const uint8_t* p = (i == m) ? par : src + i * a.row_stride;
        acc ^= ld16t<NT>(p);
      }
    }
  } else {
    if constexpr (KC > 0) {
#pragma unroll
      for (uint32_t i = 0; i < (uint32_t)KC; ++i) acc ^= ld16t<NT>(src + i * a.row_stride);
    } else {
      uint32_t i = 0;
      for (; i + 8 <= k; i += 8) {
        u32x4 v[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) v[u] = ld16t<NT>(src + (i + u) * a.row_stride);
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) acc ^= v[u];
      }
      for (; i < k; ++i) acc ^= ld16t<NT>(src + i * a.row_stride);
    }
  }
  st16t<NT>(a.out + g * a.out_stride + off, acc);
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
  a.out[g * a.out_stride + j] = acc;
}

// ---------------------------------------------------------------------------
// Ragged CSR: one wave per group.
// ---------------------------------------------------------------------------
// Right shift of a 16-byte vector by sh bytes (0..15), zero fill, branch-free:
// one 64-bit select for the 8-byte step, then 64-bit funnel shifts
// ((hi << 1) << (63 - s) is the UB-free hi << (64 - s), 0 at s = 0).
// Written without multi-way selects: the compiler turns those into divergent
// branches, each of which waits for the load (vmcnt(0)) and serialises rows.
__device__ __forceinline__ u32x4 shr_bytes_bf(u32x4 v, uint32_t sh) {
  uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
  uint64_t hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
  const bool big = sh >= 8u;
  lo = big ? hi : lo;
  hi = big ? 0ull : hi;
  const uint32_t s = (sh & 7u) * 8u;
  lo = (lo >> s) | ((hi << 1) << (63u - s));
  hi = hi >> s;
  u32x4 o;
  o.x = (uint32_t)lo;
  o.y = (uint32_t)(lo >> 32);
  o.z = (uint32_t)hi;
  o.w = (uint32_t)(hi >> 32);
  return o;
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

// XOR rows [0, cnt) of one 64-packet metadata chunk into the lane's windows,
// 8 rows per batch with every load of the batch in flight before the first
// XOR (the loop used to wait on each row's load in turn).  Every packet of
// the group is >= 16 bytes on this path.  Row j's length and offset come from
// lane j's registers via v_readlane (wave-uniform scalars).
// XOR rows [0, cnt) of one 64-packet metadata chunk into the lane's two
// windows.  Rows go in batches of B with every load of the batch issued before
// the first XOR; a lane loads only where its window overlaps the packet
// (exec-masked), so lanes past the packet end and the second window of short
// packets issue no memory requests at all.  Every packet is >= 16 B here.
template <bool NT, int B>
__device__ __forceinline__ void ragged_rows(const uint8_t* bytes, uint32_t lenr, uint32_t offlo,
                                            uint32_t offhi, uint32_t cnt, uint32_t win0,
                                            uint32_t win1, u32x4& acc0, u32x4& acc1) {
  for (uint32_t i = 0; i < cnt; i += B) {
    u32x4 r0[B], r1[B];
#pragma unroll
    for (int u = 0; u < B; ++u) {
      r0[u] = u32x4{0u, 0u, 0u, 0u};
      r1[u] = u32x4{0u, 0u, 0u, 0u};
      if (i + u < cnt) {  // wave-uniform
        const uint32_t j = i + u;
        const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)lenr, (int)j);
        const uint64_t off =
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)offhi, (int)j) << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)offlo, (int)j);
        const uint8_t* row = bytes + off;
        if (win0 < len) r0[u] = ld16t<NT>(row + (win0 + 16u <= len ? win0 : len - 16u));
        if (win1 < len) r1[u] = ld16t<NT>(row + (win1 + 16u <= len ? win1 : len - 16u));
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of their first use
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const uint32_t j = min(i + u, cnt - 1u);
      const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)lenr, (int)j);
      acc0 ^= shr_bytes_bf(r0[u], win0 + 16u <= len ? 0u : min(win0 + 16u - len, 15u));
      acc1 ^= shr_bytes_bf(r1[u], win1 + 16u <= len ? 0u : min(win1 + 16u - len, 15u));
    }
  }
}

// One wave per group.  Lane l owns parity windows at 16*l and 16*l + 1024
// (parity_len <= 1452 needs at most two), clamped so the last window ends at
// parity_len.  The group's RECEIVED packets are numbered r = 0..kr-1 (recover
// skips the lost index m: packet p = r + (r >= m)), so the lost packet's
// entries are never read and the row loop has no holes.  Packet metadata is
// loaded once, one packet per lane, and broadcast with v_readlane.
template <bool RECOVER, bool NT>
__global__ __launch_bounds__(kBlock) void ragged_xor_kernel(RaggedArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t g = (uint64_t)blockIdx.x * (kBlock / 64) +
                     (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (g >= a.n_groups) return;
  const uint32_t p0 = a.grp_ptr[g];
  const uint32_t p1 = a.grp_ptr[g + 1];
  const uint32_t k = p1 - p0;
  if (p1 < p0 || k == 0u || k > 255u) {
    if (lane == 0) atomicOr(a.err, kErrGroupSize);
    return;
  }
  uint32_t m = 0xFFFFFFFFu, plen = 0;
  if constexpr (RECOVER) {
    m = a.missing[g];
    plen = a.parity_len[g];
    if (m >= k) {
      if (lane == 0) atomicOr(a.err, kErrMissingIndex);
      return;
    }
    if (plen == 0u || plen > kMaxPacket) {
      if (lane == 0) atomicOr(a.err, kErrParityLength);
      return;
    }
  }
  const uint32_t kr = RECOVER ? k - 1u : k;  // received packets
  // metadata of received packets 0..63 (every group of <= 64 packets)
  uint32_t lenr = 0, offlo = 0, offhi = 0;
  if (lane < kr) {
    const uint32_t p = p0 + lane + (lane >= m ? 1u : 0u);
    lenr = a.pkt_len[p];
    const uint64_t o = a.pkt_off[p];
    offlo = (uint32_t)o;
    offhi = (uint32_t)(o >> 32);
  }
  // validation + parity length (+ whether any packet is shorter than 16 B)
  uint32_t mx = lenr, bad = 0, small = 0;
  if (lane < kr) {
    bad = (lenr == 0u || lenr > (RECOVER ? plen : kMaxPacket)) ? 1u : 0u;
    small = lenr < 16u ? 1u : 0u;
  }
  for (uint32_t r = 64u + lane; r < kr; r += 64u) {
    const uint32_t l = a.pkt_len[p0 + r + (r >= m ? 1u : 0u)];
    mx = max(mx, l);
    bad |= (l == 0u || l > (RECOVER ? plen : kMaxPacket)) ? 1u : 0u;
    small |= l < 16u ? 1u : 0u;
  }
  if (wave_any(bad != 0u)) {
    if (lane == 0) atomicOr(a.err, kErrPacketLength);
    return;
  }
  if constexpr (!RECOVER) {
    plen = wave_max11(min(mx, 2047u));
    if (lane == 0) a.parity_len_out[g] = (uint16_t)plen;
  }
  const bool any_small = wave_any(small != 0u);
  const uint8_t* par = RECOVER ? a.parity + a.parity_off[g] : nullptr;
  uint8_t* dst = a.out + (RECOVER ? a.out_off[g] : a.parity_off[g]);
  const uint32_t w = lane * 16u;

  if (plen >= 16u && !any_small) {
    // windows past parity_len are parked at 0xFFFF (no packet reaches them)
    const uint32_t win0 = w < plen ? min(w, plen - 16u) : 0xFFFFu;
    const uint32_t win1 = w + 1024u < plen ? min(w + 1024u, plen - 16u) : 0xFFFFu;
    u32x4 acc0 = {0u, 0u, 0u, 0u}, acc1 = {0u, 0u, 0u, 0u};
    if constexpr (RECOVER) {
      if (win0 < plen) acc0 = ld16t<NT>(par + win0);
      if (win1 < plen) acc1 = ld16t<NT>(par + win1);
    }
    for (uint32_t c = 0; c < kr; c += 64u) {
      if (c > 0) {  // groups of more than 64 packets: next metadata chunk
        lenr = offlo = offhi = 0;
        const uint32_t r = c + lane;
        if (r < kr) {
          const uint32_t p = p0 + r + (r >= m ? 1u : 0u);
          lenr = a.pkt_len[p];
          const uint64_t o = a.pkt_off[p];
          offlo = (uint32_t)o;
          offhi = (uint32_t)(o >> 32);
        }
      }
      ragged_rows<NT, 4>(a.bytes, lenr, offlo, offhi, min(64u, kr - c), win0, win1, acc0, acc1);
    }
    if (win0 < plen) st16t<NT>(dst + win0, acc0);
    if (win1 < plen) st16t<NT>(dst + win1, acc1);
  } else if (plen >= 16u) {
    // Some packet is shorter than 16 bytes (rare): per-row generic windows.
    for (uint32_t w0 = 0; w0 < plen; w0 += 1024u) {
      const uint32_t win = min(w + w0, plen - 16u);
      u32x4 acc = {0u, 0u, 0u, 0u};
      if constexpr (RECOVER) acc = ld16(par + win);
      for (uint32_t r = 0; r < kr; ++r) {
        const uint32_t p = p0 + r + (r >= m ? 1u : 0u);
        const uint32_t len = a.pkt_len[p];
        const uint8_t* row = a.bytes + a.pkt_off[p];
        acc ^= (len >= 16u) ? window16<false>(row, len, win) : window16_small(row, len, win);
      }
      if (w + w0 < plen) st16(dst + win, acc);
    }
  } else {
    // Whole group fits in one window: one lane per byte.
    if (lane < plen) {
      uint8_t acc = RECOVER ? par[lane] : (uint8_t)0;
      for (uint32_t r = 0; r < kr; ++r) {
        const uint32_t p = p0 + r + (r >= m ? 1u : 0u);
        const uint32_t len = a.pkt_len[p];
        if (lane < len) acc ^= a.bytes[a.pkt_off[p] + lane];
      }
      dst[lane] = acc;
    }
  }
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

template <bool RECOVER, bool NT, bool SM>
hipError_t launch_fixed_k(const FixedArgs& a, uint32_t C, uint32_t gpb, uint64_t blocks,
                          hipStream_t s) {
  switch (a.k) {
#define QFEC_K_CASE(KV)                                                                     \
  case KV:                                                                                   \
    hipLaunchKernelGGL((fixed_xor_kernel<KV, RECOVER, NT, SM>), dim3((uint32_t)blocks),      \
                       dim3(kBlock), 0, s, a, C, gpb);                                       \
    break;
    QFEC_K_CASE(2)
    QFEC_K_CASE(4)
    QFEC_K_CASE(5)
    QFEC_K_CASE(8)
    QFEC_K_CASE(10)
    QFEC_K_CASE(16)
#undef QFEC_K_CASE
    default:
      hipLaunchKernelGGL((fixed_xor_kernel<0, RECOVER, NT, SM>), dim3((uint32_t)blocks),
                         dim3(kBlock), 0, s, a, C, gpb);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_fixed(const FixedArgs& a0, bool nontemporal, hipStream_t s) {
  const bool recover = a0.parity != nullptr;
  if (a0.n_groups == 0) return hipSuccess;
  if (a0.L < 16u) {
    const uint64_t maxg = ((uint64_t)1 << 31) * kBlock / a0.L / 2;
    for (uint64_t g = 0; g < a0.n_groups; g += maxg) {
      FixedArgs a = a0;
      a.n_groups = std::min<uint64_t>(maxg, a0.n_groups - g);
      a.rows = a0.rows + g * a0.group_stride;
      if (recover) {
        a.parity = a0.parity + g * a0.parity_stride;
        a.missing = a0.missing + g;
      }
      a.out = a0.out + g * a0.out_stride;
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
  const uint64_t max_blocks = 0x7FFFFFFFull;
  const uint64_t maxg = max_blocks * gpb;
  for (uint64_t g = 0; g < a0.n_groups; g += maxg) {
    FixedArgs a = a0;
    a.n_groups = std::min<uint64_t>(maxg, a0.n_groups - g);
    a.rows = a0.rows + g * a0.group_stride;
    if (recover) {
      a.parity = a0.parity + g * a0.parity_stride;
      a.missing = a0.missing + g;
    }
    a.out = a0.out + g * a0.out_stride;
    const uint64_t blocks = (a.n_groups + gpb - 1) / gpb;
    hipError_t e;
    if (recover && gpb <= 8u)
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

hipError_t launch_ragged(const RaggedArgs& a0, bool recover, hipStream_t s) {
  if (a0.n_groups == 0) return hipSuccess;
  const uint64_t gpb = kBlock / 64;  // one wave per group
  const uint64_t maxg = 0x7FFFFFFFull * gpb;
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
    if (recover)
      hipLaunchKernelGGL((ragged_xor_kernel<true, true>), dim3((uint32_t)blocks), dim3(kBlock), 0,
                         s, a);
    else
      hipLaunchKernelGGL((ragged_xor_kernel<false, true>), dim3((uint32_t)blocks), dim3(kBlock),
                         0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_xor_into(const uint8_t* in, uint64_t n, uint8_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n / 16u + kBlock - 1) / kBlock;
  if (blocks < 1) blocks = 1;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(xor_into_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, s, in, n, out);
  return hipGetLastError();
}

hipError_t launch_synth_fixed(uint8_t* rows, uint32_t k, uint32_t L, uint64_t row_stride,
                              uint64_t group_stride, uint64_t g0, uint64_t n, uint64_t seed,
                              hipStream_t s) {
  const uint64_t total_rows = n * k;
  const uint64_t chunk = 0x40000000ull;  // rows per launch
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
  const uint64_t chunk = 0x40000000ull;
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
