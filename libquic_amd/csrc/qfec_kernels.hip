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

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------
// Fixed shape, L >= 16.
// ---------------------------------------------------------------------------
template <int KC, bool RECOVER, bool NT>
__global__ __launch_bounds__(kBlock) void fixed_xor_kernel(FixedArgs a, uint32_t C,
                                                           uint32_t gpb) {
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;  // group within the workgroup
  const uint32_t t = tid - gl * C;
  const uint64_t g = (uint64_t)blockIdx.x * gpb + gl;
  if (gl >= gpb || g >= a.n_groups) return;
  const uint32_t off = min(t * 16u, a.L - 16u);
  const uint8_t* src = a.rows + g * a.group_stride + off;
  const uint32_t k = KC > 0 ? (uint32_t)KC : a.k;

  u32x4 acc = {0u, 0u, 0u, 0u};
  if constexpr (RECOVER) {
    const uint32_t m = a.missing[g];
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
// a word select by sh/4, then v_alignbyte_b32 by sh%4.
__device__ __forceinline__ u32x4 shr_bytes_bf(u32x4 v, uint32_t sh) {
  const uint32_t q = sh >> 2, r = sh & 3u;
  const uint32_t s0 = q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
  const uint32_t s1 = q == 0 ? v.y : q == 1 ? v.z : q == 2 ? v.w : 0u;
  const uint32_t s2 = q == 0 ? v.z : q == 1 ? v.w : 0u;
  const uint32_t s3 = q == 0 ? v.w : 0u;
  u32x4 o;
  o.x = __builtin_amdgcn_alignbyte(s1, s0, r);
  o.y = __builtin_amdgcn_alignbyte(s2, s1, r);
  o.z = __builtin_amdgcn_alignbyte(s3, s2, r);
  o.w = __builtin_amdgcn_alignbyte(0u, s3, r);
  return o;
}

// Bytes [win, win+16) of a zero-padded packet of `len` bytes, len >= 16.
// Always ONE 16-byte load inside the packet (no exec-masked branch): a window
// that crosses the packet end loads the 16 bytes ending at its last byte and
// shifts them down; a window past the end is zeroed by a select.
template <bool NT>
__device__ __forceinline__ u32x4 window16(const uint8_t* row, uint32_t len, uint32_t win) {
  const bool full = win + 16u <= len;
  u32x4 v = ld16t<NT>(row + (full ? win : len - 16u));
  const u32x4 z = {0u, 0u, 0u, 0u};
  v = win < len ? v : z;
  return full ? v : shr_bytes_bf(v, min(win + 16u - len, 15u));
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

// Lane l of the wave owns parity windows at 16*l and 16*l + 1024 (plen <= 1452
// needs at most two), clamped so the last window ends at parity_len.  The
// group's packet lengths/offsets are loaded once, one packet per lane, and
// broadcast per row with v_readlane (no per-row scalar-load latency).
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
  uint32_t plen;
  uint32_t m = 0xFFFFFFFFu;
  if constexpr (RECOVER) {
    plen = a.parity_len[g];
    m = a.missing[g];
    if (m >= k) {
      if (lane == 0) atomicOr(a.err, kErrMissingIndex);
      return;
    }
    if (plen == 0u || plen > kMaxPacket) {
      if (lane == 0) atomicOr(a.err, kErrParityLength);
      return;
    }
    uint32_t bad = 0;
    for (uint32_t i = lane; i < k; i += 64u) {
      if (i == m) continue;  // the lost packet's entries are never read
      const uint32_t l = a.pkt_len[p0 + i];
      bad |= (l == 0u || l > plen) ? 1u : 0u;
    }
    if (wave_or(bad)) {
      if (lane == 0) atomicOr(a.err, kErrPacketLength);
      return;
    }
  } else {
    uint32_t mx = 0, bad = 0;
    for (uint32_t i = lane; i < k; i += 64u) {
      const uint32_t l = a.pkt_len[p0 + i];
      mx = max(mx, l);
      bad |= (l == 0u || l > kMaxPacket) ? 1u : 0u;
    }
    mx = wave_max(mx);
    if (wave_or(bad)) {
      if (lane == 0) atomicOr(a.err, kErrPacketLength);
      return;
    }
    plen = mx;
  }
  const uint8_t* par = RECOVER ? a.parity + a.parity_off[g] : nullptr;
  uint8_t* dst = a.out + (RECOVER ? a.out_off[g] : a.parity_off[g]);

  if (plen >= 16u) {
    const uint32_t w = lane * 16u;
    const uint32_t win0 = min(w, plen - 16u);
    const uint32_t win1 = min(w + 1024u, plen - 16u);
    const bool two = plen > 1024u;  // wave-uniform
    const uint32_t lo1 = min(1024u, plen - 16u);  // lowest byte any second window covers
    u32x4 acc0 = {0u, 0u, 0u, 0u}, acc1 = {0u, 0u, 0u, 0u};
    if constexpr (RECOVER) {
      acc0 = ld16t<NT>(par + win0);
      if (two) acc1 = ld16t<NT>(par + win1);
    }
    for (uint32_t c = 0; c < k; c += 64u) {
      const uint32_t cnt = min(64u, k - c);
      uint32_t lenr = 0, offlo = 0, offhi = 0;
      if (lane < cnt && c + lane != m) {
        lenr = a.pkt_len[p0 + c + lane];
        const uint64_t o = a.pkt_off[p0 + c + lane];
        offlo = (uint32_t)o;
        offhi = (uint32_t)(o >> 32);
      }
#pragma unroll 2
      for (uint32_t i = 0; i < cnt; ++i) {
        const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)lenr, (int)i);
        if (len == 0u) continue;  // the lost packet (wave-uniform)
        const uint64_t off = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)offhi, (int)i)
                              << 32) |
                             (uint32_t)__builtin_amdgcn_readlane((int)offlo, (int)i);
        const uint8_t* row = a.bytes + off;
        if (len >= 16u) {
          acc0 ^= window16<NT>(row, len, win0);
          if (two && len > lo1) acc1 ^= window16<NT>(row, len, win1);
        } else {
          acc0 ^= window16_small(row, len, win0);
        }
      }
    }
    if (w < plen) st16t<NT>(dst + win0, acc0);
    if (two && w + 1024u < plen) st16t<NT>(dst + win1, acc1);
  } else {
    // Whole group fits in one window: one lane per byte.
    if (lane < plen) {
      uint8_t acc = RECOVER ? par[lane] : (uint8_t)0;
      for (uint32_t i = 0; i < k; ++i) {
        if (i == m) continue;
        const uint32_t len = a.pkt_len[p0 + i];
        if (lane < len) acc ^= a.bytes[a.pkt_off[p0 + i] + lane];
      }
      dst[lane] = acc;
    }
  }
  if constexpr (!RECOVER) {
    if (lane == 0) a.parity_len_out[g] = (uint16_t)plen;
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

template <bool RECOVER, bool NT>
hipError_t launch_fixed_k(const FixedArgs& a, uint32_t C, uint32_t gpb, uint64_t blocks,
                          hipStream_t s) {
  switch (a.k) {
#define QFEC_K_CASE(KV)                                                                     \
  case KV:                                                                                   \
    hipLaunchKernelGGL((fixed_xor_kernel<KV, RECOVER, NT>), dim3((uint32_t)blocks),          \
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
      hipLaunchKernelGGL((fixed_xor_kernel<0, RECOVER, NT>), dim3((uint32_t)blocks),
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
    if (recover)
      e = nontemporal ? launch_fixed_k<true, true>(a, C, gpb, blocks, s)
                      : launch_fixed_k<true, false>(a, C, gpb, blocks, s);
    else
      e = nontemporal ? launch_fixed_k<false, true>(a, C, gpb, blocks, s)
                      : launch_fixed_k<false, false>(a, C, gpb, blocks, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_ragged(const RaggedArgs& a0, bool recover, hipStream_t s) {
  if (a0.n_groups == 0) return hipSuccess;
  const uint64_t gpb = kBlock / 64;
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
