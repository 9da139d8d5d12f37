// tune_rphase.hip — VERDICT r4 item 1: a grid-phased ragged kernel whose
// completed parities are held in registers, LDS as transient staging.
//
// ragged_phase_kernel (below): a persistent grid of one 4-wave workgroup per
// CU walks the batch in phases.  In phase p wave w of CU c owns S group slots,
// group p*S*ncu*4 + (j*ncu + c)*4 + w for slot j, so step j of all CUs covers
// one contiguous window of the batch (the fixed phased kernel's order).  Per
// group a descriptor (a pre-pass, rdesc_kernel: the group's inputs as at most
// 3 runs of 16-B chunks, each input's byte offset in the staged image, the
// output row and length) tells the wave what to stage: global_load_lds_dwordx4
// of the group's chunks into the wave's LDS ring (no per-window lookup, no
// VGPR round trip), several groups ahead (counted vmcnt), then the group is
// reduced out of LDS in the static window mapping -- lane t holds parity
// window t (set 0, 4 VGPRs per slot) and, for windows 64-90, lane t of the
// slot pair's shared set 1 (lanes 0-31 the even slot, 32-63 the odd one: 2
// VGPRs per slot) -- and the finished parity stays in registers (VGPRs and
// AGPRs: one wave per SIMD has 512) until the grid meets and stores the
// phase's parity rows.  The HBM then sees read phases and write phases.
//
//   tune_rphase [reps=5] [rounds=3] [palign=16] [slot=1536]
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

constexpr int kRpMaxIn = 16;  // inputs per group in the fast path
__device__ uint64_t* g_stamps;  // DIAG 2: per wave cycle counts

// 128-byte group descriptor (one scalar-cache line pair).
struct __attribute__((aligned(16))) RDesc {
  uint64_t base[3];   // run r: global address of its first 16-B chunk
  uint32_t nchunk;    // chunks of the staged image (all runs)
  uint32_t s12;       // first image chunk of run 1 (lo 16) and run 2 (hi 16); 0xFFFF: none
  uint64_t dst;       // output row (absolute address)
  uint32_t info;      // n_in (bits 0-7) | plen (bits 8-23) | fast (bit 31)
  uint32_t pad;
  uint16_t img[kRpMaxIn];  // byte offset of input i in the image
  uint16_t len[kRpMaxIn];  // input lengths
  uint32_t pad2[4];
};
static_assert(sizeof(RDesc) == 128, "descriptor: 128 B");

// One thread per group.  Inputs in order: encode the k packets; recover the
// k-1 received packets, then the parity row.  A run continues while the next
// input starts at most 15 bytes past the previous one's end.
template <bool RECOVER>
__global__ __launch_bounds__(256) void rdesc_kernel(RaggedArgs a, RDesc* D, uint32_t ring_chunks) {
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= a.n_groups) return;
  const uint32_t p0 = a.grp_ptr[g], k = a.grp_ptr[g + 1] - p0;
  RDesc d;
  bool fast = k >= 1 && k <= (uint32_t)kRpMaxIn;
  uint32_t m = 0xFFFFFFFFu, plen = 0;
  if constexpr (RECOVER) {
    m = a.missing[g];
    plen = a.parity_len[g];
    fast = fast && m < k && plen >= 16 && plen <= kMaxPacket;
  }
  uint32_t nin = 0, nruns = 0, S = 0, mx = 0, s1 = 0xFFFFu, s2 = 0xFFFFu;
  uint64_t ra = 0, re = 0;
  d.base[0] = d.base[1] = d.base[2] = 0;
  auto add = [&](uint64_t addr, uint32_t len) {
    if (!fast) return;
    if (len == 0 || len > kMaxPacket || (RECOVER && len > plen)) {
      fast = false;
      return;
    }
    if (nruns == 0 || !(addr >= re && addr - re < 16u)) {
      if (nruns > 0) S += (uint32_t)(((re + 15u) >> 4) - (ra >> 4));
      if (nruns == 3) {
        fast = false;
        return;
      }
      d.base[nruns] = addr & ~15ull;
      if (nruns == 1) s1 = S;
      if (nruns == 2) s2 = S;
      ra = addr;
      ++nruns;
    }
    d.img[nin] = (uint16_t)(S * 16u + (uint32_t)(addr - (ra & ~15ull)));
    d.len[nin] = (uint16_t)len;
    re = addr + len;
    mx = max(mx, len);
    ++nin;
  };
  if (fast) {
    for (uint32_t i = 0; i < k; ++i) {
      if (RECOVER && i == m) continue;
      add((uint64_t)(uintptr_t)a.bytes + a.pkt_off[p0 + i], a.pkt_len[p0 + i]);
    }
    if constexpr (RECOVER) add((uint64_t)(uintptr_t)a.parity + a.parity_off[g], plen);
  }
  if (fast) S += (uint32_t)(((re + 15u) >> 4) - (ra >> 4));
  if (!RECOVER) plen = mx;
  fast = fast && plen >= 16 && S + 64u <= ring_chunks && S * 16u < 65536u;
  for (uint32_t i = nin; i < (uint32_t)kRpMaxIn; ++i) d.img[i] = d.len[i] = 0;
  d.nchunk = fast ? S : 0;
  d.s12 = s1 | (s2 << 16);
  d.dst = (uint64_t)(uintptr_t)a.out + (RECOVER ? a.out_off[g] : a.parity_off[g]);
  d.info = nin | (plen << 8) | (fast ? 0x80000000u : 0u);
  d.pad = 0;
  d.pad2[0] = d.pad2[1] = d.pad2[2] = d.pad2[3] = 0;
  if (!RECOVER) a.parity_len_out[g] = (uint16_t)plen;
  D[g] = d;
}

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// s_waitcnt vmcnt(n) for a runtime n (the immediate is 6 bits); rounds n down
// to a multiple of 4 above 16 (a conservative wait).
template <int N>
__device__ __forceinline__ void vmwait_i() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void vmwait(uint32_t n) {
  if (n >= 63u) {
    vmwait_i<63>();
    return;
  }
  switch (n) {
#define W1(N) case N: vmwait_i<N>(); break;
    W1(0) W1(1) W1(2) W1(3) W1(4) W1(5) W1(6) W1(7) W1(8) W1(9) W1(10) W1(11) W1(12) W1(13)
    W1(14) W1(15) W1(16) W1(17) W1(18) W1(19) W1(20) W1(21) W1(22) W1(23) W1(24) W1(25)
    W1(26) W1(27) W1(28) W1(29) W1(30) W1(31) W1(32) W1(33) W1(34) W1(35) W1(36) W1(37)
    W1(38) W1(39) W1(40) W1(41) W1(42) W1(43) W1(44) W1(45) W1(46) W1(47) W1(48) W1(49)
    W1(50) W1(51) W1(52) W1(53) W1(54) W1(55) W1(56) W1(57) W1(58) W1(59) W1(60) W1(61)
    W1(62)
#undef W1
    default: vmwait_i<0>(); break;
  }
}

// first n bytes (n in 1..16) of a 16-byte window kept: dword masks
__device__ __forceinline__ uint32_t keep_dw(uint32_t n, uint32_t d) {
  const int r = (int)n - 4 * (int)d;
  return r >= 4 ? 0xFFFFFFFFu : (r <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * r)));
}

__device__ __forceinline__ u32x4 lds16(const uint8_t* p) { return *reinterpret_cast<const u32x4*>(p); }

// window at byte w of an input whose image bytes start at `img` (LDS), with
// misalignment sh = img & 15 (wave-uniform)
__device__ __forceinline__ u32x4 img_window(const uint8_t* img_al, uint32_t sh, uint32_t w) {
  const u32x4 lo = lds16(img_al + w);
  if (sh == 0u) return lo;
  const u32x4 hi = lds16(img_al + w + 16u);
  // sh is wave-uniform: the dword select is a scalar branch, then one
  // v_alignbyte per dword
  const uint32_t b = sh & 3u;
  u32x4 r;
  switch (sh >> 2) {
    case 0:
      r = u32x4{__builtin_amdgcn_alignbyte(lo.y, lo.x, b), __builtin_amdgcn_alignbyte(lo.z, lo.y, b),
                __builtin_amdgcn_alignbyte(lo.w, lo.z, b), __builtin_amdgcn_alignbyte(hi.x, lo.w, b)};
      break;
    case 1:
      r = u32x4{__builtin_amdgcn_alignbyte(lo.z, lo.y, b), __builtin_amdgcn_alignbyte(lo.w, lo.z, b),
                __builtin_amdgcn_alignbyte(hi.x, lo.w, b), __builtin_amdgcn_alignbyte(hi.y, hi.x, b)};
      break;
    case 2:
      r = u32x4{__builtin_amdgcn_alignbyte(lo.w, lo.z, b), __builtin_amdgcn_alignbyte(hi.x, lo.w, b),
                __builtin_amdgcn_alignbyte(hi.y, hi.x, b), __builtin_amdgcn_alignbyte(hi.z, hi.y, b)};
      break;
    default:
      r = u32x4{__builtin_amdgcn_alignbyte(hi.x, lo.w, b), __builtin_amdgcn_alignbyte(hi.y, hi.x, b),
                __builtin_amdgcn_alignbyte(hi.z, hi.y, b), __builtin_amdgcn_alignbyte(hi.w, hi.z, b)};
      break;
  }
  return r;
}

// the keep mask of the first n (1..16) bytes of a window, scalar: 4 dwords
struct Keep4 {
  uint32_t m[4];
};
__device__ __forceinline__ Keep4 keep_mask(uint32_t n) {
  // 128-bit mask = 2^(8n) - 1, built from two 64-bit scalar halves
  const uint64_t lo = n >= 8u ? ~0ull : ((1ull << (8u * n)) - 1ull);
  const uint64_t hi = n >= 16u ? ~0ull : (n <= 8u ? 0ull : ((1ull << (8u * (n - 8u))) - 1ull));
  Keep4 k;
  k.m[0] = rfl((uint32_t)lo);
  k.m[1] = rfl((uint32_t)(lo >> 32));
  k.m[2] = rfl((uint32_t)hi);
  k.m[3] = rfl((uint32_t)(hi >> 32));
  return k;
}

typedef uint32_t u32x32 __attribute__((ext_vector_type(32)));
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

// Parity slots in registers.  Slot j's set-0 window (4 dwords per lane) is
// dwords 4*(j%8).. of block vector B0[j/8]; the set-1 windows of the slot
// pair j/2 are dwords 4*((j%8)/2).. of B1[j/8] (lanes 0-31: the even slot,
// 32-63: the odd one).  The current block (8 slots) is assembled in cur0 /
// cur1 by a dynamic insert (s_set_gpr_idx: the index is wave-uniform), and
// moved into its block vector once per 8 groups (a switch: static indices,
// so the block vectors stay in registers -- VGPRs or AGPRs).
template <int NB>
struct ParSlots {
  u32x32 B0[NB];
  u32x16 B1[NB];
};

template <int NB, int I = 0>
__device__ __forceinline__ void park_block(ParSlots<NB>& P, uint32_t b, const u32x32& c0,
                                           const u32x16& c1) {
  if constexpr (I < NB) {
    if (b == (uint32_t)I) {
      P.B0[I] = c0;
      P.B1[I] = c1;
    } else {
      park_block<NB, I + 1>(P, b, c0, c1);
    }
  }
}

// DIAG 1: no parity stores (the read side alone)
template <bool RECOVER, int S, int RING, int DMAX, int DIAG = 0, bool LDSD = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void ragged_phase_kernel(RaggedArgs a, const RDesc* __restrict__ D, uint32_t nphase,
                         uint32_t* phase_sync) {
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[4 * RING * 16 + 64];
  // the phase's descriptors of each wave's slots, staged by LDS-DMA at the
  // phase start (LDSD): no scalar-load round trip per group
  __shared__ __attribute__((aligned(16))) RDesc s_desc[LDSD ? 4 * S : 1];
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t wv = rfl(tid >> 6);
  const uint32_t ncu = gridDim.x, cu = blockIdx.x;
  uint8_t* ring = s_ring + wv * (RING * 16);
  const bool odd_half = lane >= 32u;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  static_assert(S % 8 == 0, "slots in blocks of 8");
  constexpr int NB = S / 8;
  ParSlots<NB> P;
  u32x32 cur0;
  u32x16 cur1;
  uint64_t c_issue = 0, c_wait = 0, c_reduce = 0, c_deposit = 0, c_meet = 0, c_store = 0;
  auto stamp = [&]() -> uint64_t { return DIAG == 2 ? __builtin_amdgcn_s_memtime() : 0ull; };
  uint64_t t_ms = 0;
  for (uint32_t p = 0; p < nphase; ++p) {
    if constexpr (DIAG == 2) {
      const uint64_t t = stamp();
      if (p) c_store += t - t_ms;
    }
    const uint64_t gbase = (uint64_t)p * S * ncu * 4u;
    auto gidx = [&](uint32_t j) -> uint64_t { return gbase + ((uint64_t)j * ncu + cu) * 4u + wv; };
    // slots with a group (the batch's tail)
    uint32_t nslot = 0;
    if (gidx(0) < a.n_groups) {
      const uint64_t left = a.n_groups - gidx(0);  // groups from slot 0's on, stride ncu*4
      nslot = (uint32_t)min<uint64_t>((uint64_t)S, (left + (uint64_t)ncu * 4u - 1u) / ((uint64_t)ncu * 4u));
    }
    nslot = rfl(nslot);
    RDesc* wdesc = s_desc + (LDSD ? wv * S : 0);
    if constexpr (LDSD) {
      // 8 x 16 B per descriptor, lane l of instruction u: piece (64u + l)
      for (uint32_t u = 0; u < (uint32_t)S * 8u; u += 64u) {
        const uint32_t idx = u + lane, j = idx >> 3, part = idx & 7u;
        const uint32_t jj = j < nslot ? j : 0u;
        const uint8_t* src = reinterpret_cast<const uint8_t*>(D + gidx(jj)) + 16u * part;
        __builtin_amdgcn_global_load_lds(
            (const void*)src,
            (__attribute__((address_space(3))) void*)(reinterpret_cast<uint8_t*>(wdesc) + 16u * u),
            16, 0, 2);
      }
      vmwait_i<0>();
    }
    auto desc = [&](uint32_t j) -> const RDesc* { return LDSD ? wdesc + j : D + gidx(j); };
    uint32_t iss = 0, red = 0, head = 0, total = 0;
    uint32_t posv = 0, thru = 0;  // per in-flight group (lane j % 64): ring position, instructions
    while (red < nslot) {
      const uint64_t t_i = stamp();
      // ---- issue ahead: as many groups as the ring and DMAX allow
      while (iss < nslot && iss - red < (uint32_t)DMAX) {
        const RDesc* d = desc(iss);
        const uint32_t N = rfl(d->nchunk);
        const uint32_t A = (N + 63u) & ~63u;
        uint32_t pos;
        if (iss == red) {
          pos = (head + A <= (uint32_t)RING) ? head : 0u;
        } else {
          const uint32_t old = rfl(__builtin_amdgcn_readlane(posv, red & 63u));
          // in flight: [old, head) (head > old) or [old, end) + [0, head)
          // (head < old); head == old with groups in flight is a FULL ring
          if (head > old) {
            pos = head + A <= (uint32_t)RING ? head : (A <= old ? 0u : 0xFFFFFFFFu);
          } else if (head < old) {
            pos = head + A <= old ? head : 0xFFFFFFFFu;
          } else {
            pos = 0xFFFFFFFFu;
          }
        }
        if (pos == 0xFFFFFFFFu) break;
        const uint64_t b0 = ((uint64_t)rfl((uint32_t)(d->base[0] >> 32)) << 32) | rfl((uint32_t)d->base[0]);
        const uint64_t b1 = ((uint64_t)rfl((uint32_t)(d->base[1] >> 32)) << 32) | rfl((uint32_t)d->base[1]);
        const uint64_t b2 = ((uint64_t)rfl((uint32_t)(d->base[2] >> 32)) << 32) | rfl((uint32_t)d->base[2]);
        const uint32_t s12 = rfl(d->s12);
        const uint32_t S1 = s12 & 0xFFFFu, S2 = s12 >> 16;
        for (uint32_t q = 0; q < A; q += 64u) {
          const uint32_t c = min(q + lane, N - 1u);
          uint64_t base = b0;
          uint32_t cr = c;
          if (c >= S1) { base = b1; cr = c - S1; }
          if (c >= S2) { base = b2; cr = c - S2; }
          const uint8_t* src = reinterpret_cast<const uint8_t*>(base + 16ull * cr);
          __builtin_amdgcn_global_load_lds(
              (const void*)src, (__attribute__((address_space(3))) void*)(ring + (pos + q) * 16u), 16,
              0, 2);
        }
        total += A >> 6;
        posv = lane == (iss & 63u) ? pos : posv;
        thru = lane == (iss & 63u) ? total : thru;
        head = pos + A;
        ++iss;
      }
      // ---- wait for group `red`, reduce it out of LDS
      const uint64_t t_w = stamp();
      if constexpr (DIAG == 2) c_issue += t_w - t_i;
      vmwait(total - rfl(__builtin_amdgcn_readlane(thru, red & 63u)));
      uint64_t t_r = stamp();
      if constexpr (DIAG == 2) c_wait += t_r - t_w;
      const RDesc* d = desc(red);
      const uint32_t pos = rfl(__builtin_amdgcn_readlane(posv, red & 63u));
      const uint32_t info = rfl(d->info);
      const uint32_t nin = info & 0xFFu;
      u32x4 a0 = zero, a1 = zero;
      const uint8_t* img0 = ring + pos * 16u;
      // the image offsets and lengths as dwords: scalar loads (a 16-bit field
      // would be a VECTOR load, whose use makes the compiler wait vmcnt(0) --
      // draining every staged group in flight)
      const uint32_t* dw = reinterpret_cast<const uint32_t*>(d);
      uint32_t iw[kRpMaxIn / 2], lw[kRpMaxIn / 2];
#pragma unroll
      for (int q = 0; q < kRpMaxIn / 2; ++q) {
        iw[q] = rfl(dw[12 + q]);  // img[] at byte 48
        lw[q] = rfl(dw[20 + q]);  // len[] at byte 80
      }
#pragma unroll
      for (int i = 0; i < kRpMaxIn; ++i) {
        if ((uint32_t)i < nin) {
          const uint32_t io = (iw[i / 2] >> (16 * (i & 1))) & 0xFFFFu;
          const uint32_t ln = (lw[i / 2] >> (16 * (i & 1))) & 0xFFFFu;
          const uint32_t sh = io & 15u;
          const uint8_t* ia = img0 + (io - sh);
          const uint32_t last = (ln - 1u) >> 4;  // the input's last window
          const Keep4 km = keep_mask(ln - 16u * last);
          if (lane <= last) {
            u32x4 v = img_window(ia, sh, 16u * lane);
            const bool l = lane == last;  // the partial window's lane keeps its bytes only
            v.x &= l ? km.m[0] : ~0u;
            v.y &= l ? km.m[1] : ~0u;
            v.z &= l ? km.m[2] : ~0u;
            v.w &= l ? km.m[3] : ~0u;
            a0 ^= v;
          }
          if (ln > 1024u) {
            const uint32_t t1 = 64u + (lane & 31u);
            if (t1 <= last) {
              u32x4 v = img_window(ia, sh, 16u * t1);
              const bool l = t1 == last;
              v.x &= l ? km.m[0] : ~0u;
              v.y &= l ? km.m[1] : ~0u;
              v.z &= l ? km.m[2] : ~0u;
              v.w &= l ? km.m[3] : ~0u;
              a1 ^= v;
            }
          }
        }
      }
      {
      if constexpr (DIAG == 2) { const uint64_t t = stamp(); c_reduce += t - t_r; t_r = t; }
        const uint32_t sl = red & 7u, pr = sl >> 1;
        cur0[4u * sl] = a0.x;
        cur0[4u * sl + 1u] = a0.y;
        cur0[4u * sl + 2u] = a0.z;
        cur0[4u * sl + 3u] = a0.w;
        const bool mine = odd_half == ((red & 1u) != 0u);
        // the pair's dwords: keep the other half's lanes
        const u32x4 o1 = {cur1[4u * pr], cur1[4u * pr + 1u], cur1[4u * pr + 2u], cur1[4u * pr + 3u]};
        const u32x4 n1 = mine ? a1 : o1;
        cur1[4u * pr] = n1.x;
        cur1[4u * pr + 1u] = n1.y;
        cur1[4u * pr + 2u] = n1.z;
        cur1[4u * pr + 3u] = n1.w;
        if (sl == 7u || red + 1u == nslot) park_block<NB>(P, red >> 3, cur0, cur1);
      }
      ++red;
      if constexpr (DIAG == 2) { const uint64_t t = stamp(); c_deposit += t - t_r; }
    }
    // ---- the grid meets, then every wave stores its slots' parity rows
    uint64_t t_m = stamp();
    phase_meet(phase_sync, p + 1u);
    if constexpr (DIAG == 2) { const uint64_t t = stamp(); c_meet += t - t_m; t_ms = t; }
    if constexpr (DIAG != 1) {
#pragma unroll
      for (int j = 0; j < S; ++j) {
        if ((uint32_t)j < nslot) {
          const RDesc* d = desc(j);
          const uint32_t plen = (rfl(d->info) >> 8) & 0xFFFFu;
          uint8_t* dst = reinterpret_cast<uint8_t*>(((uint64_t)rfl((uint32_t)(d->dst >> 32)) << 32) |
                                                    rfl((uint32_t)d->dst));
          const uint32_t nw = (plen + 15u) >> 4;  // windows (plen >= 16)
          const uint32_t o = plen - 16u * (nw - 1u);  // bytes of the last one (1..16)
          const bool full_last = o == 16u;
          const uint32_t nfull = full_last ? nw : nw - 1u;
          // set 0: windows 0..63; set 1: windows 64 + (lane & 31) on this slot's half
          const u32x4 w0 = {P.B0[j / 8][4 * (j % 8)], P.B0[j / 8][4 * (j % 8) + 1],
                            P.B0[j / 8][4 * (j % 8) + 2], P.B0[j / 8][4 * (j % 8) + 3]};
          const int pr = (j % 8) / 2;
          const u32x4 w1 = {P.B1[j / 8][4 * pr], P.B1[j / 8][4 * pr + 1], P.B1[j / 8][4 * pr + 2],
                            P.B1[j / 8][4 * pr + 3]};
          if (lane < nfull) st16t<true>(dst + 16u * lane, w0);
          const uint32_t t1 = 64u + (lane & 31u);
          const bool mine = odd_half == ((j & 1) != 0);
          if (mine && t1 < nfull) st16t<true>(dst + 16u * t1, w1);
          if (!full_last) {
            // the last window: the 16 bytes ending at plen, from windows nw-2, nw-1
            const uint32_t tl = nw - 1u, tp = nw - 2u;
            u32x4 prev, cur;
            auto win = [&](uint32_t t, uint32_t comp) -> uint32_t {
              const uint32_t src_lane = t < 64u ? t : (t - 64u) + ((j & 1) ? 32u : 0u);
              const u32x4& r = t < 64u ? w0 : w1;
              const uint32_t v = comp == 0 ? r.x : comp == 1 ? r.y : comp == 2 ? r.z : r.w;
              return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)src_lane);
            };
            prev.x = win(tp, 0); prev.y = win(tp, 1); prev.z = win(tp, 2); prev.w = win(tp, 3);
            cur.x = win(tl, 0); cur.y = win(tl, 1); cur.z = win(tl, 2); cur.w = win(tl, 3);
            if (lane == 0u) st16t<true>(dst + plen - 16u, bytes16_at(prev, cur, o));
          }
        }
      }
    }
  }
  if constexpr (DIAG == 2) {
    c_store += stamp() - t_ms;
    if (lane == 0u) {
      uint64_t* o = g_stamps + ((uint64_t)blockIdx.x * 4u + wv) * 8u;
      o[0] = c_issue; o[1] = c_wait; o[2] = c_reduce; o[3] = c_deposit; o[4] = c_meet; o[5] = c_store;
    }
  }
  phase_exit(phase_sync, nullptr);
}

}  // namespace
}  // namespace qfec

using qfec::RaggedArgs;
using qfec::RDesc;

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

static RDesc* g_desc = nullptr;
static uint32_t* g_sync = nullptr;
static int g_ncu = 256;

#define BLK(REC)                                                                           \
  [=](const RaggedArgs& a) {                                                               \
    hipLaunchKernelGGL((qfec::ragged_block_kernel<REC, 4, 8, 2, true, true, 0>),          \
                       dim3((uint32_t)((a.n_groups + 7) / 8)), dim3(256), 0, 0, a);        \
  }

template <bool REC, int S, int RING, int DMAX, int DIAG = 0>
static void run_phase(const RaggedArgs& a) {
  hipLaunchKernelGGL((qfec::rdesc_kernel<REC>), dim3((uint32_t)((a.n_groups + 255) / 256)),
                     dim3(256), 0, 0, a, g_desc, (uint32_t)RING);
  const uint64_t per = (uint64_t)S * g_ncu * 4;
  const uint32_t nphase = (uint32_t)((a.n_groups + per - 1) / per);
  hipLaunchKernelGGL((qfec::ragged_phase_kernel<REC, S, RING, DMAX, DIAG>), dim3(g_ncu), dim3(256),
                     0, 0, a, (const RDesc*)g_desc, nphase, g_sync);
}

static uint64_t* g_stamps_d = nullptr;
template <bool REC, int S, int RING, int DMAX>
static void stamps_report(const RaggedArgs& a, const char* tag) {
  const size_t nw = (size_t)g_ncu * 4;
  if (!g_stamps_d) {
    CK(hipMalloc(&g_stamps_d, nw * 8 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(qfec::g_stamps), &g_stamps_d, sizeof(g_stamps_d)));
  }
  CK(hipMemset(g_stamps_d, 0, nw * 8 * 8));
  hipLaunchKernelGGL((qfec::rdesc_kernel<REC>), dim3((uint32_t)((a.n_groups + 255) / 256)),
                     dim3(256), 0, 0, a, g_desc, (uint32_t)RING);
  const uint64_t per = (uint64_t)S * g_ncu * 4;
  const uint32_t nphase = (uint32_t)((a.n_groups + per - 1) / per);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL((qfec::ragged_phase_kernel<REC, S, RING, DMAX, 2>), dim3(g_ncu), dim3(256),
                     0, 0, a, (const RDesc*)g_desc, nphase, g_sync);
  CK(hipEventRecord(e1, 0));
  CK(hipDeviceSynchronize());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<uint64_t> h(nw * 8);
  CK(hipMemcpy(h.data(), g_stamps_d, nw * 64, hipMemcpyDeviceToHost));
  double sum[6] = {0};
  for (size_t w = 0; w < nw; ++w)
    for (int i = 0; i < 6; ++i) sum[i] += (double)h[w * 8 + i];
  double tot = 0;
  for (int i = 0; i < 6; ++i) tot += sum[i];
  const char* nm[6] = {"issue", "wait", "reduce", "deposit", "meet", "store"};
  std::printf("stamps %s (S%d D%d, %.1f us): per wave mean cycles (s_memtime):", tag, S, DMAX, ms * 1e3);
  for (int i = 0; i < 6; ++i) std::printf(" %s %.0f (%.1f%%)", nm[i], sum[i] / nw, 100.0 * sum[i] / tot);
  std::printf("\n");
}

template <bool REC, int S, int RING, int DMAX>
static void run_phase_main(const RaggedArgs& a) {  // descriptors already built
  const uint64_t per = (uint64_t)S * g_ncu * 4;
  const uint32_t nphase = (uint32_t)((a.n_groups + per - 1) / per);
  hipLaunchKernelGGL((qfec::ragged_phase_kernel<REC, S, RING, DMAX, 0>), dim3(g_ncu), dim3(256),
                     0, 0, a, (const RDesc*)g_desc, nphase, g_sync);
}

template <bool REC>
static void run_desc_only(const RaggedArgs& a) {
  hipLaunchKernelGGL((qfec::rdesc_kernel<REC>), dim3((uint32_t)((a.n_groups + 255) / 256)),
                     dim3(256), 0, 0, a, g_desc, 1536u);
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const uint64_t G = 1 << 20;
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
  CK(hipMalloc(&g_desc, G * sizeof(RDesc)));
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

  std::vector<V> vs;
  vs.push_back({"product block encode", false, BLK(false)});
  vs.push_back({"phase S40 R1536 D4 encode", false, run_phase<false, 40, 1536, 4>});
  vs.push_back({"phase S40 R1536 D6 encode", false, run_phase<false, 40, 1536, 6>});
  vs.push_back({"phase S32 R2048 D6 encode", false, run_phase<false, 32, 2048, 6>});
  vs.push_back({"product block recover", true, BLK(true)});
  vs.push_back({"phase S40 R1536 D4 recover", true, run_phase<true, 40, 1536, 4>});
  vs.push_back({"phase S40 R1536 D6 recover", true, run_phase<true, 40, 1536, 6>});
  std::vector<V> diag;  // timed in this order (the main-kernel-only runs reuse the
                        // descriptors the entry before them built)
  diag.push_back({"desc pre-pass only (enc)", false, run_desc_only<false>});
  diag.push_back({"phase S40 D4 enc, main kernel only", false, run_phase_main<false, 40, 1536, 4>});
  diag.push_back({"phase S40 D4 enc, no stores", false, run_phase<false, 40, 1536, 4, 1>});
  diag.push_back({"desc pre-pass only (rec)", true, run_desc_only<true>});
  diag.push_back({"phase S40 D4 rec, main kernel only", true, run_phase_main<true, 40, 1536, 4>});
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
    if (bad) {
      int hj[64] = {0}, hw[4] = {0};
      const uint64_t S_guess = 40;
      for (uint64_t g = 0; g < G; ++g) {
        bool gb = std::memcmp(h_ref.data() + g * slot, h_v.data() + g * slot, slot) != 0;
        if (!gb) continue;
        const uint64_t per = S_guess * g_ncu * 4;
        const uint64_t r = g % per;
        const uint64_t j = r / (g_ncu * 4ull);
        hw[r % 4]++;
        if (j < 64) hj[j]++;
      }
      std::printf("  bad groups by slot (S=40 layout):");
      for (int j = 0; j < 40; ++j) std::printf(" %d", hj[j]);
      std::printf("\n  by wave: %d %d %d %d\n", hw[0], hw[1], hw[2], hw[3]);
    }
    std::printf("check %-30s == product: %s (err %u, %zu bad bytes, first at %zd = group %zd)\n",
                v.name.c_str(), ok ? "yes" : "NO", e_h, bad, (ssize_t)first,
                first == (size_t)-1 ? (ssize_t)-1 : (ssize_t)(first / slot));
    all_ok = all_ok && ok;
  }
  if (!all_ok) return 2;
  stamps_report<false, 40, 1536, 4>(ev, "encode");
  stamps_report<true, 40, 1536, 4>(rv, "recover");
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
