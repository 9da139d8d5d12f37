// tune_protect.hip — throughput of the NULL packet-protection kernels on the
// headline packet shape (1350-B payload, 22-B header), device-resident, and a
// VALU microbenchmark of the FNV-1a-128 byte step.  One process, interleaved.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_protect.hip -o tools/tune/build/tune_protect
#include "../../libquic_amd/csrc/qpp_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

template <typename T>
static T* up(const std::vector<T>& v) {
  T* d;
  CK(hipMalloc(&d, v.size() * sizeof(T)));
  CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

// pure VALU: hash `bytes` synthetic bytes per lane from registers
__global__ void fnv_valu_kernel(uint32_t bytes, uint32_t* sink) {
  qfec::Fnv128 h = qfec::fnv_init();
  uint32_t w = threadIdx.x * 0x9E3779B9u;
  for (uint32_t i = 0; i < bytes; i += 4) {
    qfec::fnv_word(h, w);
    w = w * 1664525u + 1013904223u;
  }
  if ((h.x0 ^ h.x1 ^ h.x2 ^ h.x3) == 0x12345678u) sink[0] = h.x0;
}

// pure VALU, 16-byte chunks as the staged kernels hash them (R3 or byte-serial)
template <bool R3>
__global__ void fnv_valu_chunk_kernel(uint32_t bytes, uint32_t* sink) {
  qfec::Fnv128 h = qfec::fnv_init();
  uint32_t w = threadIdx.x * 0x9E3779B9u;
  for (uint32_t i = 0; i < bytes; i += 16) {
    const qfec::u32x4 v = {w, w ^ 0x5bd1e995u, w * 3u + 1u, w + 0x27d4eb2du};
    qfec::fnv_chunk<R3>(h, v);
    w = w * 1664525u + 1013904223u;
  }
  if ((h.x0 ^ h.x1 ^ h.x2 ^ h.x3) == 0x12345678u) sink[0] = h.x0;
}

// the same with two independent packets per lane (ILP 2): does a lane's
// serial FNV chain leave the VALU idle at the 2 waves/SIMD the staged kernels run at?
__global__ void fnv_valu_chunk2_kernel(uint32_t bytes, uint32_t* sink) {
  qfec::Fnv128 h = qfec::fnv_init(), g = qfec::fnv_init();
  uint32_t w = threadIdx.x * 0x9E3779B9u, x = w ^ 0x1234567u;
  for (uint32_t i = 0; i < bytes; i += 32) {
    const qfec::u32x4 v = {w, w ^ 0x5bd1e995u, w * 3u + 1u, w + 0x27d4eb2du};
    const qfec::u32x4 u = {x, x ^ 0x5bd1e995u, x * 3u + 1u, x + 0x27d4eb2du};
    qfec::fnv_chunk<true>(h, v);
    qfec::fnv_chunk<true>(g, u);
    w = w * 1664525u + 1013904223u;
    x = x * 1664525u + 1013904223u;
  }
  if ((h.x0 ^ h.x1 ^ h.x2 ^ h.x3 ^ g.x0 ^ g.x3) == 0x12345678u) sink[0] = h.x0;
}

namespace qfec {
namespace {
// the round-2 tail store (the tune kernels below keep source-relative chunks)
__device__ __forceinline__ void store_tail(uint8_t* d, u32x4 v, uint32_t len) {
  if ((len & 15u) == 0u) return;
  if (len >= 16u) {
    st16(d + len - 16u, v);
    return;
  }
  for (uint32_t i = 0; i < len; ++i) d[i] = (uint8_t)byte_of(v, i);
}
}  // namespace
}  // namespace qfec

// null_encrypt_staged_kernel<16> with a per-wave timeline (s_memrealtime,
// 10 ns ticks): where does a wave's life go?
namespace qfec {
namespace {
__global__ __launch_bounds__(kBlock) void null_enc_timed(ProtectArgs a, uint64_t* tl) {
  constexpr uint32_t SC = 16;
  __shared__ u32x4 s_rows[kWaves][64 * (SC + 1u)];
  __shared__ StageMeta s_meta[kWaves][64];
  const uint64_t t0 = wall_clock64();
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = p < a.n;
  const uint8_t* ad = nullptr;
  const uint8_t* pt = nullptr;
  uint8_t* o = nullptr;
  uint32_t alen = 0, plen = 0;
  if (valid) {
    ad = a.bytes + a.ad_off[p];
    pt = a.bytes + a.in_off[p];
    alen = a.ad_len[p];
    plen = a.in_len[p];
    o = a.out + a.out_off[p];
  }
  s_meta[wv][lane] = StageMeta{pt, o + kTag, plen >> 4};
  const u32x4 tail = valid ? load_tail(pt, plen) : u32x4{0u, 0u, 0u, 0u};
  Fnv128 h = fnv_init();
  if (valid) fnv_span<true>(h, ad, alen);
  const uint64_t t1 = wall_clock64();
  uint64_t th = 0, tw = 0, tx = 0;
  {
    const StageMeta* meta = s_meta[wv];
    u32x4* rows = s_rows[wv];
    const uint32_t my_nfull = plen >> 4;
    const uint32_t nslab = (wave_max_u32(my_nfull) + SC - 1) / SC;
    u32x4 cur[SC], nxt[SC];
    if (nslab) stage_load<SC>(meta, lane, 0, cur);
    for (uint32_t sl = 0; sl < nslab; ++sl) {
      const uint64_t a0 = wall_clock64();
      stage_to_lds<SC>(rows, lane, cur);
      if (sl + 1u < nslab) stage_load<SC>(meta, lane, sl + 1u, nxt);
      const uint64_t a1 = wall_clock64();
#pragma unroll
      for (uint32_t j = 0; j < SC; ++j)
        if (sl * SC + j < my_nfull) fnv_chunk<true>(h, rows[lane * (SC + 1u) + j]);
      const uint64_t a2 = wall_clock64();
      __builtin_amdgcn_s_waitcnt(0x0F70);
      stage_store<SC>(meta, lane, sl, cur);
      const uint64_t a3 = wall_clock64();
#pragma unroll
      for (uint32_t j = 0; j < SC; ++j) cur[j] = nxt[j];
      tx += a1 - a0;
      th += a2 - a1;
      tw += a3 - a2;
    }
  }
  if (valid) {
    fnv_tail(h, tail, plen);
    store_tail(o + kTag, tail, plen);
    const uint32_t tag[3] = {h.x0, h.x1, h.x2};
    __builtin_memcpy(o, tag, kTag);
  }
  const uint64_t t2 = wall_clock64();
  if (lane == 0) {
    uint64_t* r = tl + 8ull * (blockIdx.x * kWaves + wv);
    r[0] = t0; r[1] = t1; r[2] = t2; r[3] = th; r[4] = tw; r[5] = tx;
  }
}
// ---------------------------------------------------------------------------
// LDS-DMA form: the payload slabs go global -> LDS by
// global_load_lds_dwordx4 (no VGPR staging: the 2 x SC u32x4 register slabs
// and the ds_write transpose disappear), NB slab buffers per wave, one wave
// per workgroup.  Instruction I of a slab: lane L loads packet
// P = (64/SC) I + L/SC, slot m = L % SC holds chunk m ^ swz(P) — the swizzle
// on the SOURCE address keeps the hashing lanes' row reads (lane q: chunk j of
// packet q at slot j ^ swz(q)) on distinct 16-B bank slots in every
// ds_read_b128 lane group.  The payload copy reads the slab back lane-linear
// (conflict-free) and stores it from the loading lane.  Waits are counted:
// per slab the wave issues exactly n_ld (loads) and n_st (stores) VMEM
// instructions (wave-uniform ballot branches), vmcnt(n) retires slab s while
// the later slabs' loads and the earlier slabs' stores stay in flight.
// ---------------------------------------------------------------------------
template <uint32_t N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15u) | ((N >> 4) << 14) | 0x0F70u);
}
template <uint32_t LO, uint32_t HI>
__device__ __forceinline__ void wait_vm_range(uint32_t n) {
  if constexpr (LO == HI) {
    wait_vm<LO>();
  } else {
    constexpr uint32_t M = (LO + HI) / 2;
    if (n <= M) wait_vm_range<LO, M>(n);
    else wait_vm_range<M + 1, HI>(n);
  }
}
// vmcnt(min(n, MAXN)) (stricter when clamped), n wave-uniform: a binary tree
// of scalar branches over the immediate forms
template <uint32_t MAXN>
__device__ __forceinline__ void wait_vm_dyn(uint32_t n) {
  n = __builtin_amdgcn_readfirstlane(n);
  wait_vm_range<0, MAXN>(n < MAXN ? n : MAXN);
}

template <uint32_t SC>
__device__ __forceinline__ uint32_t glds_swz(uint32_t P) { return (P / (16u / SC)) & (SC - 1u); }

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

template <uint32_t SC, uint32_t NB>
__global__ __launch_bounds__(64) void null_encrypt_glds_kernel(ProtectArgs a) {
  static_assert(NB >= 2 && SC >= 4 && SC <= 16, "shape");
  __shared__ __attribute__((aligned(16))) u32x4 s_buf[NB][64 * SC];
  const uint32_t lane = threadIdx.x;
  const uint64_t p = (uint64_t)blockIdx.x * 64 + lane;
  const bool valid = p < a.n;
  const uint8_t* ad = nullptr;
  const uint8_t* pt = a.bytes;
  uint8_t* o = nullptr;
  uint32_t alen = 0, plen = 0;
  if (valid) {
    ad = a.bytes + a.ad_off[p];
    pt = a.bytes + a.in_off[p];
    alen = a.ad_len[p];
    plen = a.in_len[p];
    o = a.out + a.out_off[p];
  }
  const uint32_t nfull = plen >> 4;
  uint8_t* dst = valid ? o + kTag : nullptr;
  const u32x4 tail = valid ? load_tail(pt, plen) : u32x4{0u, 0u, 0u, 0u};
  Fnv128 h = fnv_init();
  if (valid) fnv_span<true>(h, ad, alen);
  const bool overlap = valid && o + kTag < pt + plen && pt < o + kTag + plen;
  const bool inplace = wave_any_qpp(overlap);
  // this lane's loader roles
  const uint8_t* lsrc[SC];
  uint8_t* ldst[SC];
  uint32_t lnf[SC], lch[SC];
#pragma unroll
  for (uint32_t I = 0; I < SC; ++I) {
    const uint32_t P = (64u / SC) * I + lane / SC;
    lsrc[I] = (const uint8_t*)shfl64((uint64_t)pt, P);
    ldst[I] = (uint8_t*)shfl64((uint64_t)dst, P);
    lnf[I] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(P << 2), (int)nfull);
    lch[I] = (lane % SC) ^ glds_swz<SC>(P);
  }
  const uint32_t nslab = (wave_max_u32(nfull) + SC - 1) / SC;
  const uint32_t myswz = glds_swz<SC>(lane);
  uint32_t nld[NB];  // VMEM loads issued per buffered slab
#pragma unroll
  for (uint32_t b = 0; b < NB; ++b) nld[b] = 0;
  auto load = [&](uint32_t sl, uint32_t b) {
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t I = 0; I < SC; ++I) {
      const uint32_t c = sl * SC + lch[I];
      const bool act = c < lnf[I];
      if (__ballot(act)) {
        ++cnt;
        if (act)
          __builtin_amdgcn_global_load_lds((const void*)(lsrc[I] + 16u * c),
                                           (__attribute__((address_space(3))) void*)&s_buf[b][64 * I],
                                           16, 0, 0);
      }
    }
    return cnt;
  };
  // prologue: slabs 0 .. NB-2 in flight
#pragma unroll
  for (uint32_t s = 0; s + 1 < NB; ++s)
    if (s < nslab) nld[s] = load(s, s);
  uint32_t nsth[NB];  // stores issued per slab (ring; the NB-1 latest count)
#pragma unroll
  for (uint32_t b = 0; b < NB; ++b) nsth[b] = 0;
  for (uint32_t sl = 0; sl < nslab; ++sl) {
    const uint32_t b = sl % NB;
    // issue slab sl + NB - 1 into the buffer slab sl - 1 used
    const uint32_t nx = sl + NB - 1u;
    const uint32_t bn = nx % NB;
    nld[bn] = nx < nslab ? load(nx, bn) : 0u;
    // VMEM instructions issued after slab sl's loads (iteration sl-NB+1):
    // the later slabs' loads and the stores of slabs sl-NB+1 .. sl-1
    uint32_t after = 0;
#pragma unroll
    for (uint32_t k = 1; k < NB; ++k) after += nld[(sl + k) % NB] + nsth[(sl + k) % NB];
    constexpr uint32_t kMaxAfter = 2u * (NB - 1) * SC < 63u ? 2u * (NB - 1) * SC : 63u;
    wait_vm_dyn<kMaxAfter>(after);
    __builtin_amdgcn_wave_barrier();
    // hash this lane's row (all SC reads issued before the first use)
    {
      u32x4 r[SC];
#pragma unroll
      for (uint32_t j = 0; j < SC; ++j) r[j] = s_buf[b][lane * SC + (j ^ myswz)];
#pragma unroll
      for (uint32_t j = 0; j < SC; ++j)
        if (sl * SC + j < nfull) fnv_chunk<true>(h, r[j]);
    }
    // in place: the next slab's loads must have landed before these stores
    if (inplace) {
      __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
      for (uint32_t k = 0; k < NB; ++k) nsth[k] = 0;
    }
    uint32_t nst = 0;
    {
      u32x4 w[SC];
#pragma unroll
      for (uint32_t I = 0; I < SC; ++I) w[I] = s_buf[b][64 * I + lane];
#pragma unroll
      for (uint32_t I = 0; I < SC; ++I) {
        const uint32_t c = sl * SC + lch[I];
        const bool act = c < lnf[I] && ldst[I] != nullptr;
        if (__ballot(act)) {
          ++nst;
          if (act) st16g(ldst[I] + 16u * c, w[I]);
        }
      }
    }
    nsth[b] = nst;
    __builtin_amdgcn_wave_barrier();
  }
  if (!valid) return;
  fnv_tail(h, tail, plen);
  store_tail(o + kTag, tail, plen);
  const uint32_t tag[3] = {h.x0, h.x1, h.x2};
  __builtin_memcpy(o, tag, kTag);
}

// The LDS-DMA form with the product's destination-aligned split and 128-B
// line grid (line_meta); meta from LDS, not per-lane register arrays.
template <uint32_t SC, uint32_t NB>
__global__ __launch_bounds__(64) void null_encrypt_glds2_kernel(ProtectArgs a) {
  __shared__ __attribute__((aligned(16))) u32x4 s_buf[NB][64 * SC];
  __shared__ StageMeta s_meta[64];
  const uint32_t lane = threadIdx.x;
  const uint64_t p = (uint64_t)blockIdx.x * 64 + lane;
  const bool valid = p < a.n;
  const uint8_t* ad = nullptr;
  const uint8_t* pt = nullptr;
  uint8_t* o = nullptr;
  uint32_t alen = 0, plen = 0;
  if (valid) {
    ad = a.bytes + a.ad_off[p];
    pt = a.bytes + a.in_off[p];
    alen = a.ad_len[p];
    plen = a.in_len[p];
    o = a.out + a.out_off[p];
  }
  const DstSplit sp = dst_split(o + kTag, plen);
  const StageMeta m = line_meta(pt + sp.hd, o + kTag + sp.hd, sp.nmid, o + kTag + sp.hd);
  s_meta[lane] = m;
  const u32x4 head = valid ? load_head(pt, plen) : u32x4{0u, 0u, 0u, 0u};
  const u32x4 tail = valid ? load_tail(pt, plen) : u32x4{0u, 0u, 0u, 0u};
  Fnv128 h = fnv_init();
  if (valid) {
    fnv_span<true>(h, ad, alen);
    fnv_bytes(h, head, 0u, sp.hd);
  }
  const bool overlap = valid && o + kTag < pt + plen && pt < o + kTag + plen;
  const bool inplace = wave_any_qpp(overlap);
  const uint32_t li = lane / SC, lm = lane % SC;
  const uint32_t nslab = (wave_max_u32(m.nfull) + SC - 1) / SC;
  const uint32_t myswz = glds_swz<SC>(lane);
  wave_lds_order();
  uint32_t nld[NB], nsth[NB];
#pragma unroll
  for (uint32_t b = 0; b < NB; ++b) nld[b] = nsth[b] = 0;
  auto load = [&](uint32_t sl, uint32_t b) {
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t I = 0; I < SC; ++I) {
      const uint32_t P = (64u / SC) * I + li;
      const StageMeta& q = s_meta[P];
      const uint32_t c = sl * SC + (lm ^ glds_swz<SC>(P));
      const bool act = c >= q.lo && c < q.nfull;
      if (__ballot(act)) {
        ++cnt;
        if (act)
          __builtin_amdgcn_global_load_lds((const void*)(q.src + 16u * c),
                                           (__attribute__((address_space(3))) void*)&s_buf[b][64 * I],
                                           16, 0, 0);
      }
    }
    return cnt;
  };
#pragma unroll
  for (uint32_t s0 = 0; s0 + 1 < NB; ++s0)
    if (s0 < nslab) nld[s0] = load(s0, s0);
  for (uint32_t sl = 0; sl < nslab; ++sl) {
    const uint32_t b = sl % NB;
    const uint32_t nx = sl + NB - 1u;
    const uint32_t bn = nx % NB;
    nld[bn] = nx < nslab ? load(nx, bn) : 0u;
    uint32_t after = 0;
#pragma unroll
    for (uint32_t k = 1; k < NB; ++k) after += nld[(sl + k) % NB] + nsth[(sl + k) % NB];
    constexpr uint32_t kMaxAfter = 2u * (NB - 1) * SC < 63u ? 2u * (NB - 1) * SC : 63u;
    wait_vm_dyn<kMaxAfter>(after);
    __builtin_amdgcn_wave_barrier();
    {
      u32x4 r[SC];
#pragma unroll
      for (uint32_t j = 0; j < SC; ++j) r[j] = s_buf[b][lane * SC + (j ^ myswz)];
#pragma unroll
      for (uint32_t j = 0; j < SC; ++j)
        if (sl * SC + j >= m.lo && sl * SC + j < m.nfull) fnv_chunk<true>(h, r[j]);
    }
    if (inplace) {
      __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
      for (uint32_t k = 0; k < NB; ++k) nsth[k] = 0;
    }
    uint32_t nst = 0;
    {
      u32x4 w[SC];
#pragma unroll
      for (uint32_t I = 0; I < SC; ++I) w[I] = s_buf[b][64 * I + lane];
#pragma unroll
      for (uint32_t I = 0; I < SC; ++I) {
        const uint32_t P = (64u / SC) * I + li;
        const StageMeta& q = s_meta[P];
        const uint32_t c = sl * SC + (lm ^ glds_swz<SC>(P));
        const bool act = c >= q.lo && c < q.nfull && q.dst != nullptr;
        if (__ballot(act)) {
          ++nst;
          if (act) st16g(q.dst + 16u * c, w[I]);
        }
      }
    }
    nsth[b] = nst;
    __builtin_amdgcn_wave_barrier();
  }
  if (!valid) return;
  const uint32_t t0 = tail_pos(sp.hd + 16u * sp.nmid, plen);
  fnv_bytes(h, tail, t0, sp.tl);
  store_from_aligned_start(o + kTag + sp.hd + 16u * sp.nmid, tail, t0, sp.tl);
  store_to_aligned_end(o + kTag, head, 0u, sp.hd);
  const uint32_t tag[3] = {h.x0, h.x1, h.x2};
  __builtin_memcpy(o, tag, kTag);
}

// Unpadded, XOR-swizzled staging rows (64 x SC x 16 B per wave instead of
// 64 x (SC + 1) x 16 B): slot j of packet P's row at P*SC + (j ^ swz(P)),
// conflict-free for the hashing lanes' ds_read_b128 (as the LDS-DMA kernel's
// source swizzle).  With SC = 8 the block needs 38 KiB: 4 blocks per CU.
template <uint32_t SC>
__device__ __forceinline__ void stage_to_lds_swz(u32x4* rows, uint32_t lane, const u32x4 (&v)[SC]) {
  const uint32_t i = lane / SC, m = lane % SC;
  wave_lds_order();
#pragma unroll
  for (uint32_t I = 0; I < SC; ++I) {
    const uint32_t P = (64u / SC) * I + i;
    rows[P * SC + (m ^ glds_swz<SC>(P))] = v[I];
  }
  wave_lds_order();
}

template <uint32_t SC, int NT, bool INPLACE>
__device__ __forceinline__ void stage_hash_swz(Fnv128& h, const StageMeta* meta, u32x4* rows,
                                               uint32_t lane, uint32_t my_nfull, uint32_t my_lo) {
  const uint32_t nslab = (wave_max_u32(my_nfull) + SC - 1) / SC;
  const uint32_t sw = glds_swz<SC>(lane);
  u32x4 cur[SC], nxt[SC];
  if (nslab) stage_load<SC, true, NT == 1>(meta, lane, 0, cur);
  for (uint32_t sl = 0; sl < nslab; ++sl) {
    stage_to_lds_swz<SC>(rows, lane, cur);
    if (sl + 1u < nslab) stage_load<SC, true, NT == 1>(meta, lane, sl + 1u, nxt);
#pragma unroll
    for (uint32_t j = 0; j < SC; ++j)
      if (sl * SC + j >= my_lo && sl * SC + j < my_nfull)
        fnv_chunk<true>(h, rows[lane * SC + (j ^ sw)]);
    if constexpr (INPLACE) __builtin_amdgcn_s_waitcnt(0x0F70);
    stage_store<SC, true, NT != 0>(meta, lane, sl, cur);
#pragma unroll
    for (uint32_t j = 0; j < SC; ++j) cur[j] = nxt[j];
  }
}

template <uint32_t SC, int MINB>
__global__ __launch_bounds__(kBlock, MINB) void null_encrypt_swz_kernel(ProtectArgs a) {
  __shared__ u32x4 s_rows[kWaves][64 * SC];
  __shared__ StageMeta s_meta[kWaves][64];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = p < a.n;
  const uint8_t* ad = nullptr;
  const uint8_t* pt = nullptr;
  uint8_t* o = nullptr;
  uint32_t alen = 0, plen = 0;
  if (valid) {
    ad = a.bytes + a.ad_off[p];
    pt = a.bytes + a.in_off[p];
    alen = a.ad_len[p];
    plen = a.in_len[p];
    o = a.out + a.out_off[p];
  }
  const DstSplit sp = dst_split(o + kTag, plen);
  const StageMeta m = line_meta(pt + sp.hd, o + kTag + sp.hd, sp.nmid, o + kTag + sp.hd);
  s_meta[wv][lane] = m;
  const u32x4 head = valid ? load_head(pt, plen) : u32x4{0u, 0u, 0u, 0u};
  const u32x4 tail = valid ? load_tail(pt, plen) : u32x4{0u, 0u, 0u, 0u};
  Fnv128 h = fnv_init();
  if (valid) {
    fnv_span<true>(h, ad, alen);
    fnv_bytes(h, head, 0u, sp.hd);
  }
  const bool overlap = valid && o + kTag < pt + plen && pt < o + kTag + plen;
  if (wave_any_qpp(overlap))
    stage_hash_swz<SC, kNullNT, true>(h, s_meta[wv], s_rows[wv], lane, m.nfull, m.lo);
  else
    stage_hash_swz<SC, kNullNT, false>(h, s_meta[wv], s_rows[wv], lane, m.nfull, m.lo);
  if (!valid) return;
  const uint32_t t0 = tail_pos(sp.hd + 16u * sp.nmid, plen);
  fnv_bytes(h, tail, t0, sp.tl);
  store_from_aligned_start(o + kTag + sp.hd + 16u * sp.nmid, tail, t0, sp.tl);
  store_to_aligned_end(o + kTag, head, 0u, sp.hd);
  const uint32_t tag[3] = {h.x0, h.x1, h.x2};
  __builtin_memcpy(o, tag, kTag);
}

}  // namespace
}  // namespace qfec

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 21);
  const uint32_t L = 1350, H = 22;
  const int reps = 5, rounds = 3;
  // packets: [header H | payload L] records back to back; outputs tag||payload
  std::vector<uint64_t> ad_off(n), in_off(n), out_off(n), dad_off(n), dct_off(n), dout_off(n);
  std::vector<uint16_t> ad_len(n, H), in_len(n, L), ct_len(n, L + 12);
  for (uint64_t p = 0; p < n; ++p) {
    ad_off[p] = p * (H + L);
    in_off[p] = p * (H + L) + H;
    out_off[p] = p * (L + 12);
    dout_off[p] = p * L;
  }
  uint8_t *d_in, *d_out, *d_out2, *d_ok;
  CK(hipMalloc(&d_in, n * (H + L)));
  CK(hipMalloc(&d_out, n * (L + 12)));
  CK(hipMalloc(&d_out2, n * L));
  CK(hipMalloc(&d_ok, n));
  {
    std::vector<uint8_t> h(n * (H + L));
    uint64_t s = 0x243F6A8885A308D3ull;
    for (auto& b : h) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      b = (uint8_t)s;
    }
    CK(hipMemcpy(d_in, h.data(), h.size(), hipMemcpyHostToDevice));
  }
  qfec::ProtectArgs e{};
  e.bytes = d_in; e.ad_off = up(ad_off); e.ad_len = up(ad_len); e.in_off = up(in_off);
  e.in_len = up(in_len); e.out = d_out; e.out_off = up(out_off); e.n = n;
  CK(qfec::launch_null_protect(e, false, 0));
  CK(hipDeviceSynchronize());
  // decrypt input: [header | ciphertext] -> header from d_in, ciphertext in d_out
  // (two buffers: pass offsets relative to d_in? use one combined buffer instead)
  uint8_t* d_cat;
  CK(hipMalloc(&d_cat, n * (H + L + 12)));
  for (uint64_t p = 0; p < n; ++p) {
    dad_off[p] = p * (H + L + 12);
    dct_off[p] = dad_off[p] + H;
  }
  CK(hipMemcpy2D(d_cat, H + L + 12, d_in, H + L, H, n, hipMemcpyDeviceToDevice));
  CK(hipMemcpy2D(d_cat + H, H + L + 12, d_out, L + 12, L + 12, n, hipMemcpyDeviceToDevice));
  qfec::ProtectArgs d{};
  d.bytes = d_cat; d.ad_off = up(dad_off); d.ad_len = e.ad_len; d.in_off = up(dct_off);
  d.in_len = up(ct_len); d.out = d_out2; d.out_off = up(dout_off); d.ok = d_ok; d.n = n;
  CK(qfec::launch_null_protect(d, true, 0));
  CK(hipDeviceSynchronize());
  {
    std::vector<uint8_t> ok(n);
    CK(hipMemcpy(ok.data(), d_ok, n, hipMemcpyDeviceToHost));
    uint64_t good = 0;
    for (auto v : ok) good += v;
    std::printf("decrypt(encrypt) verified: %llu / %llu\n", (unsigned long long)good,
                (unsigned long long)n);
  }
  // ChaCha20-Poly1305: one key, packet numbers 1..n; seal out = ct || tag
  std::vector<uint8_t> key(32), pre(4);
  for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 7 + 1);
  for (int i = 0; i < 4; ++i) pre[i] = (uint8_t)(0xA0 + i);
  std::vector<uint32_t> kidx(n, 0);
  std::vector<uint64_t> pns(n);
  for (uint64_t p = 0; p < n; ++p) pns[p] = p + 1;
  qfec::AeadArgs as{};
  as.io = e;
  as.keys = up(key);
  as.prefixes = up(pre);
  as.key_idx = up(kidx);
  as.packet_number = up(pns);
  as.path_id = nullptr;
  CK(qfec::launch_chacha20poly1305(as, false, 0));
  CK(hipDeviceSynchronize());
  // open input: [header | ct || tag] records in a buffer of their own
  uint8_t* d_cat2;
  CK(hipMalloc(&d_cat2, n * (H + L + 12)));
  CK(hipMemcpy2D(d_cat2, H + L + 12, d_in, H + L, H, n, hipMemcpyDeviceToDevice));
  CK(hipMemcpy2D(d_cat2 + H, H + L + 12, d_out, L + 12, L + 12, n, hipMemcpyDeviceToDevice));
  qfec::AeadArgs ao = as;
  ao.io = d;
  ao.io.bytes = d_cat2;
  CK(qfec::launch_chacha20poly1305(ao, true, 0));
  CK(hipDeviceSynchronize());
  {
    std::vector<uint8_t> ok(n);
    CK(hipMemcpy(ok.data(), d_ok, n, hipMemcpyDeviceToHost));
    uint64_t good = 0;
    for (auto v : ok) good += v;
    std::printf("chacha20poly1305 open(seal) verified: %llu / %llu\n", (unsigned long long)good,
                (unsigned long long)n);
  }
  uint32_t* sink;
  CK(hipMalloc(&sink, 4));
  // LDS-DMA variants: bit-identical output to the product kernel
  uint8_t* d_outg;
  CK(hipMalloc(&d_outg, n * (L + 12)));
  qfec::ProtectArgs eg = e;
  eg.out = d_outg;
  const uint32_t gblocks = (uint32_t)((n + 63) / 64);
  std::vector<std::pair<std::string, std::function<void()>>> glds = {
      {"glds SC=16 NB=2", [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds_kernel<16, 2>), dim3(gblocks), dim3(64), 0, 0, eg); }},
      {"glds SC=8 NB=2", [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds_kernel<8, 2>), dim3(gblocks), dim3(64), 0, 0, eg); }},
      {"glds SC=8 NB=3", [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds_kernel<8, 3>), dim3(gblocks), dim3(64), 0, 0, eg); }},
      {"glds SC=4 NB=3", [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds_kernel<4, 3>), dim3(gblocks), dim3(64), 0, 0, eg); }},
      {"glds SC=4 NB=4", [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds_kernel<4, 4>), dim3(gblocks), dim3(64), 0, 0, eg); }},
      {"glds2 SC=16 NB=2", [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds2_kernel<16, 2>), dim3(gblocks), dim3(64), 0, 0, eg); }},
      {"glds2 SC=8 NB=2", [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds2_kernel<8, 2>), dim3(gblocks), dim3(64), 0, 0, eg); }},
      {"glds2 SC=8 NB=3", [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds2_kernel<8, 3>), dim3(gblocks), dim3(64), 0, 0, eg); }},
      {"swz SC=8 x4", [&] { hipLaunchKernelGGL((qfec::null_encrypt_swz_kernel<8, 4>), dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, eg); }},
      {"swz SC=8 x3", [&] { hipLaunchKernelGGL((qfec::null_encrypt_swz_kernel<8, 3>), dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, eg); }},
      {"swz SC=16 x2", [&] { hipLaunchKernelGGL((qfec::null_encrypt_swz_kernel<16, 2>), dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, eg); }},
  };
  {
    std::vector<uint8_t> ref(n * (L + 12)), got(n * (L + 12));
    CK(qfec::launch_null_protect(e, false, 0));
    CK(hipMemcpy(ref.data(), d_out, ref.size(), hipMemcpyDeviceToHost));
    for (auto& g : glds) {
      CK(hipMemset(d_outg, 0xA5, ref.size()));
      g.second();
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), d_outg, got.size(), hipMemcpyDeviceToHost));
      std::printf("%-24s output %s\n", g.first.c_str(), got == ref ? "IDENTICAL" : "DIFFERS");
    }
  }
  // the same packets with every payload and every output payload on a 128-B
  // line (record stride 1408 = 11 lines): what is unaligned loading worth?
  std::vector<uint64_t> aad(n), ain(n), aout(n);
  for (uint64_t p = 0; p < n; ++p) {
    aad[p] = p * 1408 + 106;
    ain[p] = p * 1408 + 128;
    aout[p] = p * 1408 + 116;
  }
  uint8_t *d_ain, *d_aout;
  CK(hipMalloc(&d_ain, n * 1408 + 4096));
  CK(hipMalloc(&d_aout, n * 1408 + 4096));
  CK(hipMemset(d_ain, 0x3C, n * 1408 + 4096));
  qfec::ProtectArgs ea = e;
  ea.bytes = d_ain; ea.ad_off = up(aad); ea.in_off = up(ain); ea.out = d_aout; ea.out_off = up(aout);
  const uint32_t sblocks = (uint32_t)((n + 255) / 256);
  // (a) payload aligned, output payload at +4 mod 16; (b) payload at +6 mod 16, output aligned
  std::vector<uint64_t> bad_(n), bin(n), aout2(n);
  for (uint64_t p = 0; p < n; ++p) {
    aout2[p] = p * 1408 + 120;  // dst = +132
    bad_[p] = p * 1408 + 112;
    bin[p] = p * 1408 + 134;    // src = +134 (6 mod 16)
  }
  // (c) both 16-B aligned, the payload on a line, the output payload 48 B into one
  std::vector<uint64_t> aout3(n);
  for (uint64_t p = 0; p < n; ++p) aout3[p] = p * 1408 + 164;  // dst = +176 = 48 mod 128
  qfec::ProtectArgs eC = ea;
  eC.out_off = up(aout3);
  qfec::ProtectArgs eA = ea, eB = ea;
  eA.out_off = up(aout2);
  eB.ad_off = up(bad_);
  eB.in_off = up(bin);
  struct V {
    std::string name;
    double bytes;  // algorithmic bytes (HBM) per launch
    double hashed; // bytes run through FNV per launch
    std::function<void()> run;
  };
  const double enc_b = (double)n * (H + L + L + 12), dec_b = (double)n * (H + L + 12 + L);
  const double hashed = (double)n * (H + L);
  const uint32_t vb = 4096, vgrid = 256 * 8 * 4;  // 8 waves/SIMD worth of lanes... per CU
  std::vector<V> vs = {
      {"null encrypt staged (product)", enc_b, hashed, [&] { CK(qfec::launch_null_protect(e, false, 0)); }},
      {"null decrypt staged (product)", dec_b, hashed, [&] { CK(qfec::launch_null_protect(d, true, 0)); }},
      {"chacha20poly1305 seal (product)", enc_b, hashed, [&] { CK(qfec::launch_chacha20poly1305(as, false, 0)); }},
      {"chacha20poly1305 open (product)", dec_b, hashed, [&] { CK(qfec::launch_chacha20poly1305(ao, true, 0)); }},
      {"chacha seal NT stores", enc_b, hashed, [&] {
         hipLaunchKernelGGL((qfec::c20p1305_seal_kernel<16, true>), dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, as); }},
      {"chacha open NT stores", dec_b, hashed, [&] {
         hipLaunchKernelGGL((qfec::c20p1305_open_kernel<16, false, true>), dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, ao); }},
      {"chacha20poly1305 seal (product) again", enc_b, hashed, [&] { CK(qfec::launch_chacha20poly1305(as, false, 0)); }},
      {"chacha seal NT stores again", enc_b, hashed, [&] {
         hipLaunchKernelGGL((qfec::c20p1305_seal_kernel<16, true>), dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, as); }},
      {"aes128gcm seal (product)", enc_b, hashed, [&] { CK(qfec::launch_aes128gcm(as, false, 0)); }},
      {"aes128gcm seal NT stores", enc_b, hashed, [&] {
         hipLaunchKernelGGL((qfec::aes128gcm_kernel<8, false, qfec::kGcmNB, 512, 2, true, false, true>),
                            dim3((uint32_t)((n + 511) / 512)), dim3(512), 0, 0, as); }},
      {"aes128gcm seal (product) again", enc_b, hashed, [&] { CK(qfec::launch_aes128gcm(as, false, 0)); }},
      {"aes128gcm seal NT stores again", enc_b, hashed, [&] {
         hipLaunchKernelGGL((qfec::aes128gcm_kernel<8, false, qfec::kGcmNB, 512, 2, true, false, true>),
                            dim3((uint32_t)((n + 511) / 512)), dim3(512), 0, 0, as); }},
      {"chacha20poly1305 seal SC=16", enc_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::c20p1305_seal_kernel<16>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, as); }},
      {"chacha20poly1305 open SC=16", dec_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::c20p1305_open_kernel<16>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, ao); }},
      {"chacha20poly1305 seal SC=8", enc_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::c20p1305_seal_kernel<8>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, as); }},
      {"chacha20poly1305 open SC=8", dec_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::c20p1305_open_kernel<8>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, ao); }},
      {"chacha20poly1305 seal SC=4", enc_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::c20p1305_seal_kernel<4>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, as); }},
      {"null encrypt staged SC=4", enc_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::null_encrypt_staged_kernel<4>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, e); }},
      {"null encrypt staged SC=8", enc_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::null_encrypt_staged_kernel<8>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, e); }},
      {"FNV step VALU-only (4 KiB/lane)", 0.0, (double)vgrid * 256 * vb,
       [&] { hipLaunchKernelGGL(fnv_valu_kernel, dim3(vgrid), dim3(256), 0, 0, vb, sink); }},
      {"FNV chunk VALU-only R3", 0.0, (double)vgrid * 256 * vb,
       [&] { hipLaunchKernelGGL(fnv_valu_chunk_kernel<true>, dim3(vgrid), dim3(256), 0, 0, vb, sink); }},
      // occupancy forced by dynamic LDS: 128 KiB -> 1 wave/SIMD, 64 KiB -> 2, 40 KiB -> 4
      {"FNV chunk VALU-only R3 @1 wave/SIMD", 0.0, (double)vgrid * 256 * vb,
       [&] { hipLaunchKernelGGL(fnv_valu_chunk_kernel<true>, dim3(vgrid), dim3(256), 128 << 10, 0, vb, sink); }},
      {"FNV chunk VALU-only R3 @2 waves/SIMD", 0.0, (double)vgrid * 256 * vb,
       [&] { hipLaunchKernelGGL(fnv_valu_chunk_kernel<true>, dim3(vgrid), dim3(256), 64 << 10, 0, vb, sink); }},
      {"FNV chunk VALU-only R3 @4 waves/SIMD", 0.0, (double)vgrid * 256 * vb,
       [&] { hipLaunchKernelGGL(fnv_valu_chunk_kernel<true>, dim3(vgrid), dim3(256), 40 << 10, 0, vb, sink); }},
      {"FNV 2-chain VALU-only @2 waves/SIMD", 0.0, (double)vgrid * 256 * vb,
       [&] { hipLaunchKernelGGL(fnv_valu_chunk2_kernel, dim3(vgrid), dim3(256), 64 << 10, 0, vb, sink); }},
      {"FNV 2-chain VALU-only @8 waves/SIMD", 0.0, (double)vgrid * 256 * vb,
       [&] { hipLaunchKernelGGL(fnv_valu_chunk2_kernel, dim3(vgrid), dim3(256), 0, 0, vb, sink); }},
      {"FNV chunk VALU-only serial", 0.0, (double)vgrid * 256 * vb,
       [&] { hipLaunchKernelGGL(fnv_valu_chunk_kernel<false>, dim3(vgrid), dim3(256), 0, 0, vb, sink); }},
      {"null encrypt staged serial FNV", enc_b, hashed, [&] {
         hipLaunchKernelGGL((qfec::null_encrypt_staged_kernel<16, false>), dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, e); }},
      {"glds SC=16 NB=2", enc_b, hashed, glds[0].second},
      {"glds SC=8 NB=2", enc_b, hashed, glds[1].second},
      {"glds SC=8 NB=3", enc_b, hashed, glds[2].second},
      {"glds SC=4 NB=3", enc_b, hashed, glds[3].second},
      {"glds SC=4 NB=4", enc_b, hashed, glds[4].second},
      {"glds2 SC=16 NB=2", enc_b, hashed, glds[5].second},
      {"glds2 SC=8 NB=2", enc_b, hashed, glds[6].second},
      {"glds2 SC=8 NB=3", enc_b, hashed, glds[7].second},
      {"swz SC=8 x4", enc_b, hashed, glds[8].second},
      {"swz SC=8 x3", enc_b, hashed, glds[9].second},
      {"swz SC=16 x2", enc_b, hashed, glds[10].second},
      {"null encrypt (product) again", enc_b, hashed, [&] { CK(qfec::launch_null_protect(e, false, 0)); }},
      {"swz SC=8 x4 again", enc_b, hashed, glds[8].second},
      {"ALIGNED staged (product)", enc_b, hashed, [&] { CK(qfec::launch_null_protect(ea, false, 0)); }},
      {"ALIGNED staged SC=8", enc_b, hashed, [&] { hipLaunchKernelGGL((qfec::null_encrypt_staged_kernel<8>), dim3(sblocks), dim3(256), 0, 0, ea); }},
      {"ALIGNED glds SC=16 NB=2", enc_b, hashed, [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds_kernel<16, 2>), dim3(gblocks), dim3(64), 0, 0, ea); }},
      {"ALIGNED glds SC=8 NB=2", enc_b, hashed, [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds_kernel<8, 2>), dim3(gblocks), dim3(64), 0, 0, ea); }},
      {"ALIGNED glds SC=8 NB=3", enc_b, hashed, [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds_kernel<8, 3>), dim3(gblocks), dim3(64), 0, 0, ea); }},
      {"nt staged enc SC=16", enc_b, hashed, [&] { hipLaunchKernelGGL((qfec::null_encrypt_staged_kernel<16, true, 1>), dim3(sblocks), dim3(256), 0, 0, e); }},
      {"default-store staged enc SC=16", enc_b, hashed, [&] { hipLaunchKernelGGL((qfec::null_encrypt_staged_kernel<16, true, 0>), dim3(sblocks), dim3(256), 0, 0, e); }},
      {"nt staged dec SC=16", dec_b, hashed, [&] { hipLaunchKernelGGL((qfec::null_decrypt_staged_kernel<16, true, 1>), dim3(sblocks), dim3(256), 0, 0, d); }},
      {"default-store staged dec SC=16", dec_b, hashed, [&] { hipLaunchKernelGGL((qfec::null_decrypt_staged_kernel<16, true, 0>), dim3(sblocks), dim3(256), 0, 0, d); }},
      {"SRC128-DST48 staged (product)", enc_b, hashed, [&] { CK(qfec::launch_null_protect(eC, false, 0)); }},
      {"SRC-ALIGNED staged (product)", enc_b, hashed, [&] { CK(qfec::launch_null_protect(eA, false, 0)); }},
      {"SRC-ALIGNED glds SC=16 NB=2", enc_b, hashed, [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds_kernel<16, 2>), dim3(gblocks), dim3(64), 0, 0, eA); }},
      {"DST-ALIGNED staged (product)", enc_b, hashed, [&] { CK(qfec::launch_null_protect(eB, false, 0)); }},
      {"DST-ALIGNED glds SC=16 NB=2", enc_b, hashed, [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds_kernel<16, 2>), dim3(gblocks), dim3(64), 0, 0, eB); }},
      {"ALIGNED glds SC=4 NB=3", enc_b, hashed, [&] { hipLaunchKernelGGL((qfec::null_encrypt_glds_kernel<4, 3>), dim3(gblocks), dim3(64), 0, 0, ea); }},
      {"null decrypt staged serial FNV", dec_b, hashed, [&] {
         hipLaunchKernelGGL((qfec::null_decrypt_staged_kernel<16, false>), dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, d); }},
  };
  {  // per-wave timeline of the encrypt kernel
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    uint64_t* d_tl;
    CK(hipMalloc(&d_tl, 8ull * 8 * blocks * 4));
    hipLaunchKernelGGL(qfec::null_enc_timed, dim3(blocks), dim3(256), 0, 0, e, d_tl);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(qfec::null_enc_timed, dim3(blocks), dim3(256), 0, 0, e, d_tl);
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> tl(8ull * blocks * 4);
    CK(hipMemcpy(tl.data(), d_tl, tl.size() * 8, hipMemcpyDeviceToHost));
    uint64_t mn = UINT64_MAX, mx = 0;
    double pro = 0, life = 0, hs = 0, ws = 0, xs = 0, epi = 0;
    const uint64_t W = (uint64_t)blocks * 4;
    for (uint64_t w = 0; w < W; ++w) {
      const uint64_t* r = &tl[8 * w];
      mn = std::min(mn, r[0]);
      mx = std::max(mx, r[2]);
      pro += r[1] - r[0];
      life += r[2] - r[0];
      hs += r[3];
      ws += r[4];
      xs += r[5];
      epi += (r[2] - r[1]) - (r[3] + r[4] + r[5]);
    }
    std::printf("timeline (us, mean per wave; 1 tick = 10 ns): life %.2f = prologue %.2f + "
                "lds/issue %.2f + hash %.2f + wait/store %.2f + rest %.2f; kernel span %.1f us, "
                "waves %llu\n",
                life / W / 100, pro / W / 100, xs / W / 100, hs / W / 100, ws / W / 100,
                epi / W / 100, (mx - mn) / 100.0, (unsigned long long)W);
    CK(hipFree(d_tl));
  }
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(fnv_valu_chunk_kernel<true>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(fnv_valu_chunk2_kernel),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> ms(vs.size());
  for (auto& v : vs) v.run();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(e0, 0));
      for (int q = 0; q < reps; ++q) vs[i].run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[i].push_back(t / reps);
    }
  std::printf("%-40s %10s %10s %12s\n", "variant", "ms", "HBM GB/s", "hashed GB/s");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = ms[i];
    std::sort(v.begin(), v.end());
    const double t = v[v.size() / 2] * 1e-3;
    std::printf("%-40s %10.3f %10.1f %12.1f\n", vs[i].name.c_str(), t * 1e3, vs[i].bytes / t / 1e9,
                vs[i].hashed / t / 1e9);
  }
  return 0;
}
