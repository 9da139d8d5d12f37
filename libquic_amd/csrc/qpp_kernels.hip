// qpp_kernels.hip — gfx950 kernels for QUIC packet protection around FEC:
// the NULL "encryption" libquic uses before the handshake completes
// (ENCRYPTION_NONE): a 12-byte FNV-1a-128 tag of header || payload in front
// of the payload.
//
//   encrypt  NullEncrypter::EncryptPacket   crypto/null_encrypter.cc:28-47
//   decrypt  NullDecrypter::DecryptPacket   crypto/null_decrypter.cc:38-64
//   hash     QuicUtils::FNV1a_128_Hash_Two  quic_utils.cc:110-125
//            (h = (h ^ octet) * (2^88 + 315) mod 2^128, quic_utils.cc:31-50)
//
// FNV-1a is a strict byte-serial recurrence — no associativity to split a
// packet across lanes — so the parallel axis is the packet: one lane per
// packet, every lane running its own recurrence.  The 128-bit state lives in
// four 32-bit limbs; one byte step is
//     x ^= octet;  x = x*315 + (x << 88)            (mod 2^128)
// = four v_mad_u64_u32 (the x*315 carry chain, with x0*2^24 folded into the
// third limb's addend) + one v_mul_lo_u32 + a shift/add for the top limb:
// ≈12 instructions, ≈23 VALU issue slots per byte (the 64-bit mads are
// multi-pass) — VALU-bound at ≈3.5 TB/s of hashed bytes on the chip
// (tools/tune/tune_protect.hip, register-only microbenchmark).
//
// Memory: the payload bytes move by coalesced wave loads through an LDS
// transpose (see "LDS-staged forms"); a lane loading its own packet (64
// scattered 16-B pieces per wave instruction) ran at ~0.5x.
//
// In-place encryption (QuicPacketCreator::EncryptInPlace: output == payload,
// payload shifted right by the tag) is supported: the last len % 16 bytes
// are loaded first, a slab is stored only after the next slab's loads have
// completed, and the tag is written last.  Decrypt verifies first and copies
// the payload only when the tag matches (output untouched otherwise, as the
// reference's memcpy-after-check).
#include "qfec_internal.h"

namespace qfec {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;
constexpr uint32_t kTag = 12;  // kHashSizeShort, null_encrypter.cc:15

struct Fnv128 {
  uint32_t x0, x1, x2, x3;  // little-endian limbs
};

// kOffset = 144066263297769815596495629667062367629 (quic_utils.cc:114-116)
__device__ __forceinline__ Fnv128 fnv_init() {
  const uint64_t lo = 7113472399480571277ull, hi = 7809847782465536322ull;
  return Fnv128{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}

// h = (h ^ b) * (2^88 + 315) mod 2^128
__device__ __forceinline__ void fnv_step(Fnv128& h, uint32_t b) {
  const uint32_t x0 = h.x0 ^ b;
  const uint64_t t0 = (uint64_t)x0 * 315u;
  const uint64_t t1 = (uint64_t)h.x1 * 315u + (t0 >> 32);
  // limb 2 also receives bits 0..31 of (x << 88) = x0 << 24, and its carry
  // out the bits x0 >> 8 that belong to limb 3
  const uint64_t t2 = (uint64_t)h.x2 * 315u + ((uint64_t)x0 << 24) + (t1 >> 32);
  const uint32_t r3 = h.x3 * 315u + (uint32_t)(t2 >> 32) + (h.x1 << 24);
  h.x0 = (uint32_t)t0;
  h.x1 = (uint32_t)t1;
  h.x2 = (uint32_t)t2;
  h.x3 = r3;
}

__device__ __forceinline__ void fnv_word(Fnv128& h, uint32_t w) {
  fnv_step(h, w & 0xFFu);
  fnv_step(h, (w >> 8) & 0xFFu);
  fnv_step(h, (w >> 16) & 0xFFu);
  fnv_step(h, w >> 24);
}

__device__ __forceinline__ void fnv_chunk(Fnv128& h, u32x4 v) {
  fnv_word(h, v.x);
  fnv_word(h, v.y);
  fnv_word(h, v.z);
  fnv_word(h, v.w);
}

__device__ __forceinline__ uint32_t byte_of(u32x4 v, uint32_t i) {
  const uint32_t w = i < 4u ? v.x : i < 8u ? v.y : i < 12u ? v.z : v.w;
  return (w >> (8u * (i & 3u))) & 0xFFu;
}

__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
  u32x4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) { __builtin_memcpy(p, &v, 16); }

// The last len % 16 bytes of a span as the upper bytes of one 16-byte chunk
// (len >= 16: the 16 bytes ending at the span end) or, for len < 16, the
// whole span byte by byte into bytes [0, len).
__device__ __forceinline__ u32x4 load_tail(const uint8_t* p, uint32_t len) {
  if (len >= 16u) return ld16(p + len - 16u);
  uint8_t b[16];
#pragma unroll
  for (uint32_t i = 0; i < 16u; ++i) b[i] = i < len ? p[i] : (uint8_t)0;
  u32x4 v;
  __builtin_memcpy(&v, b, 16);
  return v;
}

// Hash the bytes of a span that load_tail returned.
__device__ __forceinline__ void fnv_tail(Fnv128& h, u32x4 v, uint32_t len) {
  const uint32_t rem = len & 15u;
  if (rem == 0u) return;
  const uint32_t first = len >= 16u ? 16u - rem : 0u;
  for (uint32_t i = first; i < first + rem; ++i) fnv_step(h, byte_of(v, i));
}

// Per-lane loads (the header: a few chunks per packet) go in batches of
// kBatch 16-byte chunks issued back to back.
constexpr uint32_t kBatch = 8;

// Hash a span (no copy).
__device__ __forceinline__ void fnv_span(Fnv128& h, const uint8_t* p, uint32_t len) {
  const uint32_t nfull = len >> 4;
  const u32x4 tail = load_tail(p, len);
  for (uint32_t c = 0; c < nfull; c += kBatch) {
    u32x4 v[kBatch];
#pragma unroll
    for (uint32_t u = 0; u < kBatch; ++u) v[u] = ld16(p + 16u * min(c + u, nfull - 1u));
#pragma unroll
    for (uint32_t u = 0; u < kBatch; ++u)
      if (c + u < nfull) fnv_chunk(h, v[u]);
  }
  fnv_tail(h, tail, len);
}

// Store the tail bytes of a span (counterpart of load_tail).
__device__ __forceinline__ void store_tail(uint8_t* d, u32x4 v, uint32_t len) {
  if ((len & 15u) == 0u) return;
  if (len >= 16u) {
    st16(d + len - 16u, v);  // overlaps the last full chunk with identical bytes
    return;
  }
  for (uint32_t i = 0; i < len; ++i) d[i] = (uint8_t)byte_of(v, i);
}

// ---------------------------------------------------------------------------
// LDS-staged forms: a wave owns 64 packets (lane q hashes packet q) but the
// payload bytes are moved by coalesced wave loads — lane 8i+m of load
// instruction I fetches chunk m of the current 128-byte slab of packet 8I+i,
// so one instruction reads 8 packets x 128 contiguous bytes (8-16 cache
// lines) instead of 64 scattered 16-byte pieces — and transposed through LDS
// (row stride 144 B: the hashing lanes' ds_read_b128 hit disjoint banks).
// Encrypt stores the payload copy from the loading lanes' registers (again 8
// packets x 128 B per instruction).  The header and the last len % 16 bytes
// stay per lane (load_tail / fnv_span).
// ---------------------------------------------------------------------------
// 16-B chunks per packet per slab.  256-B slabs: the hashing of one slab
// (~2,600 VALU instructions per lane) covers the next slab's load latency at
// the 2 waves/SIMD the LDS rows allow; 128-B slabs measured 0.82x, 64-B 0.65x
// (profiles/round1/tune_protect_p4.txt).
constexpr uint32_t kSlabChunks = 16;
constexpr int kWaves = kBlock / 64;

struct StageMeta {
  const uint8_t* src;  // payload start
  uint8_t* dst;        // payload copy destination (nullptr: no copy)
  uint32_t nfull;      // full 16-B chunks
};

// Cooperative load of slab `sl` (SC chunks per packet) for the wave's 64
// packets: lane (SC*i + m) of instruction I takes chunk m of packet
// (64/SC)*I + i; SC instructions cover the 64 packets.
template <uint32_t SC>
__device__ __forceinline__ void stage_load(const StageMeta* meta, uint32_t lane, uint32_t sl,
                                           u32x4 (&v)[SC]) {
  const uint32_t i = lane / SC, m = lane % SC;
  const uint32_t c = sl * SC + m;
#pragma unroll
  for (uint32_t I = 0; I < SC; ++I) {
    const StageMeta& q = meta[(64u / SC) * I + i];
    if (c < q.nfull) v[I] = ld16(q.src + 16u * c);
  }
}

template <uint32_t SC>
__device__ __forceinline__ void stage_store(const StageMeta* meta, uint32_t lane, uint32_t sl,
                                            const u32x4 (&v)[SC]) {
  const uint32_t i = lane / SC, m = lane % SC;
  const uint32_t c = sl * SC + m;
#pragma unroll
  for (uint32_t I = 0; I < SC; ++I) {
    const StageMeta& q = meta[(64u / SC) * I + i];
    if (c < q.nfull && q.dst) st16(q.dst + 16u * c, v[I]);
  }
}

// LDS rows of SC + 1 chunks (16 B of padding: the hashing lanes' ds_read_b128
// of one row each fall on disjoint banks for SC = 4, 8).
template <uint32_t SC>
__device__ __forceinline__ void stage_to_lds(u32x4* rows, uint32_t lane, const u32x4 (&v)[SC]) {
  const uint32_t i = lane / SC, m = lane % SC;
#pragma unroll
  for (uint32_t I = 0; I < SC; ++I) rows[((64u / SC) * I + i) * (SC + 1u) + m] = v[I];
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// Hash (and, when meta[].dst is set, copy) the full chunks of the wave's 64
// payloads.  In-place safe for dst == src + 12: slab s is stored only after
// slab s+1 has been loaded AND the loads have completed (waitcnt), so no store
// overtakes a load of the 12 bytes it overwrites.
template <bool COPY, uint32_t SC>
__device__ __forceinline__ void stage_hash(Fnv128& h, const StageMeta* meta, u32x4* rows,
                                           uint32_t lane, uint32_t my_nfull) {
  const uint32_t nslab = (wave_max_u32(my_nfull) + SC - 1) / SC;
  u32x4 cur[SC], nxt[SC];
  if (nslab) stage_load<SC>(meta, lane, 0, cur);
  for (uint32_t sl = 0; sl < nslab; ++sl) {
    stage_to_lds<SC>(rows, lane, cur);
    if (sl + 1u < nslab) stage_load<SC>(meta, lane, sl + 1u, nxt);
#pragma unroll
    for (uint32_t j = 0; j < SC; ++j)
      if (sl * SC + j < my_nfull) fnv_chunk(h, rows[lane * (SC + 1u) + j]);
    if constexpr (COPY) {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the next slab's loads are done
      stage_store<SC>(meta, lane, sl, cur);
    }
#pragma unroll
    for (uint32_t j = 0; j < SC; ++j) cur[j] = nxt[j];
  }
}

template <uint32_t SC>
__global__ __launch_bounds__(kBlock) void null_encrypt_staged_kernel(ProtectArgs a) {
  __shared__ u32x4 s_rows[kWaves][64 * (SC + 1u)];
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
  s_meta[wv][lane] = StageMeta{pt, o + kTag, plen >> 4};
  // the payload's last len % 16 bytes, before any store (in place)
  const u32x4 tail = valid ? load_tail(pt, plen) : u32x4{0u, 0u, 0u, 0u};
  Fnv128 h = fnv_init();
  if (valid) fnv_span(h, ad, alen);
  stage_hash<true, SC>(h, s_meta[wv], s_rows[wv], lane, plen >> 4);
  if (!valid) return;
  fnv_tail(h, tail, plen);
  store_tail(o + kTag, tail, plen);
  const uint32_t tag[3] = {h.x0, h.x1, h.x2};
  __builtin_memcpy(o, tag, kTag);
}

template <uint32_t SC>
__global__ __launch_bounds__(kBlock) void null_decrypt_staged_kernel(ProtectArgs a) {
  __shared__ u32x4 s_rows[kWaves][64 * (SC + 1u)];
  __shared__ StageMeta s_meta[kWaves][64];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint32_t clen = p < a.n ? a.in_len[p] : 0u;
  const bool valid = p < a.n && clen >= kTag;
  if (p < a.n && !valid) a.ok[p] = 0;  // ReadHash fails (null_decrypter.cc:48-50)
  const uint8_t* ad = nullptr;
  const uint8_t* ct = nullptr;
  uint32_t alen = 0, plen = 0;
  uint32_t tag[3] = {0u, 0u, 0u};
  if (valid) {
    ad = a.bytes + a.ad_off[p];
    ct = a.bytes + a.in_off[p];
    alen = a.ad_len[p];
    plen = clen - kTag;
    __builtin_memcpy(tag, ct, kTag);
  }
  s_meta[wv][lane] = StageMeta{ct + kTag, nullptr, plen >> 4};
  const u32x4 tail = valid ? load_tail(ct + kTag, plen) : u32x4{0u, 0u, 0u, 0u};
  Fnv128 h = fnv_init();
  if (valid) fnv_span(h, ad, alen);
  stage_hash<false, SC>(h, s_meta[wv], s_rows[wv], lane, plen >> 4);
  // ComputeHash keeps the low 96 bits (null_decrypter.cc:97-106)
  bool ok = false;
  if (valid) {
    fnv_tail(h, tail, plen);
    ok = h.x0 == tag[0] && h.x1 == tag[1] && h.x2 == tag[2];
    a.ok[p] = ok ? 1 : 0;
  }
  // copy after the check (null_decrypter.cc:60-62), coalesced, verified packets only
  uint8_t* o = ok ? a.out + a.out_off[p] : nullptr;
  s_meta[wv][lane] = StageMeta{ct + kTag, o, ok ? plen >> 4 : 0u};
  const uint32_t nslab = (wave_max_u32(ok ? plen >> 4 : 0u) + SC - 1) / SC;
  for (uint32_t sl = 0; sl < nslab; ++sl) {
    u32x4 v[SC];
    stage_load<SC>(s_meta[wv], lane, sl, v);
    stage_store<SC>(s_meta[wv], lane, sl, v);
  }
  if (ok) store_tail(o, tail, plen);
}

}  // namespace

hipError_t launch_null_protect(const ProtectArgs& a0, bool decrypt, hipStream_t s) {
  const uint64_t chunk = (uint64_t)0x7FFFFFFF * kBlock;
  for (uint64_t p = 0; p < a0.n; p += chunk) {
    ProtectArgs a = a0;
    a.n = a0.n - p < chunk ? a0.n - p : chunk;
    a.ad_off += p;
    a.ad_len += p;
    a.in_off += p;
    a.in_len += p;
    a.out_off += p;
    if (decrypt) a.ok += p;
    const uint32_t blocks = (uint32_t)((a.n + kBlock - 1) / kBlock);
    if (decrypt)
      hipLaunchKernelGGL(null_decrypt_staged_kernel<kSlabChunks>, dim3(blocks), dim3(kBlock), 0, s, a);
    else
      hipLaunchKernelGGL(null_encrypt_staged_kernel<kSlabChunks>, dim3(blocks), dim3(kBlock), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace qfec
