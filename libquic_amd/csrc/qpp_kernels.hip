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
// (tools/tune/tune_protect.hip, register-only microbenchmark).  Payload
// chunks take three bytes per multiply instead (fnv_step3: the same
// recurrence, regrouped exactly).
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

[[maybe_unused]] __device__ __forceinline__ void fnv_word(Fnv128& h, uint32_t w) {
  fnv_step(h, w & 0xFFu);
  fnv_step(h, (w >> 8) & 0xFFu);
  fnv_step(h, (w >> 16) & 0xFFu);
  fnv_step(h, w >> 24);
}

// Three byte steps at once, equal to fnv_step(b0); fnv_step(b1); fnv_step(b2).
// P = 2^88 + 315 is 59 mod 256, so the state's low byte runs on its own,
// y' = 59 (y ^ b) mod 256 (`y` carries it: h.x0 & 0xFF on entry and exit),
// and XORing b into a state whose low byte is y ADDS d = (y ^ b) - y.  So
//     h3 = (h ^ b0) P^3 + d1 P^2 + d2 P                       (mod 2^128)
// with P^j = 315^j + j 315^(j-1) 2^88 (2^176 = 0 mod 2^128):
//     P^3 = 31255875 + 297675 2^88,  P^2 = 99225 + 630 2^88,  P = 315 + 2^88.
// Per three bytes: one 128 x 25-bit multiply (3 v_mad_u64_u32 + 1 mul) and a
// 40-bit product for the 2^88 column, plus full-rate 24-bit byte-chain ops,
// instead of three dependent 128 x 9-bit multiplies — ~17 instead of ~23
// VALU issue slots per byte, and one multiply instead of twelve on the
// loop-carried limb-0 chain (the d's come from the cheap y chain).
// d1, d2 lie in (-256, 256), yet every partial sum below is nonnegative: a
// negative d needs a nonzero t0 (the low byte of x0), and then
// x0 * 315^3 >= 31255875 > |99225 d1 + 315 d2| (<= 25382700), so the carries
// are plain unsigned ones (tools/tune/fnv_r3_check.c checks it all on the host).
__device__ __forceinline__ void fnv_step3(Fnv128& h, uint32_t& y, uint32_t b0, uint32_t b1,
                                          uint32_t b2) {
  constexpr uint32_t kC3 = 31255875u, kC3h = 297675u;  // 315^3, 3 * 315^2
  const uint32_t t0 = y ^ b0;
  const uint32_t y1 = (t0 * 59u) & 0xFFu;
  const uint32_t t1 = y1 ^ b1;
  const uint32_t y2 = (t1 * 59u) & 0xFFu;
  const uint32_t t2 = y2 ^ b2;
  y = (t2 * 59u) & 0xFFu;
  const int32_t d1 = (int32_t)t1 - (int32_t)y1;
  const int32_t d2 = (int32_t)t2 - (int32_t)y2;
  const uint64_t slo = (uint64_t)(int64_t)(d1 * 99225 + d2 * 315);  // low parts of d1 P^2 + d2 P
  const uint64_t shi = (uint64_t)(int64_t)(d1 * 630 + d2);          // their 2^88 coefficients
  const uint32_t x0 = h.x0 ^ b0;
  // 2^88 column mod 2^40: x * 297675 + shi, x mod 2^40 = x0 + 2^32 (x1 mod 256)
  const uint64_t u =
      (uint64_t)x0 * kC3h + shi + ((uint64_t)((h.x1 & 0xFFu) * (kC3h & 0xFFu)) << 32);
  const uint64_t q0 = (uint64_t)x0 * kC3 + slo;
  const uint64_t q1 = (uint64_t)h.x1 * kC3 + (q0 >> 32);
  const uint64_t q2 = (uint64_t)h.x2 * kC3 + (q1 >> 32) + (u << 24);
  h.x0 = (uint32_t)q0;
  h.x1 = (uint32_t)q1;
  h.x2 = (uint32_t)q2;
  h.x3 = h.x3 * kC3 + (uint32_t)(q2 >> 32);
}

// 16 bytes.  R3 (the default): five fnv_step3 + one fnv_step; otherwise 16 fnv_step.
template <bool R3 = true>
__device__ __forceinline__ void fnv_chunk(Fnv128& h, u32x4 v) {
  if constexpr (R3) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t y = h.x0 & 0xFFu;
#pragma unroll
    for (int i = 0; i < 15; i += 3)
      fnv_step3(h, y, (w[i >> 2] >> (8 * (i & 3))) & 0xFFu,
                (w[(i + 1) >> 2] >> (8 * ((i + 1) & 3))) & 0xFFu,
                (w[(i + 2) >> 2] >> (8 * ((i + 2) & 3))) & 0xFFu);
    fnv_step(h, v.w >> 24);
  } else {
    fnv_word(h, v.x);
    fnv_word(h, v.y);
    fnv_word(h, v.z);
    fnv_word(h, v.w);
  }
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

// Global-address-space forms for pointers the compiler cannot prove global
// (StageMeta entries read back from LDS): a generic pointer becomes a FLAT
// access, and FLAT loads count against lgkmcnt as well as vmcnt, so every LDS
// wait of a slab's hashing would also wait for the next slab's loads.
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef const __attribute__((address_space(1))) u32x4_a1* gld_ptr;
typedef __attribute__((address_space(1))) u32x4_a1* gst_ptr;
__device__ __forceinline__ u32x4 ld16g(const uint8_t* p) { return *(gld_ptr)p; }
__device__ __forceinline__ void st16g(uint8_t* p, u32x4 v) { *(gst_ptr)p = v; }
// nontemporal forms (streamed once: no L2 retention)
__device__ __forceinline__ u32x4 ld16gn(const uint8_t* p) {
  return __builtin_nontemporal_load((gld_ptr)p);
}
__device__ __forceinline__ void st16gn(uint8_t* p, u32x4 v) {
  __builtin_nontemporal_store(v, (gst_ptr)p);
}

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
template <bool R3 = true>
__device__ __forceinline__ void fnv_span(Fnv128& h, const uint8_t* p, uint32_t len) {
  const uint32_t nfull = len >> 4;
  const u32x4 tail = load_tail(p, len);
  for (uint32_t c = 0; c < nfull; c += kBatch) {
    u32x4 v[kBatch];
#pragma unroll
    for (uint32_t u = 0; u < kBatch; ++u) v[u] = ld16(p + 16u * min(c + u, nfull - 1u));
#pragma unroll
    for (uint32_t u = 0; u < kBatch; ++u)
      if (c + u < nfull) fnv_chunk<R3>(h, v[u]);
  }
  fnv_tail(h, tail, len);
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
  const uint8_t* src;  // payload start (chunk c at src + 16 c)
  uint8_t* dst;        // payload copy destination (nullptr: no copy)
  uint32_t nfull;      // chunks [lo, nfull) are the packet's
  uint32_t lo;         // (0 when omitted; > 0: slabs start on a 128-B line, line_meta)
};

// The staged rows pass data between lanes of one wave through LDS: the LDS
// executes a wave's accesses in program order, so no hardware wait is needed,
// but the compiler must not move a lane's own-row access across another
// lane's cooperative access (it sees no aliasing for the single lane).
// Wavefront-scope fences around a wave barrier pin that order (no s_waitcnt).
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Cooperative load of slab `sl` (SC chunks per packet) for the wave's 64
// packets: lane (SC*i + m) of instruction I takes chunk m of packet
// (64/SC)*I + i; SC instructions cover the 64 packets.
template <uint32_t SC, bool G = true, bool NT = false>
__device__ __forceinline__ void stage_load(const StageMeta* meta, uint32_t lane, uint32_t sl,
                                           u32x4 (&v)[SC]) {
  const uint32_t i = lane / SC, m = lane % SC;
  const uint32_t c = sl * SC + m;
  wave_lds_order();  // the lanes' meta entries are written (cross-lane reads follow)
#pragma unroll
  for (uint32_t I = 0; I < SC; ++I) {
    const StageMeta& q = meta[(64u / SC) * I + i];
    if (c >= q.lo && c < q.nfull)
      v[I] = NT ? ld16gn(q.src + 16u * c) : G ? ld16g(q.src + 16u * c) : ld16(q.src + 16u * c);
  }
  wave_lds_order();
}

template <uint32_t SC, bool G = true, bool NT = false>
__device__ __forceinline__ void stage_store(const StageMeta* meta, uint32_t lane, uint32_t sl,
                                            const u32x4 (&v)[SC]) {
  const uint32_t i = lane / SC, m = lane % SC;
  const uint32_t c = sl * SC + m;
  wave_lds_order();
#pragma unroll
  for (uint32_t I = 0; I < SC; ++I) {
    const StageMeta& q = meta[(64u / SC) * I + i];
    if (c >= q.lo && c < q.nfull && q.dst) {
      if (NT) st16gn(q.dst + 16u * c, v[I]);
      else if (G) st16g(q.dst + 16u * c, v[I]);
      else st16(q.dst + 16u * c, v[I]);
    }
  }
  wave_lds_order();  // before a lane rewrites its meta entry
}

// LDS rows of SC + 1 chunks (16 B of padding: the hashing lanes' ds_read_b128
// of one row each fall on disjoint banks for SC = 4, 8).
template <uint32_t SC>
__device__ __forceinline__ void stage_to_lds(u32x4* rows, uint32_t lane, const u32x4 (&v)[SC]) {
  const uint32_t i = lane / SC, m = lane % SC;
  wave_lds_order();  // earlier reads of the rows (own row, stage_from_lds) first
#pragma unroll
  for (uint32_t I = 0; I < SC; ++I) rows[((64u / SC) * I + i) * (SC + 1u) + m] = v[I];
  wave_lds_order();  // then the lanes read their own rows
}

__device__ __forceinline__ bool wave_any_qpp(bool p) { return __ballot(p) != 0ull; }

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// Hash (and, when meta[].dst is set, copy) the full chunks of the wave's 64
// payloads.  In-place safe for dst == src + 12: slab s is stored only after
// slab s+1 has been loaded AND the loads have completed (waitcnt), so no store
// overtakes a load of the 12 bytes it overwrites.
// NT: 0 default cache policy, 1 nontemporal slab loads and stores, 2 stores
// only (the NULL kernels' default: the copy's destination is not read again;
// nt stores measured +7% / +7% (encrypt / decrypt, 2^21 packets) on one box
// and +3% / +8% on another, profiles/round3/null_align/tune_protect_nt_store*.txt;
// nt LOADS cost -4% / -15%: the decrypt's copy pass re-reads the ciphertext
// the hash pass loaded.  The AEAD kernels keep default stores: nt measured
// -3% on ChaCha20-Poly1305 seal and -0.5% on AES-GCM seal, kAeadNTS)
constexpr int kNullNT = 2;
template <bool COPY, uint32_t SC, bool R3 = true, bool INPLACE = true, int NT = 0>
__device__ __forceinline__ void stage_hash(Fnv128& h, const StageMeta* meta, u32x4* rows,
                                           uint32_t lane, uint32_t my_nfull,
                                           uint32_t my_lo = 0u) {
  const uint32_t nslab = (wave_max_u32(my_nfull) + SC - 1) / SC;
  u32x4 cur[SC], nxt[SC];
  if (nslab) stage_load<SC, true, NT == 1>(meta, lane, 0, cur);
  for (uint32_t sl = 0; sl < nslab; ++sl) {
    stage_to_lds<SC>(rows, lane, cur);
    if (sl + 1u < nslab) stage_load<SC, true, NT == 1>(meta, lane, sl + 1u, nxt);
#pragma unroll
    for (uint32_t j = 0; j < SC; ++j)
      if (sl * SC + j >= my_lo && sl * SC + j < my_nfull)
        fnv_chunk<R3>(h, rows[lane * (SC + 1u) + j]);
    if constexpr (COPY) {
      // in place: vmcnt(0), the next slab's loads are done before this slab's
      // stores overwrite them; out of place the stores go out at once
      if constexpr (INPLACE) __builtin_amdgcn_s_waitcnt(0x0F70);
      stage_store<SC, true, NT != 0>(meta, lane, sl, cur);
    }
#pragma unroll
    for (uint32_t j = 0; j < SC; ++j) cur[j] = nxt[j];
  }
}

// Destination-aligned chunking.  A 16-B store that straddles a 16-B boundary
// costs the memory pipeline about as much as two: with the payload copy's
// destination unaligned (the tag shifts it by 12 from wherever the output
// sits), encrypt ran 1.86 ms on 2^21 packets against 1.45 with the output
// 16-B aligned and the input still unaligned (1.33 with both aligned;
// profiles/round3/null_align/).  So the coalesced chunks are cut where the
// DESTINATION is 16-B aligned: the first hd = (16 - dst % 16) % 16 payload
// bytes (the head) and the last (plen - hd) % 16 (the tail) are hashed and
// stored by the packet's own lane; the hash is byte-serial, so cutting the
// bytes differently changes nothing in the tag.
__device__ __forceinline__ uint32_t word_sel(u32x4 v, uint32_t w) {
  return w == 0u ? v.x : w == 1u ? v.y : w == 2u ? v.z : w == 3u ? v.w : 0u;
}
// bytes [i, i + 4) of a chunk (zero past byte 15)
__device__ __forceinline__ uint32_t bytes4_at(u32x4 v, uint32_t i) {
  return __builtin_amdgcn_alignbyte(word_sel(v, (i >> 2) + 1u), word_sel(v, i >> 2), i & 3u);
}
__device__ __forceinline__ void fnv_bytes(Fnv128& h, u32x4 v, uint32_t from, uint32_t n) {
  for (uint32_t i = from; i < from + n; ++i) fnv_step(h, byte_of(v, i));
}
// bytes [from, from + n) of v to p, n < 16, p + n 16-B aligned: peeled 1, 2, 4, 8
// (each piece lands on its own alignment)
__device__ __forceinline__ void store_to_aligned_end(uint8_t* p, u32x4 v, uint32_t from,
                                                     uint32_t n) {
  uint32_t i = 0;
  if (n & 1u) {
    p[0] = (uint8_t)byte_of(v, from);
    i = 1;
  }
  if (n & 2u) {
    *(uint16_t*)(p + i) = (uint16_t)bytes4_at(v, from + i);
    i += 2;
  }
  if (n & 4u) {
    *(uint32_t*)(p + i) = bytes4_at(v, from + i);
    i += 4;
  }
  if (n & 8u) {
    const uint64_t lo = bytes4_at(v, from + i), hi = bytes4_at(v, from + i + 4u);
    *(uint64_t*)(p + i) = lo | (hi << 32);
  }
}
// bytes [from, from + n) of v to p, n < 16, p 16-B aligned: 8, 4, 2, 1
__device__ __forceinline__ void store_from_aligned_start(uint8_t* p, u32x4 v, uint32_t from,
                                                         uint32_t n) {
  uint32_t i = 0;
  if (n & 8u) {
    const uint64_t lo = bytes4_at(v, from), hi = bytes4_at(v, from + 4u);
    *(uint64_t*)p = lo | (hi << 32);
    i = 8;
  }
  if (n & 4u) {
    *(uint32_t*)(p + i) = bytes4_at(v, from + i);
    i += 4;
  }
  if (n & 2u) {
    *(uint16_t*)(p + i) = (uint16_t)bytes4_at(v, from + i);
    i += 2;
  }
  if (n & 1u) p[i] = (uint8_t)byte_of(v, from + i);
}
// the first min(16, len) bytes of a span at bytes [0, ..) of a chunk
__device__ __forceinline__ u32x4 load_head(const uint8_t* p, uint32_t len) {
  return len >= 16u ? ld16(p) : load_tail(p, len);
}

// Split of a payload of plen bytes copied to dst: head hd bytes, nmid
// 16-B chunks starting at dst + hd (16-B aligned), tail tl bytes.
struct DstSplit {
  uint32_t hd, nmid, tl;
};
__device__ __forceinline__ DstSplit dst_split(const uint8_t* dst, uint32_t plen) {
  const uint32_t u = (uint32_t)(uintptr_t)dst & 15u;
  const uint32_t hd = min((16u - u) & 15u, plen);
  const uint32_t nmid = (plen - hd) >> 4;
  return DstSplit{hd, nmid, plen - hd - 16u * nmid};
}
// position in the load_tail chunk of payload byte x
__device__ __forceinline__ uint32_t tail_pos(uint32_t x, uint32_t plen) {
  return plen >= 16u ? x - (plen - 16u) : x;
}
// nmid 16-B chunks at src / dst, `al` (src or dst) 16-B aligned: the slab
// grid is shifted back to al's 128-B line (chunks [lo, lo + nmid) of the
// shifted grid), so every slab's run of a packet covers whole lines and a
// wave instruction touches 8 lines for 1 KiB instead of up to 12 (2^21
// packets: 1.79 -> see profiles/round3/null_align/).
__device__ __forceinline__ StageMeta line_meta(const uint8_t* src, uint8_t* dst, uint32_t nmid,
                                               const uint8_t* al) {
  const uint32_t lo = ((uint32_t)(uintptr_t)al & 127u) >> 4;
  return StageMeta{src - 16u * lo, dst ? dst - 16u * lo : nullptr, lo + nmid, lo};
}

template <uint32_t SC, bool R3 = true, int NT = kNullNT>
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
  const DstSplit sp = dst_split(o + kTag, plen);
  const StageMeta m = line_meta(pt + sp.hd, o + kTag + sp.hd, sp.nmid, o + kTag + sp.hd);
  s_meta[wv][lane] = m;
  // head and tail bytes, before any store (in place)
  const u32x4 head = valid ? load_head(pt, plen) : u32x4{0u, 0u, 0u, 0u};
  const u32x4 tail = valid ? load_tail(pt, plen) : u32x4{0u, 0u, 0u, 0u};
  Fnv128 h = fnv_init();
  if (valid) {
    fnv_span<R3>(h, ad, alen);
    fnv_bytes(h, head, 0u, sp.hd);
  }
  // does any packet of the wave write over its own payload (EncryptInPlace)?
  const bool overlap = valid && o + kTag < pt + plen && pt < o + kTag + plen;
  if (wave_any_qpp(overlap))
    stage_hash<true, SC, R3, true, NT>(h, s_meta[wv], s_rows[wv], lane, m.nfull, m.lo);
  else
    stage_hash<true, SC, R3, false, NT>(h, s_meta[wv], s_rows[wv], lane, m.nfull, m.lo);
  if (!valid) return;
  const uint32_t t0 = tail_pos(sp.hd + 16u * sp.nmid, plen);
  fnv_bytes(h, tail, t0, sp.tl);
  store_from_aligned_start(o + kTag + sp.hd + 16u * sp.nmid, tail, t0, sp.tl);
  store_to_aligned_end(o + kTag, head, 0u, sp.hd);
  const uint32_t tag[3] = {h.x0, h.x1, h.x2};
  __builtin_memcpy(o, tag, kTag);
}

template <uint32_t SC, bool R3 = true, int NT = kNullNT>
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
  uint8_t* o = nullptr;
  uint32_t alen = 0, plen = 0;
  uint32_t tag[3] = {0u, 0u, 0u};
  if (valid) {
    ad = a.bytes + a.ad_off[p];
    ct = a.bytes + a.in_off[p];
    alen = a.ad_len[p];
    plen = clen - kTag;
    o = a.out + a.out_off[p];
    __builtin_memcpy(tag, ct, kTag);
  }
  // the hash pass: chunks cut where the SOURCE is 16-B aligned (aligned loads)
  const DstSplit hs = dst_split(ct + kTag, plen);
  const StageMeta hm = line_meta(ct + kTag + hs.hd, nullptr, hs.nmid, ct + kTag + hs.hd);
  s_meta[wv][lane] = hm;
  const u32x4 head = valid ? load_head(ct + kTag, plen) : u32x4{0u, 0u, 0u, 0u};
  const u32x4 tail = valid ? load_tail(ct + kTag, plen) : u32x4{0u, 0u, 0u, 0u};
  Fnv128 h = fnv_init();
  if (valid) {
    fnv_span<R3>(h, ad, alen);
    fnv_bytes(h, head, 0u, hs.hd);
  }
  stage_hash<false, SC, R3, true, NT>(h, s_meta[wv], s_rows[wv], lane, hm.nfull, hm.lo);
  // ComputeHash keeps the low 96 bits (null_decrypter.cc:97-106)
  bool ok = false;
  if (valid) {
    fnv_bytes(h, tail, tail_pos(hs.hd + 16u * hs.nmid, plen), hs.tl);
    ok = h.x0 == tag[0] && h.x1 == tag[1] && h.x2 == tag[2];
    a.ok[p] = ok ? 1 : 0;
  }
  // copy after the check (null_decrypter.cc:60-62), coalesced, verified
  // packets only, chunks cut where the DESTINATION is 16-B aligned
  const DstSplit sp = dst_split(o, ok ? plen : 0u);
  const StageMeta cm = line_meta(ct + kTag + sp.hd, ok ? o + sp.hd : nullptr, ok ? sp.nmid : 0u,
                                 o + sp.hd);
  s_meta[wv][lane] = cm;
  // Slab s+1's loads are in flight while slab s is stored (out of place: no
  // load/store ordering hazard); a load-then-store loop parked the waves on
  // every slab's round trip (SQ_WAIT_ANY 0.76 of the decrypt's wave cycles).
  const uint32_t nslab = (wave_max_u32(ok ? cm.nfull : 0u) + SC - 1) / SC;
  u32x4 cur[SC], nxt[SC];
  if (nslab) stage_load<SC, true, NT == 1>(s_meta[wv], lane, 0, cur);
  for (uint32_t sl = 0; sl < nslab; ++sl) {
    if (sl + 1u < nslab) stage_load<SC, true, NT == 1>(s_meta[wv], lane, sl + 1u, nxt);
    stage_store<SC, true, NT != 0>(s_meta[wv], lane, sl, cur);
#pragma unroll
    for (uint32_t j = 0; j < SC; ++j) cur[j] = nxt[j];
  }
  if (ok) {
    store_to_aligned_end(o, head, 0u, sp.hd);
    store_from_aligned_start(o + sp.hd + 16u * sp.nmid, tail,
                             tail_pos(sp.hd + 16u * sp.nmid, plen), sp.tl);
  }
}

// Decrypt in ONE pass (QFEC_SCRATCH_OUTPUT): hash and copy from the same
// slab loads, as encrypt does, and the verdict afterwards — the output of a
// packet whose tag fails then holds its unverified plaintext, which is what
// BoringSSL's AEAD open leaves too and what QuicFramer::DecryptPayload
// tolerates (it decrypts into a scratch buffer and drops such a packet,
// quic_framer.cc:1884-1904).  The default two-pass kernel above keeps the
// reference NullDecrypter's output-untouched contract; this one reads the
// ciphertext once instead of twice.
template <uint32_t SC, bool R3 = true>
__global__ __launch_bounds__(kBlock) void null_decrypt_onepass_kernel(ProtectArgs a) {
  __shared__ u32x4 s_rows[kWaves][64 * (SC + 1u)];
  __shared__ StageMeta s_meta[kWaves][64];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint32_t clen = p < a.n ? a.in_len[p] : 0u;
  const bool valid = p < a.n && clen >= kTag;
  if (p < a.n && !valid) a.ok[p] = 0;  // ReadHash fails (null_decrypter.cc:48-50)
  const uint8_t* ad = nullptr;
  const uint8_t* pt = nullptr;
  uint8_t* o = nullptr;
  uint32_t alen = 0, plen = 0;
  uint32_t tag[3] = {0u, 0u, 0u};
  if (valid) {
    ad = a.bytes + a.ad_off[p];
    const uint8_t* ct = a.bytes + a.in_off[p];
    pt = ct + kTag;
    alen = a.ad_len[p];
    plen = clen - kTag;
    o = a.out + a.out_off[p];
    __builtin_memcpy(tag, ct, kTag);
  }
  const DstSplit sp = dst_split(o, plen);
  const StageMeta m = line_meta(pt + sp.hd, o + sp.hd, sp.nmid, o + sp.hd);
  s_meta[wv][lane] = m;
  const u32x4 head = valid ? load_head(pt, plen) : u32x4{0u, 0u, 0u, 0u};
  const u32x4 tail = valid ? load_tail(pt, plen) : u32x4{0u, 0u, 0u, 0u};
  Fnv128 h = fnv_init();
  if (valid) {
    fnv_span<R3>(h, ad, alen);
    fnv_bytes(h, head, 0u, sp.hd);
  }
  // output never overlaps the input (qfec.h): no in-place ordering
  stage_hash<true, SC, R3, false, kNullNT>(h, s_meta[wv], s_rows[wv], lane, m.nfull, m.lo);
  if (!valid) return;
  const uint32_t t0 = tail_pos(sp.hd + 16u * sp.nmid, plen);
  fnv_bytes(h, tail, t0, sp.tl);
  store_from_aligned_start(o + sp.hd + 16u * sp.nmid, tail, t0, sp.tl);
  store_to_aligned_end(o, head, 0u, sp.hd);
  a.ok[p] = (h.x0 == tag[0] && h.x1 == tag[1] && h.x2 == tag[2]) ? 1 : 0;
}

// ===========================================================================
// ChaCha20-Poly1305 (RFC 7539 AEAD; QUIC: 12-byte tag)
//   seal  AeadBaseEncrypter::EncryptPacket  crypto/aead_base_encrypter.cc:107-134
//         -> EVP_aead_chacha20_poly1305 seal_impl,
//            boringssl/crypto/cipher/e_chacha20poly1305.c:106-140
//   open  AeadBaseDecrypter::DecryptPacket  -> open_impl (:142-176)
// One lane per packet again (Poly1305 is a serial MAC over the packet): the
// lane generates its packet's keystream block by block (ChaCha20, counter 1..)
// while the payload moves through the same LDS-staged slabs as above; the
// ciphertext goes back into the lane's LDS row and leaves by coalesced stores.
// Poly1305 runs in five 26-bit limbs (25 v_mad_u64_u32 per 16-byte block).
// ===========================================================================
__device__ __forceinline__ uint32_t rotl32(uint32_t v, uint32_t n) {
  return __builtin_amdgcn_alignbit(v, v, 32u - n);
}

#define QPP_QR(a, b, c, d)   \
  a += b; d = rotl32(d ^ a, 16); \
  c += d; b = rotl32(b ^ c, 12); \
  a += b; d = rotl32(d ^ a, 8);  \
  c += d; b = rotl32(b ^ c, 7);

struct ChachaKey {
  uint32_t k[8];
  uint32_t n[3];
};

// One 64-byte keystream block (chacha.c:80-116) into ks[16].
__device__ __forceinline__ void chacha_block(const ChachaKey& key, uint32_t counter,
                                             uint32_t (&ks)[16]) {
  uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                    key.k[0], key.k[1], key.k[2], key.k[3],
                    key.k[4], key.k[5], key.k[6], key.k[7],
                    counter, key.n[0], key.n[1], key.n[2]};
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    QPP_QR(x[0], x[4], x[8], x[12]) QPP_QR(x[1], x[5], x[9], x[13])
    QPP_QR(x[2], x[6], x[10], x[14]) QPP_QR(x[3], x[7], x[11], x[15])
    QPP_QR(x[0], x[5], x[10], x[15]) QPP_QR(x[1], x[6], x[11], x[12])
    QPP_QR(x[2], x[7], x[8], x[13]) QPP_QR(x[3], x[4], x[9], x[14])
  }
  const uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                           key.k[0], key.k[1], key.k[2], key.k[3],
                           key.k[4], key.k[5], key.k[6], key.k[7],
                           counter, key.n[0], key.n[1], key.n[2]};
#pragma unroll
  for (int i = 0; i < 16; ++i) ks[i] = x[i] + in[i];
}
#undef QPP_QR

struct Poly1305 {
  uint32_t r0, r1, r2, r3, r4;
  uint32_t h0, h1, h2, h3, h4;
  uint32_t pad[4];
  uint32_t q0, q1, q2, q3, q4;  // r^2 mod 2^130 - 5 (poly_block2)
};

// Unreduced product of 26-bit limbs a (each < 2^27) and r (r^2 or r), into d.
__device__ __forceinline__ void poly_mul_acc(uint64_t (&d)[5], const uint32_t (&a)[5], uint32_t r0,
                                             uint32_t r1, uint32_t r2, uint32_t r3, uint32_t r4) {
  const uint32_t s1 = r1 * 5u, s2 = r2 * 5u, s3 = r3 * 5u, s4 = r4 * 5u;
  d[0] += (uint64_t)a[0] * r0 + (uint64_t)a[1] * s4 + (uint64_t)a[2] * s3 + (uint64_t)a[3] * s2 +
          (uint64_t)a[4] * s1;
  d[1] += (uint64_t)a[0] * r1 + (uint64_t)a[1] * r0 + (uint64_t)a[2] * s4 + (uint64_t)a[3] * s3 +
          (uint64_t)a[4] * s2;
  d[2] += (uint64_t)a[0] * r2 + (uint64_t)a[1] * r1 + (uint64_t)a[2] * r0 + (uint64_t)a[3] * s4 +
          (uint64_t)a[4] * s3;
  d[3] += (uint64_t)a[0] * r3 + (uint64_t)a[1] * r2 + (uint64_t)a[2] * r1 + (uint64_t)a[3] * r0 +
          (uint64_t)a[4] * s4;
  d[4] += (uint64_t)a[0] * r4 + (uint64_t)a[1] * r3 + (uint64_t)a[2] * r2 + (uint64_t)a[3] * r1 +
          (uint64_t)a[4] * r0;
}

// d (limb sums < 2^60) -> 26-bit limbs: h0..h4 with h1 < 2^26 + 2^10.
__device__ __forceinline__ void poly_carry(const uint64_t (&d0)[5], uint32_t (&h)[5]) {
  uint64_t d1 = d0[1] + (d0[0] >> 26), d2 = d0[2], d3 = d0[3], d4 = d0[4];
  d2 += d1 >> 26;
  d3 += d2 >> 26;
  d4 += d3 >> 26;
  const uint64_t c = d4 >> 26;
  const uint64_t h0 = (d0[0] & 0x3ffffffu) + c * 5u;
  h[1] = (uint32_t)(d1 & 0x3ffffffu) + (uint32_t)(h0 >> 26);
  h[0] = (uint32_t)(h0 & 0x3ffffffu);
  h[2] = (uint32_t)(d2 & 0x3ffffffu);
  h[3] = (uint32_t)(d3 & 0x3ffffffu);
  h[4] = (uint32_t)(d4 & 0x3ffffffu);
}

__device__ __forceinline__ void poly_init(Poly1305& p, const uint32_t (&k)[16]) {
  // r clamp (RFC 7539 §2.5) in 26-bit limbs
  p.r0 = k[0] & 0x3ffffffu;
  p.r1 = ((k[0] >> 26) | (k[1] << 6)) & 0x3ffff03u;
  p.r2 = ((k[1] >> 20) | (k[2] << 12)) & 0x3ffc0ffu;
  p.r3 = ((k[2] >> 14) | (k[3] << 18)) & 0x3f03fffu;
  p.r4 = (k[3] >> 8) & 0x00fffffu;
  p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0u;
  p.pad[0] = k[4];
  p.pad[1] = k[5];
  p.pad[2] = k[6];
  p.pad[3] = k[7];
  // r^2 for two blocks per step (poly_block2)
  const uint32_t r[5] = {p.r0, p.r1, p.r2, p.r3, p.r4};
  uint64_t d[5] = {0u, 0u, 0u, 0u, 0u};
  poly_mul_acc(d, r, p.r0, p.r1, p.r2, p.r3, p.r4);
  uint32_t q[5];
  poly_carry(d, q);
  p.q0 = q[0];
  p.q1 = q[1];
  p.q2 = q[2];
  p.q3 = q[3];
  p.q4 = q[4];
}

__device__ __forceinline__ void poly_limbs(u32x4 m, uint32_t (&a)[5]) {  // block + 2^128
  a[0] = m.x & 0x3ffffffu;
  a[1] = ((m.x >> 26) | (m.y << 6)) & 0x3ffffffu;
  a[2] = ((m.y >> 20) | (m.z << 12)) & 0x3ffffffu;
  a[3] = ((m.z >> 14) | (m.w << 18)) & 0x3ffffffu;
  a[4] = (m.w >> 8) | (1u << 24);
}

// Two blocks at once: h = ((h + m1) r + m2) r = (h + m1) r^2 + m2 r — two
// independent products and one carry chain, where poly_block twice is two
// products and two carry chains in series.  Limb sums stay below 2^59
// (a < 2^27, 5 r^2 < 2^28.4; the m2 r products below 2^57).
__device__ __forceinline__ void poly_block2(Poly1305& p, u32x4 m1, u32x4 m2) {
  uint32_t a[5], b[5];
  poly_limbs(m1, a);
  a[0] += p.h0;
  a[1] += p.h1;
  a[2] += p.h2;
  a[3] += p.h3;
  a[4] += p.h4;
  poly_limbs(m2, b);
  uint64_t d[5] = {0u, 0u, 0u, 0u, 0u};
  poly_mul_acc(d, a, p.q0, p.q1, p.q2, p.q3, p.q4);
  poly_mul_acc(d, b, p.r0, p.r1, p.r2, p.r3, p.r4);
  uint32_t h[5];
  poly_carry(d, h);
  p.h0 = h[0];
  p.h1 = h[1];
  p.h2 = h[2];
  p.h3 = h[3];
  p.h4 = h[4];
}

// h = (h + m + 2^128) * r mod 2^130 - 5 for one full 16-byte block.
__device__ __forceinline__ void poly_block(Poly1305& p, u32x4 m) {
  uint64_t h0 = p.h0 + (m.x & 0x3ffffffu);
  uint64_t h1 = p.h1 + (((m.x >> 26) | (m.y << 6)) & 0x3ffffffu);
  uint64_t h2 = p.h2 + (((m.y >> 20) | (m.z << 12)) & 0x3ffffffu);
  uint64_t h3 = p.h3 + (((m.z >> 14) | (m.w << 18)) & 0x3ffffffu);
  uint64_t h4 = p.h4 + ((m.w >> 8) | (1u << 24));
  const uint32_t s1 = p.r1 * 5u, s2 = p.r2 * 5u, s3 = p.r3 * 5u, s4 = p.r4 * 5u;
  const uint32_t a0 = (uint32_t)h0, a1 = (uint32_t)h1, a2 = (uint32_t)h2, a3 = (uint32_t)h3,
                 a4 = (uint32_t)h4;
  uint64_t d0 = (uint64_t)a0 * p.r0 + (uint64_t)a1 * s4 + (uint64_t)a2 * s3 +
                (uint64_t)a3 * s2 + (uint64_t)a4 * s1;
  uint64_t d1 = (uint64_t)a0 * p.r1 + (uint64_t)a1 * p.r0 + (uint64_t)a2 * s4 +
                (uint64_t)a3 * s3 + (uint64_t)a4 * s2;
  uint64_t d2 = (uint64_t)a0 * p.r2 + (uint64_t)a1 * p.r1 + (uint64_t)a2 * p.r0 +
                (uint64_t)a3 * s4 + (uint64_t)a4 * s3;
  uint64_t d3 = (uint64_t)a0 * p.r3 + (uint64_t)a1 * p.r2 + (uint64_t)a2 * p.r1 +
                (uint64_t)a3 * p.r0 + (uint64_t)a4 * s4;
  uint64_t d4 = (uint64_t)a0 * p.r4 + (uint64_t)a1 * p.r3 + (uint64_t)a2 * p.r2 +
                (uint64_t)a3 * p.r1 + (uint64_t)a4 * p.r0;
  d1 += d0 >> 26;
  d2 += d1 >> 26;
  d3 += d2 >> 26;
  d4 += d3 >> 26;
  uint32_t c = (uint32_t)(d4 >> 26);
  h0 = (d0 & 0x3ffffffu) + (uint64_t)c * 5u;
  p.h1 = (uint32_t)(d1 & 0x3ffffffu) + (uint32_t)(h0 >> 26);
  p.h0 = (uint32_t)(h0 & 0x3ffffffu);
  p.h2 = (uint32_t)(d2 & 0x3ffffffu);
  p.h3 = (uint32_t)(d3 & 0x3ffffffu);
  p.h4 = (uint32_t)(d4 & 0x3ffffffu);
}

// Final reduction + pad; returns the first 12 tag bytes as three words.
__device__ __forceinline__ void poly_finish(const Poly1305& p, uint32_t (&tag)[3]) {
  uint32_t h0 = p.h0, h1 = p.h1, h2 = p.h2, h3 = p.h3, h4 = p.h4, c;
  c = h1 >> 26; h1 &= 0x3ffffffu;
  h2 += c; c = h2 >> 26; h2 &= 0x3ffffffu;
  h3 += c; c = h3 >> 26; h3 &= 0x3ffffffu;
  h4 += c; c = h4 >> 26; h4 &= 0x3ffffffu;
  h0 += c * 5u; c = h0 >> 26; h0 &= 0x3ffffffu;
  h1 += c;
  // g = h + 5 - 2^130: select g when h >= p
  uint32_t g0 = h0 + 5u; c = g0 >> 26; g0 &= 0x3ffffffu;
  uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffffu;
  uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffffu;
  uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffffu;
  uint32_t g4 = h4 + c - (1u << 26);
  const uint32_t mask = (g4 >> 31) - 1u;  // all ones if h >= p
  h0 = (h0 & ~mask) | (g0 & mask);
  h1 = (h1 & ~mask) | (g1 & mask);
  h2 = (h2 & ~mask) | (g2 & mask);
  h3 = (h3 & ~mask) | (g3 & mask);
  h4 = (h4 & ~mask) | (g4 & mask);
  // to 4 x 32 bits, + pad mod 2^128
  // (the top word, (h3 >> 18) | (h4 << 8), only feeds tag bytes 12..15: not kept)
  const uint32_t w0 = h0 | (h1 << 26), w1 = (h1 >> 6) | (h2 << 20), w2 = (h2 >> 12) | (h3 << 14);
  uint64_t f = (uint64_t)w0 + p.pad[0];
  tag[0] = (uint32_t)f;
  f = (uint64_t)w1 + p.pad[1] + (f >> 32);
  tag[1] = (uint32_t)f;
  f = (uint64_t)w2 + p.pad[2] + (f >> 32);
  tag[2] = (uint32_t)f;
}

// Poly1305 over a per-lane span padded with zeros to 16 (the AD; short).
__device__ __forceinline__ void poly_span_padded(Poly1305& p, const uint8_t* d, uint32_t len) {
  const uint32_t nfull = len >> 4;
  for (uint32_t c = 0; c < nfull; ++c) poly_block(p, ld16(d + 16u * c));
  const uint32_t rem = len & 15u;
  if (rem) {
    uint8_t b[16];
#pragma unroll
    for (uint32_t i = 0; i < 16u; ++i) b[i] = i < rem ? d[16u * nfull + i] : (uint8_t)0;
    u32x4 v;
    __builtin_memcpy(&v, b, 16);
    poly_block(p, v);
  }
}

// Keep only the `rem` bytes of the tail chunk that load_tail put at its top
// (len >= 16) or bottom (len < 16), moved to bytes [0, rem), zero above.
// Bytes [o, o+16) of the 32 bytes lo || hi (o in 0..15) in 32-bit lanes: two
// 2-way dword selects and four v_alignbyte_b32 (no local byte array: indexed
// by a runtime value, one lived in scratch memory).
__device__ __forceinline__ u32x4 bytes16_at(u32x4 lo, u32x4 hi, uint32_t o) {
  const bool b8 = (o & 8u) != 0u, b4 = (o & 4u) != 0u;
  const uint32_t f0 = b8 ? lo.z : lo.x, f1 = b8 ? lo.w : lo.y, f2 = b8 ? hi.x : lo.z,
                 f3 = b8 ? hi.y : lo.w, f4 = b8 ? hi.z : hi.x, f5 = b8 ? hi.w : hi.y;
  const uint32_t g0 = b4 ? f1 : f0, g1 = b4 ? f2 : f1, g2 = b4 ? f3 : f2, g3 = b4 ? f4 : f3,
                 g4 = b4 ? f5 : f4;
  const uint32_t r = o & 3u;
  return u32x4{__builtin_amdgcn_alignbyte(g1, g0, r), __builtin_amdgcn_alignbyte(g2, g1, r),
               __builtin_amdgcn_alignbyte(g3, g2, r), __builtin_amdgcn_alignbyte(g4, g3, r)};
}

// The low `rem` bytes of t kept, zero above (rem in 0..16).
__device__ __forceinline__ u32x4 keep_low_bytes(u32x4 t, uint32_t rem) {
  const uint32_t k = rem * 8u;
  const uint32_t m0 = k >= 32u ? ~0u : ((1u << k) - 1u);
  const uint32_t m1 = k >= 64u ? ~0u : k <= 32u ? 0u : ((1u << (k - 32u)) - 1u);
  const uint32_t m2 = k >= 96u ? ~0u : k <= 64u ? 0u : ((1u << (k - 64u)) - 1u);
  const uint32_t m3 = k >= 128u ? ~0u : k <= 96u ? 0u : ((1u << (k - 96u)) - 1u);
  return u32x4{t.x & m0, t.y & m1, t.z & m2, t.w & m3};
}

__device__ __forceinline__ u32x4 tail_bytes(u32x4 t, uint32_t len) {
  const uint32_t rem = len & 15u;
  // len >= 16: the rem bytes sit at the top (bytes 16-rem..15): shift them down
  const u32x4 s = len >= 16u ? bytes16_at(t, u32x4{0u, 0u, 0u, 0u}, (16u - rem) & 15u) : t;
  return keep_low_bytes(len >= 16u && rem == 0u ? u32x4{0u, 0u, 0u, 0u} : s, rem);
}

__device__ __forceinline__ u32x4 ks_chunk(const uint32_t (&ks)[16], uint32_t j) {
  return j == 0 ? u32x4{ks[0], ks[1], ks[2], ks[3]}
         : j == 1 ? u32x4{ks[4], ks[5], ks[6], ks[7]}
         : j == 2 ? u32x4{ks[8], ks[9], ks[10], ks[11]}
                  : u32x4{ks[12], ks[13], ks[14], ks[15]};
}

// ks_chunk for a per-lane j (the packet tails): the empty asm pins each word
// in a VGPR, so the selects stay v_cndmask instead of being folded into one
// load at a select-chosen address — which puts ks[] in scratch (80 B per
// lane in the seal/open kernels before this).
__device__ __forceinline__ u32x4 ks_chunk_lane(const uint32_t (&ks)[16], uint32_t j) {
  uint32_t k[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    k[i] = ks[i];
    asm volatile("" : "+v"(k[i]));
  }
  const bool b2 = (j & 2u) != 0u, b1 = (j & 1u) != 0u;
  const u32x4 lo = b2 ? u32x4{k[8], k[9], k[10], k[11]} : u32x4{k[0], k[1], k[2], k[3]};
  const u32x4 hi = b2 ? u32x4{k[12], k[13], k[14], k[15]} : u32x4{k[4], k[5], k[6], k[7]};
  return b1 ? hi : lo;
}

// Transposed read back of the wave's LDS rows into the loading-lane layout.
template <uint32_t SC>
__device__ __forceinline__ void stage_from_lds(const u32x4* rows, uint32_t lane, u32x4 (&v)[SC]) {
  const uint32_t i = lane / SC, m = lane % SC;
  wave_lds_order();  // the lanes' writes to their own rows first
#pragma unroll
  for (uint32_t I = 0; I < SC; ++I) v[I] = rows[((64u / SC) * I + i) * (SC + 1u) + m];
  wave_lds_order();
}

__device__ __forceinline__ ChachaKey load_key(const AeadArgs& a, uint64_t p) {
  ChachaKey key;
  const uint32_t ki = a.key_idx[p];
  const uint8_t* kp = a.keys + 32ull * ki;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t w;
    __builtin_memcpy(&w, kp + 4 * i, 4);
    key.k[i] = w;
  }
  uint32_t pre;
  __builtin_memcpy(&pre, a.prefixes + 4ull * ki, 4);
  const uint64_t pn = ((uint64_t)(a.path_id ? a.path_id[p] : 0u) << 56) | a.packet_number[p];
  key.n[0] = pre;  // nonce = prefix || LE64(path_id << 56 | packet_number)
  key.n[1] = (uint32_t)pn;
  key.n[2] = (uint32_t)(pn >> 32);
  return key;
}

// Payload pass over the wave's packets: XOR the keystream (XOR = true) and/or
// MAC (MAC_IN: the MAC covers the input chunks; MAC_OUT: the output chunks)
// every full chunk; the transformed chunks leave through LDS by coalesced
// stores when meta[].dst is set.
// NTS: the ciphertext / plaintext leaves by nontemporal stores (kAeadNTS)
constexpr bool kAeadNTS = false;
template <uint32_t SC, bool XOR, bool MAC_IN, bool MAC_OUT, bool NTS = kAeadNTS>
__device__ __forceinline__ void aead_pass(const ChachaKey& key, Poly1305& poly,
                                          const StageMeta* meta, u32x4* rows, uint32_t lane,
                                          uint32_t my_nfull, bool store) {
  const uint32_t nslab = (wave_max_u32(my_nfull) + SC - 1) / SC;
  u32x4 buf[SC];
  if (nslab) stage_load<SC>(meta, lane, 0, buf);
  for (uint32_t sl = 0; sl < nslab; ++sl) {
    stage_to_lds<SC>(rows, lane, buf);
    if (sl + 1u < nslab) stage_load<SC>(meta, lane, sl + 1u, buf);  // regs free again
#pragma unroll
    for (uint32_t b = 0; b < SC / 4u; ++b) {
      const uint32_t c0 = sl * SC + 4u * b;
      if (c0 >= my_nfull) break;
      uint32_t ks[16];
      if constexpr (XOR) chacha_block(key, 1u + c0 / 4u, ks);
      // the MAC takes the chunks in pairs (poly_block2); a lone last chunk
      // of the packet goes through poly_block
      u32x4 mac[4];
#pragma unroll
      for (uint32_t j = 0; j < 4u; ++j) {
        u32x4& slot = rows[lane * (SC + 1u) + 4u * b + j];
        u32x4 v = slot;
        if constexpr (MAC_IN) mac[j] = v;
        if constexpr (XOR) {
          v ^= ks_chunk(ks, j);
          if (c0 + j < my_nfull) slot = v;
        }
        if constexpr (MAC_OUT) mac[j] = v;
      }
      if constexpr (MAC_IN || MAC_OUT) {
#pragma unroll
        for (uint32_t j = 0; j < 4u; j += 2u) {
          if (c0 + j + 1u < my_nfull)
            poly_block2(poly, mac[j], mac[j + 1u]);
          else if (c0 + j < my_nfull)
            poly_block(poly, mac[j]);
        }
      }
    }
    if (store) {
      u32x4 out[SC];
      stage_from_lds<SC>(rows, lane, out);
      stage_store<SC, true, NTS>(meta, lane, sl, out);
    }
  }
}

__device__ __forceinline__ void poly_lengths(Poly1305& p, uint32_t ad_len, uint32_t ct_len) {
  poly_block(p, u32x4{ad_len, 0u, ct_len, 0u});  // LE64(ad_len) || LE64(ct_len)
}

template <uint32_t SC, bool NTS = kAeadNTS>
__global__ __launch_bounds__(kBlock) void c20p1305_seal_kernel(AeadArgs a) {
  __shared__ u32x4 s_rows[kWaves][64 * (SC + 1u)];
  __shared__ StageMeta s_meta[kWaves][64];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool valid = p < a.io.n;
  const uint8_t* ad = nullptr;
  const uint8_t* pt = nullptr;
  uint8_t* o = nullptr;
  uint32_t alen = 0, plen = 0;
  ChachaKey key = {};
  Poly1305 poly = {};
  u32x4 tail = {0u, 0u, 0u, 0u};
  if (valid) {
    ad = a.io.bytes + a.io.ad_off[p];
    pt = a.io.bytes + a.io.in_off[p];
    alen = a.io.ad_len[p];
    plen = a.io.in_len[p];
    o = a.io.out + a.io.out_off[p];
    key = load_key(a, p);
    uint32_t k0[16];
    chacha_block(key, 0u, k0);  // one-time Poly1305 key (e_chacha20poly1305.c:97-99)
    poly_init(poly, k0);
    poly_span_padded(poly, ad, alen);
    tail = tail_bytes(load_tail(pt, plen), plen);  // before any store (in place)
  }
  s_meta[wv][lane] = StageMeta{pt, o, plen >> 4};
  aead_pass<SC, true, false, true, NTS>(key, poly, s_meta[wv], s_rows[wv], lane, plen >> 4, true);
  if (!valid) return;
  const uint32_t rem = plen & 15u;
  if (rem) {
    const uint32_t c = plen >> 4;
    uint32_t ks[16];
    chacha_block(key, 1u + c / 4u, ks);
    u32x4 ct = tail ^ ks_chunk_lane(ks, c & 3u);
    uint8_t b[16];
    __builtin_memcpy(b, &ct, 16);
    for (uint32_t i = rem; i < 16u; ++i) b[i] = 0;  // zero pad for the MAC
    __builtin_memcpy(&ct, b, 16);
    poly_block(poly, ct);
    for (uint32_t i = 0; i < rem; ++i) o[16u * c + i] = b[i];
  }
  poly_lengths(poly, alen, plen);
  uint32_t tag[3];
  poly_finish(poly, tag);
  __builtin_memcpy(o + plen, tag, kTag);  // ct || tag
}

// ONEPASS (QFEC_SCRATCH_OUTPUT): MAC and decrypt from the same slab loads;
// a packet whose tag fails keeps its unverified plaintext in the output, as
// BoringSSL's open_impl leaves it (e_chacha20poly1305.c:142-176 decrypts
// before it compares) — one read of the ciphertext instead of two.
template <uint32_t SC, bool ONEPASS = false, bool NTS = kAeadNTS>
__global__ __launch_bounds__(kBlock) void c20p1305_open_kernel(AeadArgs a) {
  __shared__ u32x4 s_rows[kWaves][64 * (SC + 1u)];
  __shared__ StageMeta s_meta[kWaves][64];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint32_t clen = p < a.io.n ? a.io.in_len[p] : 0u;
  const bool valid = p < a.io.n && clen >= kTag;
  if (p < a.io.n && !valid) a.io.ok[p] = 0;  // open_impl: in_len < tag_len
  const uint8_t* ad = nullptr;
  const uint8_t* ct = nullptr;
  uint32_t alen = 0, plen = 0;
  ChachaKey key = {};
  Poly1305 poly = {};
  u32x4 tail = {0u, 0u, 0u, 0u};
  uint32_t want[3] = {0u, 0u, 0u};
  if (valid) {
    ad = a.io.bytes + a.io.ad_off[p];
    ct = a.io.bytes + a.io.in_off[p];
    alen = a.io.ad_len[p];
    plen = clen - kTag;
    __builtin_memcpy(want, ct + plen, kTag);
    key = load_key(a, p);
    uint32_t k0[16];
    chacha_block(key, 0u, k0);
    poly_init(poly, k0);
    poly_span_padded(poly, ad, alen);
    tail = tail_bytes(load_tail(ct, plen), plen);
  }
  if constexpr (ONEPASS) {
    uint8_t* o = valid ? a.io.out + a.io.out_off[p] : nullptr;
    s_meta[wv][lane] = StageMeta{ct, o, plen >> 4};
    aead_pass<SC, true, true, false, NTS>(key, poly, s_meta[wv], s_rows[wv], lane, plen >> 4, true);
    if (!valid) return;
    const uint32_t rem = plen & 15u;
    if (rem) {
      poly_block(poly, tail);  // zero padded ciphertext tail
      const uint32_t c = plen >> 4;
      uint32_t ks[16];
      chacha_block(key, 1u + c / 4u, ks);
      const u32x4 pt = tail ^ ks_chunk_lane(ks, c & 3u);
      uint8_t b[16];
      __builtin_memcpy(b, &pt, 16);
      for (uint32_t i = 0; i < rem; ++i) o[16u * c + i] = b[i];
    }
    poly_lengths(poly, alen, plen);
    uint32_t tag[3];
    poly_finish(poly, tag);
    a.io.ok[p] = ((tag[0] ^ want[0]) | (tag[1] ^ want[1]) | (tag[2] ^ want[2])) == 0u ? 1 : 0;
    return;
  }
  // pass 1: MAC over the ciphertext (no output)
  s_meta[wv][lane] = StageMeta{ct, nullptr, plen >> 4};
  aead_pass<SC, false, true, false>(key, poly, s_meta[wv], s_rows[wv], lane, plen >> 4, false);
  bool ok = false;
  if (valid) {
    if (plen & 15u) poly_block(poly, tail);  // zero padded
    poly_lengths(poly, alen, plen);
    uint32_t tag[3];
    poly_finish(poly, tag);
    ok = ((tag[0] ^ want[0]) | (tag[1] ^ want[1]) | (tag[2] ^ want[2])) == 0u;
    a.io.ok[p] = ok ? 1 : 0;
  }
  // pass 2 (verified packets only): decrypt into the output
  uint8_t* o = ok ? a.io.out + a.io.out_off[p] : nullptr;
  s_meta[wv][lane] = StageMeta{ct, o, ok ? plen >> 4 : 0u};
  aead_pass<SC, true, false, false, NTS>(key, poly, s_meta[wv], s_rows[wv], lane,
                                         ok ? plen >> 4 : 0u, true);
  const uint32_t rem = plen & 15u;
  if (ok && rem) {
    const uint32_t c = plen >> 4;
    uint32_t ks[16];
    chacha_block(key, 1u + c / 4u, ks);
    const u32x4 pt = tail ^ ks_chunk_lane(ks, c & 3u);
    uint8_t b[16];
    __builtin_memcpy(b, &pt, 16);
    for (uint32_t i = 0; i < rem; ++i) o[16u * c + i] = b[i];
  }
}

// ===========================================================================
// AES-128-GCM (QUIC: 12-byte tag)
//   seal  Aes128Gcm12Encrypter::EncryptPacket = AeadBaseEncrypter::EncryptPacket
//         -> EVP_aead_aes_128_gcm aead_aes_gcm_seal,
//            boringssl/crypto/cipher/e_aes.c:1050-1091 over crypto/modes/gcm.c
//   open  Aes128Gcm12Decrypter::DecryptPacket -> aead_aes_gcm_open (:1093-1140)
// One lane per packet: its AES-128 round keys in registers (expanded per
// lane), CTR keystream one AES block per 16-byte chunk, GHASH per chunk.
// AES rounds use one T-table (Te0; Te1..3 are byte rotations of it) in LDS,
// replicated 32x so lane l reads copy l % 32: any lookup pattern costs at
// most 2 bank cycles.  GHASH uses Shoup's 4-bit tables (BoringSSL
// gcm_init_4bit / gcm_gmult_4bit) from the wave's H in LDS (256 B, one bank
// row: conflict-free) when every packet of the wave has the same key — the
// batched-by-connection case — and a bit-serial multiply otherwise.
// ===========================================================================
__constant__ uint32_t kTe0[256] = {
    0xa56363c6u, 0x847c7cf8u, 0x997777eeu, 0x8d7b7bf6u, 0x0df2f2ffu, 0xbd6b6bd6u, 0xb16f6fdeu, 0x54c5c591u,
    0x50303060u, 0x03010102u, 0xa96767ceu, 0x7d2b2b56u, 0x19fefee7u, 0x62d7d7b5u, 0xe6abab4du, 0x9a7676ecu,
    0x45caca8fu, 0x9d82821fu, 0x40c9c989u, 0x877d7dfau, 0x15fafaefu, 0xeb5959b2u, 0xc947478eu, 0x0bf0f0fbu,
    0xecadad41u, 0x67d4d4b3u, 0xfda2a25fu, 0xeaafaf45u, 0xbf9c9c23u, 0xf7a4a453u, 0x967272e4u, 0x5bc0c09bu,
    0xc2b7b775u, 0x1cfdfde1u, 0xae93933du, 0x6a26264cu, 0x5a36366cu, 0x413f3f7eu, 0x02f7f7f5u, 0x4fcccc83u,
    0x5c343468u, 0xf4a5a551u, 0x34e5e5d1u, 0x08f1f1f9u, 0x937171e2u, 0x73d8d8abu, 0x53313162u, 0x3f15152au,
    0x0c040408u, 0x52c7c795u, 0x65232346u, 0x5ec3c39du, 0x28181830u, 0xa1969637u, 0x0f05050au, 0xb59a9a2fu,
    0x0907070eu, 0x36121224u, 0x9b80801bu, 0x3de2e2dfu, 0x26ebebcdu, 0x6927274eu, 0xcdb2b27fu, 0x9f7575eau,
    0x1b090912u, 0x9e83831du, 0x742c2c58u, 0x2e1a1a34u, 0x2d1b1b36u, 0xb26e6edcu, 0xee5a5ab4u, 0xfba0a05bu,
    0xf65252a4u, 0x4d3b3b76u, 0x61d6d6b7u, 0xceb3b37du, 0x7b292952u, 0x3ee3e3ddu, 0x712f2f5eu, 0x97848413u,
    0xf55353a6u, 0x68d1d1b9u, 0x00000000u, 0x2cededc1u, 0x60202040u, 0x1ffcfce3u, 0xc8b1b179u, 0xed5b5bb6u,
    0xbe6a6ad4u, 0x46cbcb8du, 0xd9bebe67u, 0x4b393972u, 0xde4a4a94u, 0xd44c4c98u, 0xe85858b0u, 0x4acfcf85u,
    0x6bd0d0bbu, 0x2aefefc5u, 0xe5aaaa4fu, 0x16fbfbedu, 0xc5434386u, 0xd74d4d9au, 0x55333366u, 0x94858511u,
    0xcf45458au, 0x10f9f9e9u, 0x06020204u, 0x817f7ffeu, 0xf05050a0u, 0x443c3c78u, 0xba9f9f25u, 0xe3a8a84bu,
    0xf35151a2u, 0xfea3a35du, 0xc0404080u, 0x8a8f8f05u, 0xad92923fu, 0xbc9d9d21u, 0x48383870u, 0x04f5f5f1u,
    0xdfbcbc63u, 0xc1b6b677u, 0x75dadaafu, 0x63212142u, 0x30101020u, 0x1affffe5u, 0x0ef3f3fdu, 0x6dd2d2bfu,
    0x4ccdcd81u, 0x140c0c18u, 0x35131326u, 0x2fececc3u, 0xe15f5fbeu, 0xa2979735u, 0xcc444488u, 0x3917172eu,
    0x57c4c493u, 0xf2a7a755u, 0x827e7efcu, 0x473d3d7au, 0xac6464c8u, 0xe75d5dbau, 0x2b191932u, 0x957373e6u,
    0xa06060c0u, 0x98818119u, 0xd14f4f9eu, 0x7fdcdca3u, 0x66222244u, 0x7e2a2a54u, 0xab90903bu, 0x8388880bu,
    0xca46468cu, 0x29eeeec7u, 0xd3b8b86bu, 0x3c141428u, 0x79dedea7u, 0xe25e5ebcu, 0x1d0b0b16u, 0x76dbdbadu,
    0x3be0e0dbu, 0x56323264u, 0x4e3a3a74u, 0x1e0a0a14u, 0xdb494992u, 0x0a06060cu, 0x6c242448u, 0xe45c5cb8u,
    0x5dc2c29fu, 0x6ed3d3bdu, 0xefacac43u, 0xa66262c4u, 0xa8919139u, 0xa4959531u, 0x37e4e4d3u, 0x8b7979f2u,
    0x32e7e7d5u, 0x43c8c88bu, 0x5937376eu, 0xb76d6ddau, 0x8c8d8d01u, 0x64d5d5b1u, 0xd24e4e9cu, 0xe0a9a949u,
    0xb46c6cd8u, 0xfa5656acu, 0x07f4f4f3u, 0x25eaeacfu, 0xaf6565cau, 0x8e7a7af4u, 0xe9aeae47u, 0x18080810u,
    0xd5baba6fu, 0x887878f0u, 0x6f25254au, 0x722e2e5cu, 0x241c1c38u, 0xf1a6a657u, 0xc7b4b473u, 0x51c6c697u,
    0x23e8e8cbu, 0x7cdddda1u, 0x9c7474e8u, 0x211f1f3eu, 0xdd4b4b96u, 0xdcbdbd61u, 0x868b8b0du, 0x858a8a0fu,
    0x907070e0u, 0x423e3e7cu, 0xc4b5b571u, 0xaa6666ccu, 0xd8484890u, 0x05030306u, 0x01f6f6f7u, 0x120e0e1cu,
    0xa36161c2u, 0x5f35356au, 0xf95757aeu, 0xd0b9b969u, 0x91868617u, 0x58c1c199u, 0x271d1d3au, 0xb99e9e27u,
    0x38e1e1d9u, 0x13f8f8ebu, 0xb398982bu, 0x33111122u, 0xbb6969d2u, 0x70d9d9a9u, 0x898e8e07u, 0xa7949433u,
    0xb69b9b2du, 0x221e1e3cu, 0x92878715u, 0x20e9e9c9u, 0x49cece87u, 0xff5555aau, 0x78282850u, 0x7adfdfa5u,
    0x8f8c8c03u, 0xf8a1a159u, 0x80898909u, 0x170d0d1au, 0xdabfbf65u, 0x31e6e6d7u, 0xc6424284u, 0xb86868d0u,
    0xc3414182u, 0xb0999929u, 0x772d2d5au, 0x110f0f1eu, 0xcbb0b07bu, 0xfc5454a8u, 0xd6bbbb6du, 0x3a16162cu,
};

// Te0 in LDS: 256 rows of 256 B, row x = Te0[x] 64 times; lane l reads dword
// l of a row.  ds_read_b32 banks are (a/4) mod 32 per 32-lane group, so every
// lookup pattern is conflict-free, and the byte address of the lookup of
// byte k of a state word s is (byte_k(s) << 8) | 4*lane: ONE v_perm_b32 per
// lookup (the 32-copy 32 KiB layout needed a bfe + a shift-add).
constexpr uint32_t kTeBytes = 256u * 256u;  // 64 KiB

struct AesKey {
  uint32_t rk[44];  // little-endian words of the FIPS-197 round-key bytes
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32: a ^ b ^ c
}

// Te0[byte k of s] from the lane's column (lane4 = 4 * lane)
__device__ __forceinline__ uint32_t te_at(const uint32_t* te, uint32_t s, uint32_t k,
                                          uint32_t lane4) {
  const uint32_t addr = __builtin_amdgcn_perm(s, lane4, 0x0C0C0000u | ((4u + k) << 8));
  return *(const uint32_t*)((const uint8_t*)te + addr);
}

// S(byte k of s): Te0 bytes 1 and 2 are S(x)
__device__ __forceinline__ uint32_t sbox_at(const uint32_t* te, uint32_t s, uint32_t k,
                                            uint32_t lane4) {
  return (te_at(te, s, k, lane4) >> 8) & 0xFFu;
}

// FIPS-197 §5.2 key expansion in little-endian words.
__device__ __forceinline__ void aes_expand(AesKey& k, const uint8_t* key, const uint32_t* te,
                                           uint32_t lane4) {
#pragma unroll
  for (int i = 0; i < 4; ++i) __builtin_memcpy(&k.rk[i], key + 4 * i, 4);
  uint32_t rcon = 1;
#pragma unroll
  for (int i = 4; i < 44; ++i) {
    uint32_t t = k.rk[i - 1];
    if (i % 4 == 0) {
      // SubWord(RotWord(t)) (LE): byte j of the result = S(byte j+1 of t)
      t = sbox_at(te, t, 1, lane4) | (sbox_at(te, t, 2, lane4) << 8) |
          (sbox_at(te, t, 3, lane4) << 16) | (sbox_at(te, t, 0, lane4) << 24);
      t ^= rcon;
      rcon = ((rcon << 1) ^ ((rcon & 0x80u) ? 0x1Bu : 0u)) & 0xFFu;
    }
    k.rk[i] = k.rk[i - 4] ^ t;
  }
}

// NB independent blocks through the same rounds (their LDS lookups and VALU
// interleave).  Column c of a round = Te0[s_c.b0] ^ rot8 Te0[s_c+1.b1] ^
// rot16 Te0[s_c+2.b2] ^ rot24 Te0[s_c+3.b3] ^ rk: 4 perms, 4 lookups,
// 3 alignbits, 2 bitop3.  Last round: S bytes gathered by two perms.
template <int NB>
__device__ __forceinline__ void aes_encrypt_n(const AesKey& k, u32x4 (&io)[NB], const uint32_t* te,
                                              uint32_t lane4) {
  uint32_t s[NB][4];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    s[b][0] = io[b].x ^ k.rk[0];
    s[b][1] = io[b].y ^ k.rk[1];
    s[b][2] = io[b].z ^ k.rk[2];
    s[b][3] = io[b].w ^ k.rk[3];
  }
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    uint32_t t[NB][4];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        t[b][c] = xor3(xor3(te_at(te, s[b][c], 0, lane4),
                            rotl32(te_at(te, s[b][(c + 1) & 3], 1, lane4), 8),
                            rotl32(te_at(te, s[b][(c + 2) & 3], 2, lane4), 16)),
                       rotl32(te_at(te, s[b][(c + 3) & 3], 3, lane4), 24), k.rk[4 * r + c]);
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c) s[b][c] = t[b][c];
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    uint32_t o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t A = te_at(te, s[b][c], 0, lane4), B = te_at(te, s[b][(c + 1) & 3], 1, lane4);
      const uint32_t C = te_at(te, s[b][(c + 2) & 3], 2, lane4), D = te_at(te, s[b][(c + 3) & 3], 3, lane4);
      // [S(A) S(B) 0 0] and [0 0 S(C) S(D)] from bytes 1 / 2 of the entries
      o[c] = xor3(__builtin_amdgcn_perm(B, A, 0x0C0C0501u), __builtin_amdgcn_perm(D, C, 0x06020C0Cu),
                  k.rk[40 + c]);
    }
    io[b] = u32x4{o[0], o[1], o[2], o[3]};
  }
}

__device__ __forceinline__ u32x4 aes_encrypt(const AesKey& k, u32x4 in, const uint32_t* te,
                                             uint32_t lane4) {
  u32x4 v[1] = {in};
  aes_encrypt_n<1>(k, v, te, lane4);
  return v[0];
}

// ---- GHASH -----------------------------------------------------------------
// GF(2^128) elements as four big-endian 32-bit words: w[0] holds the
// coefficients of x^0..x^31 with x^0 at the MSB (SP 800-38D bit order; the
// u128 {hi, lo} of gcm.c split in words).  Multiplication by x is a right
// shift; x^128 = 1 + x + x^2 + x^7.
//
// Uniform-key waves (the batched-by-connection case) multiply with Shoup's
// 4-bit tables (gcm.c gcm_init_4bit: T[n] = n*H, nibble bit 3 = x^0) in LDS,
// but WITHOUT gcm_gmult_4bit's per-nibble reduction: the 32 nibble products
// T[n_k] * x^(4k) are summed unreduced into a 256-bit accumulator (a Horner
// chain of 4-bit shifts over the nibble position, the four words of X in
// parallel), and reduced once.  That removes the rem_4bit lookup and the
// serial dependence between nibbles.  Blocks are taken two at a time with
// aggregated reduction: Y' = (Y ^ C1)*H^2 ^ C2*H, one fold per pair (a second
// table holds n*H^2).  Each table is 256 B — one LDS bank row — so the
// wave's 64 ds_read_b128 lookups never conflict.
// Mixed-key waves fall back to the bit-serial multiply (SP 800-38D Alg. 1).
struct Gf4 {
  uint32_t w[4];
};

__device__ __forceinline__ Gf4 gf_from_block(u32x4 b) {  // block bytes -> BE words
  return Gf4{{__builtin_bswap32(b.x), __builtin_bswap32(b.y), __builtin_bswap32(b.z),
              __builtin_bswap32(b.w)}};
}

__device__ __forceinline__ u32x4 gf_to_block(const Gf4& g) {
  return u32x4{__builtin_bswap32(g.w[0]), __builtin_bswap32(g.w[1]), __builtin_bswap32(g.w[2]),
               __builtin_bswap32(g.w[3])};
}

__device__ __forceinline__ Gf4 gf_xor(const Gf4& a, const Gf4& b) {
  return Gf4{{a.w[0] ^ b.w[0], a.w[1] ^ b.w[1], a.w[2] ^ b.w[2], a.w[3] ^ b.w[3]}};
}

// low 32 bits of (hi:lo) >> r, 0 <= r < 32 (v_alignbit_b32)
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t r) {
  return __builtin_amdgcn_alignbit(hi, lo, r);
}

// v * x (REDUCE1BIT of gcm.c)
__device__ __forceinline__ Gf4 gf_mul_x(const Gf4& v) {
  const uint32_t r = (v.w[3] & 1u) ? 0xE1000000u : 0u;
  return Gf4{{(v.w[0] >> 1) ^ r, funnel(v.w[0], v.w[1], 1), funnel(v.w[1], v.w[2], 1),
              funnel(v.w[2], v.w[3], 1)}};
}

// Bit-serial X * H (SP 800-38D Algorithm 1) for waves with mixed keys.
__device__ __forceinline__ Gf4 gf_mul_bits(const Gf4& x, const Gf4& h) {
  Gf4 z{{0u, 0u, 0u, 0u}}, v = h;
  // word loop unrolled, bit loop not: x.w[q] is a constant index (x.w[i >> 5]
  // in one rolled loop kept x in scratch)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t xw = x.w[q];
#pragma unroll 1
    for (int i = 31; i >= 0; --i) {
      const uint32_t m = 0u - ((xw >> i) & 1u);
      z.w[0] ^= v.w[0] & m;
      z.w[1] ^= v.w[1] & m;
      z.w[2] ^= v.w[2] & m;
      z.w[3] ^= v.w[3] & m;
      v = gf_mul_x(v);
    }
  }
  return z;
}

// Fold a 256-bit unreduced product (a[4..7] = coefficients of x^128..x^255)
// into 128 bits: E * x^128 = E ^ E*x ^ E*x^2 ^ E*x^7, whose own overflow V
// (at most 7 bits past x^127) is folded the same way once more.
__device__ __forceinline__ Gf4 gf_fold(const uint32_t (&a)[8]) {
  const uint64_t eh = ((uint64_t)a[4] << 32) | a[5], el = ((uint64_t)a[6] << 32) | a[7];
  const uint64_t v = (el << 63) ^ (el << 62) ^ (el << 57);
  const uint64_t hi = (((uint64_t)a[0] << 32) | a[1]) ^ eh ^ (eh >> 1) ^ (eh >> 2) ^ (eh >> 7) ^
                      v ^ (v >> 1) ^ (v >> 2) ^ (v >> 7);
  const uint64_t lo = (((uint64_t)a[2] << 32) | a[3]) ^ el ^ ((el >> 1) | (eh << 63)) ^
                      ((el >> 2) | (eh << 62)) ^ ((el >> 7) | (eh << 57));
  return Gf4{{(uint32_t)(hi >> 32), (uint32_t)hi, (uint32_t)(lo >> 32), (uint32_t)lo}};
}

// Unreduced sum of X_b * T_b over NB blocks, each with its own 4-bit table
// (LDS), then one fold.  Nibble i of word q (bits 28-4i) is coefficient block
// 8q+i, i.e. a shift of 32q + 4i: the word offset q is placement, the 4i is
// the Horner chain over i.
template <int NB>
__device__ __forceinline__ Gf4 gf_mul_tables(const Gf4 (&x)[NB], const u32x4* const (&t)[NB]) {
  uint32_t a[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  // rolled: the nibble shift is the only per-step difference, and a fully
  // unrolled chain lets the compiler hoist every lookup (256+ VGPRs)
#pragma unroll 1
  for (int i = 7; i >= 0; --i) {
    if (i < 7) {
#pragma unroll
      for (int d = 7; d > 0; --d) a[d] = funnel(a[d - 1], a[d], 4);
      a[0] >>= 4;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int b = 0; b < NB; b += 2) {
        const u32x4 e1 = t[b][(x[b].w[q] >> (28 - 4 * i)) & 0xFu];
        const u32x4 e2 = t[b + 1][(x[b + 1].w[q] >> (28 - 4 * i)) & 0xFu];
        a[q] = xor3(a[q], e1.x, e2.x);
        a[q + 1] = xor3(a[q + 1], e1.y, e2.y);
        a[q + 2] = xor3(a[q + 2], e1.z, e2.z);
        a[q + 3] = xor3(a[q + 3], e1.w, e2.w);
      }
    }
  }
  return gf_fold(a);
}

// Table n*H^(j+1) (gcm_init_4bit of that power): lane 16j+n of the wave
// writes entry n of table j.
__device__ __forceinline__ void gf_table_entry(u32x4* tab, const Gf4& h, uint32_t n) {
  const Gf4 h1 = gf_mul_x(h), h2 = gf_mul_x(h1), h3 = gf_mul_x(h2);
  Gf4 e{{0u, 0u, 0u, 0u}};
  if (n & 8u) e = gf_xor(e, h);
  if (n & 4u) e = gf_xor(e, h1);
  if (n & 2u) e = gf_xor(e, h2);
  if (n & 1u) e = gf_xor(e, h3);
  tab[n] = u32x4{e.w[0], e.w[1], e.w[2], e.w[3]};
}

// GHASH blocks per step: Y' = (Y ^ C1)*H^m ^ C2*H^(m-1) ^ ... ^ Cm*H, m <= kGhNB
constexpr int kGhNB = 4;

struct Ghash {
  Gf4 y, h;
  const u32x4* tab;  // [16j .. 16j+15] = n*H^(j+1), j < kGhNB; nullptr: bit-serial
};

// Absorb the first m (1..NB) of blocks c[0..NB-1].  Table path: block b < m
// uses H^(m-b); blocks past m enter as zero (T[0] = 0) — one instruction
// stream for every m, no divergence.
template <int NB>
__device__ __forceinline__ void ghash_absorb(Ghash& g, const u32x4 (&c)[NB], uint32_t m) {
  static_assert(NB <= kGhNB && NB % 2 == 0, "tables for NB powers, blocks in pairs");
  if (g.tab) {
    Gf4 x[NB];
    const u32x4* t[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      x[b] = (uint32_t)b < m ? gf_from_block(c[b]) : Gf4{{0u, 0u, 0u, 0u}};
      t[b] = g.tab + 16u * ((uint32_t)b < m ? m - 1u - b : 0u);
    }
    x[0] = gf_xor(x[0], g.y);
    g.y = gf_mul_tables<NB>(x, t);
  } else {
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if ((uint32_t)b < m) g.y = gf_mul_bits(gf_xor(g.y, gf_from_block(c[b])), g.h);
  }
}

__device__ __forceinline__ void ghash_block(Ghash& g, u32x4 blk) {
  const u32x4 c[2] = {blk, blk};
  ghash_absorb<2>(g, c, 1u);
}

// Counter block for data chunk c: J0 + 1 + c, J0 = nonce || 0x00000001.
__device__ __forceinline__ u32x4 gcm_ctr(const uint32_t (&n)[3], uint32_t c) {
  return u32x4{n[0], n[1], n[2], __builtin_bswap32(2u + c)};
}

// Payload pass (as aead_pass for ChaCha20): XOR keystream / GHASH in or out,
// NB chunks per step (NB independent AES blocks interleaved; GHASH with
// aggregated reduction over the step).
template <uint32_t SC, int NB, bool XOR, bool MAC_IN, bool MAC_OUT, bool NTS = kAeadNTS>
__device__ __forceinline__ void gcm_pass(const AesKey& key, const uint32_t (&nonce)[3],
                                         Ghash& gh, const uint32_t* te, uint32_t copy,
                                         const StageMeta* meta, u32x4* rows, uint32_t lane,
                                         uint32_t my_nfull, bool store) {
  static_assert(SC % NB == 0u, "whole steps per slab");
  const uint32_t nslab = (wave_max_u32(my_nfull) + SC - 1) / SC;
  u32x4 buf[SC];
  if (nslab) stage_load<SC>(meta, lane, 0, buf);
  for (uint32_t sl = 0; sl < nslab; ++sl) {
    stage_to_lds<SC>(rows, lane, buf);
    if (sl + 1u < nslab) stage_load<SC>(meta, lane, sl + 1u, buf);
    for (uint32_t j = 0; j < SC; j += NB) {
      const uint32_t c = sl * SC + j;
      if (c >= my_nfull) break;
      const uint32_t m = min((uint32_t)NB, my_nfull - c);
      u32x4* slot = rows + lane * (SC + 1u) + j;
      u32x4 v[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) v[b] = slot[b];
      if constexpr (MAC_IN) ghash_absorb<NB>(gh, v, m);
      if constexpr (XOR) {
        u32x4 k[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) k[b] = gcm_ctr(nonce, c + b);
        aes_encrypt_n<NB>(key, k, te, copy);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          v[b] ^= k[b];
          slot[b] = v[b];  // chunks past the packet's end are never stored
        }
      }
      if constexpr (MAC_OUT) ghash_absorb<NB>(gh, v, m);
    }
    if (store) {
      u32x4 out[SC];
      stage_from_lds<SC>(rows, lane, out);
      stage_store<SC, true, NTS>(meta, lane, sl, out);
    }
  }
}

__device__ __forceinline__ void ghash_lengths(Ghash& g, uint32_t ad_len, uint32_t ct_len) {
  // [len(A)]_64 || [len(C)]_64 in bits, big-endian
  const uint64_t a = (uint64_t)ad_len * 8u, c = (uint64_t)ct_len * 8u;
  const u32x4 blk = gf_to_block(Gf4{{(uint32_t)(a >> 32), (uint32_t)a, (uint32_t)(c >> 32),
                                     (uint32_t)c}});
  ghash_block(g, blk);
}

__device__ __forceinline__ void ghash_span_padded(Ghash& g, const uint8_t* d, uint32_t len) {
  const uint32_t nfull = len >> 4;
  uint32_t c = 0;
  for (; c < nfull; c += 2u) {
    const u32x4 v[2] = {ld16(d + 16u * c), ld16(d + 16u * min(c + 1u, nfull - 1u))};
    ghash_absorb<2>(g, v, min(2u, nfull - c));
  }
  const uint32_t rem = len & 15u;
  if (rem) {
    uint8_t b[16];
#pragma unroll
    for (uint32_t i = 0; i < 16u; ++i) b[i] = i < rem ? d[16u * nfull + i] : (uint8_t)0;
    u32x4 v;
    __builtin_memcpy(&v, b, 16);
    ghash_block(g, v);
  }
}

// 768-thread blocks: the 64 KiB table is shared by 12 waves with 64-B slabs
// (SC = 4): LDS 154 KiB per block = one block per CU = 3 waves/SIMD, which the
// key-uniform path's SGPR round keys make fit in 168 VGPRs (148 used).
// Measured vs 512 threads / SC = 8 / 2 waves at 2^21 packets: seal +6.5%,
// open +1.3% (profiles/round1/tune_gcm_g8.txt); smaller batches and open run
// the 512-thread shape instead (launch_aes128gcm picks by batch size).
constexpr int kGcmBlock = 768;
constexpr int kGcmWPE = 3;  // waves per SIMD
constexpr int kGcmNB = 4;   // chunks per step of the payload passes

// Everything after the key setup, for one packet per lane.  Instantiated
// twice in the kernel when UNI: with the key-uniform wave's round keys as
// wave-uniform values (SGPRs, 44 VGPRs freed) and with per-lane keys.
template <uint32_t SC, bool OPEN, int NB, bool ONEPASS = false, bool NTS = kAeadNTS>
__device__ __forceinline__ void gcm_packet(const AeadArgs& a, const AesKey& key,
                                           const uint32_t (&nonce)[3], Ghash& gh,
                                           const uint32_t* s_te, uint32_t copy, StageMeta* meta,
                                           u32x4* rows, uint32_t lane, uint64_t p, bool valid,
                                           const uint8_t* ad, const uint8_t* in, uint32_t alen,
                                           uint32_t plen) {
  StageMeta* const s_meta_w = meta;
  u32x4* const s_rows_w = rows;

  u32x4 tail = {0u, 0u, 0u, 0u};
  if (valid) {
    ghash_span_padded(gh, ad, alen);
    tail = tail_bytes(load_tail(in, plen), plen);  // before any store (in place)
  }
  const uint32_t rem = plen & 15u, ctail = plen >> 4;
  if constexpr (!OPEN) {
    uint8_t* o = valid ? a.io.out + a.io.out_off[p] : nullptr;
    s_meta_w[lane] = StageMeta{in, o, plen >> 4};
    gcm_pass<SC, NB, true, false, true, NTS>(key, nonce, gh, s_te, copy, s_meta_w, s_rows_w, lane,
                                    plen >> 4, true);
    if (!valid) return;
    if (rem) {
      u32x4 ct = tail ^ aes_encrypt(key, gcm_ctr(nonce, ctail), s_te, copy);
      uint8_t b[16];
      __builtin_memcpy(b, &ct, 16);
      for (uint32_t i = rem; i < 16u; ++i) b[i] = 0;  // zero pad for GHASH
      __builtin_memcpy(&ct, b, 16);
      ghash_block(gh, ct);
      for (uint32_t i = 0; i < rem; ++i) o[16u * ctail + i] = b[i];
    }
    ghash_lengths(gh, alen, plen);
    const u32x4 ek0 = aes_encrypt(key, u32x4{nonce[0], nonce[1], nonce[2], 0x01000000u}, s_te,
                                  copy);  // E_K(J0)
    const u32x4 t = gf_to_block(gh.y) ^ ek0;
    const uint32_t tag[3] = {t.x, t.y, t.z};
    __builtin_memcpy(o + plen, tag, kTag);  // ct || tag
  } else if constexpr (ONEPASS) {
    // QFEC_SCRATCH_OUTPUT: GHASH over the ciphertext and CTR decryption from
    // the same slab loads; a failed packet keeps its unverified plaintext
    // (aead_aes_gcm_open decrypts before it compares, e_aes.c:1093-1140)
    uint32_t want[3] = {0u, 0u, 0u};
    if (valid) __builtin_memcpy(want, in + plen, kTag);
    uint8_t* o = valid ? a.io.out + a.io.out_off[p] : nullptr;
    s_meta_w[lane] = StageMeta{in, o, plen >> 4};
    gcm_pass<SC, NB, true, true, false, NTS>(key, nonce, gh, s_te, copy, s_meta_w, s_rows_w, lane,
                                    plen >> 4, true);
    if (!valid) return;
    if (rem) {
      ghash_block(gh, tail);  // zero padded ciphertext tail
      const u32x4 pt = tail ^ aes_encrypt(key, gcm_ctr(nonce, ctail), s_te, copy);
      uint8_t b[16];
      __builtin_memcpy(b, &pt, 16);
      for (uint32_t i = 0; i < rem; ++i) o[16u * ctail + i] = b[i];
    }
    ghash_lengths(gh, alen, plen);
    const u32x4 ek0 = aes_encrypt(key, u32x4{nonce[0], nonce[1], nonce[2], 0x01000000u}, s_te,
                                  copy);
    const u32x4 t = gf_to_block(gh.y) ^ ek0;
    a.io.ok[p] = ((t.x ^ want[0]) | (t.y ^ want[1]) | (t.z ^ want[2])) == 0u ? 1 : 0;
  } else {
    uint32_t want[3] = {0u, 0u, 0u};
    if (valid) __builtin_memcpy(want, in + plen, kTag);
    s_meta_w[lane] = StageMeta{in, nullptr, plen >> 4};
    gcm_pass<SC, NB, false, true, false>(key, nonce, gh, s_te, copy, s_meta_w, s_rows_w, lane,
                                     plen >> 4, false);
    bool ok = false;
    if (valid) {
      if (rem) ghash_block(gh, tail);  // zero padded
      ghash_lengths(gh, alen, plen);
      const u32x4 ek0 = aes_encrypt(key, u32x4{nonce[0], nonce[1], nonce[2], 0x01000000u}, s_te,
                                    copy);
      const u32x4 t = gf_to_block(gh.y) ^ ek0;
      ok = ((t.x ^ want[0]) | (t.y ^ want[1]) | (t.z ^ want[2])) == 0u;
      a.io.ok[p] = ok ? 1 : 0;
    }
    uint8_t* o = ok ? a.io.out + a.io.out_off[p] : nullptr;
    s_meta_w[lane] = StageMeta{in, o, ok ? plen >> 4 : 0u};
    gcm_pass<SC, NB, true, false, false, NTS>(key, nonce, gh, s_te, copy, s_meta_w, s_rows_w, lane,
                                     ok ? plen >> 4 : 0u, true);
    if (ok && rem) {
      const u32x4 pt = tail ^ aes_encrypt(key, gcm_ctr(nonce, ctail), s_te, copy);
      uint8_t b[16];
      __builtin_memcpy(b, &pt, 16);
      for (uint32_t i = 0; i < rem; ++i) o[16u * ctail + i] = b[i];
    }
  }
}

template <uint32_t SC, bool OPEN, int NB = kGcmNB, int BLOCK = kGcmBlock, int WPE = kGcmWPE,
          bool UNI = true, bool ONEPASS = false, bool NTS = kAeadNTS>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void
aes128gcm_kernel(AeadArgs a) {
  constexpr int kGcmWaves = BLOCK / 64;
  // one LDS object with the table first: it sits at LDS address 0, so the
  // v_perm result IS the lookup address (no base add per lookup)
  struct Smem {
    uint32_t te[kTeBytes / 4u];
    u32x4 tab[kGcmWaves][16 * kGhNB];  // n*H^j per wave (256-B aligned tables)
    u32x4 rows[kGcmWaves][64 * (SC + 1u)];
    StageMeta meta[kGcmWaves][64];
  };
  __shared__ Smem sm;
  uint32_t* const s_te = sm.te;
  auto& s_rows = sm.rows;
  auto& s_meta = sm.meta;
  auto& s_tab = sm.tab;
  // replicated Te0, 16-B stores (every thread of the block helps, then a barrier)
  for (uint32_t i = threadIdx.x; i < kTeBytes / 16u; i += BLOCK) {
    const uint32_t e = kTe0[i >> 4];
    reinterpret_cast<u32x4*>(s_te)[i] = u32x4{e, e, e, e};
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t copy = lane * 4u;  // the lane's byte column in every table row
  const uint64_t p = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const uint32_t inl = p < a.io.n ? a.io.in_len[p] : 0u;
  const bool valid = p < a.io.n && (!OPEN || inl >= kTag);
  if (OPEN && p < a.io.n && !valid) a.io.ok[p] = 0;  // open: in_len < tag_len
  const uint8_t* ad = nullptr;
  const uint8_t* in = nullptr;
  uint32_t alen = 0, plen = 0, kidx = 0;
  AesKey key = {};
  uint32_t nonce[3] = {0u, 0u, 0u};
  if (valid) {
    ad = a.io.bytes + a.io.ad_off[p];
    in = a.io.bytes + a.io.in_off[p];
    alen = a.io.ad_len[p];
    plen = OPEN ? inl - kTag : inl;
    kidx = a.key_idx[p];
    aes_expand(key, a.keys + 16ull * kidx, s_te, copy);
    uint32_t pre;
    __builtin_memcpy(&pre, a.prefixes + 4ull * kidx, 4);
    const uint64_t pn = ((uint64_t)(a.path_id ? a.path_id[p] : 0u) << 56) | a.packet_number[p];
    nonce[0] = pre;  // nonce = prefix || LE64(path_id << 56 | packet_number)
    nonce[1] = (uint32_t)pn;
    nonce[2] = (uint32_t)(pn >> 32);
  }
  // H = E_K(0^128); the wave shares the 4-bit tables when all its valid
  // packets use the same key (tables from the first valid lane's H)
  Ghash gh;
  gh.h = gf_from_block(valid ? aes_encrypt(key, u32x4{0u, 0u, 0u, 0u}, s_te, copy)
                             : u32x4{0u, 0u, 0u, 0u});
  gh.y = Gf4{{0u, 0u, 0u, 0u}};
  gh.tab = nullptr;
  const uint64_t vmask = __ballot(valid);
  const int src = vmask ? __builtin_ctzll(vmask) : 0;  // first valid lane
  if (vmask != 0ull) {
    const uint32_t k0 = (uint32_t)__builtin_amdgcn_readlane((int)kidx, src);
    if (__ballot(valid && kidx != k0) == 0ull) {
      Gf4 h;
#pragma unroll
      for (int i = 0; i < 4; ++i) h.w[i] = (uint32_t)__builtin_amdgcn_readlane((int)gh.h.w[i], src);
      Gf4 hp = h;  // H^(j+1) for lane 16j+n (once per wave)
      for (uint32_t j = 0; j < lane / 16u; ++j) hp = gf_mul_bits(hp, h);
      if (lane < 16u * kGhNB) gf_table_entry(s_tab[wv] + (lane & ~15u), hp, lane & 15u);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      gh.tab = s_tab[wv];
    }
  }
  if (UNI && gh.tab) {
    AesKey ks;  // the wave's key as uniform values
#pragma unroll
    for (int i = 0; i < 44; ++i) ks.rk[i] = (uint32_t)__builtin_amdgcn_readlane((int)key.rk[i], src);
    gcm_packet<SC, OPEN, NB, ONEPASS, NTS>(a, ks, nonce, gh, s_te, copy, s_meta[wv], s_rows[wv],
                                           lane, p, valid, ad, in, alen, plen);
  } else {
    gcm_packet<SC, OPEN, NB, ONEPASS, NTS>(a, key, nonce, gh, s_te, copy, s_meta[wv], s_rows[wv],
                                           lane, p, valid, ad, in, alen, plen);
  }
}

}  // namespace

hipError_t launch_null_protect(const ProtectArgs& a0, bool decrypt, hipStream_t s) {
  const uint64_t chunk = kMaxBlocks256 * kBlock;
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
    if (decrypt && a.scratch_out)
      hipLaunchKernelGGL(null_decrypt_onepass_kernel<kSlabChunks>, dim3(blocks), dim3(kBlock), 0, s, a);
    else if (decrypt)
      hipLaunchKernelGGL(null_decrypt_staged_kernel<kSlabChunks>, dim3(blocks), dim3(kBlock), 0, s, a);
    else
      hipLaunchKernelGGL(null_encrypt_staged_kernel<kSlabChunks>, dim3(blocks), dim3(kBlock), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace qfec

namespace qfec {

// AEAD slab: 256 B (16 chunks = 4 ChaCha blocks) per packet per slab: seal
// +10%, open +16% over 128-B slabs; 64-B slabs 0.82x
// (profiles/round1/tune_protect_a4.txt).
hipError_t launch_chacha20poly1305(const AeadArgs& a0, bool decrypt, hipStream_t s) {
  constexpr uint32_t SC = 16;
  const uint64_t chunk = kMaxBlocks256 * kBlock;
  for (uint64_t p = 0; p < a0.io.n; p += chunk) {
    AeadArgs a = a0;
    a.io.n = a0.io.n - p < chunk ? a0.io.n - p : chunk;
    a.io.ad_off += p;
    a.io.ad_len += p;
    a.io.in_off += p;
    a.io.in_len += p;
    a.io.out_off += p;
    if (decrypt) a.io.ok += p;
    a.key_idx += p;
    a.packet_number += p;
    if (a.path_id) a.path_id += p;
    const uint32_t blocks = (uint32_t)((a.io.n + kBlock - 1) / kBlock);
    if (decrypt && a.io.scratch_out)
      hipLaunchKernelGGL((c20p1305_open_kernel<SC, true>), dim3(blocks), dim3(kBlock), 0, s, a);
    else if (decrypt)
      hipLaunchKernelGGL(c20p1305_open_kernel<SC>, dim3(blocks), dim3(kBlock), 0, s, a);
    else
      hipLaunchKernelGGL(c20p1305_seal_kernel<SC>, dim3(blocks), dim3(kBlock), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace qfec

namespace qfec {

// AES-128-GCM block shape by batch: both shapes fill the LDS (one block per
// CU), so a grid of blocks/256 rounds leaves its last round partly idle.
// Measured seal / open (tools/tune/tune_gcm.hip, profiles/round1/tune_gcm_gq_*.txt):
// 512 threads / 128-B slabs / 2 waves per SIMD against the 768-thread shape
// (64-B slabs, 3 waves): 1.30x / 1.30x at 2^16 packets, 1.27x / 1.30x at
// 2^18, 1.04x / 1.05x at 2^20, 1.00x / 1.04x at 2^22, 0.95x / 1.01x at
// 2^23.  Seal keeps the
// 768-thread shape from 2^22 packets on (+3% at 2^21 measured earlier,
// tune_gcm_g12.txt); open always takes 512.
constexpr uint64_t kGcmSeal768From = 1ull << 22;

template <bool OPEN, int BLOCK>
hipError_t launch_gcm_shape(const AeadArgs& a0, hipStream_t s) {
  constexpr uint32_t SC = BLOCK == 768 ? 4u : 8u;
  constexpr int WPE = BLOCK == 768 ? 3 : 2;
  const uint64_t chunk = kMaxBlocks256 * 256u / BLOCK * BLOCK;  // < 2^32 work-items
  for (uint64_t p = 0; p < a0.io.n; p += chunk) {
    AeadArgs a = a0;
    a.io.n = a0.io.n - p < chunk ? a0.io.n - p : chunk;
    a.io.ad_off += p;
    a.io.ad_len += p;
    a.io.in_off += p;
    a.io.in_len += p;
    a.io.out_off += p;
    if (OPEN) a.io.ok += p;
    a.key_idx += p;
    a.packet_number += p;
    if (a.path_id) a.path_id += p;
    const uint32_t blocks = (uint32_t)((a.io.n + BLOCK - 1) / BLOCK);
    if (OPEN && a.io.scratch_out)
      hipLaunchKernelGGL((aes128gcm_kernel<SC, OPEN, kGcmNB, BLOCK, WPE, true, true>), dim3(blocks),
                         dim3(BLOCK), 0, s, a);
    else
      hipLaunchKernelGGL((aes128gcm_kernel<SC, OPEN, kGcmNB, BLOCK, WPE>), dim3(blocks),
                         dim3(BLOCK), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_aes128gcm(const AeadArgs& a, bool decrypt, hipStream_t s) {
  if (decrypt) return launch_gcm_shape<true, 512>(a, s);
  return a.io.n >= kGcmSeal768From ? launch_gcm_shape<false, 768>(a, s)
                                   : launch_gcm_shape<false, 512>(a, s);
}

}  // namespace qfec
