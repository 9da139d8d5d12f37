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
// third limb's addend) + one v_mul_lo_u32 + a shift/add for the top limb.
// The byte step is ≈10 VALU instructions per lane; a lane reads its packet in
// batches of eight 16-byte chunks issued back to back (see kBatch).
//
// In-place encryption (QuicPacketCreator::EncryptInPlace: output == payload,
// payload shifted right by the tag) is supported: the lane loads the payload's
// last 16 bytes first, never stores a chunk before the chunk after it is
// loaded, and writes the tag last.  Decrypt verifies first and copies the payload only when the tag
// matches (output untouched otherwise, as the reference's memcpy-after-check).
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

// A lane reads its packet in batches of kBatch 16-byte chunks (128 bytes, one
// L2 line's worth) issued back to back, then hashes them: the line is consumed
// while it is still in L2.  Loading chunk by chunk instead (load, hash ~170
// instructions, load the next) lets 64 lanes x 8 waves x 256 CUs of
// half-used lines fall out of L2 between a lane's consecutive chunks: 7x less
// throughput measured (tools/tune/tune_protect.hip).
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

// Hash a span and copy it to d.  d may equal p + 12 (in-place encryption):
// the tail is loaded before any store, and the last chunk of a batch is
// stored only after the next batch is loaded (its store reaches 12 bytes
// into the next chunk).
__device__ __forceinline__ void fnv_span_copy(Fnv128& h, const uint8_t* p, uint32_t len,
                                              uint8_t* d) {
  const uint32_t nfull = len >> 4;
  const u32x4 tail = load_tail(p, len);
  u32x4 pend = {0u, 0u, 0u, 0u};
  uint32_t pend_c = 0xFFFFFFFFu;  // chunk index of the deferred store
  for (uint32_t c = 0; c < nfull; c += kBatch) {
    u32x4 v[kBatch];
#pragma unroll
    for (uint32_t u = 0; u < kBatch; ++u) v[u] = ld16(p + 16u * min(c + u, nfull - 1u));
    if (pend_c != 0xFFFFFFFFu) st16(d + 16u * pend_c, pend);
    const uint32_t nb = min(kBatch, nfull - c);
#pragma unroll
    for (uint32_t u = 0; u < kBatch; ++u) {
      if (u < nb) {
        fnv_chunk(h, v[u]);
        if (u + 1u < nb) st16(d + 16u * (c + u), v[u]);
      }
    }
    pend = v[0];
#pragma unroll
    for (uint32_t u = 1; u < kBatch; ++u) pend = (u + 1u == nb) ? v[u] : pend;
    pend_c = c + nb - 1u;
  }
  if (pend_c != 0xFFFFFFFFu) st16(d + 16u * pend_c, pend);
  fnv_tail(h, tail, len);
  store_tail(d, tail, len);
}

// Plain copy of a span, batched like the hash loops (decrypt's second pass).
__device__ __forceinline__ void copy_span(const uint8_t* p, uint32_t len, uint8_t* d) {
  const uint32_t nfull = len >> 4;
  const u32x4 tail = load_tail(p, len);
  for (uint32_t c = 0; c < nfull; c += kBatch) {
    u32x4 v[kBatch];
#pragma unroll
    for (uint32_t u = 0; u < kBatch; ++u) v[u] = ld16(p + 16u * min(c + u, nfull - 1u));
#pragma unroll
    for (uint32_t u = 0; u < kBatch; ++u)
      if (c + u < nfull) st16(d + 16u * (c + u), v[u]);
  }
  store_tail(d, tail, len);
}

__global__ __launch_bounds__(kBlock) void null_encrypt_kernel(ProtectArgs a) {
  const uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= a.n) return;
  const uint8_t* ad = a.bytes + a.ad_off[p];
  const uint8_t* pt = a.bytes + a.in_off[p];
  const uint32_t alen = a.ad_len[p], plen = a.in_len[p];
  uint8_t* o = a.out + a.out_off[p];
  Fnv128 h = fnv_init();
  fnv_span(h, ad, alen);
  fnv_span_copy(h, pt, plen, o + kTag);
  // SerializeUint128Short (quic_utils.cc:175-181): low 64 bits, then the next 32
  const uint32_t tag[3] = {h.x0, h.x1, h.x2};
  __builtin_memcpy(o, tag, kTag);
}

__global__ __launch_bounds__(kBlock) void null_decrypt_kernel(ProtectArgs a) {
  const uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= a.n) return;
  const uint32_t clen = a.in_len[p];
  if (clen < kTag) {  // ReadHash fails (null_decrypter.cc:48-50)
    a.ok[p] = 0;
    return;
  }
  const uint8_t* ad = a.bytes + a.ad_off[p];
  const uint8_t* ct = a.bytes + a.in_off[p];
  const uint32_t alen = a.ad_len[p], plen = clen - kTag;
  uint32_t tag[3];
  __builtin_memcpy(tag, ct, kTag);
  Fnv128 h = fnv_init();
  fnv_span(h, ad, alen);
  fnv_span(h, ct + kTag, plen);
  // ComputeHash keeps the low 96 bits (null_decrypter.cc:97-106)
  const bool ok = h.x0 == tag[0] && h.x1 == tag[1] && h.x2 == tag[2];
  a.ok[p] = ok ? 1 : 0;
  if (!ok) return;
  // copy after the check (null_decrypter.cc:60-62); the payload is in L2 now
  copy_span(ct + kTag, plen, a.out + a.out_off[p]);
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
      hipLaunchKernelGGL(null_decrypt_kernel, dim3(blocks), dim3(kBlock), 0, s, a);
    else
      hipLaunchKernelGGL(null_encrypt_kernel, dim3(blocks), dim3(kBlock), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace qfec
