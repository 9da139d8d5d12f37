// ref_quic_shim.cc — C entry points into the REFERENCE's own packet
// protection code, compiled from /root/reference by oracle/ref/Makefile into
// oracle/_ref/libref_quic.so.  Test infrastructure only: it pins the
// restatement in oracle/qpp_oracle.c (tests/test_oracle_protect.py) and
// generates tests/golden/null_protect.npz (tests/golden/make_golden_protect.py).
// No reference source is copied: this file only calls the reference classes.
#include <stddef.h>
#include <stdint.h>

#include "net/base/int128.h"
#include "net/quic/core/crypto/null_decrypter.h"
#include "net/quic/core/crypto/null_encrypter.h"
#include "net/quic/core/quic_utils.h"

extern "C" {
#include <openssl/aes.h>
#include <openssl/chacha.h>
#include <openssl/poly1305.h>
#include "modes/internal.h"  // CRYPTO_gcm128_* (boringssl/crypto/modes)
}

#define REF_API extern "C" __attribute__((visibility("default")))

// QuicUtils::FNV1a_128_Hash_Two (quic_utils.cc:110)
REF_API void ref_fnv1a128_two(const char* d1, int n1, const char* d2, int n2, uint64_t* lo,
                              uint64_t* hi) {
  const net::uint128 h = net::QuicUtils::FNV1a_128_Hash_Two(d1, n1, d2, n2);
  *lo = net::Uint128Low64(h);
  *hi = net::Uint128High64(h);
}

// NullEncrypter::EncryptPacket (crypto/null_encrypter.cc:28)
REF_API int ref_null_encrypt(const char* ad, size_t ad_len, const char* pt, size_t pt_len,
                             char* out, size_t cap, size_t* out_len) {
  net::NullEncrypter e;
  return e.EncryptPacket(net::kDefaultPathId, 1, base::StringPiece(ad, ad_len),
                         base::StringPiece(pt, pt_len), out, out_len, cap)
             ? 1
             : 0;
}

// NullDecrypter::DecryptPacket (crypto/null_decrypter.cc:38)
REF_API int ref_null_decrypt(const char* ad, size_t ad_len, const char* ct, size_t ct_len,
                             char* out, size_t cap, size_t* out_len) {
  net::NullDecrypter d;
  return d.DecryptPacket(net::kDefaultPathId, 1, base::StringPiece(ad, ad_len),
                         base::StringPiece(ct, ct_len), out, out_len, cap)
             ? 1
             : 0;
}

// BoringSSL CRYPTO_chacha_20 (boringssl/crypto/chacha/chacha.c:118)
REF_API void ref_chacha20(uint8_t* out, const uint8_t* in, size_t len, const uint8_t* key,
                          const uint8_t* nonce, uint32_t counter) {
  CRYPTO_chacha_20(out, in, len, key, nonce, counter);
}

// BoringSSL CRYPTO_poly1305_* (boringssl/crypto/poly1305/poly1305_vec.c), one
// message fed in `nsplit` arbitrary pieces to exercise the update buffering.
REF_API void ref_poly1305(uint8_t* tag, const uint8_t* msg, size_t len, const uint8_t* key,
                          size_t split) {
  poly1305_state st;
  CRYPTO_poly1305_init(&st, key);
  if (split == 0 || split > len) split = len;
  CRYPTO_poly1305_update(&st, msg, split);
  CRYPTO_poly1305_update(&st, msg + split, len - split);
  CRYPTO_poly1305_finish(&st, tag);
}

// BoringSSL AES_set_encrypt_key + AES_encrypt (boringssl/crypto/aes/aes.c)
REF_API void ref_aes128_encrypt(uint8_t* out, const uint8_t* in, const uint8_t* key) {
  AES_KEY ks;
  AES_set_encrypt_key(key, 128, &ks);
  AES_encrypt(in, out, &ks);
}

// What aead_aes_gcm_seal (boringssl/crypto/cipher/e_aes.c:1050-1091) does,
// over the reference's own GCM mode functions (crypto/modes/gcm.c):
// setiv, aad, encrypt, tag(tag_len).  Returns 1.
REF_API int ref_aes128gcm_seal(uint8_t* out, const uint8_t* key, const uint8_t* iv, size_t iv_len,
                               const uint8_t* in, size_t in_len, const uint8_t* ad,
                               size_t ad_len, size_t tag_len) {
  AES_KEY ks;
  AES_set_encrypt_key(key, 128, &ks);
  GCM128_CONTEXT gcm;
  CRYPTO_gcm128_init(&gcm, &ks, (block128_f)AES_encrypt);
  CRYPTO_gcm128_setiv(&gcm, &ks, iv, iv_len);
  if (ad_len > 0 && !CRYPTO_gcm128_aad(&gcm, ad, ad_len)) return 0;
  if (!CRYPTO_gcm128_encrypt(&gcm, &ks, in, out, in_len)) return 0;
  CRYPTO_gcm128_tag(&gcm, out + in_len, tag_len);
  return 1;
}

// ---- CPU baselines (bench.py cpu_baseline, kind "reference") ---------------
// Batches of packets through the reference's own code on `threads` host
// threads (contiguous packet ranges), the way a connection thread would call
// it once per packet.  Packet p: header bytes[ad_off[p], +ad_len[p]), payload
// bytes[pt_off[p], +pt_len[p]); output at out + out_off[p].
#include <thread>
#include <vector>

template <typename F>
static void ref_parallel(uint64_t n, int threads, F f) {
  if (threads < 1) threads = 1;
  std::vector<std::thread> ts;
  const uint64_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const uint64_t a = t * per, b = a + per < n ? a + per : n;
    if (a >= b) break;
    ts.emplace_back([=] { f(a, b); });
  }
  for (auto& t : ts) t.join();
}

// NullEncrypter::EncryptPacket per packet (tag || payload, 12 + pt_len bytes)
REF_API void ref_null_encrypt_batch(const uint8_t* bytes, const uint64_t* ad_off,
                                    const uint16_t* ad_len, const uint64_t* pt_off,
                                    const uint16_t* pt_len, uint64_t n, uint8_t* out,
                                    const uint64_t* out_off, int threads) {
  ref_parallel(n, threads, [&](uint64_t a, uint64_t b) {
    net::NullEncrypter e;
    for (uint64_t p = a; p < b; ++p) {
      size_t olen = 0;
      e.EncryptPacket(net::kDefaultPathId, p + 1,
                      base::StringPiece((const char*)bytes + ad_off[p], ad_len[p]),
                      base::StringPiece((const char*)bytes + pt_off[p], pt_len[p]),
                      (char*)out + out_off[p], &olen, (size_t)pt_len[p] + 12);
    }
  });
}

// AES-128-GCM-12 seal per packet as AeadBaseEncrypter::EncryptPacket does it
// (aead_base_encrypter.cc:107-134): nonce = 4-byte prefix || LE64(packet
// number), then aead_aes_gcm_seal's steps over gcm.c.  The key schedule and
// GHASH table are set up once per key (SetKey / EVP_AEAD_CTX_init), the
// context is copied per packet.
REF_API void ref_quic_aes128gcm_seal_batch(const uint8_t* keys, const uint8_t* prefixes,
                                           const uint32_t* key_idx, const uint64_t* pn,
                                           uint32_t n_keys, const uint8_t* bytes,
                                           const uint64_t* ad_off, const uint16_t* ad_len,
                                           const uint64_t* pt_off, const uint16_t* pt_len,
                                           uint64_t n, uint8_t* out, const uint64_t* out_off,
                                           int threads) {
  std::vector<AES_KEY> ks(n_keys);
  std::vector<GCM128_CONTEXT> ctx(n_keys);
  for (uint32_t k = 0; k < n_keys; ++k) {
    AES_set_encrypt_key(keys + 16u * k, 128, &ks[k]);
    CRYPTO_gcm128_init(&ctx[k], &ks[k], (block128_f)AES_encrypt);
  }
  ref_parallel(n, threads, [&](uint64_t a, uint64_t b) {
    for (uint64_t p = a; p < b; ++p) {
      const uint32_t k = key_idx[p];
      uint8_t nonce[12];
      for (int i = 0; i < 4; ++i) nonce[i] = prefixes[4u * k + i];
      for (int i = 0; i < 8; ++i) nonce[4 + i] = (uint8_t)(pn[p] >> (8 * i));
      GCM128_CONTEXT g = ctx[k];
      CRYPTO_gcm128_setiv(&g, &ks[k], nonce, 12);
      if (ad_len[p]) CRYPTO_gcm128_aad(&g, bytes + ad_off[p], ad_len[p]);
      uint8_t* o = out + out_off[p];
      CRYPTO_gcm128_encrypt(&g, &ks[k], bytes + pt_off[p], o, pt_len[p]);
      CRYPTO_gcm128_tag(&g, o + pt_len[p], 12);
    }
  });
}

// ---- entropy bookkeeping (QuicSentEntropyManager) --------------------------
#include "net/quic/core/quic_sent_entropy_manager.h"

// One connection's sender: RecordPacketEntropyHash for packets 1..n_total
// (entropy[pn-1]), ClearEntropyBefore(first_pn), then GetCumulativeEntropy
// for first_pn..n_total into cum (n_total - first_pn + 1 bytes), then the
// IsValidEntropy queries in the given (non-decreasing largest) order: query q
// has missing intervals [lo[r], hi[r]) for r in range_ptr[q]..range_ptr[q+1].
REF_API void ref_sent_entropy_run(const uint8_t* entropy, uint64_t n_total, uint64_t first_pn,
                                  uint8_t* cum, uint64_t n_q, const uint64_t* largest,
                                  const uint8_t* claimed, const uint32_t* range_ptr,
                                  const uint64_t* lo, const uint64_t* hi, uint8_t* ok) {
  net::QuicSentEntropyManager m;
  for (uint64_t pn = 1; pn <= n_total; ++pn) m.RecordPacketEntropyHash(pn, entropy[pn - 1]);
  if (first_pn > 1) m.ClearEntropyBefore(first_pn);
  for (uint64_t pn = first_pn; pn <= n_total; ++pn)
    cum[pn - first_pn] = m.GetCumulativeEntropy(pn);
  for (uint64_t q = 0; q < n_q; ++q) {
    net::PacketNumberQueue missing;
    for (uint32_t r = range_ptr[q]; r < range_ptr[q + 1]; ++r) missing.Add(lo[r], hi[r]);
    ok[q] = m.IsValidEntropy(largest[q], missing, claimed[q]) ? 1 : 0;
  }
}
