/*
 * qaead_oracle.h — CPU restatement of libquic's ChaCha20-Poly1305 packet
 * protection (the AEAD negotiated for QUIC crypto, 12-byte tags).
 *
 * TEST INFRASTRUCTURE ONLY (tests/, bench.py cpu_baseline); the product never
 * links it.
 *
 * Restated (file:line in /root/reference):
 *   qo_chacha20           CRYPTO_chacha_20, boringssl/crypto/chacha/chacha.c:118-170
 *                         (RFC 7539 §2.3-2.4 block function, 32-bit counter)
 *   qo_poly1305           CRYPTO_poly1305_{init,update,finish},
 *                         boringssl/crypto/poly1305/poly1305_vec.c (x86-64 build)
 *                         (RFC 7539 §2.5; r clamped, 130-bit accumulator)
 *   qo_c20p1305_seal/open seal_impl / open_impl + poly1305_update,
 *                         boringssl/crypto/cipher/e_chacha20poly1305.c:71-200
 *                         (RFC 7539 §2.8: keystream counter 1, one-time key from
 *                         counter 0, MAC over AD|pad|CT|pad|len(AD)|len(CT),
 *                         tag truncated to tag_len)
 *   qo_quic_c20p1305_*    AeadBaseEncrypter::EncryptPacket /
 *                         AeadBaseDecrypter::DecryptPacket
 *                         (net/quic/core/crypto/aead_base_encrypter.cc:107-134,
 *                         aead_base_decrypter.cc), ChaCha20Poly1305Encrypter
 *                         (chacha20_poly1305_encrypter.cc: 32-byte key, 4-byte
 *                         nonce prefix; kAuthTagSize = 12 in the .h):
 *                         nonce = prefix(4) || LE64(path_id << 56 | packet_number)
 *                         (QuicUtils::PackPathIdAndPacketNumber quic_utils.cc:465-475)
 *
 *   qo_aes128_*           AES-128 (FIPS-197) as AES_set_encrypt_key / AES_encrypt,
 *                         boringssl/crypto/aes/aes.c (C build)
 *   qo_aes128gcm_seal/open  aead_aes_gcm_seal / _open,
 *                         boringssl/crypto/cipher/e_aes.c:1050-1140 over
 *                         CRYPTO_gcm128_* (boringssl/crypto/modes/gcm.c):
 *                         SP 800-38D GCM, any IV length, tag truncated to tag_len
 *   qo_quic_aes128gcm_*   Aes128Gcm12Encrypter / Decrypter
 *                         (crypto/aes_128_gcm_12_encrypter.cc: 16-byte key, 4-byte
 *                         nonce prefix, kAuthTagSize = 12) via AeadBaseEncrypter
 *
 * PINNED by BoringSSL's own test vectors in the reference tree
 * (boringssl/crypto/cipher/test/{chacha20_poly1305,aes_128_gcm}_tests.txt ->
 * tests/golden/{chacha20_poly1305,aes_128_gcm}.npz, tests/golden/make_golden_aead.py)
 * and by the reference's chacha.c / poly1305_vec.c / aes.c / gcm.c compiled
 * into oracle/_ref/libref_quic.so (oracle/ref/Makefile).  The AEAD glue
 * (e_chacha20poly1305.c) and AeadBaseEncrypter link BoringSSL's generated
 * err_data.c, which needs Go: not buildable here, restated.
 */
#ifndef QAEAD_ORACLE_H_
#define QAEAD_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QO_C20P1305_KEY 32u
#define QO_C20P1305_NONCE_PREFIX 4u
#define QO_QUIC_AEAD_TAG 12u /* kAuthTagSize */

void qo_chacha20(uint8_t* out, const uint8_t* in, size_t len, const uint8_t key[32],
                 const uint8_t nonce[12], uint32_t counter);
void qo_poly1305(uint8_t tag[16], const uint8_t* msg, size_t len, const uint8_t key[32]);

/* RFC 7539 AEAD with a tag_len-byte tag appended: out = ct || tag.  Returns 1. */
int qo_c20p1305_seal(uint8_t* out, const uint8_t key[32], const uint8_t nonce[12],
                     const uint8_t* in, size_t in_len, const uint8_t* ad, size_t ad_len,
                     size_t tag_len);
/* in = ct || tag; returns 1 and writes in_len - tag_len plaintext bytes when the
 * tag verifies, 0 otherwise (out untouched). */
int qo_c20p1305_open(uint8_t* out, const uint8_t key[32], const uint8_t nonce[12],
                     const uint8_t* in, size_t in_len, const uint8_t* ad, size_t ad_len,
                     size_t tag_len);

/* QUIC packet form (12-byte tag, nonce from prefix + path id + packet number). */
int qo_quic_c20p1305_encrypt(uint8_t* out, const uint8_t key[32], const uint8_t prefix[4],
                             uint8_t path_id, uint64_t packet_number, const uint8_t* ad,
                             size_t ad_len, const uint8_t* pt, size_t pt_len);
int qo_quic_c20p1305_decrypt(uint8_t* out, const uint8_t key[32], const uint8_t prefix[4],
                             uint8_t path_id, uint64_t packet_number, const uint8_t* ad,
                             size_t ad_len, const uint8_t* ct, size_t ct_len);

/* Batches (CSR as qpp_oracle.h): packet p uses key key_idx[p] (keys: 32 B each,
 * prefixes: 4 B each), packet_number[p], path_id[p] (NULL = all 0). */
void qo_quic_c20p1305_encrypt_batch(const uint8_t* keys, const uint8_t* prefixes,
                                    const uint32_t* key_idx, const uint64_t* packet_number,
                                    const uint8_t* path_id, const uint8_t* bytes,
                                    const uint64_t* ad_off, const uint16_t* ad_len,
                                    const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                                    uint8_t* out, const uint64_t* out_off, int threads);
void qo_quic_c20p1305_decrypt_batch(const uint8_t* keys, const uint8_t* prefixes,
                                    const uint32_t* key_idx, const uint64_t* packet_number,
                                    const uint8_t* path_id, const uint8_t* bytes,
                                    const uint64_t* ad_off, const uint16_t* ad_len,
                                    const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                                    uint8_t* out, const uint64_t* out_off, uint8_t* ok);

/* ---- AES-128-GCM ---- */
#define QO_AES128_KEY 16u
void qo_aes128_expand(uint32_t rk[44], const uint8_t key[16]);
void qo_aes128_encrypt(uint8_t out[16], const uint8_t in[16], const uint32_t rk[44]);
int qo_aes128gcm_seal(uint8_t* out, const uint8_t key[16], const uint8_t* iv, size_t iv_len,
                      const uint8_t* in, size_t in_len, const uint8_t* ad, size_t ad_len,
                      size_t tag_len);
int qo_aes128gcm_open(uint8_t* out, const uint8_t key[16], const uint8_t* iv, size_t iv_len,
                      const uint8_t* in, size_t in_len, const uint8_t* ad, size_t ad_len,
                      size_t tag_len);
/* Batches (keys: 16 B each, prefixes: 4 B each; as the ChaCha20 forms). */
void qo_quic_aes128gcm_encrypt_batch(const uint8_t* keys, const uint8_t* prefixes,
                                     const uint32_t* key_idx, const uint64_t* packet_number,
                                     const uint8_t* path_id, const uint8_t* bytes,
                                     const uint64_t* ad_off, const uint16_t* ad_len,
                                     const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                                     uint8_t* out, const uint64_t* out_off, int threads);
void qo_quic_aes128gcm_decrypt_batch(const uint8_t* keys, const uint8_t* prefixes,
                                     const uint32_t* key_idx, const uint64_t* packet_number,
                                     const uint8_t* path_id, const uint8_t* bytes,
                                     const uint64_t* ad_off, const uint16_t* ad_len,
                                     const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                                     uint8_t* out, const uint64_t* out_off, uint8_t* ok);

#ifdef __cplusplus
}
#endif
#endif /* QAEAD_ORACLE_H_ */
