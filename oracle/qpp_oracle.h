/*
 * qpp_oracle.h — CPU restatement of libquic's NULL packet protection
 * (the FNV-1a-128 "encryption" used before the handshake completes).
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libquic_amd/, include/)
 * links, loads or calls this code.  It is the checker used by tests/ and
 * bench.py's cpu_baseline leg for the packet-protection kernels.
 *
 * PINNED by the reference: tests/test_oracle_protect.py checks this
 * restatement byte-for-byte against the reference's own NullEncrypter /
 * NullDecrypter / QuicUtils::FNV1a_128_Hash_Two compiled from
 * /root/reference (oracle/ref/Makefile -> oracle/_ref/libref_quic.so) and
 * against fixtures that library generated (tests/golden/null_protect.npz).
 *
 * Restated functions:
 *   qo_fnv1a128_two   QuicUtils::FNV1a_128_Hash_Two  quic_utils.cc:110-125
 *                     (IncrementalHashFast :31-50; kPrime = 2^88 + 315,
 *                      kOffset = 144066263297769815596495629667062367629)
 *   qo_null_encrypt   NullEncrypter::EncryptPacket   crypto/null_encrypter.cc:28-47
 *                     (12-byte tag = SerializeUint128Short quic_utils.cc:175-181,
 *                      placed BEFORE the plaintext)
 *   qo_null_decrypt   NullDecrypter::DecryptPacket   crypto/null_decrypter.cc:38-64
 *                     (ReadHash :84-95, ComputeHash masks the top 32 bits :97-106)
 */
#ifndef QPP_ORACLE_H_
#define QPP_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QO_NULL_TAG_SIZE 12u /* kHashSizeShort, null_encrypter.cc:15 */

void qo_fnv1a128_two(const uint8_t* d1, size_t n1, const uint8_t* d2, size_t n2, uint64_t* lo,
                     uint64_t* hi);
/* 1 on success (output = 12-byte tag || plaintext), 0 if cap is too small. */
int qo_null_encrypt(const uint8_t* ad, size_t ad_len, const uint8_t* pt, size_t pt_len,
                    uint8_t* out, size_t cap, size_t* out_len);
/* 1 on success (output = plaintext), 0 on a short input, small cap or bad tag. */
int qo_null_decrypt(const uint8_t* ad, size_t ad_len, const uint8_t* ct, size_t ct_len,
                    uint8_t* out, size_t cap, size_t* out_len);

/* Batches over a CSR layout: packet p's associated data (the packet header)
 * is ad_len[p] bytes at bytes + ad_off[p], its payload in_len[p] bytes at
 * bytes + in_off[p]; its output goes to out + out_off[p] (in_len + 12 bytes
 * for encrypt, in_len - 12 for decrypt).  Decrypt writes ok[p] = 1/0. */
void qo_null_encrypt_batch(const uint8_t* bytes, const uint64_t* ad_off, const uint16_t* ad_len,
                           const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                           uint8_t* out, const uint64_t* out_off);
void qo_null_decrypt_batch(const uint8_t* bytes, const uint64_t* ad_off, const uint16_t* ad_len,
                           const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                           uint8_t* out, const uint64_t* out_off, uint8_t* ok);
/* multi-threaded encrypt batch (cpu_baseline) */
void qo_null_encrypt_batch_mt(const uint8_t* bytes, const uint64_t* ad_off,
                              const uint16_t* ad_len, const uint64_t* in_off,
                              const uint16_t* in_len, uint64_t n, uint8_t* out,
                              const uint64_t* out_off, int threads);

#ifdef __cplusplus
}
#endif
#endif /* QPP_ORACLE_H_ */
