/* qpp_oracle.c — see qpp_oracle.h (test infrastructure only). */
#include "qpp_oracle.h"

#include <pthread.h>
#include <string.h>

typedef unsigned __int128 u128;

/* quic_utils.cc:31-50 (IncrementalHashFast): h = (h ^ octet) * kPrime. */
static u128 fnv_update(u128 h, const uint8_t* d, size_t n) {
  const u128 prime = ((u128)16777216 << 64) + 315; /* 2^88 + 315 */
  for (size_t i = 0; i < n; ++i) h = (h ^ d[i]) * prime;
  return h;
}

/* quic_utils.cc:110-125 */
void qo_fnv1a128_two(const uint8_t* d1, size_t n1, const uint8_t* d2, size_t n2, uint64_t* lo,
                     uint64_t* hi) {
  const u128 offset = ((u128)UINT64_C(7809847782465536322) << 64) | UINT64_C(7113472399480571277);
  u128 h = fnv_update(offset, d1, n1);
  if (d2 != NULL) h = fnv_update(h, d2, n2);
  *lo = (uint64_t)h;
  *hi = (uint64_t)(h >> 64);
}

/* null_encrypter.cc:28-47 + SerializeUint128Short quic_utils.cc:175-181 */
int qo_null_encrypt(const uint8_t* ad, size_t ad_len, const uint8_t* pt, size_t pt_len,
                    uint8_t* out, size_t cap, size_t* out_len) {
  const size_t len = pt_len + QO_NULL_TAG_SIZE;
  if (cap < len) return 0;
  uint64_t lo, hi;
  qo_fnv1a128_two(ad, ad_len, pt, pt_len, &lo, &hi);
  memmove(out + QO_NULL_TAG_SIZE, pt, pt_len);
  memcpy(out, &lo, 8);         /* little-endian host, as the reference assumes */
  memcpy(out + 8, &hi, 4);
  *out_len = len;
  return 1;
}

/* null_decrypter.cc:38-64, ReadHash :84-95, ComputeHash :97-106 */
int qo_null_decrypt(const uint8_t* ad, size_t ad_len, const uint8_t* ct, size_t ct_len,
                    uint8_t* out, size_t cap, size_t* out_len) {
  if (ct_len < QO_NULL_TAG_SIZE) return 0;
  uint64_t tlo;
  uint32_t thi;
  memcpy(&tlo, ct, 8);
  memcpy(&thi, ct + 8, 4);
  const uint8_t* pt = ct + QO_NULL_TAG_SIZE;
  const size_t pt_len = ct_len - QO_NULL_TAG_SIZE;
  if (pt_len > cap) return 0;
  uint64_t lo, hi;
  qo_fnv1a128_two(ad, ad_len, pt, pt_len, &lo, &hi);
  if (lo != tlo || (uint32_t)hi != thi) return 0;
  memmove(out, pt, pt_len);
  *out_len = pt_len;
  return 1;
}

void qo_null_encrypt_batch(const uint8_t* bytes, const uint64_t* ad_off, const uint16_t* ad_len,
                           const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                           uint8_t* out, const uint64_t* out_off) {
  for (uint64_t p = 0; p < n; ++p) {
    size_t ol;
    qo_null_encrypt(bytes + ad_off[p], ad_len[p], bytes + in_off[p], in_len[p], out + out_off[p],
                    (size_t)in_len[p] + QO_NULL_TAG_SIZE, &ol);
  }
}

void qo_null_decrypt_batch(const uint8_t* bytes, const uint64_t* ad_off, const uint16_t* ad_len,
                           const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                           uint8_t* out, const uint64_t* out_off, uint8_t* ok) {
  for (uint64_t p = 0; p < n; ++p) {
    size_t ol;
    const size_t cap = in_len[p] >= QO_NULL_TAG_SIZE ? in_len[p] - QO_NULL_TAG_SIZE : 0;
    ok[p] = (uint8_t)qo_null_decrypt(bytes + ad_off[p], ad_len[p], bytes + in_off[p], in_len[p],
                                     out + out_off[p], cap, &ol);
  }
}

struct enc_job {
  const uint8_t* bytes;
  const uint64_t *ad_off, *in_off, *out_off;
  const uint16_t *ad_len, *in_len;
  uint8_t* out;
  uint64_t p0, p1;
};

static void* enc_worker(void* arg) {
  struct enc_job* j = (struct enc_job*)arg;
  qo_null_encrypt_batch(j->bytes, j->ad_off + j->p0, j->ad_len + j->p0, j->in_off + j->p0,
                        j->in_len + j->p0, j->p1 - j->p0, j->out, j->out_off + j->p0);
  return NULL;
}

void qo_null_encrypt_batch_mt(const uint8_t* bytes, const uint64_t* ad_off,
                              const uint16_t* ad_len, const uint64_t* in_off,
                              const uint16_t* in_len, uint64_t n, uint8_t* out,
                              const uint64_t* out_off, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  struct enc_job jobs[256];
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (struct enc_job){bytes, ad_off, in_off, out_off, ad_len, in_len, out,
                               n * (uint64_t)t / (uint64_t)threads,
                               n * (uint64_t)(t + 1) / (uint64_t)threads};
    pthread_create(&th[t], NULL, enc_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}
