/* qaead_oracle.c — see qaead_oracle.h (test infrastructure only). */
#include "qaead_oracle.h"

#include <pthread.h>
#include <string.h>

static uint32_t ld32(const uint8_t* p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}
static void st32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static uint64_t ld64(const uint8_t* p) { return (uint64_t)ld32(p) | (uint64_t)ld32(p + 4) << 32; }
static void st64(uint8_t* p, uint64_t v) { st32(p, (uint32_t)v); st32(p + 4, (uint32_t)(v >> 32)); }

#define ROTL(v, n) (((v) << (n)) | ((v) >> (32 - (n))))
#define QR(a, b, c, d)                                   \
  a += b; d ^= a; d = ROTL(d, 16);                       \
  c += d; b ^= c; b = ROTL(b, 12);                       \
  a += b; d ^= a; d = ROTL(d, 8);                        \
  c += d; b ^= c; b = ROTL(b, 7);

/* RFC 7539 §2.3 block function (chacha.c:80-116) */
static void chacha_block(uint8_t out[64], const uint32_t in[16]) {
  uint32_t x[16];
  memcpy(x, in, sizeof(x));
  for (int i = 0; i < 10; ++i) {
    QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13])
    QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
    QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12])
    QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
  }
  for (int i = 0; i < 16; ++i) st32(out + 4 * i, x[i] + in[i]);
}

/* chacha.c:118-170 */
void qo_chacha20(uint8_t* out, const uint8_t* in, size_t len, const uint8_t key[32],
                 const uint8_t nonce[12], uint32_t counter) {
  static const uint8_t sigma[16] = "expand 32-byte k";
  uint32_t st[16];
  for (int i = 0; i < 4; ++i) st[i] = ld32(sigma + 4 * i);
  for (int i = 0; i < 8; ++i) st[4 + i] = ld32(key + 4 * i);
  st[12] = counter;
  for (int i = 0; i < 3; ++i) st[13 + i] = ld32(nonce + 4 * i);
  uint8_t ks[64];
  while (len > 0) {
    chacha_block(ks, st);
    const size_t n = len < 64 ? len : 64;
    for (size_t i = 0; i < n; ++i) out[i] = in[i] ^ ks[i];
    out += n; in += n; len -= n;
    st[12]++;
  }
}

/* Poly1305 (RFC 7539 §2.5), 44/44/42-bit limbs with 128-bit products. */
typedef unsigned __int128 u128;
typedef struct { uint64_t r0, r1, r2, s1, s2, h0, h1, h2, pad0, pad1; } poly_state;

static void poly_init(poly_state* p, const uint8_t key[32]) {
  const uint64_t t0 = ld64(key), t1 = ld64(key + 8);
  p->r0 = t0 & 0xffc0fffffffull;
  p->r1 = ((t0 >> 44) | (t1 << 20)) & 0xfffffc0ffffull;
  p->r2 = (t1 >> 24) & 0x00ffffffc0full;
  p->s1 = p->r1 * (5 << 2);
  p->s2 = p->r2 * (5 << 2);
  p->h0 = p->h1 = p->h2 = 0;
  p->pad0 = ld64(key + 16);
  p->pad1 = ld64(key + 24);
}

/* one 16-byte block with the 2^128 bit (hibit = 1<<40 in limb 2) */
static void poly_block(poly_state* p, const uint8_t m[16], uint64_t hibit) {
  const uint64_t t0 = ld64(m), t1 = ld64(m + 8);
  uint64_t h0 = p->h0 + (t0 & 0xfffffffffffull);
  uint64_t h1 = p->h1 + (((t0 >> 44) | (t1 << 20)) & 0xfffffffffffull);
  uint64_t h2 = p->h2 + (((t1 >> 24)) & 0x3ffffffffffull) + hibit;
  const u128 d0 = (u128)h0 * p->r0 + (u128)h1 * p->s2 + (u128)h2 * p->s1;
  u128 d1 = (u128)h0 * p->r1 + (u128)h1 * p->r0 + (u128)h2 * p->s2;
  u128 d2 = (u128)h0 * p->r2 + (u128)h1 * p->r1 + (u128)h2 * p->r0;
  uint64_t c = (uint64_t)(d0 >> 44);
  h0 = (uint64_t)d0 & 0xfffffffffffull;
  d1 += c;
  c = (uint64_t)(d1 >> 44);
  h1 = (uint64_t)d1 & 0xfffffffffffull;
  d2 += c;
  c = (uint64_t)(d2 >> 42);
  h2 = (uint64_t)d2 & 0x3ffffffffffull;
  h0 += c * 5;
  c = h0 >> 44;
  h0 &= 0xfffffffffffull;
  h1 += c;
  p->h0 = h0; p->h1 = h1; p->h2 = h2;
}

static void poly_finish(poly_state* p, uint8_t tag[16]) {
  uint64_t h0 = p->h0, h1 = p->h1, h2 = p->h2, c;
  c = h1 >> 44; h1 &= 0xfffffffffffull;
  h2 += c; c = h2 >> 42; h2 &= 0x3ffffffffffull;
  h0 += c * 5; c = h0 >> 44; h0 &= 0xfffffffffffull;
  h1 += c; c = h1 >> 44; h1 &= 0xfffffffffffull;
  h2 += c; c = h2 >> 42; h2 &= 0x3ffffffffffull;
  h0 += c * 5; c = h0 >> 44; h0 &= 0xfffffffffffull;
  h1 += c;
  /* h - p */
  uint64_t g0 = h0 + 5; c = g0 >> 44; g0 &= 0xfffffffffffull;
  uint64_t g1 = h1 + c; c = g1 >> 44; g1 &= 0xfffffffffffull;
  uint64_t g2 = h2 + c - (1ull << 42);
  c = (g2 >> 63) - 1; /* all ones if h >= p */
  g0 &= c; g1 &= c; g2 &= c;
  c = ~c;
  h0 = (h0 & c) | g0; h1 = (h1 & c) | g1; h2 = (h2 & c) | g2;
  /* h + pad mod 2^128 */
  const uint64_t lo = h0 | (h1 << 44), hi = (h1 >> 20) | (h2 << 24);
  u128 t = ((u128)hi << 64 | lo) + ((u128)p->pad1 << 64 | p->pad0);
  st64(tag, (uint64_t)t);
  st64(tag + 8, (uint64_t)(t >> 64));
}

static void poly_update(poly_state* p, const uint8_t* m, size_t len) {
  for (; len >= 16; m += 16, len -= 16) poly_block(p, m, 1ull << 40);
  if (len) { /* partial final block: m || 0x01 || zeros, no hibit */
    uint8_t b[16] = {0};
    memcpy(b, m, len);
    b[len] = 1;
    poly_block(p, b, 0);
  }
}

/* poly1305_update_padded_16 (e_chacha20poly1305.c:177-184): data then zeros
 * up to a multiple of 16 — every block a full block (2^128 bit set). */
static void poly_update_padded16(poly_state* p, const uint8_t* m, size_t len) {
  for (; len >= 16; m += 16, len -= 16) poly_block(p, m, 1ull << 40);
  if (len) {
    uint8_t b[16] = {0};
    memcpy(b, m, len);
    poly_block(p, b, 1ull << 40);
  }
}

void qo_poly1305(uint8_t tag[16], const uint8_t* msg, size_t len, const uint8_t key[32]) {
  poly_state p;
  poly_init(&p, key);
  poly_update(&p, msg, len);
  poly_finish(&p, tag);
}

/* e_chacha20poly1305.c:71-105, 186-200: MAC over AD|pad16|CT|pad16|len|len */
static void aead_tag(uint8_t tag[16], const uint8_t key[32], const uint8_t nonce[12],
                     const uint8_t* ad, size_t ad_len, const uint8_t* ct, size_t ct_len) {
  uint8_t pk[32] = {0};
  qo_chacha20(pk, pk, 32, key, nonce, 0);
  poly_state p;
  poly_init(&p, pk);
  poly_update_padded16(&p, ad, ad_len);
  poly_update_padded16(&p, ct, ct_len);
  uint8_t lens[16];
  st64(lens, ad_len);
  st64(lens + 8, ct_len);
  poly_update(&p, lens, 16);
  poly_finish(&p, tag);
}

int qo_c20p1305_seal(uint8_t* out, const uint8_t key[32], const uint8_t nonce[12],
                     const uint8_t* in, size_t in_len, const uint8_t* ad, size_t ad_len,
                     size_t tag_len) {
  qo_chacha20(out, in, in_len, key, nonce, 1);
  uint8_t tag[16];
  aead_tag(tag, key, nonce, ad, ad_len, out, in_len);
  memcpy(out + in_len, tag, tag_len);
  return 1;
}

int qo_c20p1305_open(uint8_t* out, const uint8_t key[32], const uint8_t nonce[12],
                     const uint8_t* in, size_t in_len, const uint8_t* ad, size_t ad_len,
                     size_t tag_len) {
  if (in_len < tag_len) return 0;
  const size_t pt_len = in_len - tag_len;
  uint8_t tag[16];
  aead_tag(tag, key, nonce, ad, ad_len, in, pt_len);
  uint8_t diff = 0;
  for (size_t i = 0; i < tag_len; ++i) diff |= (uint8_t)(tag[i] ^ in[pt_len + i]);
  if (diff) return 0;
  qo_chacha20(out, in, pt_len, key, nonce, 1);
  return 1;
}

/* aead_base_encrypter.cc:120-126 */
static void quic_nonce(uint8_t nonce[12], const uint8_t prefix[4], uint8_t path_id,
                       uint64_t packet_number) {
  memcpy(nonce, prefix, 4);
  st64(nonce + 4, ((uint64_t)path_id << 56) | packet_number);
}

int qo_quic_c20p1305_encrypt(uint8_t* out, const uint8_t key[32], const uint8_t prefix[4],
                             uint8_t path_id, uint64_t packet_number, const uint8_t* ad,
                             size_t ad_len, const uint8_t* pt, size_t pt_len) {
  uint8_t nonce[12];
  quic_nonce(nonce, prefix, path_id, packet_number);
  return qo_c20p1305_seal(out, key, nonce, pt, pt_len, ad, ad_len, QO_QUIC_AEAD_TAG);
}

int qo_quic_c20p1305_decrypt(uint8_t* out, const uint8_t key[32], const uint8_t prefix[4],
                             uint8_t path_id, uint64_t packet_number, const uint8_t* ad,
                             size_t ad_len, const uint8_t* ct, size_t ct_len) {
  uint8_t nonce[12];
  quic_nonce(nonce, prefix, path_id, packet_number);
  return qo_c20p1305_open(out, key, nonce, ct, ct_len, ad, ad_len, QO_QUIC_AEAD_TAG);
}

struct c20_job {
  const uint8_t *keys, *prefixes, *path_id, *bytes;
  const uint32_t* key_idx;
  const uint64_t *packet_number, *ad_off, *in_off, *out_off;
  const uint16_t *ad_len, *in_len;
  uint8_t* out;
  uint64_t p0, p1;
};

static void* c20_worker(void* arg) {
  const struct c20_job* j = (const struct c20_job*)arg;
  for (uint64_t p = j->p0; p < j->p1; ++p) {
    const uint32_t k = j->key_idx[p];
    qo_quic_c20p1305_encrypt(j->out + j->out_off[p], j->keys + 32ull * k,
                             j->prefixes + 4ull * k, j->path_id ? j->path_id[p] : 0,
                             j->packet_number[p], j->bytes + j->ad_off[p], j->ad_len[p],
                             j->bytes + j->in_off[p], j->in_len[p]);
  }
  return NULL;
}

void qo_quic_c20p1305_encrypt_batch(const uint8_t* keys, const uint8_t* prefixes,
                                    const uint32_t* key_idx, const uint64_t* packet_number,
                                    const uint8_t* path_id, const uint8_t* bytes,
                                    const uint64_t* ad_off, const uint16_t* ad_len,
                                    const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                                    uint8_t* out, const uint64_t* out_off, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  struct c20_job jobs[256];
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (struct c20_job){keys, prefixes, path_id, bytes, key_idx, packet_number, ad_off,
                               in_off, out_off, ad_len, in_len, out,
                               n * (uint64_t)t / (uint64_t)threads,
                               n * (uint64_t)(t + 1) / (uint64_t)threads};
    if (threads == 1) c20_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, c20_worker, &jobs[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}

void qo_quic_c20p1305_decrypt_batch(const uint8_t* keys, const uint8_t* prefixes,
                                    const uint32_t* key_idx, const uint64_t* packet_number,
                                    const uint8_t* path_id, const uint8_t* bytes,
                                    const uint64_t* ad_off, const uint16_t* ad_len,
                                    const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                                    uint8_t* out, const uint64_t* out_off, uint8_t* ok) {
  for (uint64_t p = 0; p < n; ++p) {
    const uint32_t k = key_idx[p];
    ok[p] = (uint8_t)qo_quic_c20p1305_decrypt(out + out_off[p], keys + 32ull * k,
                                              prefixes + 4ull * k, path_id ? path_id[p] : 0,
                                              packet_number[p], bytes + ad_off[p], ad_len[p],
                                              bytes + in_off[p], in_len[p]);
  }
}
