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

/* ======================================================================== */
/* AES-128 (FIPS-197 §5.1-5.2), byte-oriented                                */
/* ======================================================================== */
static uint8_t g_sbox[256];
static int g_sbox_ready = 0;

static uint8_t gf_mul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
    b >>= 1;
  }
  return r;
}

/* S-box from its definition: multiplicative inverse in GF(2^8) + affine map */
static void sbox_init(void) {
  if (g_sbox_ready) return;
  for (int x = 0; x < 256; ++x) {
    uint8_t inv = 0;
    for (int y = 1; y < 256 && x; ++y)
      if (gf_mul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
    uint8_t s = inv;
    for (int i = 1; i < 5; ++i) s ^= (uint8_t)((inv << i) | (inv >> (8 - i)));
    g_sbox[x] = (uint8_t)(s ^ 0x63);
  }
  g_sbox_ready = 1;
}

void qo_aes128_expand(uint32_t rk[44], const uint8_t key[16]) {
  sbox_init();
  /* words big-endian as FIPS-197 (w[i] = key[4i..4i+3]) */
  for (int i = 0; i < 4; ++i)
    rk[i] = (uint32_t)key[4 * i] << 24 | (uint32_t)key[4 * i + 1] << 16 |
            (uint32_t)key[4 * i + 2] << 8 | key[4 * i + 3];
  uint8_t rcon = 1;
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk[i - 1];
    if (i % 4 == 0) {
      t = (t << 8) | (t >> 24); /* RotWord */
      t = (uint32_t)g_sbox[t >> 24] << 24 | (uint32_t)g_sbox[(t >> 16) & 0xff] << 16 |
          (uint32_t)g_sbox[(t >> 8) & 0xff] << 8 | g_sbox[t & 0xff];
      t ^= (uint32_t)rcon << 24;
      rcon = gf_mul(rcon, 2);
    }
    rk[i] = rk[i - 4] ^ t;
  }
}

void qo_aes128_encrypt(uint8_t out[16], const uint8_t in[16], const uint32_t rk[44]) {
  sbox_init();
  uint8_t s[16];
  for (int i = 0; i < 16; ++i) s[i] = in[i] ^ (uint8_t)(rk[i / 4] >> (24 - 8 * (i % 4)));
  for (int r = 1; r <= 10; ++r) {
    uint8_t t[16];
    for (int i = 0; i < 16; ++i) t[i] = g_sbox[s[i]];             /* SubBytes */
    for (int c = 0; c < 4; ++c)                                       /* ShiftRows */
      for (int rr = 0; rr < 4; ++rr) s[4 * c + rr] = t[4 * ((c + rr) % 4) + rr];
    if (r != 10) {                                                    /* MixColumns */
      for (int c = 0; c < 4; ++c) {
        const uint8_t a0 = s[4 * c], a1 = s[4 * c + 1], a2 = s[4 * c + 2], a3 = s[4 * c + 3];
        s[4 * c] = gf_mul(a0, 2) ^ gf_mul(a1, 3) ^ a2 ^ a3;
        s[4 * c + 1] = a0 ^ gf_mul(a1, 2) ^ gf_mul(a2, 3) ^ a3;
        s[4 * c + 2] = a0 ^ a1 ^ gf_mul(a2, 2) ^ gf_mul(a3, 3);
        s[4 * c + 3] = gf_mul(a0, 3) ^ a1 ^ a2 ^ gf_mul(a3, 2);
      }
    }
    for (int i = 0; i < 16; ++i) s[i] ^= (uint8_t)(rk[4 * r + i / 4] >> (24 - 8 * (i % 4)));
  }
  memcpy(out, s, 16);
}

/* ======================================================================== */
/* GCM (SP 800-38D §6.3-7): bitwise GF(2^128) multiply, Algorithm 1          */
/* ======================================================================== */
static void gf128_mul(uint8_t x[16], const uint8_t h[16]) {
  uint8_t z[16] = {0}, v[16];
  memcpy(v, h, 16);
  for (int i = 0; i < 128; ++i) {
    if (x[i / 8] & (0x80 >> (i % 8)))
      for (int j = 0; j < 16; ++j) z[j] ^= v[j];
    const int lsb = v[15] & 1;
    for (int j = 15; j > 0; --j) v[j] = (uint8_t)((v[j] >> 1) | (v[j - 1] << 7));
    v[0] >>= 1;
    if (lsb) v[0] ^= 0xe1;
  }
  memcpy(x, z, 16);
}

static void ghash_update(uint8_t y[16], const uint8_t h[16], const uint8_t* d, size_t len) {
  for (; len > 0;) {
    const size_t n = len < 16 ? len : 16;
    for (size_t i = 0; i < n; ++i) y[i] ^= d[i]; /* zero padded block */
    gf128_mul(y, h);
    d += n; len -= n;
  }
}

static void inc32(uint8_t ctr[16]) {
  for (int i = 15; i >= 12; --i)
    if (++ctr[i]) break;
}

static void gcm_core(uint8_t tag[16], uint8_t* out, const uint8_t key[16], const uint8_t* iv,
                     size_t iv_len, const uint8_t* in, size_t in_len, const uint8_t* ad,
                     size_t ad_len, int decrypt) {
  uint32_t rk[44];
  qo_aes128_expand(rk, key);
  uint8_t h[16] = {0}, j0[16] = {0}, y[16] = {0};
  qo_aes128_encrypt(h, h, rk);
  if (iv_len == 12) {
    memcpy(j0, iv, 12);
    j0[15] = 1;
  } else {
    ghash_update(j0, h, iv, iv_len);
    uint8_t lb[16] = {0};
    st64(lb + 8, 0);
    const uint64_t bits = (uint64_t)iv_len * 8;
    for (int i = 0; i < 8; ++i) lb[15 - i] = (uint8_t)(bits >> (8 * i));
    ghash_update(j0, h, lb, 16);
  }
  ghash_update(y, h, ad, ad_len);
  /* GCTR from inc32(J0); MAC over the ciphertext */
  uint8_t ctr[16], ks[16];
  memcpy(ctr, j0, 16);
  const uint8_t* src = in;
  for (size_t off = 0; off < in_len; off += 16) {
    inc32(ctr);
    qo_aes128_encrypt(ks, ctr, rk);
    const size_t n = in_len - off < 16 ? in_len - off : 16;
    if (out)
      for (size_t i = 0; i < n; ++i) out[off + i] = src[off + i] ^ ks[i];
  }
  ghash_update(y, h, decrypt ? in : out, in_len);
  uint8_t lens[16];
  const uint64_t ab = (uint64_t)ad_len * 8, cb = (uint64_t)in_len * 8;
  for (int i = 0; i < 8; ++i) {
    lens[7 - i] = (uint8_t)(ab >> (8 * i));
    lens[15 - i] = (uint8_t)(cb >> (8 * i));
  }
  ghash_update(y, h, lens, 16);
  qo_aes128_encrypt(ks, j0, rk);
  for (int i = 0; i < 16; ++i) tag[i] = y[i] ^ ks[i];
}

int qo_aes128gcm_seal(uint8_t* out, const uint8_t key[16], const uint8_t* iv, size_t iv_len,
                      const uint8_t* in, size_t in_len, const uint8_t* ad, size_t ad_len,
                      size_t tag_len) {
  uint8_t tag[16];
  gcm_core(tag, out, key, iv, iv_len, in, in_len, ad, ad_len, 0);
  memcpy(out + in_len, tag, tag_len);
  return 1;
}

int qo_aes128gcm_open(uint8_t* out, const uint8_t key[16], const uint8_t* iv, size_t iv_len,
                      const uint8_t* in, size_t in_len, const uint8_t* ad, size_t ad_len,
                      size_t tag_len) {
  if (in_len < tag_len) return 0;
  const size_t pt_len = in_len - tag_len;
  uint8_t tag[16];
  gcm_core(tag, NULL, key, iv, iv_len, in, pt_len, ad, ad_len, 1); /* MAC only */
  uint8_t diff = 0;
  for (size_t i = 0; i < tag_len; ++i) diff |= (uint8_t)(tag[i] ^ in[pt_len + i]);
  if (diff) return 0;
  gcm_core(tag, out, key, iv, iv_len, in, pt_len, ad, ad_len, 1);
  return 1;
}

struct gcm_job {
  const uint8_t *keys, *prefixes, *path_id, *bytes;
  const uint32_t* key_idx;
  const uint64_t *packet_number, *ad_off, *in_off, *out_off;
  const uint16_t *ad_len, *in_len;
  uint8_t* out;
  uint8_t* ok;
  uint64_t p0, p1;
};

static void* gcm_worker(void* arg) {
  const struct gcm_job* j = (const struct gcm_job*)arg;
  for (uint64_t p = j->p0; p < j->p1; ++p) {
    const uint32_t k = j->key_idx[p];
    uint8_t nonce[12];
    quic_nonce(nonce, j->prefixes + 4ull * k, j->path_id ? j->path_id[p] : 0,
               j->packet_number[p]);
    if (j->ok)
      j->ok[p] = (uint8_t)qo_aes128gcm_open(j->out + j->out_off[p], j->keys + 16ull * k, nonce,
                                            12, j->bytes + j->in_off[p], j->in_len[p],
                                            j->bytes + j->ad_off[p], j->ad_len[p],
                                            QO_QUIC_AEAD_TAG);
    else
      qo_aes128gcm_seal(j->out + j->out_off[p], j->keys + 16ull * k, nonce, 12,
                        j->bytes + j->in_off[p], j->in_len[p], j->bytes + j->ad_off[p],
                        j->ad_len[p], QO_QUIC_AEAD_TAG);
  }
  return NULL;
}

static void gcm_batch(const uint8_t* keys, const uint8_t* prefixes, const uint32_t* key_idx,
                      const uint64_t* packet_number, const uint8_t* path_id,
                      const uint8_t* bytes, const uint64_t* ad_off, const uint16_t* ad_len,
                      const uint64_t* in_off, const uint16_t* in_len, uint64_t n, uint8_t* out,
                      const uint64_t* out_off, uint8_t* ok, int threads) {
  sbox_init();
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  struct gcm_job jobs[256];
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (struct gcm_job){keys, prefixes, path_id, bytes, key_idx, packet_number, ad_off,
                               in_off, out_off, ad_len, in_len, out, ok,
                               n * (uint64_t)t / (uint64_t)threads,
                               n * (uint64_t)(t + 1) / (uint64_t)threads};
    if (threads == 1) gcm_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, gcm_worker, &jobs[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}

void qo_quic_aes128gcm_encrypt_batch(const uint8_t* keys, const uint8_t* prefixes,
                                     const uint32_t* key_idx, const uint64_t* packet_number,
                                     const uint8_t* path_id, const uint8_t* bytes,
                                     const uint64_t* ad_off, const uint16_t* ad_len,
                                     const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                                     uint8_t* out, const uint64_t* out_off, int threads) {
  gcm_batch(keys, prefixes, key_idx, packet_number, path_id, bytes, ad_off, ad_len, in_off,
            in_len, n, out, out_off, NULL, threads);
}

void qo_quic_aes128gcm_decrypt_batch(const uint8_t* keys, const uint8_t* prefixes,
                                     const uint32_t* key_idx, const uint64_t* packet_number,
                                     const uint8_t* path_id, const uint8_t* bytes,
                                     const uint64_t* ad_off, const uint16_t* ad_len,
                                     const uint64_t* in_off, const uint16_t* in_len, uint64_t n,
                                     uint8_t* out, const uint64_t* out_off, uint8_t* ok) {
  gcm_batch(keys, prefixes, key_idx, packet_number, path_id, bytes, ad_off, ad_len, in_off,
            in_len, n, out, out_off, ok, 1);
}
