/* fnv_r3_check.c — host check of fnv_step3 (libquic_amd/csrc/qpp_kernels.hip):
 * three FNV-1a-128 byte steps per multiply, against the byte-serial recurrence
 * of the reference (quic_utils.cc:31-54: h = (h ^ octet) * (2^88 + 315) mod 2^128).
 * build + run: gcc -O2 -o /tmp/fnv_r3_check tools/tune/fnv_r3_check.c && /tmp/fnv_r3_check */
#include <stdint.h>
#include <stdio.h>

typedef unsigned __int128 u128;
typedef struct {
  uint32_t x0, x1, x2, x3;
} Fnv128;

static u128 to128(Fnv128 h) {
  return ((u128)h.x3 << 96) | ((u128)h.x2 << 64) | ((u128)h.x1 << 32) | h.x0;
}

static Fnv128 from128(u128 v) {
  Fnv128 h = {(uint32_t)v, (uint32_t)(v >> 32), (uint32_t)(v >> 64), (uint32_t)(v >> 96)};
  return h;
}

/* the device function, in C */
static void fnv_step3(Fnv128* h, uint32_t* y, uint32_t b0, uint32_t b1, uint32_t b2) {
  const uint32_t kC3 = 31255875u, kC3h = 297675u;
  const uint32_t t0 = *y ^ b0;
  const uint32_t y1 = (t0 * 59u) & 0xFFu;
  const uint32_t t1 = y1 ^ b1;
  const uint32_t y2 = (t1 * 59u) & 0xFFu;
  const uint32_t t2 = y2 ^ b2;
  *y = (t2 * 59u) & 0xFFu;
  const int32_t d1 = (int32_t)t1 - (int32_t)y1;
  const int32_t d2 = (int32_t)t2 - (int32_t)y2;
  const uint64_t slo = (uint64_t)(int64_t)(d1 * 99225 + d2 * 315);
  const uint64_t shi = (uint64_t)(int64_t)(d1 * 630 + d2);
  const uint32_t x0 = h->x0 ^ b0;
  const uint64_t u =
      (uint64_t)x0 * kC3h + shi + ((uint64_t)((h->x1 & 0xFFu) * (kC3h & 0xFFu)) << 32);
  const uint64_t q0 = (uint64_t)x0 * kC3 + slo;
  const uint64_t q1 = (uint64_t)h->x1 * kC3 + (q0 >> 32);
  const uint64_t q2 = (uint64_t)h->x2 * kC3 + (q1 >> 32) + (u << 24);
  h->x0 = (uint32_t)q0;
  h->x1 = (uint32_t)q1;
  h->x2 = (uint32_t)q2;
  h->x3 = h->x3 * kC3 + (uint32_t)(q2 >> 32);
}

static uint64_t rs = 0x243F6A8885A308D3ull;
static uint64_t rnd(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return rs;
}

int main(void) {
  const u128 prime = ((u128)16777216 << 64) + 315;
  long bad = 0, n = 0;
  for (int t = 0; t < 4000000; ++t) {
    Fnv128 h = {(uint32_t)rnd(), (uint32_t)rnd(), (uint32_t)rnd(), (uint32_t)rnd()};
    if (t % 5 == 0) h.x0 = (h.x0 & 0xFFFFFF00u) | (uint32_t)(t & 0xFF);
    if (t % 7 == 0) h.x0 = (uint32_t)(t & 3); /* tiny low limb: the carry edge */
    uint32_t b[3] = {(uint32_t)rnd() & 255u, (uint32_t)rnd() & 255u, (uint32_t)rnd() & 255u};
    if (t % 3 == 0) b[1] = b[2] = 0;
    u128 want = to128(h);
    for (int i = 0; i < 3; ++i) want = (want ^ b[i]) * prime;
    uint32_t y = h.x0 & 0xFFu;
    fnv_step3(&h, &y, b[0], b[1], b[2]);
    bad += to128(h) != want || y != (h.x0 & 0xFFu);
    ++n;
  }
  /* 16-byte chunks as the kernel hashes them (5 x fnv_step3 + 1 serial byte),
   * from the FNV offset basis, over a 3.2 MB stream */
  u128 w = ((u128)7809847782465536322ull << 64) | 7113472399480571277ull;
  Fnv128 h = from128(w);
  for (int c = 0; c < 200000; ++c) {
    uint8_t d[16];
    for (int i = 0; i < 16; ++i) d[i] = (uint8_t)rnd();
    for (int i = 0; i < 16; ++i) w = (w ^ d[i]) * prime;
    uint32_t y = h.x0 & 0xFFu;
    for (int i = 0; i < 15; i += 3) fnv_step3(&h, &y, d[i], d[i + 1], d[i + 2]);
    h = from128((to128(h) ^ d[15]) * prime);
  }
  bad += to128(h) != w;
  printf("fnv_step3 vs byte-serial FNV-1a-128: %ld mismatches over %ld random triples + a 3.2 MB stream\n",
         bad, n);
  return bad != 0;
}
