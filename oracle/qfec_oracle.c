/*
 * qfec_oracle.c — CPU restatement of the QUIC FEC group (XOR parity).
 *
 * TEST INFRASTRUCTURE ONLY — see qfec_oracle.h for the contract, the
 * reference citations and the "parity unpinned" status.  This file is the
 * checker for the HIP product path and the `cpu_baseline` leg of bench.py;
 * the product never links it.
 *
 * Algorithm (historical QuicFecGroup::UpdateParity /
 * QuicFecGroupInterface::XorBuffers; the source files are absent from the
 * snapshot, evidence Makefile:5332-5384):
 *   - the first packet initialises the parity (copy + zero fill),
 *   - each later packet is XORed into it, word-wise (uint64) then a byte tail,
 *   - parity_len = max payload length; shorter payloads are zero padded
 *     (QuicDataWriter::WritePadding fills 0x00, quic_data_writer.cc:136-143),
 *   - revive = parity XOR every received payload; its length is parity_len and
 *     the zero tail parses as one PADDING frame (quic_framer.cc:1224-1231).
 */
#define _POSIX_C_SOURCE 199309L
#include "qfec_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

uint64_t qo_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline uint64_t row_key(uint64_t seed, uint64_t g, uint32_t i) {
  return seed ^ ((g * 256u + i) << 32);
}

uint8_t qo_synth_byte(uint64_t seed, uint64_t g, uint32_t i, uint32_t j) {
  uint64_t w = qo_splitmix64(row_key(seed, g, i) ^ (uint64_t)(j >> 3));
  return (uint8_t)(w >> (8 * (j & 7)));
}

void qo_synth_row(uint64_t seed, uint64_t g, uint32_t i, uint32_t len, uint8_t* out) {
  uint64_t key = row_key(seed, g, i);
  uint32_t words = len / 8;
  for (uint32_t w = 0; w < words; ++w) {
    uint64_t v = qo_splitmix64(key ^ w);
    memcpy(out + 8 * (size_t)w, &v, 8); /* little-endian host */
  }
  if (len & 7) {
    uint64_t v = qo_splitmix64(key ^ words);
    memcpy(out + 8 * (size_t)words, &v, len & 7);
  }
}

void qo_synth_fixed(uint64_t seed, uint64_t g0, uint64_t n, uint32_t k, uint32_t L,
                    uint64_t row_stride, uint64_t group_stride, uint8_t* rows) {
  for (uint64_t g = 0; g < n; ++g)
    for (uint32_t i = 0; i < k; ++i)
      qo_synth_row(seed, g0 + g, i, L, rows + g * group_stride + i * row_stride);
}

uint32_t qo_ragged_k(uint64_t seed, uint64_t g, uint32_t kmin, uint32_t kmax) {
  return kmin + (uint32_t)(qo_splitmix64(seed ^ (0x6Bull << 56) ^ g) % (kmax - kmin + 1));
}

uint32_t qo_ragged_len(uint64_t seed, uint64_t g, uint32_t i, uint32_t lmin, uint32_t lmax) {
  return lmin +
         (uint32_t)(qo_splitmix64(seed ^ (0x4Cull << 56) ^ (g * 256u + i)) % (lmax - lmin + 1));
}

uint32_t qo_drop_index(uint64_t seed, uint64_t g, uint32_t k) {
  return (uint32_t)(qo_splitmix64(seed ^ (0x44ull << 56) ^ g) % k);
}

/* QuicFecGroupInterface::XorBuffers (historical): out ^= in, word then byte. */
void qo_xor_buffers(const uint8_t* in, size_t n, uint8_t* out) {
  size_t w = n / 8;
  for (size_t x = 0; x < w; ++x) {
    uint64_t a, b;
    memcpy(&a, in + 8 * x, 8);
    memcpy(&b, out + 8 * x, 8);
    b ^= a;
    memcpy(out + 8 * x, &b, 8);
  }
  for (size_t j = 8 * w; j < n; ++j) out[j] ^= in[j];
}

static int len_ok(uint32_t len) { return len >= 1 && len <= QO_MAX_PACKET_SIZE; }

int qo_group_encode(const uint8_t* const* payloads, const uint32_t* lens, uint32_t k,
                    uint8_t* parity) {
  if (k < 1 || k > QO_MAX_GROUP_PACKETS) return QO_INVALID_FEC_DATA;
  uint32_t plen = 0;
  for (uint32_t i = 0; i < k; ++i) {
    if (!len_ok(lens[i])) return QO_INVALID_FEC_DATA;
    if (lens[i] > plen) plen = lens[i];
  }
  /* UpdateParity: the first packet initialises the parity, zero filled. */
  memset(parity, 0, plen);
  memcpy(parity, payloads[0], lens[0]);
  for (uint32_t i = 1; i < k; ++i) qo_xor_buffers(payloads[i], lens[i], parity);
  return (int)plen;
}

int qo_group_recover(const uint8_t* const* payloads, const uint32_t* lens, uint32_t k,
                     const uint8_t* parity, uint32_t parity_len, uint32_t m, uint8_t* out) {
  if (k < 1 || k > QO_MAX_GROUP_PACKETS || m >= k || !len_ok(parity_len))
    return QO_INVALID_FEC_DATA;
  /* UpdateFec seeds the accumulator with the redundancy, then every received
   * data packet is folded in; Revive hands out the accumulator. */
  memcpy(out, parity, parity_len);
  for (uint32_t i = 0; i < k; ++i) {
    if (i == m) continue;
    if (!len_ok(lens[i]) || lens[i] > parity_len) return QO_INVALID_FEC_DATA;
    qo_xor_buffers(payloads[i], lens[i], out);
  }
  return (int)parity_len;
}

int qo_encode_fixed(const uint8_t* rows, uint32_t k, uint32_t L, uint64_t row_stride,
                    uint64_t group_stride, uint64_t n, uint8_t* parity, uint64_t parity_stride) {
  if (k < 1 || k > QO_MAX_GROUP_PACKETS || !len_ok(L)) return QO_INVALID_FEC_DATA;
  for (uint64_t g = 0; g < n; ++g) {
    const uint8_t* base = rows + g * group_stride;
    uint8_t* p = parity + g * parity_stride;
    memcpy(p, base, L);
    for (uint32_t i = 1; i < k; ++i) qo_xor_buffers(base + i * row_stride, L, p);
  }
  return QO_OK;
}

int qo_recover_fixed(const uint8_t* rows, const uint8_t* parity, const uint8_t* missing,
                     uint32_t k, uint32_t L, uint64_t row_stride, uint64_t group_stride,
                     uint64_t parity_stride, uint64_t n, uint8_t* out, uint64_t out_stride) {
  if (k < 1 || k > QO_MAX_GROUP_PACKETS || !len_ok(L)) return QO_INVALID_FEC_DATA;
  for (uint64_t g = 0; g < n; ++g)
    if (missing[g] >= k) return QO_INVALID_FEC_DATA;
  for (uint64_t g = 0; g < n; ++g) {
    const uint8_t* base = rows + g * group_stride;
    uint8_t* o = out + g * out_stride;
    memcpy(o, parity + g * parity_stride, L);
    for (uint32_t i = 0; i < k; ++i)
      if (i != missing[g]) qo_xor_buffers(base + i * row_stride, L, o);
  }
  return QO_OK;
}

int qo_encode_ragged(const uint8_t* bytes, const uint64_t* pkt_off, const uint16_t* pkt_len,
                     const uint32_t* grp_ptr, uint64_t n, uint8_t* parity,
                     const uint64_t* parity_off, uint16_t* parity_len) {
  for (uint64_t g = 0; g < n; ++g) {
    uint32_t p0 = grp_ptr[g], p1 = grp_ptr[g + 1];
    uint32_t k = p1 - p0;
    if (p1 < p0 || k < 1 || k > QO_MAX_GROUP_PACKETS) return QO_INVALID_FEC_DATA;
    uint32_t plen = 0;
    for (uint32_t i = p0; i < p1; ++i) {
      if (!len_ok(pkt_len[i])) return QO_INVALID_FEC_DATA;
      if (pkt_len[i] > plen) plen = pkt_len[i];
    }
    uint8_t* p = parity + parity_off[g];
    memset(p, 0, plen);
    for (uint32_t i = p0; i < p1; ++i) qo_xor_buffers(bytes + pkt_off[i], pkt_len[i], p);
    parity_len[g] = (uint16_t)plen;
  }
  return QO_OK;
}

int qo_recover_ragged(const uint8_t* bytes, const uint64_t* pkt_off, const uint16_t* pkt_len,
                      const uint32_t* grp_ptr, uint64_t n, const uint8_t* parity,
                      const uint64_t* parity_off, const uint16_t* parity_len,
                      const uint8_t* missing, uint8_t* out, const uint64_t* out_off) {
  for (uint64_t g = 0; g < n; ++g) {
    uint32_t p0 = grp_ptr[g], p1 = grp_ptr[g + 1];
    uint32_t k = p1 - p0;
    uint32_t plen = parity_len[g];
    if (p1 < p0 || k < 1 || k > QO_MAX_GROUP_PACKETS || missing[g] >= k || !len_ok(plen))
      return QO_INVALID_FEC_DATA;
    uint8_t* o = out + out_off[g];
    memcpy(o, parity + parity_off[g], plen);
    for (uint32_t i = 0; i < k; ++i) {
      if (i == missing[g]) continue;
      uint32_t len = pkt_len[p0 + i];
      if (!len_ok(len) || len > plen) return QO_INVALID_FEC_DATA;
      qo_xor_buffers(bytes + pkt_off[p0 + i], len, o);
    }
  }
  return QO_OK;
}

/* ---- multi-threaded CPU baseline: contiguous group split, std pthreads ---- */
typedef struct {
  const uint8_t* rows;
  const uint8_t* parity_in;
  const uint8_t* missing;
  uint32_t k, L;
  uint64_t g0, n;
  uint8_t* out;
  int rc;
} qo_job;

static void* qo_job_run(void* arg) {
  qo_job* j = (qo_job*)arg;
  uint64_t gs = (uint64_t)j->k * j->L;
  if (j->parity_in)
    j->rc = qo_recover_fixed(j->rows + j->g0 * gs, j->parity_in + j->g0 * j->L,
                             j->missing + j->g0, j->k, j->L, j->L, gs, j->L, j->n,
                             j->out + j->g0 * j->L, j->L);
  else
    j->rc = qo_encode_fixed(j->rows + j->g0 * gs, j->k, j->L, j->L, gs, j->n,
                            j->out + j->g0 * j->L, j->L);
  return NULL;
}

static int qo_run_mt(const uint8_t* rows, const uint8_t* parity_in, const uint8_t* missing,
                     uint32_t k, uint32_t L, uint64_t n, uint8_t* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  qo_job jobs[256];
  pthread_t tid[256];
  uint64_t per = (n + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; ++t) {
    uint64_t g0 = per * t;
    if (g0 >= n) break;
    uint64_t cnt = (g0 + per > n) ? n - g0 : per;
    qo_job tmp = {rows, parity_in, missing, k, L, g0, cnt, out, 0};
    jobs[t] = tmp;
    if (pthread_create(&tid[t], NULL, qo_job_run, &jobs[t]) != 0) return QO_INVALID_FEC_DATA;
    ++started;
  }
  int rc = QO_OK;
  for (int t = 0; t < started; ++t) {
    pthread_join(tid[t], NULL);
    if (jobs[t].rc != QO_OK) rc = jobs[t].rc;
  }
  return rc;
}

int qo_encode_fixed_mt(const uint8_t* rows, uint32_t k, uint32_t L, uint64_t n,
                       uint8_t* parity, int threads) {
  return qo_run_mt(rows, NULL, NULL, k, L, n, parity, threads);
}

int qo_recover_fixed_mt(const uint8_t* rows, const uint8_t* parity, const uint8_t* missing,
                        uint32_t k, uint32_t L, uint64_t n, uint8_t* out, int threads) {
  return qo_run_mt(rows, parity, missing, k, L, n, out, threads);
}

uint64_t qo_fnv1a64(const uint8_t* p, size_t n, uint64_t h) {
  if (h == 0) h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; ++i) {
    h ^= p[i];
    h *= 0x100000001b3ull;
  }
  return h;
}

/* ---- digests ------------------------------------------------------------ */
typedef struct {
  const uint8_t* base;
  uint64_t g0, n, stride;
  uint32_t L;
  const uint64_t* off;
  const uint16_t* len;
  uint64_t* hashes;
} qo_hash_job;

static void* qo_hash_run(void* arg) {
  qo_hash_job* j = (qo_hash_job*)arg;
  for (uint64_t g = j->g0; g < j->g0 + j->n; ++g) {
    const uint8_t* p = j->off ? j->base + j->off[g] : j->base + g * j->stride;
    size_t l = j->len ? j->len[g] : j->L;
    j->hashes[g] = qo_fnv1a64(p, l, 0);
  }
  return NULL;
}

uint64_t qo_group_digest(const uint8_t* base, uint64_t n, uint64_t stride, uint32_t L,
                         const uint64_t* off, const uint16_t* len, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  uint64_t* hashes = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
  qo_hash_job jobs[256];
  pthread_t tid[256];
  uint64_t per = (n + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; ++t) {
    uint64_t g0 = per * t;
    if (g0 >= n) break;
    qo_hash_job j = {base, g0, (g0 + per > n) ? n - g0 : per, stride, L, off, len, hashes};
    jobs[t] = j;
    pthread_create(&tid[t], NULL, qo_hash_run, &jobs[t]);
    ++started;
  }
  for (int t = 0; t < started; ++t) pthread_join(tid[t], NULL);
  uint64_t d = qo_fnv1a64((const uint8_t*)hashes, n * sizeof(uint64_t), 0);
  free(hashes);
  return d;
}

typedef struct {
  uint64_t seed, drop_seed, g0, n;
  uint32_t k, L;
  uint64_t* ph; /* per-group parity hash */
  uint64_t* rh; /* per-group revived-row hash */
} qo_dig_job;

static void* qo_dig_run(void* arg) {
  qo_dig_job* j = (qo_dig_job*)arg;
  uint8_t* rows = (uint8_t*)malloc((size_t)j->k * j->L);
  uint8_t* par = (uint8_t*)malloc(j->L);
  for (uint64_t g = 0; g < j->n; ++g) {
    uint64_t gg = j->g0 + g;
    qo_synth_fixed(j->seed, gg, 1, j->k, j->L, j->L, (uint64_t)j->k * j->L, rows);
    qo_encode_fixed(rows, j->k, j->L, j->L, (uint64_t)j->k * j->L, 1, par, j->L);
    j->ph[g] = qo_fnv1a64(par, j->L, 0);
    uint32_t m = qo_drop_index(j->drop_seed, gg, j->k);
    j->rh[g] = qo_fnv1a64(rows + (size_t)m * j->L, j->L, 0);
  }
  free(rows);
  free(par);
  return NULL;
}

void qo_fixed_digests(uint64_t seed, uint64_t drop_seed, uint64_t g0, uint64_t n, uint32_t k,
                      uint32_t L, int threads, uint64_t* parity_digest,
                      uint64_t* recovered_digest) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  uint64_t* ph = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
  uint64_t* rh = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
  qo_dig_job jobs[256];
  pthread_t tid[256];
  uint64_t per = (n + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; ++t) {
    uint64_t a = per * t;
    if (a >= n) break;
    qo_dig_job j = {seed, drop_seed, g0 + a, (a + per > n) ? n - a : per, k, L, ph + a, rh + a};
    jobs[t] = j;
    pthread_create(&tid[t], NULL, qo_dig_run, &jobs[t]);
    ++started;
  }
  for (int t = 0; t < started; ++t) pthread_join(tid[t], NULL);
  *parity_digest = qo_fnv1a64((const uint8_t*)ph, n * sizeof(uint64_t), 0);
  *recovered_digest = qo_fnv1a64((const uint8_t*)rh, n * sizeof(uint64_t), 0);
  free(ph);
  free(rh);
}

/* Ragged (configs[3]) digests without materialising the batch: group g has
 * k = qo_ragged_k(seed, g, kmin, kmax) packets of qo_ragged_len(seed, g, i,
 * lmin, lmax) bytes filled by qo_synth_row; its parity is parity_len = max len
 * bytes (zero padded XOR, as qo_encode_ragged), its revived row the lost
 * packet qo_drop_index(drop_seed, g, k) zero padded to parity_len (as
 * qo_recover_ragged). */
typedef struct {
  uint64_t seed, drop_seed, g0, n;
  uint32_t kmin, kmax, lmin, lmax;
  uint64_t *ph, *rh;
} qo_rdig_job;

static void* qo_rdig_run(void* arg) {
  qo_rdig_job* j = (qo_rdig_job*)arg;
  uint8_t row[QO_MAX_PACKET_SIZE], par[QO_MAX_PACKET_SIZE], lost[QO_MAX_PACKET_SIZE];
  for (uint64_t g = 0; g < j->n; ++g) {
    const uint64_t gg = j->g0 + g;
    const uint32_t k = qo_ragged_k(j->seed, gg, j->kmin, j->kmax);
    const uint32_t m = qo_drop_index(j->drop_seed, gg, k);
    uint32_t plen = 0;
    memset(par, 0, sizeof(par));
    memset(lost, 0, sizeof(lost));
    for (uint32_t i = 0; i < k; ++i) {
      const uint32_t len = qo_ragged_len(j->seed, gg, i, j->lmin, j->lmax);
      qo_synth_row(j->seed, gg, i, len, row);
      for (uint32_t b = 0; b < len; ++b) par[b] ^= row[b];
      if (i == m) memcpy(lost, row, len);
      if (len > plen) plen = len;
    }
    j->ph[g] = qo_fnv1a64(par, plen, 0);
    j->rh[g] = qo_fnv1a64(lost, plen, 0);
  }
  return NULL;
}

void qo_ragged_digests(uint64_t seed, uint64_t drop_seed, uint64_t g0, uint64_t n, uint32_t kmin,
                       uint32_t kmax, uint32_t lmin, uint32_t lmax, int threads,
                       uint64_t* parity_digest, uint64_t* recovered_digest) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  uint64_t* ph = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
  uint64_t* rh = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
  qo_rdig_job jobs[256];
  pthread_t tid[256];
  uint64_t per = (n + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; ++t) {
    uint64_t a = per * t;
    if (a >= n) break;
    qo_rdig_job jb = {seed, drop_seed, g0 + a, (a + per > n) ? n - a : per,
                      kmin, kmax, lmin, lmax, ph + a, rh + a};
    jobs[t] = jb;
    pthread_create(&tid[t], NULL, qo_rdig_run, &jobs[t]);
    ++started;
  }
  for (int t = 0; t < started; ++t) pthread_join(tid[t], NULL);
  *parity_digest = qo_fnv1a64((const uint8_t*)ph, n * sizeof(uint64_t), 0);
  *recovered_digest = qo_fnv1a64((const uint8_t*)rh, n * sizeof(uint64_t), 0);
  free(ph);
  free(rh);
}

double qo_time_single_group_ns(uint32_t k, uint32_t L, uint64_t iters) {
  uint8_t* rows = (uint8_t*)malloc((size_t)k * L);
  uint8_t par[QO_MAX_PACKET_SIZE], out[QO_MAX_PACKET_SIZE];
  qo_synth_fixed(0x51554943u, 0, 1, k, L, L, (uint64_t)k * L, rows);
  uint8_t m = (uint8_t)qo_drop_index(0x51554945u, 0, k);
  volatile uint8_t sink = 0;
  for (int w = 0; w < 1000; ++w) {
    qo_encode_fixed(rows, k, L, L, (uint64_t)k * L, 1, par, L);
    qo_recover_fixed(rows, par, &m, k, L, L, (uint64_t)k * L, L, 1, out, L);
  }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (uint64_t it = 0; it < iters; ++it) {
    qo_encode_fixed(rows, k, L, L, (uint64_t)k * L, 1, par, L);
    qo_recover_fixed(rows, par, &m, k, L, L, (uint64_t)k * L, L, 1, out, L);
    sink ^= out[it % L];
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  (void)sink;
  free(rows);
  return ((t1.tv_sec - t0.tv_sec) * 1e9 + (t1.tv_nsec - t0.tv_nsec)) / (double)iters;
}
