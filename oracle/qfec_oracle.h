/*
 * qfec_oracle.h — CPU restatement of the QUIC FEC group arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libquic_amd/, include/)
 * links, loads or calls this code.  It is the checker used by tests/,
 * __graft_entry__.smoke() and bench.py's `cpu_baseline` leg.
 *
 * PARITY UNPINNED (by the reference): the libquic snapshot under
 * /root/reference no longer contains the FEC implementation
 * (quic_fec_group{,_interface}.cc are named only by the stale
 * Makefile:5332-5384; src/net/quic/core/quic_protocol.h:373 "FEC related fields
 * are removed from wire format"), and no test, vector or fixture in the
 * reference pins FEC results.  This restatement follows SURVEY.md Appendix A
 * (the historical QuicFecGroup contract) plus the in-tree constraints:
 *   - kMaxPacketSize = 1452        quic_protocol.h:66
 *   - k <= 255 (uint8 group offset) quic_framer.cc:1126-1136
 *   - zero padding                  quic_data_writer.cc:136-143,
 *                                   PADDING_FRAME = 0 quic_protocol.h:259,
 *                                   parsed as "rest of packet" quic_framer.cc:1224-1231
 *   - QUIC_INVALID_FEC_DATA = 5     quic_protocol.h:537-538
 * It is cross-checked against an independent NumPy restatement
 * (oracle/qfec_np.py) and against algebraic identities (tests/test_oracle.py).
 */
#ifndef QFEC_ORACLE_H_
#define QFEC_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QO_MAX_PACKET_SIZE 1452u /* kMaxPacketSize, quic_protocol.h:66 */
#define QO_MAX_GROUP_PACKETS 255u /* uint8 offset, quic_framer.cc:1126 */
#define QO_OK 0
#define QO_INVALID_FEC_DATA (-5) /* -QUIC_INVALID_FEC_DATA, quic_protocol.h:538 */

/* ---- synthetic inputs (counter-based) ---- */
uint64_t qo_splitmix64(uint64_t x);
/* byte j of packet (g, i): little-endian byte j%8 of
 * splitmix64(seed ^ ((g*256 + i) << 32) ^ (j/8)) */
uint8_t qo_synth_byte(uint64_t seed, uint64_t g, uint32_t i, uint32_t j);
void qo_synth_row(uint64_t seed, uint64_t g, uint32_t i, uint32_t len, uint8_t* out);
/* rows laid out [n][k][row_stride]; bytes [L, row_stride) are left untouched */
void qo_synth_fixed(uint64_t seed, uint64_t g0, uint64_t n, uint32_t k, uint32_t L,
                    uint64_t row_stride, uint64_t group_stride, uint8_t* rows);
/* ragged shapes: k_g in [kmin,kmax], len in [lmin,lmax] */
uint32_t qo_ragged_k(uint64_t seed, uint64_t g, uint32_t kmin, uint32_t kmax);
uint32_t qo_ragged_len(uint64_t seed, uint64_t g, uint32_t i, uint32_t lmin, uint32_t lmax);
uint32_t qo_drop_index(uint64_t seed, uint64_t g, uint32_t k);

/* ---- the FEC group (Appendix A), one group at a time ---- */
/* XorBuffers: out[j] ^= in[j], word-wise + byte tail. */
void qo_xor_buffers(const uint8_t* in, size_t n, uint8_t* out);

/* Encode one group. payloads[i] has lens[i] bytes.  parity receives
 * parity_len = max lens[i] bytes.  Returns parity_len or QO_INVALID_FEC_DATA. */
int qo_group_encode(const uint8_t* const* payloads, const uint32_t* lens, uint32_t k,
                    uint8_t* parity);
/* Recover packet m.  payloads[m] / lens[m] are ignored.  Returns parity_len. */
int qo_group_recover(const uint8_t* const* payloads, const uint32_t* lens, uint32_t k,
                     const uint8_t* parity, uint32_t parity_len, uint32_t m, uint8_t* out);

/* ---- batch forms mirroring the C-ABI shapes (include/qfec.h) ---- */
int qo_encode_fixed(const uint8_t* rows, uint32_t k, uint32_t L, uint64_t row_stride,
                    uint64_t group_stride, uint64_t n, uint8_t* parity, uint64_t parity_stride);
int qo_recover_fixed(const uint8_t* rows, const uint8_t* parity, const uint8_t* missing,
                     uint32_t k, uint32_t L, uint64_t row_stride, uint64_t group_stride,
                     uint64_t parity_stride, uint64_t n, uint8_t* out, uint64_t out_stride);
int qo_encode_ragged(const uint8_t* bytes, const uint64_t* pkt_off, const uint16_t* pkt_len,
                     const uint32_t* grp_ptr, uint64_t n, uint8_t* parity,
                     const uint64_t* parity_off, uint16_t* parity_len);
int qo_recover_ragged(const uint8_t* bytes, const uint64_t* pkt_off, const uint16_t* pkt_len,
                      const uint32_t* grp_ptr, uint64_t n, const uint8_t* parity,
                      const uint64_t* parity_off, const uint16_t* parity_len,
                      const uint8_t* missing, uint8_t* out, const uint64_t* out_off);

/* multi-threaded fixed encode/recover for the CPU baseline (contiguous split) */
int qo_encode_fixed_mt(const uint8_t* rows, uint32_t k, uint32_t L, uint64_t n,
                       uint8_t* parity, int threads);
int qo_recover_fixed_mt(const uint8_t* rows, const uint8_t* parity, const uint8_t* missing,
                        uint32_t k, uint32_t L, uint64_t n, uint8_t* out, int threads);

/* configs[0] timer: mean ns for encode + recover of ONE group of k x L
 * (1 core), over `iters` repetitions after a warm-up. */
double qo_time_single_group_ns(uint32_t k, uint32_t L, uint64_t iters);

/* FNV-1a 64 over a buffer (checksums for large-size property tests) */
uint64_t qo_fnv1a64(const uint8_t* p, size_t n, uint64_t h);

/* "Checksum of checksums": FNV-1a over the sequence of per-group FNV-1a
 * hashes (each group's bytes [0, len_g) at base + g*stride, or at base + off[g]
 * when off != NULL with lengths len[g]).  Order-sensitive, multi-threaded. */
uint64_t qo_group_digest(const uint8_t* base, uint64_t n, uint64_t stride, uint32_t L,
                         const uint64_t* off, const uint16_t* len, int threads);
/* Digests of the full fixed-shape workload without materialising it:
 * groups g0..g0+n-1 of synth rows (k x L), parity digest and the digest of the
 * rows a recover with drop indices qo_drop_index(drop_seed, g, k) revives. */
void qo_fixed_digests(uint64_t seed, uint64_t drop_seed, uint64_t g0, uint64_t n, uint32_t k,
                      uint32_t L, int threads, uint64_t* parity_digest,
                      uint64_t* recovered_digest);

/* The same for the ragged configs[3] workload (qo_ragged_k / qo_ragged_len
 * shapes, qo_synth_row bytes): digests of the parity rows (parity_len = max
 * len bytes each) and of the revived rows (the lost packet zero padded to
 * parity_len).  Layout independent: the digests cover the bytes of each row. */
void qo_ragged_digests(uint64_t seed, uint64_t drop_seed, uint64_t g0, uint64_t n, uint32_t kmin,
                       uint32_t kmax, uint32_t lmin, uint32_t lmax, int threads,
                       uint64_t* parity_digest, uint64_t* recovered_digest);

#ifdef __cplusplus
}
#endif
#endif /* QFEC_ORACLE_H_ */
