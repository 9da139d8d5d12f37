/*
 * qent_oracle.h — CPU restatement of libquic's packet-entropy bookkeeping
 * (QUIC versions <= 33: one entropy bit per packet, acks carry the XOR of the
 * entropy hashes of every packet they acknowledge).  SURVEY.md §8(f) rank 4.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libquic_amd/, include/)
 * links, loads or calls this code.  It is the checker used by tests/ and
 * bench.py's cpu_baseline leg for the batched entropy kernels.
 *
 * PINNED by the reference: tests/test_oracle_entropy.py checks it against the
 * reference's own QuicSentEntropyManager (quic_sent_entropy_manager.cc)
 * compiled from /root/reference into oracle/_ref/libref_quic.so.
 *
 * Restated (batched over connections):
 *   packet entropy        QuicFramer::GetPacketEntropyHash   quic_framer.cc:351-354
 *                         (entropy_flag << (packet_number % 8))
 *   cumulative entropy    QuicSentEntropyManager::GetCumulativeEntropy /
 *                         UpdateCumulativeEntropy            quic_sent_entropy_manager.cc:33-41, :57-66
 *   ack validation        QuicSentEntropyManager::IsValidEntropy  :68-96
 *                         (called from QuicConnection::ValidateAckFrame,
 *                          quic_connection.cc:854)
 *
 * Batch layout.  Connection c holds the entropy hashes of its sent packets
 * first_pn[c] .. first_pn[c] + n_c - 1 at entropy[conn_ptr[c] .. conn_ptr[c+1])
 * (the manager's deque after ClearEntropyBefore(first_pn[c])) and
 * cum_base[c] = the cumulative entropy through first_pn[c] - 1.
 * cum[i] = cum_base[c] ^ entropy[conn_ptr[c]] ^ ... ^ entropy[i].
 * Ack a (connection ack_conn[a]): largest_observed[a], its missing packets as
 * disjoint ranges [range_lo, range_hi) (the PacketNumberQueue intervals,
 * range_ptr CSR), the claimed hash.  ok[a] = IsValidEntropy's result; where
 * the reference's behaviour is undefined (a missing packet above the largest
 * recorded one: deque index out of range; largest_observed below the window:
 * DCHECK) the batch form answers 0.
 */
#ifndef QENT_ORACLE_H_
#define QENT_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

uint8_t qo_packet_entropy_hash(int entropy_flag, uint64_t packet_number);
void qo_entropy_cumulative_batch(const uint8_t* entropy, const uint64_t* conn_ptr,
                                 const uint8_t* cum_base, uint64_t n_conns, uint8_t* cum);
void qo_entropy_validate_batch(const uint8_t* cum, const uint64_t* conn_ptr,
                               const uint64_t* first_pn, const uint8_t* cum_base,
                               const uint32_t* ack_conn, const uint64_t* largest_observed,
                               const uint8_t* claimed, const uint32_t* range_ptr,
                               const uint64_t* range_lo, const uint64_t* range_hi,
                               uint64_t n_acks, uint8_t* ok);

#ifdef __cplusplus
}
#endif
#endif /* QENT_ORACLE_H_ */
