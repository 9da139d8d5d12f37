/* qent_oracle.c — see qent_oracle.h (TEST INFRASTRUCTURE ONLY). */
#include "qent_oracle.h"

/* quic_framer.cc:351-354 */
uint8_t qo_packet_entropy_hash(int entropy_flag, uint64_t packet_number) {
  return (uint8_t)((entropy_flag ? 1u : 0u) << (packet_number % 8u));
}

/* UpdateCumulativeEntropy (quic_sent_entropy_manager.cc:33-41): walk forward
 * XORing each packet's hash — here once over the whole window. */
void qo_entropy_cumulative_batch(const uint8_t* entropy, const uint64_t* conn_ptr,
                                 const uint8_t* cum_base, uint64_t n_conns, uint8_t* cum) {
  for (uint64_t c = 0; c < n_conns; ++c) {
    uint8_t h = cum_base ? cum_base[c] : 0u;
    for (uint64_t i = conn_ptr[c]; i < conn_ptr[c + 1]; ++i) {
      h ^= entropy[i];
      cum[i] = h;
    }
  }
}

/* Cumulative entropy through packet pn of connection c (pn >= first - 1). */
static uint8_t cum_at(const uint8_t* cum, uint64_t base_idx, uint64_t first, uint8_t base,
                      uint64_t pn) {
  return pn < first ? base : cum[base_idx + (pn - first)];
}

/* IsValidEntropy (quic_sent_entropy_manager.cc:68-96). */
void qo_entropy_validate_batch(const uint8_t* cum, const uint64_t* conn_ptr,
                               const uint64_t* first_pn, const uint8_t* cum_base,
                               const uint32_t* ack_conn, const uint64_t* largest_observed,
                               const uint8_t* claimed, const uint32_t* range_ptr,
                               const uint64_t* range_lo, const uint64_t* range_hi,
                               uint64_t n_acks, uint8_t* ok) {
  for (uint64_t a = 0; a < n_acks; ++a) {
    const uint32_t c = ack_conn[a];
    const uint64_t b = conn_ptr[c], n = conn_ptr[c + 1] - b, first = first_pn[c];
    const uint8_t base = cum_base ? cum_base[c] : 0u;
    const uint64_t last = first + n - 1; /* GetLargestPacketWithEntropy (:27-29) */
    const uint64_t lo_obs = largest_observed[a];
    int good = 1;
    /* "largest_observed > GetLargestPacketWithEntropy() -> false" (:75-77);
     * below the window: the reference's DCHECK (:71) — 0 here */
    if (lo_obs + 1 < first || lo_obs > last) good = 0;
    uint8_t expected = good ? cum_at(cum, b, first, base, lo_obs) : 0u;
    for (uint32_t r = range_ptr[a]; good && r < range_ptr[a + 1]; ++r) {
      const uint64_t lo = range_lo[r], hi = range_hi[r];
      if (lo >= hi) continue; /* empty interval */
      /* "missing_packets.Min() < GetSmallestPacketWithEntropy() -> false"
       * (:78-81); above the largest recorded: undefined there, 0 here */
      if (lo < first || hi - 1 > last) {
        good = 0;
        break;
      }
      /* XOR of the hashes of lo .. hi-1 (:86-92) */
      expected ^= (uint8_t)(cum_at(cum, b, first, base, hi - 1) ^
                            cum_at(cum, b, first, base, lo - 1));
    }
    ok[a] = (uint8_t)(good && expected == claimed[a]);
  }
}
