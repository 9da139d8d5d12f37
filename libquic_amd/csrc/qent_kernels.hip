// qent_kernels.hip — gfx950 kernels for libquic's packet-entropy bookkeeping
// (QUIC <= v33), batched over connections:
//
//   cumulative  QuicSentEntropyManager::GetCumulativeEntropy /
//               UpdateCumulativeEntropy  quic_sent_entropy_manager.cc:33-41, :57-66
//               (and the receiver's EntropyTracker::EntropyHash,
//                quic_received_packet_manager.cc:40-56, with 0 for packets
//                not received)
//   validate    QuicSentEntropyManager::IsValidEntropy  :68-96
//               (QuicConnection::ValidateAckFrame, quic_connection.cc:854)
//
// One byte per packet: HBM-bound byte work, no MFMA.  The cumulative hash is
// a segmented prefix XOR: one wave per connection walks its window 256 bytes
// at a time (4 per lane: a lane-local prefix, then a 6-step wave scan of the
// lane totals with ds_swizzle-free shuffles, carried across chunks).
// Validation is one lane per ack: every missing interval [lo, hi) costs two
// cumulative bytes (cum[hi-1] ^ cum[lo-1]) instead of a walk over the packets.
#include "qfec_internal.h"

namespace qfec {
namespace {

constexpr int kEntBlock = 256;
constexpr int kEntWaves = kEntBlock / 64;

__global__ __launch_bounds__(kEntBlock) void entropy_scan_kernel(EntropyScanArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t c = (uint64_t)blockIdx.x * kEntWaves + (threadIdx.x >> 6); c < a.n_conns;
       c += (uint64_t)gridDim.x * kEntWaves) {  // wave-uniform
    const uint64_t b = a.conn_ptr[c], end = a.conn_ptr[c + 1];
    uint32_t carry = a.cum_base ? a.cum_base[c] : 0u;
    for (uint64_t off = b; off < end; off += 256u) {
      const uint64_t i0 = off + 4u * lane;
      uint32_t x[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = i0 + j < end ? a.entropy[i0 + j] : 0u;
      x[1] ^= x[0];
      x[2] ^= x[1];
      x[3] ^= x[2];
      // inclusive wave scan of the lane totals
      uint32_t s = x[3];
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)s, d, 64);
        if (lane >= (uint32_t)d) s ^= v;
      }
      const uint32_t pre = carry ^ s ^ x[3];  // carry-in ^ exclusive prefix
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i0 + j < end) a.cum[i0 + j] = (uint8_t)(x[j] ^ pre);
      carry ^= (uint32_t)__shfl((int)s, 63, 64);
    }
  }
}

__device__ __forceinline__ uint32_t cum_at(const uint8_t* cum, uint64_t b, uint64_t first,
                                           uint32_t base, uint64_t pn) {
  return pn < first ? base : cum[b + (pn - first)];
}

__global__ __launch_bounds__(kEntBlock) void entropy_validate_kernel(EntropyValidateArgs a) {
  for (uint64_t q = (uint64_t)blockIdx.x * kEntBlock + threadIdx.x; q < a.n_acks;
       q += (uint64_t)gridDim.x * kEntBlock) {
    const uint32_t c = a.ack_conn[q];
    bool good = c < a.n_conns;
    uint32_t expected = 0u;
    if (good) {
      const uint64_t b = a.conn_ptr[c], n = a.conn_ptr[c + 1] - b, first = a.first_pn[c];
      const uint32_t base = a.cum_base ? a.cum_base[c] : 0u;
      const uint64_t last = first + n - 1u, largest = a.largest_observed[q];
      // largest above the largest recorded packet: false (:75-77); below the
      // window: the reference's DCHECK (:71), false here
      good = largest + 1u >= first && largest <= last;
      if (good) expected = cum_at(a.cum, b, first, base, largest);
      for (uint32_t r = a.range_ptr[q]; good && r < a.range_ptr[q + 1]; ++r) {
        const uint64_t lo = a.range_lo[r], hi = a.range_hi[r];
        if (lo >= hi) continue;
        // a missing packet below the window: false (:78-81); above the
        // largest recorded: out of the deque in the reference, false here
        if (lo < first || hi - 1u > last) {
          good = false;
          break;
        }
        expected ^= cum_at(a.cum, b, first, base, hi - 1u) ^ cum_at(a.cum, b, first, base, lo - 1u);
      }
    }
    a.ok[q] = (good && expected == a.claimed[q]) ? 1 : 0;
  }
}

uint32_t grid_for(uint64_t items, uint64_t per_block) {
  const uint64_t g = (items + per_block - 1) / per_block;
  return (uint32_t)(g < (1ull << 20) ? (g ? g : 1) : (1ull << 20));
}

}  // namespace

hipError_t launch_entropy_scan(const EntropyScanArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(entropy_scan_kernel, dim3(grid_for(a.n_conns, kEntWaves)), dim3(kEntBlock),
                     0, s, a);
  return hipGetLastError();
}

hipError_t launch_entropy_validate(const EntropyValidateArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(entropy_validate_kernel, dim3(grid_for(a.n_acks, kEntBlock)),
                     dim3(kEntBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace qfec
