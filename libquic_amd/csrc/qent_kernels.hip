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
// a segmented prefix XOR: a group of LPC lanes per connection walks its
// window 16*LPC bytes at a time (16 per lane: a lane-local prefix, then a
// shuffle scan of the lane totals inside the group, carried across steps),
// 64/LPC connections per wave.
// Validation is one lane per ack: every missing interval [lo, hi) costs two
// cumulative bytes (cum[hi-1] ^ cum[lo-1]) instead of a walk over the packets.
#include "qfec_internal.h"

namespace qfec {
namespace {

constexpr int kEntBlock = 256;
constexpr int kEntWaves = kEntBlock / 64;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Prefix XOR over the 16 bytes of a chunk (little-endian: byte i of the
// result = byte 0 ^ ... ^ byte i), carry-in c (0..255) XORed into every byte.
__device__ __forceinline__ u32x4 prefix16(u32x4 v, uint32_t c) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t run = c * 0x01010101u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t x = w[i];
    x ^= x << 8;
    x ^= x << 16;
    w[i] = x ^ run;
    run = (w[i] >> 24) * 0x01010101u;
  }
  return u32x4{w[0], w[1], w[2], w[3]};
}

// LPC lanes per connection, 16 bytes per lane: a wave scans 64/LPC
// connections at once, 16*LPC bytes of each per step (chunk-local prefix,
// then a log2(LPC)-step shuffle scan of the lane totals inside the lane
// group, carried across steps).  Windows of a few hundred packets — the
// usual case — take one step, so the dependent loads (pointers, then bytes)
// of 64/LPC connections overlap in one wave instead of one connection per
// wave.
template <int LPC>
__global__ __launch_bounds__(kEntBlock) void entropy_scan_kernel(EntropyScanArgs a) {
  constexpr int kPerWave = 64 / LPC;
  const uint32_t lane = threadIdx.x & 63u, sub = lane % LPC;
  for (uint64_t c0 = ((uint64_t)blockIdx.x * kEntWaves + (threadIdx.x >> 6)) * kPerWave;
       c0 < a.n_conns; c0 += (uint64_t)gridDim.x * kEntWaves * kPerWave) {
    const uint64_t c = c0 + lane / LPC;
    const bool live = c < a.n_conns;
    const uint64_t b = live ? a.conn_ptr[c] : 0u, end = live ? a.conn_ptr[c + 1] : 0u;
    uint32_t carry = live && a.cum_base ? a.cum_base[c] : 0u;
    const uint64_t len = end - b;
    // steps: the longest window of the wave's connections (loop is wave-uniform)
    uint64_t mx = len;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t y = (uint64_t)__shfl_xor((long long)mx, o, 64);
      mx = y > mx ? y : mx;
    }
    for (uint64_t off = 0; off < mx; off += 16u * LPC) {
      const uint64_t i0 = b + off + 16u * sub;
      const uint32_t nb = i0 >= end ? 0u : (uint32_t)min((uint64_t)16u, end - i0);
      u32x4 v = {0u, 0u, 0u, 0u};
      if (nb == 16u) {
        __builtin_memcpy(&v, a.entropy + i0, 16);
      } else if (nb) {
        uint8_t t[16];
#pragma unroll
        for (uint32_t j = 0; j < 16u; ++j) t[j] = j < nb ? a.entropy[i0 + j] : (uint8_t)0;
        __builtin_memcpy(&v, t, 16);
      }
      const u32x4 loc = prefix16(v, 0u);
      const uint32_t tot = loc.w >> 24;  // zero bytes past the window keep it exact
      uint32_t s = tot;
#pragma unroll
      for (int d = 1; d < LPC; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)s, d, LPC);
        if (sub >= (uint32_t)d) s ^= y;
      }
      const u32x4 out = prefix16(v, carry ^ s ^ tot);  // carry-in ^ exclusive prefix
      if (nb == 16u) {
        __builtin_memcpy(a.cum + i0, &out, 16);
      } else if (nb) {
        uint8_t t[16];
        __builtin_memcpy(t, &out, 16);
        for (uint32_t j = 0; j < nb; ++j) a.cum[i0 + j] = t[j];
      }
      carry ^= (uint32_t)__shfl((int)s, LPC - 1, LPC);
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

// Lanes per connection from the mean window (unknown: 16): 8 (128-B steps) up
// to 64.
hipError_t launch_entropy_scan(const EntropyScanArgs& a, hipStream_t s, uint64_t total_bytes) {
  const uint64_t mean = a.n_conns && total_bytes ? total_bytes / a.n_conns : 256u;
  if (mean <= 128u)
    hipLaunchKernelGGL(entropy_scan_kernel<8>, dim3(grid_for(a.n_conns, kEntWaves * 8)),
                       dim3(kEntBlock), 0, s, a);
  else if (mean <= 256u)
    hipLaunchKernelGGL(entropy_scan_kernel<16>, dim3(grid_for(a.n_conns, kEntWaves * 4)),
                       dim3(kEntBlock), 0, s, a);
  else if (mean <= 512u)
    hipLaunchKernelGGL(entropy_scan_kernel<32>, dim3(grid_for(a.n_conns, kEntWaves * 2)),
                       dim3(kEntBlock), 0, s, a);
  else
    hipLaunchKernelGGL(entropy_scan_kernel<64>, dim3(grid_for(a.n_conns, kEntWaves)),
                       dim3(kEntBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_entropy_validate(const EntropyValidateArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(entropy_validate_kernel, dim3(grid_for(a.n_acks, kEntBlock)),
                     dim3(kEntBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace qfec
