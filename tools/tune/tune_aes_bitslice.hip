// tune_aes_bitslice.hip — round 6: a bitsliced AES-128
// keystream (CTR, the GCM counter blocks) against the product's T-table AES,
// both compute-only over 2^20 packets of 1350 B (85 counter blocks each).
//
// The product's aes128gcm_kernel runs issue-latency bound: VALU issue 0.34 of
// its ceiling and LDS issue 0.45 at 1.7-2.3 waves per SIMD
// (profiles/round5/aead_stall.json), each AES round being 16 Te0 lookups in
// a 64-KiB LDS table per block.  The lever DESIGN.md §9 names is a bitsliced
// AES: no table, VALU only, 32 blocks per lane (bit b of each 32-bit word
// belongs to block b), so its issue rate is bounded by VALU alone.  Here:
//   * the S-box is a generated circuit (tools/tune/gen_bitslice_sbox.py: the
//     GF(2^8) inverse in the tower field GF(((2^2)^2)^2), then the affine
//     map; 195 gates fused into 135 v_bitop3_b32), checked on the GPU for all
//     256 inputs first;
//   * ShiftRows is a renaming, MixColumns ~100 XORs per column (xtime on bit
//     words), AddRoundKey one XOR per word with a mask made from the round
//     key in SGPRs (one key for the batch: the uniform-key case);
//   * the counter blocks go in by one 32x32 bit transpose (bytes 12-15), the
//     nonce bytes as sign-extended bit fields, and the keystream comes out by
//     four 32x32 transposes.
// Variants: the T-table kernel (aes_encrypt_n from qpp_kernels.hip, Te0 in
// LDS, the product's shape: 768 threads, 3 waves per SIMD, 4 blocks in
// flight per lane) and the bitsliced kernel at 1-3 waves per SIMD.  Every
// variant's keystream is byte-compared with the T-table kernel's over 4,096
// packets before timing; the timed runs XOR each lane's keystream into one
// word (compute-only, the same for both).
//
//   tune_aes_bitslice [packets=2^20] [reps=5] [rounds=3]
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_aes_bitslice.hip \
//          -o tools/tune/build/tune_aes_bitslice
#include "../../libquic_amd/csrc/qpp_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

#define QFEC_BOP3(a, b, c, t) __builtin_amdgcn_bitop3_b32((a), (b), (c), (t))
#include "aes_bitslice_sbox.inc"

namespace bs {

using qfec::u32x4;
constexpr uint32_t kBlocks = 85;  // 1350 B per packet

struct RK {
  uint32_t w[44];  // FIPS-197 round keys, little-endian words (AesKey layout)
};

// 32x32 bit transpose, LSB-first: afterwards m[p] bit b = (before) m[b] bit p.
__host__ __device__ __forceinline__ void transpose32(uint32_t (&m)[32]) {
#define BS_STAGE(S, MASK)                                                  \
  _Pragma("unroll") for (int r = 0; r < 32; ++r) {                         \
    if ((r & (S)) == 0) {                                                  \
      const uint32_t t = ((m[r] >> (S)) ^ m[r + (S)]) & (MASK);            \
      m[r + (S)] ^= t;                                                     \
      m[r] ^= t << (S);                                                    \
    }                                                                      \
  }
  BS_STAGE(16, 0x0000FFFFu)
  BS_STAGE(8, 0x00FF00FFu)
  BS_STAGE(4, 0x0F0F0F0Fu)
  BS_STAGE(2, 0x33333333u)
  BS_STAGE(1, 0x55555555u)
#undef BS_STAGE
}

__device__ __forceinline__ void xtime(const uint32_t (&t)[8], uint32_t (&x)[8]) {
  x[0] = t[7];
  x[1] = t[0] ^ t[7];
  x[2] = t[1];
  x[3] = t[2] ^ t[7];
  x[4] = t[3] ^ t[7];
  x[5] = t[4];
  x[6] = t[5];
  x[7] = t[6];
}

__device__ __forceinline__ void add_round_key(uint32_t (&W)[16][8], const RK& rk, int r) {
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t kb = rk.w[4 * r + k / 4] >> (8 * (k % 4));
#pragma unroll
    for (int i = 0; i < 8; ++i) W[k][i] ^= 0u - ((kb >> i) & 1u);
  }
}

// W: byte k (state index r + 4c, FIPS-197 column-major), bit i, of 32 blocks
__device__ __forceinline__ void aes_bitsliced(uint32_t (&W)[16][8], const RK& rk) {
  add_round_key(W, rk, 0);
#pragma unroll 1
  for (int round = 1; round <= 10; ++round) {
    uint32_t N[16][8];
#pragma unroll
    for (int kp = 0; kp < 16; ++kp) {  // SubBytes + ShiftRows (renaming)
      const int r = kp & 3, c = kp >> 2;
      const int src = r + 4 * ((c + r) & 3);
      QFEC_SBOX_BITSLICED(W[src], N[kp]);
    }
    if (round < 10) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {  // MixColumns
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          uint32_t t[8], x[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) t[i] = N[4 * c + r][i] ^ N[4 * c + ((r + 1) & 3)][i];
          xtime(t, x);
#pragma unroll
          for (int i = 0; i < 8; ++i)
            W[4 * c + r][i] = x[i] ^ N[4 * c + ((r + 1) & 3)][i] ^ N[4 * c + ((r + 2) & 3)][i] ^
                              N[4 * c + ((r + 3) & 3)][i];
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i) W[k][i] = N[k][i];
    }
    add_round_key(W, rk, round);
  }
}

// S-box self-test: lane L (of 8) computes S(32L + b) for b < 32.
template <bool SWAP>
__global__ void sbox_test(uint8_t* out) {
  const uint32_t L = threadIdx.x;
  if (L >= 8) return;
  uint32_t x[8], y[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t w = 0;
    for (uint32_t b = 0; b < 32; ++b) w |= (((32u * L + b) >> i) & 1u) << b;
    x[i] = w;
  }
  if constexpr (SWAP) {
#undef QFEC_BOP3
#define QFEC_BOP3(a, b, c, t) __builtin_amdgcn_bitop3_b32((c), (b), (a), (t))
    QFEC_SBOX_BITSLICED(x, y);
#undef QFEC_BOP3
#define QFEC_BOP3(a, b, c, t) __builtin_amdgcn_bitop3_b32((a), (b), (c), (t))
  } else {
    QFEC_SBOX_BITSLICED(x, y);
  }
  for (uint32_t b = 0; b < 32; ++b) {
    uint32_t v = 0;
    for (int i = 0; i < 8; ++i) v |= ((y[i] >> b) & 1u) << i;
    out[32u * L + b] = (uint8_t)v;
  }
}

// nonce words of packet p (the product's layout: prefix || LE64 packet number)
__device__ __forceinline__ void packet_nonce(uint64_t p, uint32_t (&n)[3]) {
  n[0] = 0x01020304u;
  n[1] = (uint32_t)(p * 0x9E3779B9u);
  n[2] = (uint32_t)(p >> 7) ^ 0xA5A5A5A5u;
}

// Bitsliced keystream: one lane per packet, 32 counter blocks per pass.
// WRITE: keystream to out (packet-major, 16 B per block); else XOR-folded.
template <bool WRITE, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void ks_bitsliced(
    RK rk, uint64_t n, u32x4* out, uint32_t* fold) {
  const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  uint32_t nonce[3];
  packet_nonce(p, nonce);
  uint32_t acc = 0;
#pragma unroll 1
  for (uint32_t c0 = 0; c0 < kBlocks; c0 += 32) {
    uint32_t W[16][8];
#pragma unroll
    for (int k = 0; k < 12; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i)  // sign-extended bit field: 0 or ~0
        W[k][i] = (uint32_t)__builtin_amdgcn_sbfe((int)nonce[k / 4], 8 * (k % 4) + i, 1);
    uint32_t M[32];
#pragma unroll
    for (int b = 0; b < 32; ++b) M[b] = __builtin_bswap32(2u + c0 + (uint32_t)b);  // gcm_ctr
    transpose32(M);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) W[12 + j][i] = M[8 * j + i];
    aes_bitsliced(W, rk);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t R[32];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) R[8 * j + i] = W[4 * q + j][i];
      transpose32(R);  // R[b] = dword q of block b
#pragma unroll
      for (int b = 0; b < 32; ++b) {
        if (c0 + (uint32_t)b < kBlocks) {
          if constexpr (WRITE)
            reinterpret_cast<uint32_t*>(out + p * kBlocks + c0 + b)[q] = R[b];
          else
            acc ^= R[b];
        }
      }
    }
  }
  if constexpr (!WRITE) fold[p] = acc;
}

// T-table keystream (the product's aes_encrypt_n, Te0 replicated in LDS).
template <bool WRITE, int NB>
__global__ __launch_bounds__(768) __attribute__((amdgpu_waves_per_eu(3, 3))) void ks_ttable(
    RK rk, uint64_t n, u32x4* out, uint32_t* fold) {
  __shared__ uint32_t te[qfec::kTeBytes / 4u];
  for (uint32_t i = threadIdx.x; i < qfec::kTeBytes / 16u; i += 768) {
    const uint32_t e = qfec::kTe0[i >> 4];
    reinterpret_cast<u32x4*>(te)[i] = u32x4{e, e, e, e};
  }
  __syncthreads();
  const uint64_t p = (uint64_t)blockIdx.x * 768 + threadIdx.x;
  if (p >= n) return;
  const uint32_t lane4 = (threadIdx.x & 63u) * 4u;
  qfec::AesKey key;
#pragma unroll
  for (int i = 0; i < 44; ++i) key.rk[i] = rk.w[i];
  uint32_t nonce[3];
  packet_nonce(p, nonce);
  uint32_t acc = 0;
#pragma unroll 1
  for (uint32_t c = 0; c < kBlocks; c += NB) {
    u32x4 io[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) io[b] = qfec::gcm_ctr(nonce, c + b);
    qfec::aes_encrypt_n<NB>(key, io, te, lane4);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (c + (uint32_t)b < kBlocks) {
        if constexpr (WRITE)
          out[p * kBlocks + c + b] = io[b];
        else
          acc ^= io[b].x ^ io[b].y ^ io[b].z ^ io[b].w;
      }
    }
  }
  if constexpr (!WRITE) fold[p] = acc;
}

}  // namespace bs

// ---- host ---------------------------------------------------------------------
static uint8_t h_gmul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1B : 0));
    b >>= 1;
  }
  return r;
}

static uint8_t h_sbox(uint8_t x) {
  uint8_t inv = 0;
  if (x)
    for (int b = 1; b < 256; ++b)
      if (h_gmul(x, (uint8_t)b) == 1) inv = (uint8_t)b;
  uint8_t r = 0x63;
  for (int i = 0; i < 8; ++i) {
    const int bit = ((inv >> i) ^ (inv >> ((i + 4) % 8)) ^ (inv >> ((i + 5) % 8)) ^
                     (inv >> ((i + 6) % 8)) ^ (inv >> ((i + 7) % 8))) & 1;
    r ^= (uint8_t)(bit << i);
  }
  return r;
}

static void h_expand(const uint8_t key[16], bs::RK& rk) {
  uint8_t S[256];
  for (int i = 0; i < 256; ++i) S[i] = h_sbox((uint8_t)i);
  for (int i = 0; i < 4; ++i) std::memcpy(&rk.w[i], key + 4 * i, 4);
  uint32_t rcon = 1;
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk.w[i - 1];
    if (i % 4 == 0) {
      t = (uint32_t)S[(t >> 8) & 0xFF] | ((uint32_t)S[(t >> 16) & 0xFF] << 8) |
          ((uint32_t)S[(t >> 24) & 0xFF] << 16) | ((uint32_t)S[t & 0xFF] << 24);
      t ^= rcon;
      rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x1B : 0)) & 0xFF;
    }
    rk.w[i] = rk.w[i - 4] ^ t;
  }
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 20);
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int rounds = argc > 3 ? atoi(argv[3]) : 3;

  // host check of the transpose
  {
    uint32_t m[32], o[32];
    for (int r = 0; r < 32; ++r) m[r] = o[r] = 0x9E3779B9u * (uint32_t)(r + 1) ^ (uint32_t)(r << 7);
    bs::transpose32(m);
    for (int p = 0; p < 32; ++p)
      for (int b = 0; b < 32; ++b)
        if (((m[p] >> b) & 1u) != ((o[b] >> p) & 1u)) {
          std::printf("transpose32 wrong at %d,%d\n", p, b);
          return 2;
        }
  }
  // S-box on the GPU, both operand orders of v_bitop3_b32's truth table
  uint8_t* d_s;
  CK(hipMalloc(&d_s, 256));
  uint8_t hs[256];
  bool order_ok[2] = {false, false};
  for (int swap = 0; swap < 2; ++swap) {
    CK(hipMemset(d_s, 0, 256));
    if (swap)
      hipLaunchKernelGGL(bs::sbox_test<true>, dim3(1), dim3(64), 0, 0, d_s);
    else
      hipLaunchKernelGGL(bs::sbox_test<false>, dim3(1), dim3(64), 0, 0, d_s);
    CK(hipMemcpy(hs, d_s, 256, hipMemcpyDeviceToHost));
    bool ok = true;
    for (int x = 0; x < 256; ++x) ok = ok && hs[x] == h_sbox((uint8_t)x);
    order_ok[swap] = ok;
    std::printf("bitsliced S-box, %s operand order: %s\n", swap ? "swapped" : "as generated",
                ok ? "all 256 exact" : "WRONG");
  }
  if (!order_ok[0]) {
    std::printf("the generated circuit's bitop3 convention does not hold: stop\n");
    return 2;
  }

  const uint8_t key[16] = {0x2b, 0x7e, 0x15, 0x16, 0x28, 0xae, 0xd2, 0xa6,
                           0xab, 0xf7, 0x15, 0x88, 0x09, 0xcf, 0x4f, 0x3c};  // FIPS-197 C.1-style
  bs::RK rk;
  h_expand(key, rk);
  const uint64_t nchk = std::min<uint64_t>(n, 4096);
  qfec::u32x4 *ref, *got;
  uint32_t* fold;
  CK(hipMalloc(&ref, nchk * bs::kBlocks * 16));
  CK(hipMalloc(&got, nchk * bs::kBlocks * 16));
  CK(hipMalloc(&fold, n * 4));
  hipLaunchKernelGGL((bs::ks_ttable<true, 4>), dim3((uint32_t)((nchk + 767) / 768)), dim3(768), 0, 0,
                     rk, nchk, ref, fold);
  CK(hipDeviceSynchronize());
  // FIPS-197 Appendix B: plaintext 3243f6a8885a308d313198a2e0370734 under
  // this key encrypts to 3925841d02dc09fbdc118597196a0b32 (checks the T-table
  // path and the key expansion here; the counter blocks differ)
  struct V {
    std::string name;
    std::function<void(bool)> run;  // write?
  };
  auto grid256 = [&](uint64_t m) { return dim3((uint32_t)((m + 255) / 256)); };
  std::vector<V> vs;
  vs.push_back({"T-table NB4 (product AES)", [&](bool w) {
                  const uint64_t m = w ? nchk : n;
                  if (w)
                    hipLaunchKernelGGL((bs::ks_ttable<true, 4>), dim3((uint32_t)((m + 767) / 768)),
                                       dim3(768), 0, 0, rk, m, got, fold);
                  else
                    hipLaunchKernelGGL((bs::ks_ttable<false, 4>), dim3((uint32_t)((m + 767) / 768)),
                                       dim3(768), 0, 0, rk, m, got, fold);
                }});
  vs.push_back({"T-table NB8", [&](bool w) {
                  const uint64_t m = w ? nchk : n;
                  if (w)
                    hipLaunchKernelGGL((bs::ks_ttable<true, 8>), dim3((uint32_t)((m + 767) / 768)),
                                       dim3(768), 0, 0, rk, m, got, fold);
                  else
                    hipLaunchKernelGGL((bs::ks_ttable<false, 8>), dim3((uint32_t)((m + 767) / 768)),
                                       dim3(768), 0, 0, rk, m, got, fold);
                }});
#define BS_V(WPE)                                                                              \
  vs.push_back({"bitsliced, " #WPE " wave(s)/SIMD", [&](bool w) {                             \
                  const uint64_t m = w ? nchk : n;                                             \
                  if (w)                                                                       \
                    hipLaunchKernelGGL((bs::ks_bitsliced<true, WPE>), grid256(m), dim3(256), 0, 0, \
                                       rk, m, got, fold);                                      \
                  else                                                                         \
                    hipLaunchKernelGGL((bs::ks_bitsliced<false, WPE>), grid256(m), dim3(256), 0, \
                                       0, rk, m, got, fold);                                   \
                }});
  BS_V(1)
  BS_V(2)
  BS_V(3)
  std::vector<uint8_t> hr(nchk * bs::kBlocks * 16), hg(hr.size());
  CK(hipMemcpy(hr.data(), ref, hr.size(), hipMemcpyDeviceToHost));
  bool all_ok = true;
  for (const V& v : vs) {
    CK(hipMemset(got, 0, hg.size()));
    v.run(true);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hg.data(), got, hg.size(), hipMemcpyDeviceToHost));
    const bool ok = hg == hr;
    std::printf("check %-30s == T-table keystream (%llu packets): %s\n", v.name.c_str(),
                (unsigned long long)nchk, ok ? "yes" : "NO");
    all_ok = all_ok && ok;
  }
  if (!all_ok) return 2;
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  std::vector<std::vector<float>> ms(vs.size());
  for (int rd = 0; rd < rounds; ++rd)
    for (size_t i = 0; i < vs.size(); ++i) {
      vs[i].run(false);
      CK(hipEventRecord(t0, 0));
      for (int q = 0; q < reps; ++q) vs[i].run(false);
      CK(hipEventRecord(t1, 0));
      CK(hipEventSynchronize(t1));
      float m = 0;
      CK(hipEventElapsedTime(&m, t0, t1));
      ms[i].push_back(m / reps);
    }
  const double blocks = (double)n * bs::kBlocks;
  std::printf("\n%llu packets x %u counter blocks (1350 B), keystream only (XOR-folded)\n",
              (unsigned long long)n, bs::kBlocks);
  for (size_t i = 0; i < vs.size(); ++i) {
    std::vector<float> s = ms[i];
    std::sort(s.begin(), s.end());
    const double sec = s[s.size() / 2] * 1e-3;
    std::printf("%-30s median %9.1f us  %8.1f GB/s of keystream  %7.2f Gblocks/s\n",
                vs[i].name.c_str(), sec * 1e6, blocks * 16 / sec / 1e9, blocks / sec / 1e9);
  }
  return 0;
}
