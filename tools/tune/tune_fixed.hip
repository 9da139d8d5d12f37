// tune_fixed.hip — variant/ceiling study for the fixed-shape FEC XOR kernel
// (10 x 1350 B rows, 1M groups).  Not product code: it includes the product
// kernels verbatim and times them next to experimental variants and streaming
// ceilings, interleaved in one process (cdna_hip_programming.md §5.4 rule 24).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_fixed.hip -o tools/tune/build/tune_fixed
#include "../../libquic_amd/csrc/qfec_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,            \
                   hipGetErrorString(e_));                                       \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

namespace tune {
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld(const uint8_t* p) {
  u32x4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ u32x4 ldnt(const uint8_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ void st(uint8_t* p, u32x4 v) { __builtin_memcpy(p, &v, 16); }
__device__ __forceinline__ void stnt(uint8_t* p, u32x4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

// Ceiling: 10 aligned streams -> 1 (out[j] = XOR_r in[r*M + j]).
__global__ __launch_bounds__(256) void ceil_10to1(const uint8_t* in, uint8_t* out, uint64_t M) {
  const uint64_t n16 = M / 16;
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < n16;
       j += (uint64_t)gridDim.x * 256) {
    u32x4 acc = ld(in + 16 * j);
#pragma unroll
    for (int r = 1; r < 10; ++r) acc ^= ld(in + r * M + 16 * j);
    st(out + 16 * j, acc);
  }
}

// Ceiling: plain copy (read B, write B).
__global__ __launch_bounds__(256) void ceil_copy(const uint8_t* in, uint8_t* out, uint64_t B) {
  const uint64_t n16 = B / 16;
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < n16;
       j += (uint64_t)gridDim.x * 256)
    st(out + 16 * j, ld(in + 16 * j));
}

// Ceiling: read only (XOR-reduce to one word per thread).
__global__ __launch_bounds__(256) void ceil_read(const uint8_t* in, uint8_t* out, uint64_t B) {
  const uint64_t n16 = B / 16;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < n16;
       j += (uint64_t)gridDim.x * 256)
    acc ^= ld(in + 16 * j);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[threadIdx.x] = 1;
}

// Variant: product mapping, block size BS, NT loads / NT stores options.
template <int BS, bool NTL, bool NTS>
__global__ __launch_bounds__(BS) void v_block(const uint8_t* rows, uint8_t* out, uint64_t n,
                                              uint32_t C, uint32_t gpb) {
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;
  const uint32_t t = tid - gl * C;
  const uint64_t g = (uint64_t)blockIdx.x * gpb + gl;
  if (gl >= gpb || g >= n) return;
  const uint32_t off = min(t * 16u, 1350u - 16u);
  const uint8_t* src = rows + g * 13500u + off;
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 10; ++i) acc ^= NTL ? ldnt(src + i * 1350) : ld(src + i * 1350);
  if (NTS)
    stnt(out + g * 1350u + off, acc);
  else
    st(out + g * 1350u + off, acc);
}

// Variant: persistent grid-stride, two group-sets in flight per iteration.
__global__ __launch_bounds__(256) void v_persist2(const uint8_t* rows, uint8_t* out, uint64_t n,
                                                  uint32_t C, uint32_t gpb) {
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;
  const uint32_t t = tid - gl * C;
  if (gl >= gpb) return;
  const uint32_t off = min(t * 16u, 1350u - 16u);
  const uint64_t nsets = (n + gpb - 1) / gpb;
  for (uint64_t s = blockIdx.x; s < nsets; s += 2ull * gridDim.x) {
    const uint64_t g0 = s * gpb + gl;
    const uint64_t g1 = (s + gridDim.x) * gpb + gl;
    const bool v0 = g0 < n, v1 = (s + gridDim.x) < nsets && g1 < n;
    u32x4 a0 = {0, 0, 0, 0}, a1 = {0, 0, 0, 0};
    u32x4 r0[10], r1[10];
    const uint8_t* s0 = rows + g0 * 13500u + off;
    const uint8_t* s1 = rows + g1 * 13500u + off;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      if (v0) r0[i] = ld(s0 + i * 1350);
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      if (v1) r1[i] = ld(s1 + i * 1350);
    }
    if (v0) {
#pragma unroll
      for (int i = 0; i < 10; ++i) a0 ^= r0[i];
      st(out + g0 * 1350u + off, a0);
    }
    if (v1) {
#pragma unroll
      for (int i = 0; i < 10; ++i) a1 ^= r1[i];
      st(out + g1 * 1350u + off, a1);
    }
  }
}

// Variant: aligned global loads; the unaligned 16-B window is assembled from
// two aligned 16-B loads (same cache lines) with byte funnel shifts.
__device__ __forceinline__ u32x4 funnel(u32x4 a, u32x4 b, uint32_t sh /*0..15 bytes*/) {
  uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  const uint32_t q = sh >> 2, r = (sh & 3u) * 8u;
  uint32_t o[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    uint32_t v = w[i];
    v = (q == 1) ? w[i + 1] : v;
    v = (q == 2) ? w[i + 2] : v;
    v = (q == 3) ? w[i + 3] : v;
    o[i] = v;
  }
  u32x4 res;
  res.x = r ? (uint32_t)((((uint64_t)o[1] << 32) | o[0]) >> r) : o[0];
  res.y = r ? (uint32_t)((((uint64_t)o[2] << 32) | o[1]) >> r) : o[1];
  res.z = r ? (uint32_t)((((uint64_t)o[3] << 32) | o[2]) >> r) : o[2];
  res.w = r ? (uint32_t)((((uint64_t)o[4] << 32) | o[3]) >> r) : o[3];
  return res;
}

__global__ __launch_bounds__(256) void v_aligned2(const uint8_t* rows, uint8_t* out, uint64_t n,
                                                  uint32_t C, uint32_t gpb) {
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;
  const uint32_t t = tid - gl * C;
  const uint64_t g = (uint64_t)blockIdx.x * gpb + gl;
  if (gl >= gpb || g >= n) return;
  const uint32_t off = min(t * 16u, 1350u - 16u);
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uintptr_t a = (uintptr_t)(rows + g * 13500u + i * 1350u + off);
    const uintptr_t al = a & ~(uintptr_t)15;
    const uint32_t sh = (uint32_t)(a & 15);
    u32x4 lo = ld((const uint8_t*)al);
    u32x4 hi = sh ? ld((const uint8_t*)al + 16) : lo;  // never past the row's last line
    acc ^= funnel(lo, hi, sh);
  }
  st(out + g * 1350u + off, acc);
}

// Variant: raw buffer loads/stores with explicit cache-policy aux bits
// (gfx94x/gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16).
template <int LAUX, int SAUX, int GPT>
__global__ __launch_bounds__(256) void v_buf(const uint8_t* rows, uint8_t* out, uint64_t n,
                                             uint32_t C, uint32_t gpb) {
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;
  const uint32_t t = tid - gl * C;
  if (gl >= gpb) return;
  const uint64_t gb = (uint64_t)blockIdx.x * gpb * GPT;  // first group of the block
  const uint64_t ng = min((uint64_t)gpb * GPT, n - gb);
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(rows + gb * 13500u), (short)0, (int)(ng * 13500u), 0x00020000);
  __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(out + gb * 1350u), (short)0, (int)(ng * 1350u), 0x00020000);
  const uint32_t off = min(t * 16u, 1350u - 16u);
  u32x4 acc[GPT];
  u32x4 r[GPT][10];
#pragma unroll
  for (int q = 0; q < GPT; ++q) {
    const uint32_t g = gl + q * gpb;
#pragma unroll
    for (int i = 0; i < 10; ++i)
      r[q][i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rs, g * 13500u + i * 1350u + off, 0, LAUX));
  }
#pragma unroll
  for (int q = 0; q < GPT; ++q) {
    acc[q] = r[q][0];
#pragma unroll
    for (int i = 1; i < 10; ++i) acc[q] ^= r[q][i];
    const uint32_t g = gl + q * gpb;
    if (g < ng)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, acc[q]), ws, g * 1350u + off, 0, SAUX);
  }
}

// Better ceilings: U independent 16-B loads in flight per lane, each block
// sweeping a contiguous 256*U*16-byte chunk per iteration.
template <int U>
__global__ __launch_bounds__(256) void ceil_read_u(const uint8_t* in, uint8_t* out, uint64_t B) {
  const uint64_t chunk = 256ull * U * 16;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t base = (uint64_t)blockIdx.x * chunk; base + chunk <= B;
       base += (uint64_t)gridDim.x * chunk) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld(in + base + (u * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[threadIdx.x] = 1;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void ceil_copy_u(const uint8_t* in, uint8_t* out, uint64_t B) {
  const uint64_t chunk = 256ull * U * 16;
  for (uint64_t base = (uint64_t)blockIdx.x * chunk; base + chunk <= B;
       base += (uint64_t)gridDim.x * chunk) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = NT ? ldnt(in + base + (u * 256 + threadIdx.x) * 16)
                : ld(in + base + (u * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT)
        stnt(out + base + (u * 256 + threadIdx.x) * 16, v[u]);
      else
        st(out + base + (u * 256 + threadIdx.x) * 16, v[u]);
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void ceil_read_nt(const uint8_t* in, uint8_t* out, uint64_t B) {
  const uint64_t chunk = 256ull * U * 16;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t base = (uint64_t)blockIdx.x * chunk; base + chunk <= B;
       base += (uint64_t)gridDim.x * chunk) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ldnt(in + base + (u * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[threadIdx.x] = 1;
}

// LDS-DMA read ceiling: every wave streams 1 KiB pieces into its own LDS ring
// (global_load_lds_dwordx4), U pieces in flight, then touches one dword.
template <int U, int AUX>
__global__ __launch_bounds__(256) void ceil_read_lds(const uint8_t* in, uint8_t* out, uint64_t B) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[4][U][1024];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t chunk = 256ull * U * 16;
  uint32_t acc = 0;
  for (uint64_t base = (uint64_t)blockIdx.x * chunk; base + chunk <= B;
       base += (uint64_t)gridDim.x * chunk) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_amdgcn_global_load_lds((const void*)(in + base + (u * 256 + threadIdx.x) * 16),
                                       (__attribute__((address_space(3))) void*)&ring[w][u][0],
                                       16, 0, AUX);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc ^= reinterpret_cast<const uint32_t*>(&ring[w][0][0])[lane];
  }
  if (acc == 0x12345678u) out[threadIdx.x] = 1;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void ceil_write(uint8_t* out, uint64_t B) {
  const uint64_t chunk = 256ull * U * 16;
  const u32x4 v = {threadIdx.x, 1u, 2u, 3u};
  for (uint64_t base = (uint64_t)blockIdx.x * chunk; base + chunk <= B;
       base += (uint64_t)gridDim.x * chunk) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT)
        stnt(out + base + (u * 256 + threadIdx.x) * 16, v);
      else
        st(out + base + (u * 256 + threadIdx.x) * 16, v);
    }
  }
}

// Persistent, software-pipelined: lanes keep the next group-set's 10 loads in
// flight while XOR-ing and storing the current one (nt loads and stores).
__global__ __launch_bounds__(256) void v_pipe(const uint8_t* rows, uint8_t* out, uint64_t n,
                                              uint32_t C, uint32_t gpb) {
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;
  const uint32_t t = tid - gl * C;
  if (gl >= gpb) return;
  const uint32_t off = min(t * 16u, 1350u - 16u);
  const uint64_t nsets = (n + gpb - 1) / gpb;
  uint64_t s = blockIdx.x;
  if (s >= nsets) return;
  u32x4 cur[10], nxt[10];
  {
    const uint64_t g = min(s * gpb + gl, n - 1);
#pragma unroll
    for (int i = 0; i < 10; ++i) cur[i] = ldnt(rows + g * 13500u + i * 1350u + off);
  }
  for (;;) {
    const uint64_t sn = s + gridDim.x;
    const bool more = sn < nsets;
    if (more) {
      const uint64_t g = min(sn * gpb + gl, n - 1);
#pragma unroll
      for (int i = 0; i < 10; ++i) nxt[i] = ldnt(rows + g * 13500u + i * 1350u + off);
    }
    u32x4 acc = cur[0];
#pragma unroll
    for (int i = 1; i < 10; ++i) acc ^= cur[i];
    const uint64_t g = s * gpb + gl;
    if (g < n) stnt(out + g * 1350u + off, acc);
    if (!more) break;
#pragma unroll
    for (int i = 0; i < 10; ++i) cur[i] = nxt[i];
    s = sn;
  }
}

// LDS-staged group tile: the block's GPB consecutive groups (GPB*13500 B,
// contiguous in HBM) arrive by 16-B-aligned nt LDS-DMA pieces; lanes then read
// their (unaligned) row windows from LDS as 3 x ds_read_b64 + byte funnel.
__device__ __forceinline__ u32x4 lds_read16(const uint8_t* tile, uint32_t a) {
  const uint32_t a8 = a & ~7u, sh = a & 7u;
  const uint64_t* q = reinterpret_cast<const uint64_t*>(tile + a8);
  const uint64_t x0 = q[0], x1 = q[1], x2 = q[2];
  const uint32_t w0 = (uint32_t)x0, w1 = (uint32_t)(x0 >> 32), w2 = (uint32_t)x1,
                 w3 = (uint32_t)(x1 >> 32), w4 = (uint32_t)x2, w5 = (uint32_t)(x2 >> 32);
  const bool hi = sh >= 4;
  const uint32_t r = sh & 3u;
  const uint32_t s0 = hi ? w1 : w0, s1 = hi ? w2 : w1, s2 = hi ? w3 : w2, s3 = hi ? w4 : w3,
                 s4 = hi ? w5 : w4;
  u32x4 o;
  o.x = __builtin_amdgcn_alignbyte(s1, s0, r);
  o.y = __builtin_amdgcn_alignbyte(s2, s1, r);
  o.z = __builtin_amdgcn_alignbyte(s3, s2, r);
  o.w = __builtin_amdgcn_alignbyte(s4, s3, r);
  return o;
}

template <int GPB, int AUX>
__global__ __launch_bounds__(256) void v_lds(const uint8_t* rows, uint8_t* out, uint64_t n) {
  constexpr uint32_t C = 85;
  constexpr uint32_t TILE = GPB * 13500u;
  __shared__ __attribute__((aligned(16))) uint8_t tile[TILE + 48];
  const uint64_t g0 = (uint64_t)blockIdx.x * GPB;
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C, t = tid - gl * C;
  const uint32_t off = min(t * 16u, 1334u);
  if (g0 + GPB >= n) {  // the block touching the buffer end: direct loads
    if (gl < GPB && g0 + gl < n) {
      const uint8_t* src = rows + (g0 + gl) * 13500u + off;
      u32x4 acc = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < 10; ++i) acc ^= ldnt(src + i * 1350u);
      stnt(out + (g0 + gl) * 1350u + off, acc);
    }
    return;
  }
  const uint64_t S = g0 * 13500u;
  const uint64_t A = S & ~15ull;
  const uint32_t head = (uint32_t)(S - A);
  const uint32_t nchunk = (head + TILE + 15u) / 16u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63u;
  for (uint32_t c0 = wave * 64u; c0 < nchunk; c0 += 256u) {
    const uint32_t c = c0 + lane;
    if (c < nchunk)
      __builtin_amdgcn_global_load_lds((const void*)(rows + A + 16ull * c),
                                       (__attribute__((address_space(3))) void*)&tile[c0 * 16u],
                                       16, 0, AUX);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (gl < GPB) {
    u32x4 acc = {0, 0, 0, 0};
    const uint32_t base = head + gl * 13500u + off;
#pragma unroll
    for (int i = 0; i < 10; ++i) acc ^= lds_read16(tile, base + i * 1350u);
    stnt(out + (g0 + gl) * 1350u + off, acc);
  }
}

// Mix ceiling: each block reads a contiguous, aligned 40 KiB tile (10 nt
// pieces per lane) and writes 4 KiB contiguous aligned (1 nt piece per lane):
// exactly the 10:1 byte mix of the FEC encode with ideal contiguity.
template <bool NTS>
__global__ __launch_bounds__(256) void ceil_mix10(const uint8_t* in, uint8_t* out, uint64_t tiles) {
  for (uint64_t b = blockIdx.x; b < tiles; b += gridDim.x) {
    const uint8_t* src = in + b * 40960u;
    u32x4 acc = ldnt(src + threadIdx.x * 16u);
    u32x4 v[9];
#pragma unroll
    for (int u = 1; u < 10; ++u) v[u - 1] = ldnt(src + (u * 256u + threadIdx.x) * 16u);
#pragma unroll
    for (int u = 0; u < 9; ++u) acc ^= v[u];
    if (NTS)
      stnt(out + b * 4096u + threadIdx.x * 16u, acc);
    else
      st(out + b * 4096u + threadIdx.x * 16u, acc);
  }
}

// Product mapping without the parity store (value kept live): read side only.
__global__ __launch_bounds__(256) void v_nostore(const uint8_t* rows, uint8_t* out, uint64_t n,
                                                 uint32_t C, uint32_t gpb) {
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;
  const uint32_t t = tid - gl * C;
  const uint64_t g = (uint64_t)blockIdx.x * gpb + gl;
  if (gl >= gpb || g >= n) return;
  const uint32_t off = min(t * 16u, 1350u - 16u);
  const uint8_t* src = rows + g * 13500u + off;
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 10; ++i) acc ^= ldnt(src + i * 1350);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9abcdef1u) out[g] = 1;
}

// Output-layout probes: same reads as the product, parity written to
// (MODE 0) g*PS (padded rows), (MODE 1) a 4 KiB slot per block.
template <int MODE, uint32_t PS>
__global__ __launch_bounds__(256) void v_outlayout(const uint8_t* rows, uint8_t* out, uint64_t n,
                                                   uint32_t C, uint32_t gpb) {
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;
  const uint32_t t = tid - gl * C;
  const uint64_t g = (uint64_t)blockIdx.x * gpb + gl;
  if (gl >= gpb || g >= n) return;
  const uint32_t off = min(t * 16u, 1350u - 16u);
  const uint8_t* src = rows + g * 13500u + off;
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 10; ++i) acc ^= ldnt(src + i * 1350);
  if (MODE == 0)
    stnt(out + g * PS + off, acc);
  else
    stnt(out + (uint64_t)blockIdx.x * 4096u + gl * 1350u + off, acc);
}

// Recover variants.  R_all: load every row AND the parity (k+1 loads, no
// address depends on missing[g]), drop row m with a select after the fact.
__global__ __launch_bounds__(256) void r_all(const uint8_t* rows, const uint8_t* par,
                                             const uint8_t* miss, uint8_t* out, uint64_t n,
                                             uint32_t C, uint32_t gpb) {
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;
  const uint32_t t = tid - gl * C;
  const uint64_t g = (uint64_t)blockIdx.x * gpb + gl;
  if (gl >= gpb || g >= n) return;
  const uint32_t off = min(t * 16u, 1350u - 16u);
  const uint8_t* src = rows + g * 13500u + off;
  u32x4 v[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) v[i] = ldnt(src + i * 1350);
  u32x4 acc = ldnt(par + g * 1350u + off);
  const uint32_t m = miss[g];
#pragma unroll
  for (int i = 0; i < 10; ++i) acc ^= (i == (int)m) ? u32x4{0, 0, 0, 0} : v[i];
  stnt(out + g * 1350u + off, acc);
}

// R_blockm: the block's missing indices arrive by one scalar 8-byte load of
// the aligned word that covers them (uniform), so no per-lane dependent load.
__global__ __launch_bounds__(256) void r_blockm(const uint8_t* rows, const uint8_t* par,
                                                const uint8_t* miss, uint8_t* out, uint64_t n,
                                                uint32_t C, uint32_t gpb) {
  const uint32_t tid = threadIdx.x;
  const uint32_t gl = tid / C;
  const uint32_t t = tid - gl * C;
  const uint64_t gb = (uint64_t)blockIdx.x * gpb;
  const uint64_t g = gb + gl;
  // 16 bytes starting at the 8-aligned word below gb cover gb..gb+gpb-1 (gpb <= 8)
  const uint64_t a8 = gb & ~7ull;
  const uint64_t* mw = reinterpret_cast<const uint64_t*>(miss + a8);
  const uint64_t w0 = __builtin_nontemporal_load(mw), w1 = (a8 + 8 < n) ? mw[1] : 0ull;
  if (gl >= gpb || g >= n) return;
  const uint32_t sh = (uint32_t)(g - a8);
  const uint32_t m = (uint32_t)(((sh < 8) ? (w0 >> (8 * sh)) : (w1 >> (8 * (sh - 8)))) & 0xFF);
  const uint32_t off = min(t * 16u, 1350u - 16u);
  const uint8_t* src = rows + g * 13500u + off;
  const uint8_t* pp = par + g * 1350u + off;
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 10; ++i) acc ^= ldnt(i == (int)m ? pp : src + i * 1350);
  stnt(out + g * 1350u + off, acc);
}

__global__ void fill(uint8_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n / 8;
       i += (uint64_t)gridDim.x * 256) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z ^= z >> 29;
    reinterpret_cast<uint64_t*>(p)[i] = z * 0xBF58476D1CE4E5B9ull;
  }
}

}  // namespace tune

int main(int argc, char** argv) {
  const uint64_t G = 1 << 20, k = 10, L = 1350;
  const uint64_t rows_b = G * k * L, par_b = G * L;
  const double alg = (double)(rows_b + par_b);
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  uint8_t *rows, *par, *out, *rows_pad, *miss;
  CK(hipMalloc(&rows, rows_b + 4096));
  CK(hipMalloc(&rows_pad, G * k * 1360 + 4096));
  CK(hipMalloc(&par, par_b + 4096));
  CK(hipMalloc(&out, par_b + 4096));
  CK(hipMalloc(&miss, G));
  CK(hipMemset(miss, 3, G));
  hipLaunchKernelGGL(tune::fill, dim3(8192), dim3(256), 0, 0, rows, rows_b);
  hipLaunchKernelGGL(tune::fill, dim3(8192), dim3(256), 0, 0, rows_pad, G * k * 1360);
  CK(hipDeviceSynchronize());
  uint32_t* d_err;
  CK(hipMalloc(&d_err, 4));
  CK(hipMemset(d_err, 0, 4));

  const uint32_t C = 85, gpb = 3;
  const uint64_t blocks = (G + gpb - 1) / gpb;
  struct V {
    std::string name;
    double bytes;
    std::function<void()> run;
  };
  std::vector<V> vs;
  auto prod = [&](bool nt, bool recover, uint64_t rs) {
    qfec::FixedArgs a{};
    a.rows = rs == L ? rows : rows_pad;
    a.parity = recover ? par : nullptr;
    a.missing = recover ? miss : nullptr;
    a.out = out;
    a.row_stride = rs;
    a.group_stride = k * rs;
    a.parity_stride = L;
    a.out_stride = L;
    a.n_groups = G;
    a.k = k;
    a.L = L;
    a.err = d_err;
    CK(qfec::launch_fixed(a, nt, 0));
  };
  vs.push_back({"product encode", alg, [&] { prod(false, false, L); }});
  vs.push_back({"product encode NT", alg, [&] { prod(true, false, L); }});
  vs.push_back({"product recover", alg, [&] { prod(false, true, L); }});
  vs.push_back({"product recover NT", alg, [&] { prod(true, true, L); }});
  vs.push_back({"r_all (k+1 loads, no addr dependency)", alg, [&] {
                  hipLaunchKernelGGL(tune::r_all, dim3(blocks), dim3(256), 0, 0, rows, par, miss,
                                     out, G, C, gpb);
                }});
  vs.push_back({"r_blockm (scalar missing word)", alg, [&] {
                  hipLaunchKernelGGL(tune::r_blockm, dim3(blocks), dim3(256), 0, 0, rows, par,
                                     miss, out, G, C, gpb);
                }});
  vs.push_back({"v_block<512>", alg, [&] {
                  hipLaunchKernelGGL((tune::v_block<512, false, false>), dim3((G + 5) / 6),
                                     dim3(512), 0, 0, rows, out, G, C, 6u);
                }});
  vs.push_back({"v_block<1024>", alg, [&] {
                  hipLaunchKernelGGL((tune::v_block<1024, false, false>), dim3((G + 11) / 12),
                                     dim3(1024), 0, 0, rows, out, G, C, 12u);
                }});
  vs.push_back({"v_block<256> NT store", alg, [&] {
                  hipLaunchKernelGGL((tune::v_block<256, false, true>), dim3(blocks), dim3(256), 0,
                                     0, rows, out, G, C, gpb);
                }});
  vs.push_back({"v_block<256> NT load+store", alg, [&] {
                  hipLaunchKernelGGL((tune::v_block<256, true, true>), dim3(blocks), dim3(256), 0,
                                     0, rows, out, G, C, gpb);
                }});
  vs.push_back({"v_block<256> NT load", alg, [&] {
                  hipLaunchKernelGGL((tune::v_block<256, true, false>), dim3(blocks), dim3(256), 0,
                                     0, rows, out, G, C, gpb);
                }});
#define BUFV(LA, SA, GPT)                                                                    \
  vs.push_back({"v_buf load" #LA " store" #SA " gpt" #GPT, alg, [&] {                          \
                  hipLaunchKernelGGL((tune::v_buf<LA, SA, GPT>), dim3((G + gpb * GPT - 1) /    \
                                                                       (gpb * GPT)),          \
                                     dim3(256), 0, 0, rows, out, G, C, gpb);                   \
                }});
  BUFV(0, 0, 1)
  BUFV(2, 2, 1)
  BUFV(0, 2, 1)
  BUFV(18, 2, 1)
  BUFV(2, 2, 2)
#undef BUFV
  const uint64_t M = par_b & ~15ull;
  const uint64_t RB = (rows_b / (256 * 16 * 16)) * (256 * 16 * 16);
  vs.push_back({"CEIL read U=4 grid 4096", (double)RB, [&] {
                  hipLaunchKernelGGL((tune::ceil_read_u<4>), dim3(4096), dim3(256), 0, 0, rows,
                                     out, RB);
                }});
  vs.push_back({"CEIL read U=8 grid 8192", (double)RB, [&] {
                  hipLaunchKernelGGL((tune::ceil_read_u<8>), dim3(8192), dim3(256), 0, 0, rows,
                                     out, RB);
                }});
  vs.push_back({"CEIL read U=16 grid 4096", (double)RB, [&] {
                  hipLaunchKernelGGL((tune::ceil_read_u<16>), dim3(4096), dim3(256), 0, 0, rows,
                                     out, RB);
                }});
  vs.push_back({"CEIL read NT U=8 grid 8192", (double)RB, [&] {
                  hipLaunchKernelGGL((tune::ceil_read_nt<8>), dim3(8192), dim3(256), 0, 0, rows,
                                     out, RB);
                }});
  vs.push_back({"CEIL read NT U=16 grid 4096", (double)RB, [&] {
                  hipLaunchKernelGGL((tune::ceil_read_nt<16>), dim3(4096), dim3(256), 0, 0, rows,
                                     out, RB);
                }});
  vs.push_back({"CEIL read NT U=8 base+2 (misaligned)", (double)RB, [&] {
                  hipLaunchKernelGGL((tune::ceil_read_nt<8>), dim3(8192), dim3(256), 0, 0,
                                     rows + 2, out, RB);
                }});
  vs.push_back({"CEIL read NT U=8 base+6 (misaligned)", (double)RB, [&] {
                  hipLaunchKernelGGL((tune::ceil_read_nt<8>), dim3(8192), dim3(256), 0, 0,
                                     rows + 6, out, RB);
                }});
  {
    const uint64_t tiles = rows_b / 40960u;
    const double mb = tiles * (40960.0 + 4096.0);
    vs.push_back({"CEIL mix 10:1 contiguous nt/nt grid 8192", mb, [&, tiles] {
                    hipLaunchKernelGGL((tune::ceil_mix10<true>), dim3(8192), dim3(256), 0, 0, rows,
                                       rows_pad, tiles);
                  }});
    vs.push_back({"CEIL mix 10:1 contiguous nt/plain grid 8192", mb, [&, tiles] {
                    hipLaunchKernelGGL((tune::ceil_mix10<false>), dim3(8192), dim3(256), 0, 0,
                                       rows, rows_pad, tiles);
                  }});
    vs.push_back({"CEIL mix 10:1 contiguous nt/nt 1 tile/block", mb, [&, tiles] {
                    hipLaunchKernelGGL((tune::ceil_mix10<true>), dim3((uint32_t)tiles), dim3(256),
                                       0, 0, rows, rows_pad, tiles);
                  }});
  }
  vs.push_back({"v_out parity stride 1408 (128B-aligned rows)", alg, [&] {
                  hipLaunchKernelGGL((tune::v_outlayout<0, 1408>), dim3(blocks), dim3(256), 0, 0,
                                     rows, rows_pad, G, C, gpb);
                }});
  vs.push_back({"v_out parity stride 1360", alg, [&] {
                  hipLaunchKernelGGL((tune::v_outlayout<0, 1360>), dim3(blocks), dim3(256), 0, 0,
                                     rows, rows_pad, G, C, gpb);
                }});
  vs.push_back({"v_out 4KiB slot per block", alg, [&] {
                  hipLaunchKernelGGL((tune::v_outlayout<1, 0>), dim3(blocks), dim3(256), 0, 0,
                                     rows, rows_pad, G, C, gpb);
                }});
  vs.push_back({"v_out parity stride 1350 (=product NT)", alg, [&] {
                  hipLaunchKernelGGL((tune::v_outlayout<0, 1350>), dim3(blocks), dim3(256), 0, 0,
                                     rows, rows_pad, G, C, gpb);
                }});
  vs.push_back({"v_out parity stride 1350 -> out buffer", alg, [&] {
                  hipLaunchKernelGGL((tune::v_outlayout<0, 1350>), dim3(blocks), dim3(256), 0, 0,
                                     rows, out, G, C, gpb);
                }});
  vs.push_back({"v_block<256> NT load+store -> rows_pad", alg, [&] {
                  hipLaunchKernelGGL((tune::v_block<256, true, true>), dim3(blocks), dim3(256), 0,
                                     0, rows, rows_pad, G, C, gpb);
                }});
  vs.push_back({"v_nostore (reads only, alg bytes=read)", (double)rows_b, [&] {
                  hipLaunchKernelGGL(tune::v_nostore, dim3(blocks), dim3(256), 0, 0, rows, out, G,
                                     C, gpb);
                }});
  vs.push_back({"v_lds<3> nt", alg, [&] {
                  hipLaunchKernelGGL((tune::v_lds<3, 2>), dim3((G + 2) / 3), dim3(256), 0, 0,
                                     rows, out, G);
                }});
  vs.push_back({"v_lds<3> default", alg, [&] {
                  hipLaunchKernelGGL((tune::v_lds<3, 0>), dim3((G + 2) / 3), dim3(256), 0, 0,
                                     rows, out, G);
                }});
  vs.push_back({"v_lds<2> nt", alg, [&] {
                  hipLaunchKernelGGL((tune::v_lds<2, 2>), dim3((G + 1) / 2), dim3(256), 0, 0,
                                     rows, out, G);
                }});
  for (int gr : {512}) {
    vs.push_back({"v_pipe grid=" + std::to_string(gr), alg, [&, gr] {
                    hipLaunchKernelGGL(tune::v_pipe, dim3(gr), dim3(256), 0, 0, rows, out, G, C,
                                       gpb);
                  }});
  }
  vs.push_back({"CEIL read LDS-DMA U=8", (double)RB, [&] {
                  hipLaunchKernelGGL((tune::ceil_read_lds<8, 0>), dim3(8192), dim3(256), 0, 0,
                                     rows, out, RB);
                }});
  vs.push_back({"CEIL read LDS-DMA U=8 nt", (double)RB, [&] {
                  hipLaunchKernelGGL((tune::ceil_read_lds<8, 2>), dim3(8192), dim3(256), 0, 0,
                                     rows, out, RB);
                }});
  vs.push_back({"CEIL read LDS-DMA U=16 nt", (double)RB, [&] {
                  hipLaunchKernelGGL((tune::ceil_read_lds<16, 2>), dim3(4096), dim3(256), 0, 0,
                                     rows, out, RB);
                }});
  vs.push_back({"CEIL write 7GB", (double)(RB / 2), [&] {
                  hipLaunchKernelGGL((tune::ceil_write<8, false>), dim3(8192), dim3(256), 0, 0,
                                     rows_pad, RB / 2);
                }});
  vs.push_back({"CEIL write NT 7GB", (double)(RB / 2), [&] {
                  hipLaunchKernelGGL((tune::ceil_write<8, true>), dim3(8192), dim3(256), 0, 0,
                                     rows_pad, RB / 2);
                }});
  const uint64_t HB = RB / 2;
  vs.push_back({"CEIL copy U=8 7GB", 2.0 * HB, [&] {
                  hipLaunchKernelGGL((tune::ceil_copy_u<8, false>), dim3(8192), dim3(256), 0, 0,
                                     rows, rows_pad, HB);
                }});
  vs.push_back({"CEIL copy U=8 NT 7GB", 2.0 * HB, [&] {
                  hipLaunchKernelGGL((tune::ceil_copy_u<8, true>), dim3(8192), dim3(256), 0, 0,
                                     rows, rows_pad, HB);
                }});
  vs.push_back({"CEIL 10->1 aligned streams", 11.0 * M, [&] {
                  hipLaunchKernelGGL(tune::ceil_10to1, dim3(8192), dim3(256), 0, 0, rows, out, M);
                }});

  {  // correctness of the LDS-staged variants against the product kernel
    std::vector<uint8_t> h1(par_b), h2(par_b);
    prod(true, false, L);
    CK(hipMemcpy(h1.data(), out, par_b, hipMemcpyDeviceToHost));
    for (int variant = 0; variant < 2; ++variant) {
      CK(hipMemset(out, 0, par_b));
      if (variant == 0)
        hipLaunchKernelGGL((tune::v_lds<3, 2>), dim3((G + 2) / 3), dim3(256), 0, 0, rows, out, G);
      else
        hipLaunchKernelGGL((tune::v_lds<2, 2>), dim3((G + 1) / 2), dim3(256), 0, 0, rows, out, G);
      CK(hipMemcpy(h2.data(), out, par_b, hipMemcpyDeviceToHost));
      std::printf("v_lds variant %d matches product: %s\n", variant,
                  h1 == h2 ? "yes" : "NO");
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> res(vs.size());
  for (auto& v : vs) v.run();  // warm
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(e0, 0));
      for (int q = 0; q < reps; ++q) vs[i].run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      res[i].push_back(vs[i].bytes / (ms / reps * 1e-3) / 1e9);
    }
  }
  std::printf("%-44s %10s %10s %8s\n", "variant", "med GB/s", "max GB/s", "%8TB/s");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = res[i];
    std::sort(v.begin(), v.end());
    std::printf("%-44s %10.1f %10.1f %7.1f%%\n", vs[i].name.c_str(), v[v.size() / 2], v.back(),
                v[v.size() / 2] / 80.0);
  }
  return 0;
}
