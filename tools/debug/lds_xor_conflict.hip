// lds_xor_conflict.hip — does a wave's ds_xor_b32 give the right result when
// several of its lanes hit the SAME LDS address in one instruction?  (The
// ragged flat-window kernels: idle lanes XORed into one spare window gave
// wrong parity in other windows, profiles/round2/tune_rw_f.txt.)
//
// Each wave owns an LDS array of 368 dwords (the component-major accumulator,
// 92 windows x 4).  Pattern P decides each lane's target window per
// instruction; every lane XORs a per-(wave, instr, lane) random value into
// the 4 components of its window (4 ds_xor_b32, offsets 0/368/736/1104 B, as
// ragged_flat_kernel does).  The host recomputes every wave's final array.
//   P0: lane l -> window l (no two lanes alike)
//   P1: lanes < A -> window l, lanes >= A -> window 91 (64-A lanes alike)
//   P2: all 64 lanes -> window 91
//   P3: lane l -> window l/2 (pairs alike)
//   P4: lane l -> window (l + 64*it) % 91, it = instruction (no conflicts)
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/debug/lds_xor_conflict.hip -o tools/debug/build/lds_xor_conflict
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kWin = 92, kInstr = 10, kWaves = 4;

__device__ __host__ inline uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__device__ __host__ inline uint32_t target(int P, uint32_t lane, uint32_t it, uint32_t A) {
  switch (P) {
    case 0: return lane;
    case 1: return lane < A ? lane : 91u;
    case 2: return 91u;
    case 3: return lane / 2u;
    default: return (lane + 64u * it) % 91u;
  }
}

template <int FENCE>
__global__ __launch_bounds__(256) void k(uint32_t* out, int P, uint32_t A) {
  __shared__ uint32_t acc[kWaves][4 * kWin];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t w = blockIdx.x * kWaves + wv;
  for (uint32_t i = lane; i < 4u * kWin; i += 64u) acc[wv][i] = 0u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uint32_t v[kInstr][4], t[kInstr];
#pragma unroll
  for (int it = 0; it < kInstr; ++it) {
    t[it] = target(P, lane, it, A);
    for (int c = 0; c < 4; ++c) v[it][c] = hash32(w * 0x9E3779B9u ^ (it * 64u + lane) * 4u + c);
  }
#pragma unroll
  for (int it = 0; it < kInstr; ++it) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
      __hip_atomic_fetch_xor(&acc[wv][c * kWin + t[it]], v[it][c], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WAVEFRONT);
    if (FENCE) __builtin_amdgcn_s_waitcnt(0xC07F);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (uint32_t i = lane; i < 4u * kWin; i += 64u) out[(size_t)w * 4 * kWin + i] = acc[wv][i];
}

int main(int argc, char** argv) {
  const uint32_t blocks = argc > 1 ? atoi(argv[1]) : 65536;
  const uint32_t nw = blocks * kWaves;
  uint32_t* d;
  hipMalloc(&d, (size_t)nw * 4 * kWin * 4);
  std::vector<uint32_t> h((size_t)nw * 4 * kWin), want(4 * kWin);
  int rc = 0;
  struct Case { int P; uint32_t A; };
  const Case cases[] = {{0, 0}, {1, 48}, {1, 32}, {1, 8}, {2, 0}, {3, 0}, {4, 0}};
  for (int fence = 0; fence < 2; ++fence) {
    for (const Case& c : cases) {
      hipMemset(d, 0xFF, (size_t)nw * 4 * kWin * 4);
      if (fence) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, d, c.P, c.A);
      else hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, d, c.P, c.A);
      hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
      uint64_t bad_waves = 0, bad_words = 0, bad_spare = 0;
      for (uint32_t w = 0; w < nw; ++w) {
        std::fill(want.begin(), want.end(), 0u);
        for (uint32_t it = 0; it < kInstr; ++it)
          for (uint32_t lane = 0; lane < 64; ++lane)
            for (uint32_t cc = 0; cc < 4; ++cc)
              want[cc * kWin + target(c.P, lane, it, c.A)] ^=
                  hash32(w * 0x9E3779B9u ^ (it * 64u + lane) * 4u + cc);
        bool bad = false;
        for (uint32_t i = 0; i < 4 * kWin; ++i) {
          if (h[(size_t)w * 4 * kWin + i] != want[i]) {
            bad = true;
            ++bad_words;
            if (i % kWin == 91) ++bad_spare;
          }
        }
        bad_waves += bad;
      }
      std::printf("fence %d P%d A %2u: bad waves %llu of %u, bad words %llu (in window 91: %llu)\n",
                  fence, c.P, c.A, (unsigned long long)bad_waves, nw,
                  (unsigned long long)bad_words, (unsigned long long)bad_spare);
      if (bad_waves) rc = 1;
    }
  }
  return rc;
}
