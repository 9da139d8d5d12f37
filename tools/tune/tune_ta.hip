// tune_ta.hip — the texture-address (TA) cost model of 16-B vector loads on
// gfx950, which bounds the FEC kernels: per CU, how many
// cycles does one wave-wide load instruction occupy, depending on its active
// lanes, alignment and width?  Every variant re-reads an L2-resident buffer
// (2 MiB per XCD, so HBM is out of the picture) from 16 waves per CU, 64
// loads per lane; time -> load instructions per CU per microsecond.
//   A full64  : 64 lanes, consecutive 16-B windows (1 KiB per instruction)
//   B half32  : 32 active lanes (exec mask), consecutive
//   C quarter : 16 active lanes
//   D unalign : 64 lanes, windows at +2 B (the fixed kernel's rows)
//   E bcast   : 64 lanes, one address
//   F dwordx2 : 64 lanes x 8 B, consecutive
//   G dword   : 64 lanes x 4 B
//   H scatter : 64 lanes, 16 B each from 64 different 128-B lines
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_ta.hip -o tools/tune/build/tune_ta
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kIters = 64;

template <int V>
__global__ __launch_bounds__(256) void ta_kernel(const uint8_t* buf, uint32_t span, uint32_t* sink) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = (blockIdx.x * 4u + (threadIdx.x >> 6));
  uint32_t acc = 0;
  uint32_t base = (wave * 4096u) % span;
  const bool active = V == 1 ? lane < 32u : V == 2 ? lane < 16u : true;
  if (active) {
#pragma unroll 8
    for (int i = 0; i < kIters; ++i) {
      const uint32_t b = (base + (uint32_t)i * 1024u) % span;
      if constexpr (V <= 2) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(buf + b + 16u * lane);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      } else if constexpr (V == 3) {
        u32x4 v;
        __builtin_memcpy(&v, buf + b + 2u + 16u * lane, 16);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      } else if constexpr (V == 4) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(buf + b);
        acc ^= v.x ^ v.y ^ v.z ^ v.w ^ lane;
      } else if constexpr (V == 5) {
        const u32x2 v = *reinterpret_cast<const u32x2*>(buf + b + 8u * lane);
        acc ^= v.x ^ v.y;
      } else if constexpr (V == 6) {
        acc ^= *reinterpret_cast<const uint32_t*>(buf + b + 4u * lane);
      } else {
        const u32x4 v = *reinterpret_cast<const u32x4*>(buf + (b + 128u * lane) % span);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads
}

int main(int argc, char** argv) {
  const uint32_t span = 2u << 20;  // 2 MiB: L2-resident on every XCD
  uint8_t* buf;
  uint32_t* sink;
  if (hipMalloc(&buf, span + 4096) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 2;
  (void)hipMemset(buf, 1, span + 4096);
  const int blocks = 256 * 4 * 8;  // 4 blocks (16 waves) per CU, 8 rounds
  const char* names[] = {"A full64 (16 B x 64, consecutive)", "B half32 (32 active lanes)",
                         "C quarter (16 active lanes)",       "D unaligned +2 B (64 lanes)",
                         "E broadcast (64 lanes, 1 address)", "F dwordx2 (8 B x 64)",
                         "G dword (4 B x 64)",                "H scatter (64 lines)"};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int V = 0; V < 8; ++V) {
    auto launch = [&] {
      switch (V) {
        case 0: hipLaunchKernelGGL(ta_kernel<0>, dim3(blocks), dim3(256), 0, 0, buf, span, sink); break;
        case 1: hipLaunchKernelGGL(ta_kernel<1>, dim3(blocks), dim3(256), 0, 0, buf, span, sink); break;
        case 2: hipLaunchKernelGGL(ta_kernel<2>, dim3(blocks), dim3(256), 0, 0, buf, span, sink); break;
        case 3: hipLaunchKernelGGL(ta_kernel<3>, dim3(blocks), dim3(256), 0, 0, buf, span, sink); break;
        case 4: hipLaunchKernelGGL(ta_kernel<4>, dim3(blocks), dim3(256), 0, 0, buf, span, sink); break;
        case 5: hipLaunchKernelGGL(ta_kernel<5>, dim3(blocks), dim3(256), 0, 0, buf, span, sink); break;
        case 6: hipLaunchKernelGGL(ta_kernel<6>, dim3(blocks), dim3(256), 0, 0, buf, span, sink); break;
        default: hipLaunchKernelGGL(ta_kernel<7>, dim3(blocks), dim3(256), 0, 0, buf, span, sink); break;
      }
    };
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 10; ++r) launch();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double instr_per_cu = (double)blocks * 4 * kIters * 10 / 256;
    const double us = ms * 1e3;
    std::printf("%-36s %8.3f ms  %7.1f load instr / CU / us  (%.1f cycles each at 2.4 GHz)\n",
                names[V], ms / 10, instr_per_cu / us, 2400.0 * us / instr_per_cu);
  }
  return 0;
}
