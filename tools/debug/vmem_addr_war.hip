// vmem_addr_war.hip — does a VALU instruction that overwrites a vector load's
// ADDRESS VGPRs right after the load issues corrupt the load on gfx950?
//
// Found while chasing wrong parity in one build of the ragged flat-window
// kernel: the failing build, alone among semantically identical
// builds, issues `global_load_dwordx4 v[18:21], v[12:13]` and then at once
// `v_lshrrev_b64 v[12:13], ...` — a 64-bit shift writing the load's address
// pair in the next instruction.  Each variant below issues a 16-B load, then
// (inline asm, nothing between) one instruction that overwrites the address
// pair, then waits; every lane checks the 16 bytes it got against the buffer
// at its original address.
//   V0: v_lshrrev_b64 addr, 0, other      (the failing build's pattern)
//   V1: v_lshl_add_u64 addr, other, 0, 0  (64-bit add, seen in passing builds)
//   V2: v_mov_b64 addr, other
//   V3: s_nop 0, then V0
//   V4: s_nop 4, then V0
//   V5: no overwrite (control)
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/debug/vmem_addr_war.hip -o tools/debug/build/vmem_addr_war
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int V>
__global__ __launch_bounds__(256) void war_kernel(const uint8_t* buf, uint64_t n16, int iters,
                                                  uint32_t* bad) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t nbad = 0;
  for (int it = 0; it < iters; ++it) {
    // a pseudo-random 16-B window per lane and iteration, at an odd offset
    uint64_t w = (tid * 0x9E3779B97F4A7C15ull + (uint64_t)it * 0xBF58476D1CE4E5B9ull) % n16;
    const uint8_t* p = buf + w * 16 + (w & 7);
    uint64_t addr = (uint64_t)p;
    // another VALID window of the buffer: a load that picked up the new address
    // value reads wrong bytes instead of faulting
    const uint64_t other = (uint64_t)(buf + ((w * 7919u + 12345u) % n16) * 16 + 3);
    u32x4 v;
    if constexpr (V == 0) {
      asm volatile("global_load_dwordx4 %0, %1, off\n\t"
                   "v_lshrrev_b64 %1, 0, %2\n\t"
                   "s_waitcnt vmcnt(0)"
                   : "=&v"(v), "+&v"(addr) : "v"(other) : "memory");
    } else if constexpr (V == 1) {
      asm volatile("global_load_dwordx4 %0, %1, off\n\t"
                   "v_lshl_add_u64 %1, %2, 0, 0\n\t"
                   "s_waitcnt vmcnt(0)"
                   : "=&v"(v), "+&v"(addr) : "v"(other) : "memory");
    } else if constexpr (V == 2) {
      asm volatile("global_load_dwordx4 %0, %1, off\n\t"
                   "v_mov_b64 %1, %2\n\t"
                   "s_waitcnt vmcnt(0)"
                   : "=&v"(v), "+&v"(addr) : "v"(other) : "memory");
    } else if constexpr (V == 3) {
      asm volatile("global_load_dwordx4 %0, %1, off\n\t"
                   "s_nop 0\n\t"
                   "v_lshrrev_b64 %1, 0, %2\n\t"
                   "s_waitcnt vmcnt(0)"
                   : "=&v"(v), "+&v"(addr) : "v"(other) : "memory");
    } else if constexpr (V == 4) {
      asm volatile("global_load_dwordx4 %0, %1, off\n\t"
                   "s_nop 4\n\t"
                   "v_lshrrev_b64 %1, 0, %2\n\t"
                   "s_waitcnt vmcnt(0)"
                   : "=&v"(v), "+&v"(addr) : "v"(other) : "memory");
    } else {
      asm volatile("global_load_dwordx4 %0, %1, off\n\t"
                   "s_waitcnt vmcnt(0)"
                   : "=&v"(v), "+&v"(addr) :  : "memory");
    }
    u32x4 want;
    __builtin_memcpy(&want, p, 16);
    if (v.x != want.x || v.y != want.y || v.z != want.z || v.w != want.w) ++nbad;
  }
  if (nbad) atomicAdd(bad, nbad);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 64;
  const uint64_t bytes = 1ull << 30;
  uint8_t* buf;
  uint32_t* bad;
  if (hipMalloc(&buf, bytes + 64) != hipSuccess || hipMalloc(&bad, 4) != hipSuccess) return 2;
  std::vector<uint8_t> h(bytes + 64);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)((i * 2654435761u) >> 7);
  (void)hipMemcpy(buf, h.data(), h.size(), hipMemcpyHostToDevice);
  const uint64_t n16 = bytes / 16 - 1;
  const dim3 grid(16384), blk(256);
  const char* names[] = {"V0 v_lshrrev_b64 overwrites addr", "V1 v_lshl_add_u64 overwrites addr",
                         "V2 v_mov_b64 overwrites addr", "V3 s_nop 0 + v_lshrrev_b64",
                         "V4 s_nop 4 + v_lshrrev_b64", "V5 control (no overwrite)"};
  int rc = 0;
  for (int rep = 0; rep < 2; ++rep) {
    for (int V = 0; V < 6; ++V) {
      (void)hipMemset(bad, 0, 4);
      switch (V) {
        case 0: hipLaunchKernelGGL(war_kernel<0>, grid, blk, 0, 0, buf, n16, iters, bad); break;
        case 1: hipLaunchKernelGGL(war_kernel<1>, grid, blk, 0, 0, buf, n16, iters, bad); break;
        case 2: hipLaunchKernelGGL(war_kernel<2>, grid, blk, 0, 0, buf, n16, iters, bad); break;
        case 3: hipLaunchKernelGGL(war_kernel<3>, grid, blk, 0, 0, buf, n16, iters, bad); break;
        case 4: hipLaunchKernelGGL(war_kernel<4>, grid, blk, 0, 0, buf, n16, iters, bad); break;
        default: hipLaunchKernelGGL(war_kernel<5>, grid, blk, 0, 0, buf, n16, iters, bad); break;
      }
      uint32_t hb = 0;
      if (hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost) != hipSuccess) return 3;
      std::printf("rep %d %-36s wrong loads %u of %llu\n", rep, names[V], hb,
                  (unsigned long long)grid.x * blk.x * iters);
      if (hb && V == 5) rc = 1;
    }
  }
  return rc;
}
