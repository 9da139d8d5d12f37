// unaligned_load_clobber.hip — tools/debug/shift_operand_war.hip replays the
// failing round-1 ragged build's instruction sequence and gets wrong results
// only while the shift amount lives in v55, the last VGPR of a 56-VGPR
// allocation, and then that register holds the low dword of the 16-B window
// the wave just loaded into v[22:25].  Is it the load that writes the
// wave's last VGPR?
//
// Each lane puts sentinels in the allocation's last VGPR (v55 under
// amdgpu_num_vgpr(56)) and in v40, issues ONE global load into v[22:25]
// (or v[22:23] / v22), waits, and reads the sentinels back.  Variants: the
// load's byte misalignment (aligned 16 B, +1, +2, +4, +8, random), nt or
// default cache policy, width (dwordx4, dwordx2, dword), and 1 or 8 blocks
// per CU.  A changed sentinel is classified against the loaded bytes
// (dword 0 of the window, the dword before it, the aligned dword holding
// the first byte).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/debug/unaligned_load_clobber.hip -o tools/debug/build/unaligned_load_clobber
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

// MIS: byte offset added to a 16-B aligned address (-1 = random 0..15)
// W: 4 = dwordx4, 2 = dwordx2, 1 = dword.  NT: nt bit.
template <int MIS, int W, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(56))) void clobber_kernel(
    const uint8_t* buf, uint64_t n16, int iters, uint32_t* res) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t n55 = 0, n40 = 0, d0 = 0, dprev = 0, dal = 0;
  for (int it = 0; it < iters; ++it) {
    const uint64_t w = (tid * 0x9E3779B97F4A7C15ull + (uint64_t)it * 0xBF58476D1CE4E5B9ull) % n16;
    const uint32_t mis = MIS >= 0 ? (uint32_t)MIS : (uint32_t)(w >> 40) & 15u;
    const uint8_t* p = buf + 16 + w * 16 + mis;
    const uint64_t addr = (uint64_t)p;
    const uint32_t s55 = 0x5A5A0000u ^ (uint32_t)tid, s40 = 0xA5A50000u ^ (uint32_t)it;
    uint32_t o55, o40;
    if constexpr (W == 4) {
      if constexpr (NT)
        asm volatile("v_mov_b32_e32 v55, %2\n\t"
                     "v_mov_b32_e32 v40, %3\n\t"
                     "global_load_dwordx4 v[22:25], %4, off nt\n\t"
                     "s_waitcnt vmcnt(0)\n\t"
                     "v_mov_b32_e32 %0, v55\n\t"
                     "v_mov_b32_e32 %1, v40"
                     : "=v"(o55), "=v"(o40)
                     : "v"(s55), "v"(s40), "v"(addr)
                     : "v22", "v23", "v24", "v25", "v40", "v55", "memory");
      else
        asm volatile("v_mov_b32_e32 v55, %2\n\t"
                     "v_mov_b32_e32 v40, %3\n\t"
                     "global_load_dwordx4 v[22:25], %4, off\n\t"
                     "s_waitcnt vmcnt(0)\n\t"
                     "v_mov_b32_e32 %0, v55\n\t"
                     "v_mov_b32_e32 %1, v40"
                     : "=v"(o55), "=v"(o40)
                     : "v"(s55), "v"(s40), "v"(addr)
                     : "v22", "v23", "v24", "v25", "v40", "v55", "memory");
    } else if constexpr (W == 2) {
      asm volatile("v_mov_b32_e32 v55, %2\n\t"
                   "v_mov_b32_e32 v40, %3\n\t"
                   "global_load_dwordx2 v[22:23], %4, off nt\n\t"
                   "s_waitcnt vmcnt(0)\n\t"
                   "v_mov_b32_e32 %0, v55\n\t"
                   "v_mov_b32_e32 %1, v40"
                   : "=v"(o55), "=v"(o40)
                   : "v"(s55), "v"(s40), "v"(addr)
                   : "v22", "v23", "v40", "v55", "memory");
    } else {
      asm volatile("v_mov_b32_e32 v55, %2\n\t"
                   "v_mov_b32_e32 v40, %3\n\t"
                   "global_load_dword v22, %4, off nt\n\t"
                   "s_waitcnt vmcnt(0)\n\t"
                   "v_mov_b32_e32 %0, v55\n\t"
                   "v_mov_b32_e32 %1, v40"
                   : "=v"(o55), "=v"(o40)
                   : "v"(s55), "v"(s40), "v"(addr)
                   : "v22", "v40", "v55", "memory");
    }
    n40 += o40 != s40;
    if (o55 != s55) {
      ++n55;
      uint32_t a, b, c;
      __builtin_memcpy(&a, p, 4);
      __builtin_memcpy(&b, p - 4, 4);
      __builtin_memcpy(&c, (const uint8_t*)((uint64_t)p & ~3ull), 4);
      d0 += o55 == a;
      dprev += o55 == b;
      dal += o55 == c;
    }
  }
  if (n55 | n40) {
    atomicAdd(&res[0], n55);
    atomicAdd(&res[1], n40);
    atomicAdd(&res[2], d0);
    atomicAdd(&res[3], dprev);
    atomicAdd(&res[4], dal);
  }
}

struct Var {
  const char* name;
  void (*k)(const uint8_t*, uint64_t, int, uint32_t*);
};

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 64;
  const uint64_t nbytes = 1ull << 32, n16 = nbytes / 16 - 4;
  uint8_t* buf;
  CK(hipMalloc(&buf, nbytes));
  std::vector<uint8_t> h(1 << 24);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)((i * 2654435761u) >> 11);
  for (uint64_t o = 0; o < nbytes; o += h.size())
    CK(hipMemcpy(buf + o, h.data(), h.size(), hipMemcpyHostToDevice));
  uint32_t* res;
  CK(hipMalloc(&res, 32));
  const Var vs[] = {
      {"x4 nt  aligned", clobber_kernel<0, 4, true>},  {"x4 nt  +1", clobber_kernel<1, 4, true>},
      {"x4 nt  +2", clobber_kernel<2, 4, true>},       {"x4 nt  +4", clobber_kernel<4, 4, true>},
      {"x4 nt  +8", clobber_kernel<8, 4, true>},       {"x4 nt  random", clobber_kernel<-1, 4, true>},
      {"x4 def random", clobber_kernel<-1, 4, false>}, {"x2 nt  random", clobber_kernel<-1, 2, true>},
      {"x1 nt  random", clobber_kernel<-1, 1, true>},
  };
  for (int bpc : {8, 1}) {
    const dim3 grid(256 * bpc), blk(256);
    const int it = iters * (bpc == 1 ? 8 : 1);
    for (const auto& v : vs) {
      CK(hipMemset(res, 0, 32));
      hipLaunchKernelGGL(v.k, grid, blk, 0, 0, buf, n16, it, res);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      uint32_t r[5];
      CK(hipMemcpy(r, res, 20, hipMemcpyDeviceToHost));
      std::printf("%d blk/CU %-16s loads %10llu  v55 changed %7u (= dword0 %u, = dword before %u, "
                  "= aligned dword %u)  v40 changed %u\n",
                  bpc, v.name, (unsigned long long)grid.x * 256ull * it, r[0], r[2], r[3], r[4],
                  r[1]);
    }
  }
  return 0;
}
