// last_vgpr_operand.hip — narrowing tools/debug/shift_operand_war.hip: in the
// failing round-1 sequence the instruction right before
//     v_lshlrev_b64 v[22:23], v55, v[22:23]      (v55 = last VGPR of 56)
// is `v_lshrrev_b64 v[0:1], v54, v[0:1]`, and the shift amount the failing
// instruction used equals the value just written to v0.  The load-only probe
// (unaligned_load_clobber.hip) never changes v55, so the suspect is the
// operand read of the wave's last VGPR right after a write of v0.
//
// Each variant (inline asm, explicit registers, kernel limited to NV VGPRs so
// the named "last" register is the allocation's last) sets the shift amount
// register R = 63, then one instruction writes v[0:1] with a sentinel whose
// low 6 bits are 5, then the 64-bit shift reads R:
//   out = v[22:23] << R   must be  in << 63;   with R read as v0: in << 5.
// Variants:
//   A: R = v55 of 56, v[0:1] written by v_lshrrev_b64 right before (the failing pair)
//   B: A with s_nop 1 between the two instructions
//   C: R = v40 of 56 (not the last register)
//   D: R = v55 of 56, v[0:1] written by v_mov_b32 ×2 right before
//   E: R = v55 of 56, nothing written to v0 in between (control)
//   F: R = v63 of 64 (last register of a 64-VGPR allocation), v[0:1] by v_lshrrev_b64
//   G: A with a 32-bit shift (v_lshlrev_b32 v22, v55, v22)
//   H: A after a 16-B global load + s_waitcnt (the failing build's timing)
// 1 or 8 blocks per CU (4 waves each).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/debug/last_vgpr_operand.hip -o tools/debug/build/last_vgpr_operand
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

#define PRE "v_mov_b32_e32 v22, %2\n\tv_mov_b32_e32 v23, %3\n\tv_mov_b32_e32 v0, 0\n\tv_mov_b32_e32 v1, 0\n\tv_mov_b32_e32 v54, 0\n\t"
#define POST "v_mov_b32_e32 %0, v22\n\tv_mov_b32_e32 %1, v23"

template <int V>
__device__ __forceinline__ void body(uint32_t lo, uint32_t hi, uint32_t sent, const uint8_t* p,
                                     uint32_t& o0, uint32_t& o1) {
  if constexpr (V == 0) {  // A
    asm volatile(PRE "v_mov_b32_e32 v55, 63\n\t"
                 "v_mov_b32_e32 v0, %4\n\tv_mov_b32_e32 v1, %4\n\t"
                 "s_nop 4\n\t"
                 "v_lshrrev_b64 v[0:1], v54, v[0:1]\n\t"
                 "v_lshlrev_b64 v[22:23], v55, v[22:23]\n\t" POST
                 : "=v"(o0), "=v"(o1) : "v"(lo), "v"(hi), "v"(sent)
                 : "v0", "v1", "v22", "v23", "v54", "v55");
  } else if constexpr (V == 1) {  // B
    asm volatile(PRE "v_mov_b32_e32 v55, 63\n\t"
                 "v_mov_b32_e32 v0, %4\n\tv_mov_b32_e32 v1, %4\n\t"
                 "s_nop 4\n\t"
                 "v_lshrrev_b64 v[0:1], v54, v[0:1]\n\t"
                 "s_nop 1\n\t"
                 "v_lshlrev_b64 v[22:23], v55, v[22:23]\n\t" POST
                 : "=v"(o0), "=v"(o1) : "v"(lo), "v"(hi), "v"(sent)
                 : "v0", "v1", "v22", "v23", "v54", "v55");
  } else if constexpr (V == 2) {  // C
    asm volatile(PRE "v_mov_b32_e32 v40, 63\n\t"
                 "v_mov_b32_e32 v0, %4\n\tv_mov_b32_e32 v1, %4\n\t"
                 "s_nop 4\n\t"
                 "v_lshrrev_b64 v[0:1], v54, v[0:1]\n\t"
                 "v_lshlrev_b64 v[22:23], v40, v[22:23]\n\t" POST
                 : "=v"(o0), "=v"(o1) : "v"(lo), "v"(hi), "v"(sent)
                 : "v0", "v1", "v22", "v23", "v40", "v54");
  } else if constexpr (V == 3) {  // D
    asm volatile(PRE "v_mov_b32_e32 v55, 63\n\t"
                 "s_nop 4\n\t"
                 "v_mov_b32_e32 v0, %4\n\tv_mov_b32_e32 v1, %4\n\t"
                 "v_lshlrev_b64 v[22:23], v55, v[22:23]\n\t" POST
                 : "=v"(o0), "=v"(o1) : "v"(lo), "v"(hi), "v"(sent)
                 : "v0", "v1", "v22", "v23", "v54", "v55");
  } else if constexpr (V == 4) {  // E
    asm volatile(PRE "v_mov_b32_e32 v55, 63\n\t"
                 "v_mov_b32_e32 v0, %4\n\tv_mov_b32_e32 v1, %4\n\t"
                 "s_nop 4\n\t"
                 "v_lshrrev_b64 v[26:27], v54, v[0:1]\n\t"
                 "v_lshlrev_b64 v[22:23], v55, v[22:23]\n\t" POST
                 : "=v"(o0), "=v"(o1) : "v"(lo), "v"(hi), "v"(sent)
                 : "v0", "v1", "v22", "v23", "v26", "v27", "v54", "v55");
  } else if constexpr (V == 5) {  // F
    asm volatile(PRE "v_mov_b32_e32 v63, 63\n\t"
                 "v_mov_b32_e32 v0, %4\n\tv_mov_b32_e32 v1, %4\n\t"
                 "s_nop 4\n\t"
                 "v_lshrrev_b64 v[0:1], v54, v[0:1]\n\t"
                 "v_lshlrev_b64 v[22:23], v63, v[22:23]\n\t" POST
                 : "=v"(o0), "=v"(o1) : "v"(lo), "v"(hi), "v"(sent)
                 : "v0", "v1", "v22", "v23", "v54", "v63");
  } else if constexpr (V == 6) {  // G
    asm volatile(PRE "v_mov_b32_e32 v55, 31\n\t"
                 "v_mov_b32_e32 v0, %4\n\tv_mov_b32_e32 v1, %4\n\t"
                 "s_nop 4\n\t"
                 "v_lshrrev_b64 v[0:1], v54, v[0:1]\n\t"
                 "v_lshlrev_b32_e32 v22, v55, v22\n\t"
                 "v_mov_b32_e32 v23, 0\n\t" POST
                 : "=v"(o0), "=v"(o1) : "v"(lo), "v"(hi), "v"(sent)
                 : "v0", "v1", "v22", "v23", "v54", "v55");
  } else {  // H
    asm volatile(PRE "v_mov_b32_e32 v55, 63\n\t"
                 "global_load_dwordx4 v[24:27], %5, off nt\n\t"
                 "v_mov_b32_e32 v0, %4\n\tv_mov_b32_e32 v1, %4\n\t"
                 "s_waitcnt vmcnt(0)\n\t"
                 "v_lshrrev_b64 v[0:1], v54, v[0:1]\n\t"
                 "v_lshlrev_b64 v[22:23], v55, v[22:23]\n\t" POST
                 : "=v"(o0), "=v"(o1) : "v"(lo), "v"(hi), "v"(sent), "v"(p)
                 : "v0", "v1", "v22", "v23", "v24", "v25", "v26", "v27", "v54", "v55", "memory");
  }
}

template <int V>
__device__ __forceinline__ void probe_loop(const uint8_t* buf, uint64_t n16, int iters,
                                           uint32_t* res) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t bad = 0, as_v0 = 0;
  for (int it = 0; it < iters; ++it) {
    const uint64_t w = (tid * 0x9E3779B97F4A7C15ull + (uint64_t)it * 0xBF58476D1CE4E5B9ull) % n16;
    const uint32_t lo = (uint32_t)(w * 2654435761u) | 1u, hi = (uint32_t)(w >> 17);
    const uint32_t sent = ((uint32_t)it << 6) | 5u;  // low 6 bits 5
    uint32_t o0, o1;
    body<V>(lo, hi, sent, buf + w * 16 + (w & 7), o0, o1);
    const uint64_t in = ((uint64_t)hi << 32) | lo;
    const uint64_t want = V == 6 ? (uint64_t)(lo << 31) : in << 63;
    const uint64_t got = ((uint64_t)o1 << 32) | o0;
    if (got != want) {
      ++bad;
      as_v0 += got == (V == 6 ? (uint64_t)(lo << 5) : in << 5);
    }
  }
  if (bad) {
    atomicAdd(&res[0], bad);
    atomicAdd(&res[1], as_v0);
  }
}

template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(56))) void probe56(
    const uint8_t* buf, uint64_t n16, int iters, uint32_t* res) {
  probe_loop<V>(buf, n16, iters, res);
}
template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(64))) void probe64(
    const uint8_t* buf, uint64_t n16, int iters, uint32_t* res) {
  probe_loop<V>(buf, n16, iters, res);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 256;
  const uint64_t nbytes = 1ull << 32, n16 = nbytes / 16 - 4;
  uint8_t* buf;
  CK(hipMalloc(&buf, nbytes));
  CK(hipMemset(buf, 0x3c, nbytes));
  uint32_t* res;
  CK(hipMalloc(&res, 8));
  struct Var {
    const char* name;
    void (*k)(const uint8_t*, uint64_t, int, uint32_t*);
  } vs[] = {
      {"A v55/56 after v_lshrrev_b64 v[0:1]", probe56<0>},
      {"B A + s_nop 1", probe56<1>},
      {"C v40/56", probe56<2>},
      {"D v55/56 after v_mov v0,v1", probe56<3>},
      {"E v55/56, v0 not written (control)", probe56<4>},
      {"F v63/64 after v_lshrrev_b64 v[0:1]", probe64<5>},
      {"G A with a 32-bit shift", probe56<6>},
      {"H A after a 16-B load + wait", probe56<7>},
  };
  for (int bpc : {8, 1}) {
    const dim3 grid(256 * bpc), blk(256);
    const int it = iters * (bpc == 1 ? 8 : 1);
    for (const auto& v : vs) {
      CK(hipMemset(res, 0, 8));
      hipLaunchKernelGGL(v.k, grid, blk, 0, 0, buf, n16, it, res);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      uint32_t r[2];
      CK(hipMemcpy(r, res, 8, hipMemcpyDeviceToHost));
      std::printf("%d blk/CU %-40s ops %10llu  wrong %8u  (shift amount = v0: %u)\n", bpc, v.name,
                  (unsigned long long)grid.x * 256ull * it, r[0], r[1]);
    }
  }
  return 0;
}
