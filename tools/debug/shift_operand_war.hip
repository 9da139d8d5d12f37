// shift_operand_war.hip — replays, in inline asm with the same registers, the
// instruction sequence of the failing round-1 ragged build
// (ragged_xor_kernel<recover, nt, U = 4, ACC = 2> at 9ecab67, unroll slot 0:
// tools/debug/anomaly_diag.hip showed its wrong groups are explained, window
// by window, as the funnel shift `(w1 << 1) << v55` having used the low dword
// of the 16-B window just loaded into v[22:25] as its shift amount instead of
// v55 — DESIGN.md §4):
//
//   global_load_dwordx4 v[22:25], v[0:1], off nt
//   v_cmp_lt_u32_e64 s[16:17], 7, v52            ; sh > 7
//   v_lshlrev_b32 v54, 3, v52                    ; s = 8 sh
//   v_bitop3_b32 v55, v54, 63, 56 bitop3:0x6c    ; 63 - (s & 56)
//   v_add_u32 v53, ...                           ; (unrelated)
//   s_waitcnt vmcnt(0)
//   v_cndmask_b32_e64 v11, v25, 0, s[16:17]  ... v0, v22, v24
//   v_lshlrev_b64 v[22:23], 1, v[10:11]
//   v_lshrrev_b64 v[0:1], v54, v[0:1]
//   v_lshlrev_b64 v[22:23], v55, v[22:23]        ; <- the read that went wrong
//   v_or_b32 v1, v23, v1 / v_or_b32 v0, v22, v0 / v_lshrrev_b64 v[10:11], v54, v[10:11]
//
// Every lane loads a pseudo-random 16-B window of a large buffer (sh = 0:
// r0/r1 must equal the window) and counts r0/r1 mismatches, and how many of
// them match "shift amount = loaded dword 0".  Variants:
//   V0: the sequence as above, the kernel limited to 56 VGPRs (v55 the last)
//   V1: V0 with s_nop 7 between s_waitcnt and the first v_cndmask
//   V2: V0 with the shift amount in v40 instead of v55
//   V3: V0 without v_bitop3 (v55 = 63 by v_mov_b32 before the load)
//   V4: V0 with the load's destination not overwritten (v_lshlrev_b64 into v[26:27])
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/debug/shift_operand_war.hip -o tools/debug/build/shift_operand_war
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

#define SEQ_HEAD                                                   \
  "global_load_dwordx4 v[22:25], v[0:1], off nt\n\t"               \
  "v_cmp_lt_u32_e64 s[16:17], 7, v52\n\t"                          \
  "v_lshlrev_b32_e32 v54, 3, v52\n\t"

#define SEQ_MID                                                    \
  "v_add_u32_e32 v53, 0xfffff3f0, v54\n\t"                         \
  "s_waitcnt vmcnt(0)\n\t"

#define SEQ_SEL                                                    \
  "v_cndmask_b32_e64 v11, v25, 0, s[16:17]\n\t"                    \
  "v_cndmask_b32_e64 v10, v24, 0, s[16:17]\n\t"                    \
  "v_cndmask_b32_e64 v1, v23, v25, s[16:17]\n\t"                   \
  "v_cndmask_b32_e64 v0, v22, v24, s[16:17]\n\t"

template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(56))) void replay_kernel(
    const uint8_t* buf, uint64_t n16, int iters, uint32_t* bad) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t nbad = 0, nexpl = 0;
  for (int it = 0; it < iters; ++it) {
    const uint64_t w = (tid * 0x9E3779B97F4A7C15ull + (uint64_t)it * 0xBF58476D1CE4E5B9ull) % n16;
    const uint8_t* p = buf + w * 16 + (w & 7);
    uint64_t r0 = (uint64_t)p, r1;
    const uint32_t sh = 0;
    if constexpr (V == 0) {
      asm volatile(SEQ_HEAD "v_bitop3_b32 v55, v54, 63, 56 bitop3:0x6c\n\t" SEQ_MID SEQ_SEL
                   "v_lshlrev_b64 v[22:23], 1, v[10:11]\n\t"
                   "v_lshrrev_b64 v[0:1], v54, v[0:1]\n\t"
                   "v_lshlrev_b64 v[22:23], v55, v[22:23]\n\t"
                   "v_or_b32_e32 v1, v23, v1\n\t"
                   "v_or_b32_e32 v0, v22, v0\n\t"
                   "v_lshrrev_b64 v[10:11], v54, v[10:11]"
                   : "+{v[0:1]}"(r0), "={v[10:11]}"(r1)
                   : "{v52}"(sh)
                   : "v22", "v23", "v24", "v25", "v53", "v54", "v55", "s16", "s17", "memory");
    } else if constexpr (V == 1) {
      asm volatile(SEQ_HEAD "v_bitop3_b32 v55, v54, 63, 56 bitop3:0x6c\n\t" SEQ_MID
                   "s_nop 7\n\t" SEQ_SEL
                   "v_lshlrev_b64 v[22:23], 1, v[10:11]\n\t"
                   "v_lshrrev_b64 v[0:1], v54, v[0:1]\n\t"
                   "v_lshlrev_b64 v[22:23], v55, v[22:23]\n\t"
                   "v_or_b32_e32 v1, v23, v1\n\t"
                   "v_or_b32_e32 v0, v22, v0\n\t"
                   "v_lshrrev_b64 v[10:11], v54, v[10:11]"
                   : "+{v[0:1]}"(r0), "={v[10:11]}"(r1)
                   : "{v52}"(sh)
                   : "v22", "v23", "v24", "v25", "v53", "v54", "v55", "s16", "s17", "memory");
    } else if constexpr (V == 2) {
      asm volatile(SEQ_HEAD "v_bitop3_b32 v40, v54, 63, 56 bitop3:0x6c\n\t" SEQ_MID SEQ_SEL
                   "v_lshlrev_b64 v[22:23], 1, v[10:11]\n\t"
                   "v_lshrrev_b64 v[0:1], v54, v[0:1]\n\t"
                   "v_lshlrev_b64 v[22:23], v40, v[22:23]\n\t"
                   "v_or_b32_e32 v1, v23, v1\n\t"
                   "v_or_b32_e32 v0, v22, v0\n\t"
                   "v_lshrrev_b64 v[10:11], v54, v[10:11]"
                   : "+{v[0:1]}"(r0), "={v[10:11]}"(r1)
                   : "{v52}"(sh)
                   : "v22", "v23", "v24", "v25", "v40", "v53", "v54", "s16", "s17", "memory");
    } else if constexpr (V == 3) {
      asm volatile("v_mov_b32_e32 v55, 63\n\t" SEQ_HEAD SEQ_MID SEQ_SEL
                   "v_lshlrev_b64 v[22:23], 1, v[10:11]\n\t"
                   "v_lshrrev_b64 v[0:1], v54, v[0:1]\n\t"
                   "v_lshlrev_b64 v[22:23], v55, v[22:23]\n\t"
                   "v_or_b32_e32 v1, v23, v1\n\t"
                   "v_or_b32_e32 v0, v22, v0\n\t"
                   "v_lshrrev_b64 v[10:11], v54, v[10:11]"
                   : "+{v[0:1]}"(r0), "={v[10:11]}"(r1)
                   : "{v52}"(sh)
                   : "v22", "v23", "v24", "v25", "v53", "v54", "v55", "s16", "s17", "memory");
    } else {
      asm volatile(SEQ_HEAD "v_bitop3_b32 v55, v54, 63, 56 bitop3:0x6c\n\t" SEQ_MID SEQ_SEL
                   "v_lshlrev_b64 v[26:27], 1, v[10:11]\n\t"
                   "v_lshrrev_b64 v[0:1], v54, v[0:1]\n\t"
                   "v_lshlrev_b64 v[26:27], v55, v[26:27]\n\t"
                   "v_or_b32_e32 v1, v27, v1\n\t"
                   "v_or_b32_e32 v0, v26, v0\n\t"
                   "v_lshrrev_b64 v[10:11], v54, v[10:11]"
                   : "+{v[0:1]}"(r0), "={v[10:11]}"(r1)
                   : "{v52}"(sh)
                   : "v22", "v23", "v24", "v25", "v26", "v27", "v53", "v54", "v55", "s16", "s17",
                     "memory");
    }
    // reference: the same window by ordinary loads
    uint64_t w0, w1;
    __builtin_memcpy(&w0, p, 8);
    __builtin_memcpy(&w1, p + 8, 8);
    if (r0 != w0 || r1 != w1) {
      ++nbad;
      const uint32_t k = ((uint32_t)w0 & 63u) + 1u;  // shift amount = loaded dword 0
      if (k < 64u && r0 == (w0 | (w1 << k))) ++nexpl;
    }
  }
  if (nbad) {
    atomicAdd(&bad[0], nbad);
    atomicAdd(&bad[1], nexpl);
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 64;
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  const uint64_t nbytes = 1ull << 32, n16 = nbytes / 16 - 1;
  uint8_t* buf;
  CK(hipMalloc(&buf, nbytes));
  std::vector<uint8_t> h(1 << 24);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)((i * 2654435761u) >> 11);
  for (uint64_t o = 0; o < nbytes; o += h.size()) CK(hipMemcpy(buf + o, h.data(), h.size(), hipMemcpyHostToDevice));
  uint32_t* bad;
  CK(hipMalloc(&bad, 8));
  const dim3 grid(256 * 8 * 4), blk(256);  // 8 blocks per CU
  const char* names[] = {"V0 replay (v55 last VGPR)", "V1 s_nop 7 after the wait",
                         "V2 shift amount in v40", "V3 no v_bitop3 (v_mov 63 before the load)",
                         "V4 load registers not overwritten"};
  for (int r = 0; r < rounds; ++r)
    for (int v = 0; v < 5; ++v) {
      CK(hipMemset(bad, 0, 8));
      switch (v) {
        case 0: hipLaunchKernelGGL(replay_kernel<0>, grid, blk, 0, 0, buf, n16, iters, bad); break;
        case 1: hipLaunchKernelGGL(replay_kernel<1>, grid, blk, 0, 0, buf, n16, iters, bad); break;
        case 2: hipLaunchKernelGGL(replay_kernel<2>, grid, blk, 0, 0, buf, n16, iters, bad); break;
        case 3: hipLaunchKernelGGL(replay_kernel<3>, grid, blk, 0, 0, buf, n16, iters, bad); break;
        default: hipLaunchKernelGGL(replay_kernel<4>, grid, blk, 0, 0, buf, n16, iters, bad); break;
      }
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      uint32_t hb[2];
      CK(hipMemcpy(hb, bad, 8, hipMemcpyDeviceToHost));
      std::printf("round %d %-44s wrong %u of %llu windows (%u as 'shift = loaded dword 0')\n", r,
                  names[v], hb[0], (unsigned long long)grid.x * 256ull * iters, hb[1]);
    }
  return 0;
}
