// last_vgpr_ops.hip — which instructions are affected by the last-VGPR operand
// read of tools/debug/last_vgpr_operand.hip (a 64-bit shift whose 32-bit
// amount is the allocation's last VGPR shifts by v0's value), and is it v0?
//
// Each variant sets the last register (v55 of a 56-VGPR kernel) to a known
// operand, v0 = X and v1 = Y (distinct), then runs ONE instruction reading the
// last register; the result is classified as right, "operand read as v0",
// "operand read as v1", or other.  8 blocks per CU (the failure needs
// several waves per SIMD).
//   I0 v_lshlrev_b64  v[22:23], v55, v[22:23]         (positive control)
//   I1 v_lshrrev_b64  v[22:23], v55, v[22:23]
//   I2 v_lshl_add_u64 v[22:23], v[22:23], v55, v[24:25]   (amount as src1)
//   I3 v_mad_u64_u32  v[22:23], s[20:21], v55, v24, v[26:27]
//   I4 v_cvt_f64_u32  v[22:23], v55
//   I5 v_mul_lo_u32   v22, v55, v24                    (32-bit control)
//   I6 v_lshlrev_b64  v[22:23], v55, v[22:23] in a 64-VGPR kernel (v55 not last)
//   I7 v_lshlrev_b64  v[22:23], v63, v[22:23] in a 64-VGPR kernel (v63 last)
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/debug/last_vgpr_ops.hip -o tools/debug/build/last_vgpr_ops
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

// operands: %2 = a (value in the last register), %3/%4 = lo/hi of the 64-bit
// input, %5 = X (v0), %6 = Y (v1), %7 = K (v24); output %0/%1 = v22/v23
#define SETUP(LAST)                                                                   \
  "v_mov_b32_e32 " LAST ", %2\n\tv_mov_b32_e32 v22, %3\n\tv_mov_b32_e32 v23, %4\n\t" \
  "v_mov_b32_e32 v24, %7\n\tv_mov_b32_e32 v25, %4\n\tv_mov_b32_e32 v26, %3\n\t"       \
  "v_mov_b32_e32 v27, %7\n\tv_mov_b32_e32 v0, %5\n\tv_mov_b32_e32 v1, %6\n\ts_nop 4\n\t"
#define OUT "\n\ts_nop 4\n\tv_mov_b32_e32 %0, v22\n\tv_mov_b32_e32 %1, v23"
#define OPS(LAST)                                                                    \
  : "=v"(o0), "=v"(o1)                                                               \
  : "v"(a), "v"(lo), "v"(hi), "v"(X), "v"(Y), "v"(K)                                 \
  : "v0", "v1", "v22", "v23", "v24", "v25", "v26", "v27", LAST, "s20", "s21"

__device__ __forceinline__ uint64_t ref(int V, uint32_t a, uint64_t in, uint32_t K) {
  const uint64_t acc = ((uint64_t)K << 32) | (uint32_t)in;  // v[26:27] = {lo, K}
  const uint64_t c = ((uint64_t)(uint32_t)(in >> 32) << 32) | K;  // v[24:25] = {K, hi}
  switch (V) {
    case 0: case 6: case 7: return in << (a & 63);
    case 1: return in >> (a & 63);
    case 2: return (in << (a & 7)) + c;
    case 3: return (uint64_t)a * K + acc;
    case 4: { double d = (double)a; uint64_t u; __builtin_memcpy(&u, &d, 8); return u; }
    default: return ((uint64_t)(uint32_t)(in >> 32) << 32) | (uint32_t)(a * K);
  }
}

template <int V>
__device__ __forceinline__ void run(uint32_t a, uint32_t lo, uint32_t hi, uint32_t X, uint32_t Y,
                                    uint32_t K, uint32_t& o0, uint32_t& o1) {
  if constexpr (V == 0)
    asm volatile(SETUP("v55") "v_lshlrev_b64 v[22:23], v55, v[22:23]" OUT OPS("v55"));
  else if constexpr (V == 1)
    asm volatile(SETUP("v55") "v_lshrrev_b64 v[22:23], v55, v[22:23]" OUT OPS("v55"));
  else if constexpr (V == 2)
    asm volatile(SETUP("v55") "v_lshl_add_u64 v[22:23], v[22:23], v55, v[24:25]" OUT OPS("v55"));
  else if constexpr (V == 3)
    asm volatile(SETUP("v55") "v_mad_u64_u32 v[22:23], s[20:21], v55, v24, v[26:27]" OUT OPS("v55"));
  else if constexpr (V == 4)
    asm volatile(SETUP("v55") "v_cvt_f64_u32_e32 v[22:23], v55" OUT OPS("v55"));
  else if constexpr (V == 5)
    asm volatile(SETUP("v55") "v_mul_lo_u32 v22, v55, v24" OUT OPS("v55"));
  else if constexpr (V == 6)  // v63 touched so that the allocation is 64
    asm volatile("v_mov_b32_e32 v63, 0\n\t" SETUP("v55") "v_lshlrev_b64 v[22:23], v55, v[22:23]" OUT
                 : "=v"(o0), "=v"(o1)
                 : "v"(a), "v"(lo), "v"(hi), "v"(X), "v"(Y), "v"(K)
                 : "v0", "v1", "v22", "v23", "v24", "v25", "v26", "v27", "v55", "v63", "s20", "s21");
  else
    asm volatile(SETUP("v63") "v_lshlrev_b64 v[22:23], v63, v[22:23]" OUT OPS("v63"));
}

template <int V>
__device__ __forceinline__ void loop(int iters, uint32_t* res) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t n_ok = 0, n_v0 = 0, n_v1 = 0, n_other = 0;
  for (int it = 0; it < iters; ++it) {
    const uint64_t h = (tid * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)it * 0xBF58476D1CE4E5B9ull);
    const uint32_t lo = (uint32_t)h | 1u, hi = (uint32_t)(h >> 32) | 0x10000u;
    // the last register's value and the two decoys differ in every field used
    uint32_t a = 40u + (uint32_t)(h >> 59), X = 0x3000u + 5u + (uint32_t)((h >> 20) & 0xF00u),
             Y = 0x7000u + 9u + (uint32_t)((h >> 28) & 0xF00u);
    if (V == 2) a = 3u, X = 0x3005u, Y = 0x7006u;
    const uint32_t K = (uint32_t)(h >> 13) | 3u;
    uint32_t o0, o1;
    run<V>(a, lo, hi, X, Y, K, o0, o1);
    const uint64_t in = ((uint64_t)hi << 32) | lo, got = ((uint64_t)o1 << 32) | o0;
    if (got == ref(V, a, in, K)) ++n_ok;
    else if (got == ref(V, X, in, K)) ++n_v0;
    else if (got == ref(V, Y, in, K)) ++n_v1;
    else ++n_other;
  }
  atomicAdd(&res[0], n_ok);
  atomicAdd(&res[1], n_v0);
  atomicAdd(&res[2], n_v1);
  atomicAdd(&res[3], n_other);
}

template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(56))) void k56(int iters,
                                                                                 uint32_t* res) {
  loop<V>(iters, res);
}
template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(64))) void k64(int iters,
                                                                                 uint32_t* res) {
  loop<V>(iters, res);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 256;
  uint32_t* res;
  CK(hipMalloc(&res, 16));
  struct Var {
    const char* name;
    void (*k)(int, uint32_t*);
  } vs[] = {
      {"I0 v_lshlrev_b64, amount v55 (last of 56)", k56<0>},
      {"I1 v_lshrrev_b64, amount v55 (last)", k56<1>},
      {"I2 v_lshl_add_u64, amount v55 (last)", k56<2>},
      {"I3 v_mad_u64_u32, src0 v55 (last)", k56<3>},
      {"I4 v_cvt_f64_u32, src v55 (last)", k56<4>},
      {"I5 v_mul_lo_u32, src0 v55 (last)", k56<5>},
      {"I6 v_lshlrev_b64, amount v55 (not last of 64)", k64<6>},
      {"I7 v_lshlrev_b64, amount v63 (last of 64)", k64<7>},
  };
  for (const auto& v : vs) {
    CK(hipMemset(res, 0, 16));
    hipLaunchKernelGGL(v.k, dim3(256 * 8), dim3(256), 0, 0, iters, res);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    uint32_t r[4];
    CK(hipMemcpy(r, res, 16, hipMemcpyDeviceToHost));
    std::printf("%-48s right %9u  read as v0 %8u  read as v1 %8u  other %8u\n", v.name, r[0], r[1],
                r[2], r[3]);
  }
  return 0;
}
