// place_cpol.hip — cache-policy bits of the fixed encode's loads and parity
// stores against the parity-placement modes.  The encode body
// of the product (3 groups per 256-lane workgroup, 10 row loads per lane in
// flight) with its 16-B loads and stores as inline-asm VECTOR memory
// instructions carrying explicit gfx950 cache-policy bits (nt / sc0 / sc1),
// timed over several parity destinations (separate buffers, the head and the
// tail of the rows' allocation) in interleaved rounds of one process.
// Round 1 measured only nt vs default stores (place_policy.hip).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/place_cpol.hip -o tools/tune/build/place_cpol
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int LP, int SP>
__device__ __forceinline__ void enc_body(const uint8_t* src, uint8_t* dst) {
  u32x4 r0, r1, r2, r3, r4, r5, r6, r7, r8, r9;
#define L10(POLSTR)                                                                           \
  asm volatile("global_load_dwordx4 %0, %10, off offset:0 " POLSTR "\n\t"                    \
               "global_load_dwordx4 %1, %10, off offset:1350 " POLSTR "\n\t"                 \
               "global_load_dwordx4 %2, %10, off offset:2700 " POLSTR "\n\t"                 \
               "global_load_dwordx4 %3, %10, off offset:4050 " POLSTR "\n\t"                 \
               "global_load_dwordx4 %4, %11, off offset:0 " POLSTR "\n\t"                    \
               "global_load_dwordx4 %5, %11, off offset:1350 " POLSTR "\n\t"                 \
               "global_load_dwordx4 %6, %11, off offset:2700 " POLSTR "\n\t"                 \
               "global_load_dwordx4 %7, %11, off offset:4050 " POLSTR "\n\t"                 \
               "global_load_dwordx4 %8, %12, off offset:0 " POLSTR "\n\t"                    \
               "global_load_dwordx4 %9, %12, off offset:1350 " POLSTR "\n\t"                 \
               "s_waitcnt vmcnt(0)"                                                           \
               : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), \
                 "=&v"(r7), "=&v"(r8), "=&v"(r9)                                              \
               : "v"(src), "v"(src + 5400), "v"(src + 10800)                                  \
               : "memory")
  if constexpr (LP == 0) L10("nt");
  else if constexpr (LP == 1) L10("nt sc1");
  else if constexpr (LP == 2) L10("sc1");
  else L10("");
#undef L10
  const u32x4 acc = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ r8 ^ r9;
#define S1(POLSTR) asm volatile("global_store_dwordx4 %0, %1, off " POLSTR : : "v"(dst), "v"(acc) : "memory")
  if constexpr (SP == 0) S1("nt");
  else if constexpr (SP == 1) S1("nt sc0");
  else if constexpr (SP == 2) S1("nt sc1");
  else if constexpr (SP == 3) S1("nt sc0 sc1");
  else if constexpr (SP == 4) S1("sc0 sc1");
  else S1("sc1");
#undef S1
}

template <int LP, int SP>
__global__ __launch_bounds__(256) void enc_cpol(const uint8_t* rows, uint8_t* out, uint64_t n) {
  const uint32_t C = 85u, gpb = 3u;
  const uint32_t gl = threadIdx.x / C, t = threadIdx.x - gl * C;
  const uint64_t g = (uint64_t)blockIdx.x * gpb + gl;
  if (gl >= gpb || g >= n) return;
  const uint32_t off = min(t * 16u, 1350u - 16u);
  enc_body<LP, SP>(rows + g * 13500u + off, out + g * 1350u + off);
}

__global__ void fill(uint8_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8;
       i += (uint64_t)gridDim.x * blockDim.x)
    reinterpret_cast<uint64_t*>(p)[i] = i * 0x9E3779B97F4A7C15ull;
}

__global__ void ref_enc(const uint8_t* rows, uint8_t* out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * 1350u) return;
  const uint64_t g = i / 1350u, j = i - g * 1350u;
  uint8_t a = 0;
  for (int r = 0; r < 10; ++r) a ^= rows[g * 13500u + r * 1350u + j];
  out[i] = a;
}

int main(int argc, char** argv) {
  const uint64_t G = 1 << 20, k = 10, L = 1350;
  const uint64_t rows_b = G * k * L, par_b = G * L;
  const int reps = argc > 1 ? atoi(argv[1]) : 5, rounds = argc > 2 ? atoi(argv[2]) : 3;
  const uint64_t MB = 1ull << 20, front = (par_b + 2 * MB) & ~(2 * MB - 1);
  const uint64_t rows_end = front + ((rows_b + 2 * MB) & ~(2 * MB - 1));
  uint8_t* base;
  CK(hipMalloc(&base, rows_end + 4096 * MB + par_b + 2 * MB));
  uint8_t* rows = base + front;
  std::vector<uint8_t*> outs(3);
  for (auto& o : outs) CK(hipMalloc(&o, par_b + 4096));
  uint8_t* want;
  CK(hipMalloc(&want, par_b));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, rows, rows_b);
  hipLaunchKernelGGL(ref_enc, dim3((uint32_t)((par_b + 255) / 256)), dim3(256), 0, 0, rows, want,
                     G);
  CK(hipDeviceSynchronize());
  std::vector<std::pair<std::string, uint8_t*>> dst = {
      {"head", base}, {"sep1", outs[0]}, {"sep2", outs[1]}, {"sep3", outs[2]},
      {"tail4G", base + rows_end + 4096 * MB}};
  struct K {
    std::string name;
    void (*k)(const uint8_t*, uint8_t*, uint64_t);
  };
  std::vector<K> ks = {
      {"ld nt / st nt (product)", enc_cpol<0, 0>}, {"ld nt / st nt sc0", enc_cpol<0, 1>},
      {"ld nt / st nt sc1", enc_cpol<0, 2>},       {"ld nt / st nt sc0 sc1", enc_cpol<0, 3>},
      {"ld nt / st sc0 sc1", enc_cpol<0, 4>},      {"ld nt / st sc1", enc_cpol<0, 5>},
      {"ld nt sc1 / st nt", enc_cpol<1, 0>},       {"ld sc1 / st nt", enc_cpol<2, 0>},
      {"ld dflt / st nt", enc_cpol<3, 0>},
  };
  // correctness of every variant (a byte compare on the device via host copy)
  std::vector<uint8_t> h_want(par_b), h_got(par_b);
  CK(hipMemcpy(h_want.data(), want, par_b, hipMemcpyDeviceToHost));
  const dim3 grid((uint32_t)((G + 2) / 3)), blk(256);
  for (auto& kk : ks) {
    CK(hipMemset(outs[0], 0, par_b));
    hipLaunchKernelGGL(kk.k, grid, blk, 0, 0, rows, outs[0], G);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h_got.data(), outs[0], par_b, hipMemcpyDeviceToHost));
    std::printf("%-26s exact: %s\n", kk.name.c_str(), h_got == h_want ? "yes" : "NO");
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> res(ks.size() * dst.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t d = 0; d < dst.size(); ++d)
      for (size_t i = 0; i < ks.size(); ++i) {
        hipLaunchKernelGGL(ks[i].k, grid, blk, 0, 0, rows, dst[d].second, G);
        CK(hipEventRecord(e0, 0));
        for (int q = 0; q < reps; ++q)
          hipLaunchKernelGGL(ks[i].k, grid, blk, 0, 0, rows, dst[d].second, G);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        res[d * ks.size() + i].push_back((double)(rows_b + par_b) / (ms / reps * 1e-3) / 8e12);
      }
  std::printf("%-26s", "frac of 8 TB/s (median)");
  for (auto& d : dst) std::printf(" %8s", d.first.c_str());
  std::printf("\n");
  for (size_t i = 0; i < ks.size(); ++i) {
    std::printf("%-26s", ks[i].name.c_str());
    for (size_t d = 0; d < dst.size(); ++d) {
      auto v = res[d * ks.size() + i];
      std::sort(v.begin(), v.end());
      std::printf(" %8.4f", v[v.size() / 2]);
    }
    std::printf("\n");
  }
  return 0;
}
