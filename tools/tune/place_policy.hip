// place_policy.hip — does the cache policy of the parity stores change the
// parity-placement modes (place_fixed.hip)?  For every parity
// destination of place_fixed, the product encode (nt loads + nt stores) and
// the same kernel with default-policy stores (nt loads) are timed side by
// side.  Interleaved rounds in one process.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/place_policy.hip -o tools/tune/build/place_policy
#include "../../libquic_amd/csrc/qfec_kernels.hip"

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

// the product kernel's encode body with a choice of store policy
template <bool NTS>
__global__ __launch_bounds__(256) void enc_policy(const uint8_t* rows, uint8_t* out, uint64_t n) {
  const uint32_t C = 85u, gpb = 3u;
  const uint32_t gl = threadIdx.x / C, t = threadIdx.x - gl * C;
  const uint64_t g = (uint64_t)blockIdx.x * gpb + gl;
  if (gl >= gpb || g >= n) return;
  const uint32_t off = min(t * 16u, 1350u - 16u);
  const uint8_t* src = rows + g * 13500u + off;
  qfec::u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < 10; ++i) acc ^= qfec::ld16t<true>(src + i * 1350);
  qfec::st16t<NTS>(out + g * 1350u + off, acc);
}

__global__ void fill(uint8_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8;
       i += (uint64_t)gridDim.x * blockDim.x)
    reinterpret_cast<uint64_t*>(p)[i] = i * 0x9E3779B97F4A7C15ull;
}

int main(int argc, char** argv) {
  const uint64_t G = 1 << 20, k = 10, L = 1350;
  const uint64_t rows_b = G * k * L, par_b = G * L;
  const int reps = argc > 1 ? atoi(argv[1]) : 10, rounds = argc > 2 ? atoi(argv[2]) : 5;
  // arena = [parity slot | rows | gap ... parity slots at growing offsets]
  const uint64_t MB = 1ull << 20, front = (par_b + 2 * MB) & ~(2 * MB - 1);
  const uint64_t rows_end = front + ((rows_b + 2 * MB) & ~(2 * MB - 1));
  const uint64_t gaps[] = {0, 64 * MB, 4096 * MB};
  uint8_t* base;
  CK(hipMalloc(&base, rows_end + 4096 * MB + par_b + 2 * MB));
  uint8_t* arena = base + front;  // rows
  std::vector<uint8_t*> outs(4);
  for (auto& o : outs) CK(hipMalloc(&o, par_b + 4096));
  uint32_t* d_err;
  CK(hipMalloc(&d_err, 4));
  CK(hipMemset(d_err, 0, 4));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, arena, rows_b);
  CK(hipDeviceSynchronize());
  std::vector<std::pair<std::string, uint8_t*>> dst = {
      {"arena head (parity before rows)", base},
      {"separate #1", outs[0]}, {"separate #2", outs[1]}, {"separate #3", outs[2]},
      {"separate #4", outs[3]}};
  for (uint64_t g : gaps)
    dst.push_back({"arena tail + " + std::to_string(g / MB) + " MiB", base + rows_end + g});
  bool xcd = false;
  auto run = [&](uint8_t* out) {
    qfec::FixedArgs a{};
    a.rows = arena;
    a.out = out;
    a.row_stride = L;
    a.group_stride = k * L;
    a.parity_stride = L;
    a.out_stride = L;
    a.n_groups = G;
    a.k = k;
    a.L = L;
    a.err = d_err;
    if (xcd) {
      hipLaunchKernelGGL(enc_policy<false>, dim3((uint32_t)((G + 2) / 3)), dim3(256), 0, 0, arena,
                         out, G);
      CK(hipGetLastError());
    } else {
      CK(qfec::launch_fixed(a, true, 0));
    }
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> res(2 * dst.size());
  for (auto& d : dst) run(d.second);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < 2 * dst.size(); ++i) {
      xcd = (i & 1) != 0;
      CK(hipEventRecord(e0, 0));
      for (int q = 0; q < reps; ++q) run(dst[i / 2].second);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      res[i].push_back((double)(rows_b + par_b) / (ms / reps * 1e-3) / 1e9);
    }
  for (size_t i = 0; i < 2 * dst.size(); ++i) {
    auto v = res[i];
    std::sort(v.begin(), v.end());
    std::printf("%-34s %-8s %8.1f GB/s  (%.1f%% of 8 TB/s)  out=%p\n", dst[i / 2].first.c_str(),
                (i & 1) ? "st-dflt" : "product", v[v.size() / 2], v[v.size() / 2] / 80.0,
                (void*)dst[i / 2].second);
  }
  return 0;
}
