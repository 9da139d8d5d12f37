// place_spread.hip — does spreading the concurrently active groups over the
// whole batch change the parity-placement modes (place_fixed.hip, DESIGN.md
// §4)?  Block b takes logical block (b % S) * ceil(n / S) + b / S (S = 8 is
// the XCD-aware order), so the groups in flight at any moment lie in S
// regions across the rows and the parity instead of one window.  For every
// parity destination of place_fixed: the product and S = 64, 512, 4096.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/place_spread.hip -o tools/tune/build/place_spread
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

// the product kernel's encode body (nt) with a spread block order
template <uint32_t S>
__global__ __launch_bounds__(256) void enc_spread(const uint8_t* rows, uint8_t* out, uint64_t n) {
  const uint32_t nb = gridDim.x, b = blockIdx.x;
  const uint32_t q = nb / S, r = nb % S, x = b % S;
  const uint32_t lb = (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + b / S;
  const uint32_t C = 85u, gpb = 3u;
  const uint32_t gl = threadIdx.x / C, t = threadIdx.x - gl * C;
  const uint64_t g = (uint64_t)lb * gpb + gl;
  if (gl >= gpb || g >= n) return;
  const uint32_t off = min(t * 16u, 1350u - 16u);
  const uint8_t* src = rows + g * 13500u + off;
  qfec::u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < 10; ++i) acc ^= qfec::ld16t<true>(src + i * 1350);
  qfec::st16t<true>(out + g * 1350u + off, acc);
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
  int mode = 0;
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
    const dim3 grid((uint32_t)((G + 2) / 3));
    if (mode == 1) hipLaunchKernelGGL(enc_spread<64>, grid, dim3(256), 0, 0, arena, out, G);
    if (mode == 2) hipLaunchKernelGGL(enc_spread<512>, grid, dim3(256), 0, 0, arena, out, G);
    if (mode == 3) hipLaunchKernelGGL(enc_spread<4096>, grid, dim3(256), 0, 0, arena, out, G);
    if (mode == 0) CK(qfec::launch_fixed(a, true, 0));
    CK(hipGetLastError());
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> res(4 * dst.size());
  for (auto& d : dst) run(d.second);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < 4 * dst.size(); ++i) {
      mode = (int)(i & 3);
      CK(hipEventRecord(e0, 0));
      for (int q = 0; q < reps; ++q) run(dst[i / 4].second);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      res[i].push_back((double)(rows_b + par_b) / (ms / reps * 1e-3) / 1e9);
    }
  const char* names[4] = {"product", "S=64", "S=512", "S=4096"};
  for (size_t i = 0; i < 4 * dst.size(); ++i) {
    auto v = res[i];
    std::sort(v.begin(), v.end());
    std::printf("%-34s %-8s %8.1f GB/s  (%.1f%% of 8 TB/s)  out=%p\n", dst[i / 4].first.c_str(),
                names[i & 3], v[v.size() / 2], v[v.size() / 2] / 80.0,
                (void*)dst[i / 4].second);
  }
  return 0;
}
