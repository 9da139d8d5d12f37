// place_2d.hip — is the placement mode of the fixed encode set
// by where the ROWS landed or where the PARITY landed?  Three separately
// allocated 14.2 GB row buffers (same bytes) x three parity buffers, the
// product encode timed for all nine pairs in interleaved rounds of one
// process.  A row-driven mode shows as rows that are slow with every parity
// buffer; a parity-driven one as a parity column slow with every rows.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/place_2d.hip -o tools/tune/build/place_2d
#include "../../libquic_amd/csrc/qfec_kernels.hip"

#include <algorithm>
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

__global__ __launch_bounds__(256) void write_only(uint8_t* p, uint64_t n16, uint32_t v) {
  const qfec::u32x4 x = {v, v, v, v};
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < n16; w += (uint64_t)gridDim.x * 256)
    qfec::st16t<true>(p + 16u * w, x);
}

__global__ void fill(uint8_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8;
       i += (uint64_t)gridDim.x * blockDim.x)
    reinterpret_cast<uint64_t*>(p)[i] = i * 0x9E3779B97F4A7C15ull;
}

int main(int argc, char** argv) {
  const uint64_t G = 1 << 20, k = 10, L = 1350;
  const uint64_t rows_b = G * k * L, par_b = G * L;
  const int reps = argc > 1 ? atoi(argv[1]) : 5, rounds = argc > 2 ? atoi(argv[2]) : 3;
  const int NR = 3, NP = 3;
  std::vector<uint8_t*> rows(NR), par(NP);
  for (auto& r : rows) {
    CK(hipMalloc(&r, rows_b));
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, r, rows_b);
  }
  for (auto& p : par) CK(hipMalloc(&p, par_b + 4096));
  uint32_t* d_err;
  CK(hipMalloc(&d_err, 4));
  CK(hipMemset(d_err, 0, 4));
  CK(hipDeviceSynchronize());
  auto run = [&](int i, int j) {
    qfec::FixedArgs a{};
    a.rows = rows[i];
    a.out = par[j];
    a.row_stride = L;
    a.group_stride = k * L;
    a.parity_stride = L;
    a.out_stride = L;
    a.n_groups = G;
    a.k = k;
    a.L = L;
    a.err = d_err;
    CK(qfec::launch_fixed(a, true, 0));
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> res(NR * NP);
  for (int r = 0; r < rounds; ++r)
    for (int i = 0; i < NR; ++i)
      for (int j = 0; j < NP; ++j) {
        run(i, j);
        CK(hipEventRecord(e0, 0));
        for (int q = 0; q < reps; ++q) run(i, j);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        res[i * NP + j].push_back((double)(rows_b + par_b) / (ms / reps * 1e-3) / 8e12);
      }
  // pure streaming read of each rows buffer, pure streaming write of each parity buffer
  uint8_t* sink;
  CK(hipMalloc(&sink, 4096));
  std::vector<double> rd(NR), wr(NP);
  for (int i = 0; i < NR; ++i) {
    std::vector<double> v;
    for (int q = 0; q < 5; ++q) {
      CK(hipEventRecord(e0, 0));
      CK(qfec::launch_stream_probe(rows[i], rows_b / 16 * 16, sink, false, 0));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.push_back(rows_b / (ms * 1e-3) / 8e12);
    }
    std::sort(v.begin(), v.end());
    rd[i] = v[2];
  }
  for (int j = 0; j < NP; ++j) {
    std::vector<double> v;
    for (int q = 0; q < 5; ++q) {
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(write_only, dim3(16384), dim3(256), 0, 0, par[j], par_b / 16, (uint32_t)q);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.push_back(par_b / (ms * 1e-3) / 8e12);
    }
    std::sort(v.begin(), v.end());
    wr[j] = v[2];
  }
  std::printf("frac of 8 TB/s (median)   ");
  for (int j = 0; j < NP; ++j) std::printf("   par%d", j);
  std::printf("\n");
  for (int i = 0; i < NR; ++i) {
    std::printf("rows%d read %.4f  ", i, rd[i]);
    for (int j = 0; j < NP; ++j) {
      auto v = res[i * NP + j];
      std::sort(v.begin(), v.end());
      std::printf(" %.4f", v[v.size() / 2]);
    }
    std::printf("\n");
  }
  std::printf("parity write-only:");
  for (int j = 0; j < NP; ++j) std::printf(" par%d %.4f", j, wr[j]);
  std::printf("\n");
  return 0;
}
