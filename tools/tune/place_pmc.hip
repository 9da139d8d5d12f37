// place_pmc.hip — what differs in the memory system between the slow and the
// fast placement mode of the fixed encode kernel?  The same
// rows are encoded into parity destinations known to land in different modes
// (the head of the rows' own allocation: always slow; separate buffers and
// the arena tail 4 GiB past the rows: mostly fast), `reps` launches each, in
// a fixed order, each launch timed by HIP events and printed with its
// dispatch index so that a rocprofv3 --pmc pass's per-dispatch counters can
// be matched to the destination (tools/place_pmc.py).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/place_pmc.hip -o tools/tune/build/place_pmc
#include "../../libquic_amd/csrc/qfec_kernels.hip"

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

__global__ void fill(uint8_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8;
       i += (uint64_t)gridDim.x * blockDim.x)
    reinterpret_cast<uint64_t*>(p)[i] = i * 0x9E3779B97F4A7C15ull;
}

int main(int argc, char** argv) {
  const uint64_t G = 1 << 20, k = 10, L = 1350;
  const uint64_t rows_b = G * k * L, par_b = G * L;
  const int reps = argc > 1 ? atoi(argv[1]) : 3;
  const uint64_t MB = 1ull << 20, front = (par_b + 2 * MB) & ~(2 * MB - 1);
  const uint64_t rows_end = front + ((rows_b + 2 * MB) & ~(2 * MB - 1));
  uint8_t* base;
  CK(hipMalloc(&base, rows_end + 4096 * MB + par_b + 2 * MB));
  uint8_t* rows = base + front;
  std::vector<uint8_t*> outs(3);
  for (auto& o : outs) CK(hipMalloc(&o, par_b + 4096));
  uint32_t* d_err;
  CK(hipMalloc(&d_err, 4));
  CK(hipMemset(d_err, 0, 4));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, rows, rows_b);
  CK(hipDeviceSynchronize());
  std::vector<std::pair<std::string, uint8_t*>> dst = {
      {"head", base}, {"sep1", outs[0]}, {"sep2", outs[1]}, {"sep3", outs[2]},
      {"tail4G", base + rows_end + 4096 * MB}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // dispatch 0 is the fill kernel
  int dispatch = 1;
  for (auto& d : dst) {
    for (int r = 0; r < reps; ++r) {
      qfec::FixedArgs a{};
      a.rows = rows;
      a.out = d.second;
      a.row_stride = L;
      a.group_stride = k * L;
      a.parity_stride = L;
      a.out_stride = L;
      a.n_groups = G;
      a.k = k;
      a.L = L;
      a.err = d_err;
      CK(hipEventRecord(e0, 0));
      CK(qfec::launch_fixed(a, true, 0));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("dispatch %d dst %s rep %d us %.1f frac %.4f out %p\n", dispatch++,
                  d.first.c_str(), r, ms * 1e3,
                  (double)(rows_b + par_b) / (ms * 1e-3) / 8e12, (void*)d.second);
    }
  }
  return 0;
}
