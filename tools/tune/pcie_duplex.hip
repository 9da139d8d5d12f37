// pcie_duplex.hip — the host link's one-way and both-ways ceilings, measured
// the ways the FEC path can move bytes (round 3's probe
// timed torch copy_ on two streams and reported 57.3 GB/s "shared", which the
// fused leg's 68 GB/s combined contradicted).
//
// Pinned host buffers (hipHostMalloc, device-mapped), device buffers; every
// figure is bytes moved / wall time between events (GB/s, 1e9), median of
// `reps` runs:
//   dma_h2d, dma_d2h        hipMemcpyAsync alone, one stream
//   dma_both                H2D and D2H at once on two non-blocking streams
//   dma_both_chunked        the same as 64-MiB chunks, 4 streams each way
//   dma_both_2streams_chunkN  N-MiB chunks, one stream each way
//   zc_read                 a kernel reading mapped host memory into HBM (the
//                           QFEC_PTR_MAPPED input side)
//   zc_write                a kernel writing HBM to mapped host memory
//   zc_read + dma_d2h       kernel reads one way while DMA copies the other
//   dma_h2d + zc_write      DMA in, kernel writes out
//   zc_both                 one kernel reads host->HBM while another writes HBM->host
// Prints one JSON line.  HSA_ENABLE_SDMA=0 in the environment moves the DMA
// copies to blit kernels (the runtime's other path); run both ways.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/pcie_duplex.hip \
//          -o tools/tune/build/pcie_duplex
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

// grid-stride 16-B copy; src or dst may be mapped host memory
__global__ __launch_bounds__(256) void copy16(const u32x4* __restrict__ src,
                                              u32x4* __restrict__ dst, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const size_t B = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024) << 20;  // MiB
  const int reps = argc > 2 ? atoi(argv[2]) : 7;
  const size_t chunk = 64ull << 20;
  uint8_t *h_in, *h_out, *d_in, *d_out;
  CK(hipHostMalloc(&h_in, B, hipHostMallocDefault));
  CK(hipHostMalloc(&h_out, B, hipHostMallocDefault));
  CK(hipMalloc(&d_in, B));
  CK(hipMalloc(&d_out, B));
  for (size_t i = 0; i < B; i += 4096) h_in[i] = (uint8_t)i;
  CK(hipMemset(d_out, 1, B));
  hipStream_t s[8];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int dev = 0, ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const uint32_t grid = (uint32_t)ncu * 8u;

  // runs f(stream list) with s[0] as the timing stream: every other stream
  // waits on e0 and s[0] waits on them at the end
  auto timed = [&](auto f, int nstreams) {
    std::vector<double> r;
    for (int q = 0; q < reps + 1; ++q) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s[0]));
      for (int i = 1; i < nstreams; ++i) CK(hipStreamWaitEvent(s[i], e0, 0));
      f();
      hipEvent_t done[8];
      for (int i = 1; i < nstreams; ++i) {
        CK(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
        CK(hipEventRecord(done[i], s[i]));
        CK(hipStreamWaitEvent(s[0], done[i], 0));
      }
      CK(hipEventRecord(e1, s[0]));
      CK(hipEventSynchronize(e1));
      for (int i = 1; i < nstreams; ++i) CK(hipEventDestroy(done[i]));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (q) r.push_back(ms * 1e-3);
    }
    return med(r);
  };
  const uint64_t n16 = B / 16;
  auto h2d = [&](hipStream_t st) { CK(hipMemcpyAsync(d_in, h_in, B, hipMemcpyHostToDevice, st)); };
  auto d2h = [&](hipStream_t st) { CK(hipMemcpyAsync(h_out, d_out, B, hipMemcpyDeviceToHost, st)); };
  auto zcr = [&](hipStream_t st) {
    hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, st, (const u32x4*)h_in, (u32x4*)d_in, n16);
  };
  auto zcw = [&](hipStream_t st) {
    hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, st, (const u32x4*)d_out, (u32x4*)h_out, n16);
  };
  const double g = B / 1e9;
  const double t_h2d = timed([&] { h2d(s[0]); }, 1);
  const double t_d2h = timed([&] { d2h(s[0]); }, 1);
  const double t_both = timed([&] { h2d(s[0]); d2h(s[1]); }, 2);
  const double t_chunk = timed([&] {
    for (size_t o = 0, c = 0; o < B; o += chunk, ++c) {
      const size_t n = std::min(chunk, B - o);
      CK(hipMemcpyAsync(d_in + o, h_in + o, n, hipMemcpyHostToDevice, s[c % 4]));
      CK(hipMemcpyAsync(h_out + o, d_out + o, n, hipMemcpyDeviceToHost, s[4 + c % 4]));
    }
  }, 8);
  // one stream per direction, chunked (the fused leg's duplex schedule)
  auto chunk2 = [&](size_t ch) {
    return timed([&] {
      for (size_t o = 0; o < B; o += ch) {
        const size_t n = std::min(ch, B - o);
        CK(hipMemcpyAsync(d_in + o, h_in + o, n, hipMemcpyHostToDevice, s[0]));
        CK(hipMemcpyAsync(h_out + o, d_out + o, n, hipMemcpyDeviceToHost, s[1]));
      }
    }, 2);
  };
  const double t_c2_16 = chunk2(16ull << 20), t_c2_64 = chunk2(64ull << 20),
               t_c2_256 = chunk2(256ull << 20);
  const double t_zcr = timed([&] { zcr(s[0]); }, 1);
  const double t_zcw = timed([&] { zcw(s[0]); }, 1);
  const double t_zcr_d2h = timed([&] { zcr(s[0]); d2h(s[1]); }, 2);
  const double t_h2d_zcw = timed([&] { h2d(s[0]); zcw(s[1]); }, 2);
  const double t_zc_both = timed([&] { zcr(s[0]); zcw(s[1]); }, 2);
  const char* sdma = std::getenv("HSA_ENABLE_SDMA");
  std::printf("{\"bytes_each_way\": %zu, \"HSA_ENABLE_SDMA\": \"%s\", "
              "\"dma_h2d\": %.2f, \"dma_d2h\": %.2f, \"dma_both_combined\": %.2f, "
              "\"dma_both_chunked_combined\": %.2f, \"zc_read\": %.2f, \"zc_write\": %.2f, "
              "\"zc_read_plus_dma_d2h_combined\": %.2f, \"dma_h2d_plus_zc_write_combined\": %.2f, "
              "\"zc_both_combined\": %.2f, \"dma_both_2streams_chunk16M\": %.2f, "
              "\"dma_both_2streams_chunk64M\": %.2f, \"dma_both_2streams_chunk256M\": %.2f, "
              "\"unit\": \"GB/s\"}\n",
              B, sdma ? sdma : "(unset)", g / t_h2d, g / t_d2h, 2 * g / t_both, 2 * g / t_chunk,
              g / t_zcr, g / t_zcw, 2 * g / t_zcr_d2h, 2 * g / t_h2d_zcw, 2 * g / t_zc_both,
              2 * g / t_c2_16, 2 * g / t_c2_64, 2 * g / t_c2_256);
  // check the data arrived (one byte per page)
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> chk(B);
  CK(hipMemcpy(chk.data(), d_in, B, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < B; i += 4096)
    if (chk[i] != (uint8_t)i) {
      std::fprintf(stderr, "H2D data mismatch at %zu\n", i);
      return 2;
    }
  for (size_t i = 0; i < B; i += 4096)
    if (h_out[i] != 1) {
      std::fprintf(stderr, "D2H data mismatch at %zu\n", i);
      return 2;
    }
  return 0;
}
