// tune_hostbw.hip — how fast can W workgroups read a small batch out of
// host-mapped (pinned) memory?  The small-batch service reads a 64-group job
// (864 KB: 64 x 10 x 1350 B) over PCIe with its 8 workgroups (one CU each);
// round 5's stamps put those reads at ~20 us (43 GB/s) against the link's
// 57 GB/s for a DMA copy.  This probe times one kernel per size that reads
// `bytes` of mapped host memory with W workgroups of 512 lanes, every lane
// issuing its 16-B loads (P in flight) before one XOR and one store per lane,
// for W = 1 .. 64 and sizes 14 KB (one group) .. 3.5 MB; HIP events around
// `reps` back-to-back launches (the launch gap is measured separately with an
// empty kernel and subtracted).  (where the 64-group
// flush's time goes.)
//
//   tune_hostbw [reps=200]
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_hostbw.hip \
//          -o tools/tune/build/tune_hostbw
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 512;
constexpr int kP = 8;  // loads in flight per lane

// lane t of workgroup w reads 16-B chunks c = (w * 512 + t) + i * W * 512
__global__ __launch_bounds__(kThreads) void read_kernel(const u32x4* __restrict__ src, uint64_t n16,
                                                        u32x4* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * kThreads;
  const uint64_t t = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (uint64_t c = t; c < n16; c += stride * kP) {
    u32x4 v[kP];
#pragma unroll
    for (int i = 0; i < kP; ++i) {
      const uint64_t ci = c + (uint64_t)i * stride;
      v[i] = ci < n16 ? __builtin_nontemporal_load(src + ci) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < kP; ++i) acc ^= v[i];
  }
  out[t] = acc;
}

__global__ void empty_kernel() {}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  const uint64_t maxb = 3600000;
  void* h;
  CK(hipHostMalloc(&h, maxb, hipHostMallocMapped | hipHostMallocPortable));
  for (uint64_t i = 0; i < maxb; ++i) static_cast<uint8_t*>(h)[i] = (uint8_t)(i * 131u);
  void* hd;
  CK(hipHostGetDevicePointer(&hd, h, 0));
  u32x4* out;
  CK(hipMalloc(&out, 64 * kThreads * sizeof(u32x4)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto time_us = [&](auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3 / reps;
  };
  const double gap = time_us([&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0); });
  std::printf("empty kernel back to back: %.2f us per launch (subtracted below)\n", gap);
  const uint64_t sizes[] = {13500, 108000, 216000, 432000, 864000, 1728000, 3456000};
  const int wgs[] = {1, 2, 4, 8, 16, 32, 64};
  std::printf("%10s", "bytes \\ W");
  for (int w : wgs) std::printf(" %14d", w);
  std::printf("\n");
  for (uint64_t bytes : sizes) {
    std::printf("%10llu", (unsigned long long)bytes);
    for (int w : wgs) {
      const uint64_t n16 = bytes / 16;
      const double us = time_us([&] {
        hipLaunchKernelGGL(read_kernel, dim3(w), dim3(kThreads), 0, 0,
                           static_cast<const u32x4*>(hd), n16, out);
      });
      const double t = std::max(us - gap, 0.01);
      std::printf(" %5.1fus %5.1fGB", t, bytes / t / 1e3);
    }
    std::printf("\n");
  }
  CK(hipHostFree(h));
  return 0;
}
