// tune_lds_unaligned.hip — does ds_read_b128 at a byte-granular LDS address
// return the right bytes on gfx950 (unaligned DS access), and at what rate
// next to 16-B aligned reads?  Used by the NULL-encrypt realignment design.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_lds_unaligned.hip -o tools/tune/build/tune_lds_unaligned
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

// correctness: lane l reads 16 B at byte offset l*48 + ((sh + l) & 31)
__global__ void check(const uint32_t* in, uint32_t* out, uint32_t sh) {
  __shared__ __attribute__((aligned(16))) uint8_t s[64 * 48 + 64];
  for (int i = threadIdx.x; i < (64 * 48 + 64) / 4; i += 64) ((uint32_t*)s)[i] = in[i];
  __syncthreads();
  const uint32_t off = threadIdx.x * 48 + ((sh + threadIdx.x) & 31);
  ((u32x4*)out)[threadIdx.x] = *(const u32x4_a1*)(s + off);
}

// rate: every lane reads 16 B per step from its own 272-B row (stride of the
// staged rows) at byte offset 16 j + sh (sh = 0: aligned)
template <bool UNAL>
__global__ __launch_bounds__(256) void rate(uint32_t iters, uint32_t shift, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t s[256 * 272 + 64];
  for (int i = threadIdx.x; i < (256 * 272 + 64) / 4; i += 256) ((uint32_t*)s)[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t sh = UNAL ? ((threadIdx.x * 7 + shift) & 15) : 0;
  const uint8_t* row = s + threadIdx.x * 272 + sh;
  uint32_t acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const u32x4 v = *(const u32x4_a1*)(row + 16 * j);
      acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    asm volatile("" : "+v"(acc));
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  std::vector<uint32_t> h((64 * 48 + 64) / 4);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(i * 0x9E3779B9u + 0x1234567u);
  uint32_t *din, *dout;
  CK(hipMalloc(&din, h.size() * 4));
  CK(hipMalloc(&dout, 64 * 16));
  CK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const uint8_t* hb = (const uint8_t*)h.data();
  int bad = 0;
  for (uint32_t sh = 0; sh < 32; ++sh) {
    hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, din, dout, sh);
    std::vector<uint8_t> o(64 * 16);
    CK(hipMemcpy(o.data(), dout, o.size(), hipMemcpyDeviceToHost));
    for (int l = 0; l < 64; ++l) {
      const uint32_t off = l * 48 + ((sh + l) & 31);
      for (int b = 0; b < 16; ++b)
        if (o[l * 16 + b] != hb[off + b]) ++bad;
    }
  }
  std::printf("unaligned ds_read_b128: %d wrong bytes over 32 x 64 lanes x 16 B\n", bad);
  uint32_t* sink;
  CK(hipMalloc(&sink, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t iters = 4096, grid = 256 * 2;
  for (int rep = 0; rep < 2; ++rep)
    for (int u = 0; u < 2; ++u) {
      CK(hipEventRecord(e0));
      if (u) hipLaunchKernelGGL(rate<true>, dim3(grid), dim3(256), 0, 0, iters, 3u, sink);
      else hipLaunchKernelGGL(rate<false>, dim3(grid), dim3(256), 0, 0, iters, 3u, sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double reads = (double)grid * 4 * iters * 16;  // wave-instructions
      std::printf("%s: %.3f ms, %.2f LDS cycles... per wave-read (at 2.4 GHz, 256 CUs)\n",
                  u ? "unaligned" : "aligned  ", ms, ms * 1e-3 * 2.4e9 * 256 / reads);
    }
  return bad ? 1 : 0;
}
