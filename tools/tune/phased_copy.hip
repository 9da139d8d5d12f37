// phased_copy.hip — does separating a copy's reads and writes in time (the
// phased FEC kernel's grid-wide phases) lift it above the
// box's copy ceiling?  The NULL protection kernels are a copy plus a hash
// and run at ~0.81 of the nt 16-B streaming copy (~4.8-5.0 TB/s, 0.60-0.63 of
// 8 TB/s): if a phased copy beats the streaming copy by
// a wide margin, a phased NULL kernel is worth building; if not, the copy
// ceiling is the NULL kernels' bound.
//
// Kernels (4 GiB source, 4 GiB destination, bytes read + written / time):
//   read      nt 16-B streaming read (qfec stream_probe<false>)
//   write     nt 16-B streaming store of a register value
//   copy      nt 16-B streaming copy (qfec stream_probe<true>)
//   phased R+S  one workgroup of 256 lanes per CU, persistent: per phase each
//             workgroup loads R steps of 4 KiB into VGPRs and S steps into LDS
//             (S <= 40: 160 KiB), meets the grid (qfec::phase_meet), stores
//             them; chunks of consecutive workgroups are contiguous
// Every copy is checked byte for byte against the source.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/phased_copy.hip \
//          -o tools/tune/build/phased_copy
#include "../../libquic_amd/csrc/qfec_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
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

using qfec::u32x4;

__global__ __launch_bounds__(256) void write_probe(uint8_t* dst, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  const u32x4 v = {threadIdx.x, blockIdx.x, 1u, 2u};
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride)
    qfec::st16t<true>(dst + 16u * i, v);
}

template <int R, int S>
__global__ __launch_bounds__(256) void phased_copy(const uint8_t* __restrict__ src,
                                                   uint8_t* __restrict__ dst, uint64_t n,
                                                   uint32_t* ps, uint32_t nphase) {
  __shared__ u32x4 s_buf[S > 0 ? S : 1][256];
  constexpr uint64_t kStep = 256u * 16u;
  constexpr uint64_t kChunk = (uint64_t)(R + S) * kStep;
  const uint32_t t = threadIdx.x;
  for (uint32_t p = 0; p < nphase; ++p) {
    const uint64_t base = ((uint64_t)p * gridDim.x + blockIdx.x) * kChunk + 16u * t;
    u32x4 v[R > 0 ? R : 1];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint64_t o = base + (uint64_t)s * kStep;
      if (o < n) s_buf[s][t] = qfec::ld16t<true>(src + o);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t o = base + (uint64_t)(S + r) * kStep;
      v[r] = qfec::ld16t<true>(src + (o < n ? o : 0));
    }
    qfec::phase_meet(ps, p + 1u);
#pragma unroll 4
    for (int s = 0; s < S; ++s) {
      const uint64_t o = base + (uint64_t)s * kStep;
      if (o < n) qfec::st16t<true>(dst + o, s_buf[s][t]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t o = base + (uint64_t)(S + r) * kStep;
      if (o < n) qfec::st16t<true>(dst + o, v[r]);
    }
  }
  qfec::phase_exit(ps, nullptr);
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const uint64_t n = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 4096) << 20;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int rounds = argc > 3 ? atoi(argv[3]) : 3;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t *src, *dst;
  uint32_t* ps;
  CK(hipMalloc(&src, n));
  CK(hipMalloc(&dst, n));
  CK(hipMalloc(&ps, 64 * 4 * 32));
  CK(hipMemset(ps, 0, 64 * 4 * 32));
  CK(qfec::launch_synth_fixed(src, 1, (uint32_t)(n >> 20), n >> 20, n >> 20, 0, 1 << 20,
                              0x5EEDull, 0));
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> h_src(n), h_dst(n);
  CK(hipMemcpy(h_src.data(), src, n, hipMemcpyDeviceToHost));

  struct V {
    std::string name;
    double bytes;  // moved per launch
    bool check;
    std::function<void()> run;
  };
  auto phased = [&](auto kern, uint64_t chunk) {
    const uint32_t np = (uint32_t)((n + chunk * ncu - 1) / (chunk * ncu));
    return [=] { hipLaunchKernelGGL(kern, dim3(ncu), dim3(256), 0, 0, src, dst, n, ps, np); };
  };
  const uint64_t kStep = 4096;
  std::vector<V> vs = {
      {"read (nt stream)", (double)n, false,
       [&] { CK(qfec::launch_stream_probe(src, n, dst, false, 0)); }},
      {"write (nt stream)", (double)n, false,
       [&] { hipLaunchKernelGGL(write_probe, dim3(ncu * 16), dim3(256), 0, 0, dst, n / 16); }},
      {"copy (nt stream)", 2.0 * n, true,
       [&] { CK(qfec::launch_stream_probe(src, n, dst, true, 0)); }},
      {"phased 0+40 (LDS)", 2.0 * n, true, phased(phased_copy<0, 40>, 40 * kStep)},
      {"phased 32+40", 2.0 * n, true, phased(phased_copy<32, 40>, 72 * kStep)},
      {"phased 64+40", 2.0 * n, true, phased(phased_copy<64, 40>, 104 * kStep)},
      {"phased 64+0 (VGPR)", 2.0 * n, true, phased(phased_copy<64, 0>, 64 * kStep)},
      {"copy (nt stream) again", 2.0 * n, true,
       [&] { CK(qfec::launch_stream_probe(src, n, dst, true, 0)); }},
  };
  bool ok = true;
  for (const V& v : vs) {
    if (!v.check) continue;
    CK(hipMemset(dst, 0, n));
    v.run();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h_dst.data(), dst, n, hipMemcpyDeviceToHost));
    const bool same = h_dst == h_src;
    std::printf("check %-24s %s\n", v.name.c_str(), same ? "exact" : "MISMATCH");
    ok = ok && same;
  }
  if (!ok) return 2;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < vs.size(); ++i) {
      vs[i].run();
      CK(hipEventRecord(e0, 0));
      for (int q = 0; q < reps; ++q) vs[i].run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float m = 0;
      CK(hipEventElapsedTime(&m, e0, e1));
      ms[i].push_back(m / reps);
    }
  uint32_t h_ps[64 * 20];
  CK(hipMemcpy(h_ps, ps, sizeof(h_ps), hipMemcpyDeviceToHost));
  std::printf("\n%llu MiB each way, %d CUs; GB/s = bytes read + written / time (median of %d)\n",
              (unsigned long long)(n >> 20), ncu, rounds);
  for (size_t i = 0; i < vs.size(); ++i) {
    std::vector<float> s = ms[i];
    std::sort(s.begin(), s.end());
    const double sec = s[s.size() / 2] * 1e-3;
    std::printf("%-26s %9.1f us  %8.1f GB/s  %.4f of 8 TB/s\n", vs[i].name.c_str(), sec * 1e6,
                vs[i].bytes / sec / 1e9, vs[i].bytes / sec / 8e12);
  }
  std::printf("abandoned phased launches: %u\n", h_ps[64 * 19]);
  return 0;
}
