// tune_ragged.hip — A/B study of the ragged (CSR) FEC XOR kernels: the current
// product (flat-window, LDS accumulator) kernel, the previous two-windows-per-
// lane kernel (prev_ragged.inc, git fbed0d3), cache policies, and packed vs
// padded packet layouts (BASELINE configs[3] padding study).  One process, interleaved rounds.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_ragged.hip -o tools/tune/build/tune_ragged
#include "../../libquic_amd/csrc/qfec_kernels.hip"
#include "prev_ragged.inc"
#include "pipe_ragged.inc"

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,            \
                   hipGetErrorString(e_));                                       \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

static uint64_t sm64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Layout {
  std::vector<uint32_t> ptr;
  std::vector<uint16_t> len;
  std::vector<uint64_t> off;
  uint64_t bytes = 0;
  double alg = 0;
};

static Layout make_layout(uint64_t G, uint64_t stride /*0 = packed*/) {
  const uint64_t seed = 0x51554944;
  Layout l;
  l.ptr.push_back(0);
  double sum = 0, psum = 0;
  for (uint64_t g = 0; g < G; ++g) {
    const uint32_t k = 5 + (uint32_t)(sm64(seed ^ (0x6Bull << 56) ^ g) % 11);
    uint32_t mx = 0;
    for (uint32_t i = 0; i < k; ++i) {
      const uint32_t ln = 64 + (uint32_t)(sm64(seed ^ (0x4Cull << 56) ^ (g * 256 + i)) % 1287);
      l.len.push_back((uint16_t)ln);
      l.off.push_back(stride ? l.len.size() * 0 + (l.off.size()) * stride : l.bytes);
      l.bytes = stride ? (l.off.back() + stride) : l.bytes + ln;
      sum += ln;
      mx = std::max(mx, ln);
    }
    psum += mx;
    l.ptr.push_back((uint32_t)l.len.size());
  }
  l.alg = sum + psum;
  return l;
}

template <typename T>
static T* up(const std::vector<T>& v) {
  T* d;
  CK(hipMalloc(&d, v.size() * sizeof(T)));
  CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const uint64_t G = 1 << 20;
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  struct Set {
    std::string name;
    Layout l;
    uint8_t* data;
    uint64_t* off;
    uint16_t* len;
    uint32_t* ptr;
  };
  std::vector<Set> sets;
  for (uint64_t stride : {0ull, 1360ull, 1408ull}) {
    Set s;
    s.name = stride ? "stride" + std::to_string(stride) : "packed";
    s.l = make_layout(G, stride);
    CK(hipMalloc(&s.data, s.l.bytes + 4096));
    s.off = up(s.l.off);
    s.len = up(s.l.len);
    s.ptr = up(s.l.ptr);
    CK(qfec::launch_synth_ragged(s.data, s.off, s.len, s.ptr, 0, G, 0x51554944, 0));
    sets.push_back(s);
  }
  std::vector<uint64_t> poff(G);
  for (uint64_t g = 0; g < G; ++g) poff[g] = g * 1452;
  uint64_t* d_poff = up(poff);
  uint8_t *par, *par2;
  uint16_t* plen;
  uint32_t* err;
  CK(hipMalloc(&par, G * 1452));
  CK(hipMalloc(&par2, G * 1452));
  CK(hipMalloc(&plen, G * 2));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  CK(hipDeviceSynchronize());

  auto args = [&](const Set& s, uint8_t* out) {
    qfec::RaggedArgs a{};
    a.bytes = s.data;
    a.pkt_off = s.off;
    a.pkt_len = s.len;
    a.grp_ptr = s.ptr;
    a.parity_off = d_poff;
    a.parity_len_out = plen;
    a.out = out;
    a.n_groups = G;
    a.err = err;
    return a;
  };
  struct V {
    std::string name;
    double bytes;
    std::function<void()> run;
  };
  std::vector<V> vs;
  for (auto& s : sets) {
    auto a = args(s, par);
    vs.push_back({"product (nt) " + s.name, s.l.alg,
                  [=] { CK(qfec::launch_ragged(a, false, 0)); }});
    if (s.name == "packed") {
      vs.push_back({"product default-policy " + s.name, s.l.alg, [=] {
                      hipLaunchKernelGGL((qfec::ragged_xor_kernel<false, false>),
                                         dim3((uint32_t)((G + 3) / 4)), dim3(256), 0, 0, a);
                    }});
#define TP(NAME, GRID)                                                                      \
  vs.push_back({NAME, s.l.alg, [=] {                                                        \
                  hipLaunchKernelGGL((qfec::ragged_pipe_kernel<false, true>), dim3(GRID),     \
                                     dim3(256), 0, 0, a);                                    \
                }});
      TP("pipe grid 1024", 1024)
      TP("pipe grid 2048", 2048)
      TP("pipe grid 4096", 4096)
      TP("pipe grid 8192", 8192)
      TP("pipe grid 16384", 16384)
#undef TP
      vs.push_back({"prev (2 fixed windows/lane, nt) " + s.name, s.l.alg, [=] {
                      hipLaunchKernelGGL((qfec::prev_ragged_xor_kernel<false, true>),
                                         dim3((uint32_t)((G + 3) / 4)), dim3(256), 0, 0, a);
                    }});
      vs.push_back({"prev default-policy " + s.name, s.l.alg, [=] {
                      hipLaunchKernelGGL((qfec::prev_ragged_xor_kernel<false, false>),
                                         dim3((uint32_t)((G + 3) / 4)), dim3(256), 0, 0, a);
                    }});
    }
  }
  // correctness: product == prev on the packed set
  {
    auto a1 = args(sets[0], par);
    auto a2 = args(sets[0], par2);
    CK(hipMemset(par, 0, G * 1452));
    CK(hipMemset(par2, 0, G * 1452));
    CK(qfec::launch_ragged(a1, false, 0));
    hipLaunchKernelGGL((qfec::prev_ragged_xor_kernel<false, true>), dim3((uint32_t)((G + 3) / 4)),
                       dim3(256), 0, 0, a2);
    std::vector<uint8_t> h1(G * 1452), h2(G * 1452);
    CK(hipMemcpy(h1.data(), par, G * 1452, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), par2, G * 1452, hipMemcpyDeviceToHost));
    std::printf("product == prev: %s\n", h1 == h2 ? "yes" : "NO");
    // host reference on a sample of groups
    const Layout& L0 = sets[0].l;
    std::vector<uint8_t> data(L0.bytes);
    CK(hipMemcpy(data.data(), sets[0].data, L0.bytes, hipMemcpyDeviceToHost));
    int badp = 0, bado = 0;
    for (uint64_t g = 0; g < G; g += 997) {
      uint8_t ref[1452] = {0};
      uint32_t mx = 0;
      for (uint32_t p = L0.ptr[g]; p < L0.ptr[g + 1]; ++p) {
        for (uint32_t j = 0; j < L0.len[p]; ++j) ref[j] ^= data[L0.off[p] + j];
        mx = std::max<uint32_t>(mx, L0.len[p]);
      }
      badp += memcmp(ref, &h1[g * 1452], mx) != 0;
      bado += memcmp(ref, &h2[g * 1452], mx) != 0;
    }
    std::printf("host check: product bad groups %d, prev bad groups %d\n", badp, bado);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> res(vs.size());
  for (auto& v : vs) v.run();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(e0, 0));
      for (int q = 0; q < reps; ++q) vs[i].run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      res[i].push_back(vs[i].bytes / (ms / reps * 1e-3) / 1e9);
    }
  }
  std::printf("%-44s %10s %10s %8s\n", "variant", "med GB/s", "max GB/s", "%8TB/s");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = res[i];
    std::sort(v.begin(), v.end());
    std::printf("%-44s %10.1f %10.1f %7.1f%%\n", vs[i].name.c_str(), v[v.size() / 2], v.back(),
                v[v.size() / 2] / 80.0);
  }
  return 0;
}
