// tune_xcd.hip — XCD-aware workgroup order for the fixed-shape FEC kernels:
// fixed_xor_kernel<..., XCD = true> (the blocks that share an XCD take one
// contiguous share of the groups, so the 128-B lines two neighbouring
// workgroups both touch meet in one L2) against the product's blockIdx order,
// headline shape 2^20 x 10 x 1350, nt.  Outputs compared byte for byte; every
// timed variant writes the same buffers (where the parity lands moves the rate
// by up to 10%).  One process, interleaved rounds.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_xcd.hip -o tools/tune/build/tune_xcd
#include "../../libquic_amd/csrc/qfec_kernels.hip"

#include <algorithm>
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

template <bool REC, bool XCD>
static void launch(const qfec::FixedArgs& a, uint32_t C, uint32_t gpb, uint64_t blocks) {
  hipLaunchKernelGGL((qfec::fixed_xor_kernel<10, REC, true, REC, XCD>), dim3((uint32_t)blocks),
                     dim3(256), 0, 0, a, C, gpb);
  CK(hipGetLastError());
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const uint64_t G = 1ull << 20;
  const uint32_t k = 10, L = 1350, C = (L + 15) / 16, gpb = 256 / C;
  const uint64_t blocks = (G + gpb - 1) / gpb;
  uint8_t *rows, *par, *out, *chk, *miss;
  uint32_t* err;
  CK(hipMalloc(&rows, G * k * L));
  CK(hipMalloc(&par, G * L));
  CK(hipMalloc(&out, G * L));
  CK(hipMalloc(&chk, G * L));
  CK(hipMalloc(&miss, G));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  CK(qfec::launch_synth_fixed(rows, k, L, L, (uint64_t)k * L, 0, G, 0x51554943ull, 0));
  std::vector<uint8_t> m(G);
  for (uint64_t g = 0; g < G; ++g) m[g] = (uint8_t)(sm64(0x51554945ull ^ g) % k);
  CK(hipMemcpy(miss, m.data(), G, hipMemcpyHostToDevice));
  qfec::FixedArgs e{};
  e.rows = rows;
  e.out = par;
  e.row_stride = L;
  e.group_stride = (uint64_t)k * L;
  e.parity_stride = L;
  e.out_stride = L;
  e.n_groups = G;
  e.k = k;
  e.L = L;
  e.err = err;
  qfec::FixedArgs r = e;
  r.parity = par;
  r.missing = miss;
  r.out = out;
  CK(qfec::launch_fixed(e, true, 0));
  CK(qfec::launch_fixed(r, true, 0));
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> want_p(G * L), want_o(G * L), got(G * L), h_rows(2 * k * L);
  CK(hipMemcpy(want_p.data(), par, G * L, hipMemcpyDeviceToHost));
  CK(hipMemcpy(want_o.data(), out, G * L, hipMemcpyDeviceToHost));
  // the product's recovered rows == the lost rows (first two groups)
  CK(hipMemcpy(h_rows.data(), rows, h_rows.size(), hipMemcpyDeviceToHost));
  bool ok_prod = true;
  for (uint64_t g = 0; g < 2; ++g)
    ok_prod = ok_prod && std::equal(want_o.begin() + g * L, want_o.begin() + (g + 1) * L,
                                    h_rows.begin() + (g * k + m[g]) * L);
  qfec::FixedArgs ec = e, rc = r;
  ec.out = chk;
  rc.out = chk;
  launch<false, true>(ec, C, gpb, blocks);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(got.data(), chk, G * L, hipMemcpyDeviceToHost));
  const bool ok_e = got == want_p;
  launch<true, true>(rc, C, gpb, blocks);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(got.data(), chk, G * L, hipMemcpyDeviceToHost));
  const bool ok_r = got == want_o;
  uint32_t he;
  CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
  std::printf("product revives lost rows: %s; XCD encode == product: %s; XCD recover == product: %s (err %u)\n",
              ok_prod ? "yes" : "NO", ok_e ? "yes" : "NO", ok_r ? "yes" : "NO", he);
  struct V {
    std::string name;
    std::function<void()> run;
  };
  std::vector<V> vs = {
      {"product encode", [&] { CK(qfec::launch_fixed(e, true, 0)); }},
      {"XCD encode", [&] { launch<false, true>(e, C, gpb, blocks); }},
      {"product recover", [&] { CK(qfec::launch_fixed(r, true, 0)); }},
      {"XCD recover", [&] { launch<true, true>(r, C, gpb, blocks); }},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> res(vs.size());
  const double alg = (double)G * (k * L + L);  // 14,850 B/group both ways
  for (int q = 0; q < rounds; ++q)
    for (size_t i = 0; i < vs.size(); ++i) {
      vs[i].run();
      CK(hipEventRecord(e0, 0));
      for (int t = 0; t < reps; ++t) vs[i].run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      res[i].push_back(alg / (ms / reps * 1e-3) / 1e9);
    }
  std::printf("%-24s %10s %10s %8s\n", "variant", "med GB/s", "max GB/s", "%8TB/s");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = res[i];
    std::sort(v.begin(), v.end());
    std::printf("%-24s %10.1f %10.1f %7.1f%%\n", vs[i].name.c_str(), v[v.size() / 2], v.back(),
                v[v.size() / 2] / 80.0);
  }
  return ok_prod && ok_e && ok_r && he == 0 ? 0 : 1;
}
