// tune_multi.hip — A/B of the ragged kernels: GPW groups per wave
// (ragged_multi_kernel; the product runs GPW = 2) against one group per wave
// (ragged_xor_kernel), branch-free / aligned-chunk / XCD variants, encode and
// recover on the BASELINE configs[3] batch (2^20 groups, k 5-15, 64-1350 B,
// packed CSR).  Every variant's output bytes are compared with the product's.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_multi.hip -o tools/tune/build/tune_multi
// run:   tune_multi [reps] [rounds] [kmin] [kspan] [align16] [packed_out]
//        packed_out = 1: parity / revived rows back to back (offset = running sum of
//        parity lengths) instead of 1452-byte slots
#include "../../libquic_amd/csrc/qfec_kernels.hip"
#include "al_ragged.inc"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

template <typename T>
static T* up(const std::vector<T>& v) {
  T* d;
  CK(hipMalloc(&d, v.size() * sizeof(T)));
  CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

using qfec::RaggedArgs;

template <bool REC, int GPW, int WAVES, int U = 2>
static void launch_multi(const RaggedArgs& a, uint64_t G) {
  const uint64_t per = (uint64_t)GPW * WAVES;
  hipLaunchKernelGGL((qfec::ragged_multi_kernel<REC, true, GPW, U, WAVES>),
                     dim3((uint32_t)((G + per - 1) / per)), dim3(64 * WAVES), 0, 0, a);
}

template <bool REC, int U>
static void launch_bf(const RaggedArgs& a, uint64_t G) {
  hipLaunchKernelGGL((qfec::ragged_xor_kernel<REC, true, U, 4, 1, true>),
                     dim3((uint32_t)((G + 3) / 4)), dim3(256), 0, 0, a);
}

template <bool REC, int U>
static void launch_al(const RaggedArgs& a, uint64_t G) {
  hipLaunchKernelGGL((qfec::ragged_al_kernel<REC, true, U, 4, 1>),
                     dim3((uint32_t)((G + 3) / 4)), dim3(256), 0, 0, a);
}

template <bool REC>
static void launch_1g(const RaggedArgs& a, uint64_t G) {
  hipLaunchKernelGGL((qfec::ragged_xor_kernel<REC, true>), dim3((uint32_t)((G + 3) / 4)), dim3(256),
                     0, 0, a);
}

template <bool REC>
static void launch_xcd(const RaggedArgs& a, uint64_t G) {
  hipLaunchKernelGGL((qfec::ragged_xor_kernel<REC, true, 2, 4, 1, false, true>),
                     dim3((uint32_t)((G + 3) / 4)), dim3(256), 0, 0, a);
}

int main(int argc, char** argv) {
  const uint64_t G = 1 << 20;
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const uint32_t kmin = argc > 3 ? atoi(argv[3]) : 5, kspan = argc > 4 ? atoi(argv[4]) : 11;
  const bool align16 = argc > 5 && atoi(argv[5]) != 0;
  const bool packed_out = argc > 6 && atoi(argv[6]) != 0;
  uint64_t out_pos = 0;
  const uint64_t seed = 0x51554944;
  std::vector<uint32_t> ptr{0};
  std::vector<uint16_t> len, plen_h(G);
  std::vector<uint64_t> off, poff(G);
  std::vector<uint8_t> miss(G);
  uint64_t bytes = 0;
  double enc_alg = 0, rec_alg = 0;
  for (uint64_t g = 0; g < G; ++g) {
    const uint32_t k = kmin + (uint32_t)(sm64(seed ^ (0x6Bull << 56) ^ g) % kspan);
    miss[g] = (uint8_t)(sm64(seed ^ (0x4Dull << 56) ^ g) % k);
    uint32_t mx = 0;
    double s = 0, sm = 0;
    for (uint32_t i = 0; i < k; ++i) {
      uint32_t ln = 64 + (uint32_t)(sm64(seed ^ (0x4Cull << 56) ^ (g * 256 + i)) % 1287);
      if (align16) ln = std::min(1440u, (ln + 15u) & ~15u);  // 16-B multiples: aligned starts
      len.push_back((uint16_t)ln);
      off.push_back(bytes);
      bytes += ln;
      s += ln;
      if (i != miss[g]) sm += ln;
      mx = std::max(mx, ln);
    }
    enc_alg += s + mx;
    rec_alg += sm + 2.0 * mx;
    ptr.push_back((uint32_t)len.size());
    poff[g] = packed_out ? out_pos : g * 1452;
    out_pos += mx;
  }
  uint8_t* data;
  CK(hipMalloc(&data, bytes + 4096));
  uint64_t* d_off = up(off);
  uint16_t* d_len = up(len);
  uint32_t* d_ptr = up(ptr);
  uint64_t* d_poff = up(poff);
  uint8_t* d_miss = up(miss);
  CK(qfec::launch_synth_ragged(data, d_off, d_len, d_ptr, 0, G, seed, 0));
  uint8_t *par, *out, *chk;
  uint16_t *plen, *plen2;
  uint32_t* err;
  CK(hipMalloc(&par, G * 1452));
  CK(hipMalloc(&out, G * 1452));
  CK(hipMalloc(&chk, G * 1452));
  CK(hipMalloc(&plen, G * 2));
  CK(hipMalloc(&plen2, G * 2));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  CK(hipMemset(par, 0, G * 1452));
  CK(hipDeviceSynchronize());

  RaggedArgs e{};
  e.bytes = data;
  e.pkt_off = d_off;
  e.pkt_len = d_len;
  e.grp_ptr = d_ptr;
  e.parity_off = d_poff;
  e.parity_len_out = plen;
  e.out = par;
  e.n_groups = G;
  e.err = err;
  CK(qfec::launch_ragged(e, false, 0));  // reference parity for the recover runs
  CK(hipDeviceSynchronize());
  RaggedArgs r = e;
  r.parity = par;
  r.parity_len = plen;
  r.missing = d_miss;
  r.out_off = d_poff;
  r.parity_len_out = nullptr;
  r.out = out;
  RaggedArgs e2 = e;  // timed encodes write elsewhere
  e2.out = out;
  e2.parity_len_out = plen2;

  struct V {
    std::string name;
    bool rec;
    std::function<void(const RaggedArgs&)> run;
  };
  std::vector<V> vs;
  vs.push_back({"product encode", false, [](const RaggedArgs& a) { CK(qfec::launch_ragged(a, false, 0)); }});
  vs.push_back({"BF U2 encode", false, [=](const RaggedArgs& a) { launch_bf<false, 2>(a, G); }});
  vs.push_back({"AL U2 encode", false, [=](const RaggedArgs& a) { launch_al<false, 2>(a, G); }});
  vs.push_back({"AL U4 encode", false, [=](const RaggedArgs& a) { launch_al<false, 4>(a, G); }});
  vs.push_back({"AL U6 encode", false, [=](const RaggedArgs& a) { launch_al<false, 6>(a, G); }});
  vs.push_back({"AL U8 encode", false, [=](const RaggedArgs& a) { launch_al<false, 8>(a, G); }});
  vs.push_back({"BF U3 encode", false, [=](const RaggedArgs& a) { launch_bf<false, 3>(a, G); }});
  vs.push_back({"BF U4 encode", false, [=](const RaggedArgs& a) { launch_bf<false, 4>(a, G); }});
  vs.push_back({"BF U6 encode", false, [=](const RaggedArgs& a) { launch_bf<false, 6>(a, G); }});
  vs.push_back({"multi2 w4 encode", false, [=](const RaggedArgs& a) { launch_multi<false, 2, 4>(a, G); }});
  vs.push_back({"multi2 w4 U1 encode", false, [=](const RaggedArgs& a) { launch_multi<false, 2, 4, 1>(a, G); }});
  vs.push_back({"multi2 w4 U3 encode", false, [=](const RaggedArgs& a) { launch_multi<false, 2, 4, 3>(a, G); }});
  vs.push_back({"multi2 w2 encode", false, [=](const RaggedArgs& a) { launch_multi<false, 2, 2>(a, G); }});
  vs.push_back({"multi2 w8 encode", false, [=](const RaggedArgs& a) { launch_multi<false, 2, 8>(a, G); }});
  vs.push_back({"1 group/wave encode", false, [=](const RaggedArgs& a) { launch_1g<false>(a, G); }});
  vs.push_back({"multi3 w4 encode", false, [=](const RaggedArgs& a) { launch_multi<false, 3, 4>(a, G); }});
  vs.push_back({"product XCD encode", false, [=](const RaggedArgs& a) { launch_xcd<false>(a, G); }});
  vs.push_back({"product recover", true, [](const RaggedArgs& a) { CK(qfec::launch_ragged(a, true, 0)); }});
  vs.push_back({"BF U2 recover", true, [=](const RaggedArgs& a) { launch_bf<true, 2>(a, G); }});
  vs.push_back({"AL U2 recover", true, [=](const RaggedArgs& a) { launch_al<true, 2>(a, G); }});
  vs.push_back({"AL U4 recover", true, [=](const RaggedArgs& a) { launch_al<true, 4>(a, G); }});
  vs.push_back({"AL U6 recover", true, [=](const RaggedArgs& a) { launch_al<true, 6>(a, G); }});
  vs.push_back({"AL U8 recover", true, [=](const RaggedArgs& a) { launch_al<true, 8>(a, G); }});
  vs.push_back({"BF U3 recover", true, [=](const RaggedArgs& a) { launch_bf<true, 3>(a, G); }});
  vs.push_back({"BF U4 recover", true, [=](const RaggedArgs& a) { launch_bf<true, 4>(a, G); }});
  vs.push_back({"BF U6 recover", true, [=](const RaggedArgs& a) { launch_bf<true, 6>(a, G); }});
  vs.push_back({"multi2 w4 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2, 4>(a, G); }});
  vs.push_back({"multi2 w4 U1 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2, 4, 1>(a, G); }});
  vs.push_back({"multi2 w4 U3 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2, 4, 3>(a, G); }});
  vs.push_back({"multi2 w2 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2, 2>(a, G); }});
  vs.push_back({"multi2 w8 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2, 8>(a, G); }});
  vs.push_back({"1 group/wave recover", true, [=](const RaggedArgs& a) { launch_1g<true>(a, G); }});
  vs.push_back({"multi3 w4 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 3, 4>(a, G); }});
  vs.push_back({"product XCD recover", true, [=](const RaggedArgs& a) { launch_xcd<true>(a, G); }});

  // correctness: each variant's output (and parity lengths) == the product's
  std::vector<uint8_t> want_e(G * 1452), want_r(G * 1452), got(G * 1452);
  std::vector<uint16_t> want_pl(G), got_pl(G);
  CK(hipMemcpy(want_e.data(), par, G * 1452, hipMemcpyDeviceToHost));
  CK(hipMemcpy(want_pl.data(), plen, G * 2, hipMemcpyDeviceToHost));
  CK(hipMemset(out, 0, G * 1452));
  CK(qfec::launch_ragged(r, true, 0));
  CK(hipMemcpy(want_r.data(), out, G * 1452, hipMemcpyDeviceToHost));
  {  // the product against a host XOR on a sample
    std::vector<uint8_t> h(bytes);
    CK(hipMemcpy(h.data(), data, bytes, hipMemcpyDeviceToHost));
    int bad = 0;
    for (uint64_t g = 0; g < G; g += 997) {
      uint8_t ref[1452] = {0}, rv[1452] = {0};
      uint32_t mx = 0;
      for (uint32_t p = ptr[g]; p < ptr[g + 1]; ++p) {
        for (uint32_t j = 0; j < len[p]; ++j) ref[j] ^= h[off[p] + j];
        mx = std::max<uint32_t>(mx, len[p]);
      }
      std::memcpy(rv, ref, mx);
      for (uint32_t p = ptr[g]; p < ptr[g + 1]; ++p)
        if (p - ptr[g] != miss[g])
          for (uint32_t j = 0; j < len[p]; ++j) rv[j] ^= h[off[p] + j];
      const uint32_t lm = len[ptr[g] + miss[g]];
      bad += memcmp(ref, &want_e[poff[g]], mx) != 0 || want_pl[g] != mx;
      bad += memcmp(rv, &want_r[poff[g]], lm) != 0;
    }
    std::printf("product vs host XOR: bad groups %d\n", bad);
  }
  bool all_ok = true;
  for (auto& v : vs) {
    CK(hipMemset(out, 0, G * 1452));
    CK(hipMemset(plen2, 0, G * 2));
    v.run(v.rec ? r : e2);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), out, G * 1452, hipMemcpyDeviceToHost));
    bool same = got == (v.rec ? want_r : want_e);
    if (!v.rec) {
      CK(hipMemcpy(got_pl.data(), plen2, G * 2, hipMemcpyDeviceToHost));
      same = same && got_pl == want_pl;
    }
    uint32_t he;
    CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
    std::printf("%-24s == product: %s (err %u)\n", v.name.c_str(), same ? "yes" : "NO", he);
    all_ok = all_ok && same && he == 0;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> res(vs.size());
  for (int q = 0; q < rounds; ++q) {
    for (size_t i = 0; i < vs.size(); ++i) {
      const RaggedArgs& a = vs[i].rec ? r : e2;
      vs[i].run(a);
      CK(hipEventRecord(e0, 0));
      for (int t = 0; t < reps; ++t) vs[i].run(a);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      res[i].push_back((vs[i].rec ? rec_alg : enc_alg) / (ms / reps * 1e-3) / 1e9);
    }
  }
  std::printf("k %u..%u, %llu groups, %.3f GB packets\n", kmin, kmin + kspan - 1,
              (unsigned long long)G, bytes / 1e9);
  std::printf("%-24s %10s %10s %8s\n", "variant", "med GB/s", "max GB/s", "%8TB/s");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = res[i];
    std::sort(v.begin(), v.end());
    std::printf("%-24s %10.1f %10.1f %7.1f%%\n", vs[i].name.c_str(), v[v.size() / 2], v.back(),
                v[v.size() / 2] / 80.0);
  }
  return all_ok ? 0 : 1;
}
