// tune_gcm2.hip — round 5: AES-128-GCM-12 seal shapes
// against the stall picture of profiles/round5/aead_stall.json (issue-latency
// bound: 2.3 waves per SIMD, a third of the wave cycles waiting on operands).
// Variants trade counter blocks in flight per lane (NB) against waves per
// SIMD (BLOCK / WPE, which cap the VGPRs) and slab size (SC, the LDS rows);
// every variant's ciphertexts and tags are byte-compared with the product's.
//   tune_gcm2 [packets=2^22]
#include "../../libquic_amd/csrc/qpp_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

template <typename T>
static T* up(const std::vector<T>& v) {
  T* d;
  CK(hipMalloc(&d, v.size() * sizeof(T)));
  CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

template <uint32_t SC, int NB, int BLOCK, int WPE>
static void seal(const qfec::AeadArgs& a) {
  hipLaunchKernelGGL((qfec::aes128gcm_kernel<SC, false, NB, BLOCK, WPE>),
                     dim3((uint32_t)((a.io.n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, 0, a);
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 22);
  const uint32_t L = 1350, H = 22;
  const int reps = 3, rounds = 3;
  std::vector<uint64_t> ad_off(n), in_off(n), out_off(n);
  std::vector<uint16_t> ad_len(n, H), in_len(n, L);
  for (uint64_t p = 0; p < n; ++p) {
    ad_off[p] = p * (H + L);
    in_off[p] = p * (H + L) + H;
    out_off[p] = p * (L + 12);
  }
  uint8_t *d_in, *d_ref, *d_out;
  CK(hipMalloc(&d_in, n * (H + L)));
  CK(hipMalloc(&d_ref, n * (L + 12)));
  CK(hipMalloc(&d_out, n * (L + 12)));
  {
    std::vector<uint8_t> h(n * (H + L));
    uint64_t s = 0x243F6A8885A308D3ull;
    for (auto& b : h) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      b = (uint8_t)s;
    }
    CK(hipMemcpy(d_in, h.data(), h.size(), hipMemcpyHostToDevice));
  }
  std::vector<uint8_t> key(16), pre(4);
  for (int i = 0; i < 16; ++i) key[i] = (uint8_t)(i * 11 + 3);
  for (int i = 0; i < 4; ++i) pre[i] = (uint8_t)(0xB0 + i);
  std::vector<uint32_t> kidx(n, 0);
  std::vector<uint64_t> pns(n);
  for (uint64_t p = 0; p < n; ++p) pns[p] = p + 1;
  qfec::AeadArgs a{};
  a.io.bytes = d_in;
  a.io.ad_off = up(ad_off);
  a.io.ad_len = up(ad_len);
  a.io.in_off = up(in_off);
  a.io.in_len = up(in_len);
  a.io.out = d_ref;
  a.io.out_off = up(out_off);
  a.io.n = n;
  a.keys = up(key);
  a.prefixes = up(pre);
  a.key_idx = up(kidx);
  a.packet_number = up(pns);
  a.path_id = nullptr;
  CK(qfec::launch_aes128gcm(a, false, 0));
  CK(hipDeviceSynchronize());
  qfec::AeadArgs b = a;
  b.io.out = d_out;

  struct V {
    std::string name;
    std::function<void(const qfec::AeadArgs&)> run;
  };
  std::vector<V> vs = {
      {"product (launch_aes128gcm)", [](const qfec::AeadArgs& x) { CK(qfec::launch_aes128gcm(x, false, 0)); }},
      {"SC4 NB4 768 WPE3 (product shape)", seal<4, 4, 768, 3>},
      {"SC8 NB4 512 WPE2", seal<8, 4, 512, 2>},
      {"SC2 NB2 1024 WPE4", seal<2, 2, 1024, 4>},
      {"SC4 NB2 768 WPE3", seal<4, 2, 768, 3>},
      {"SC8 NB2 512 WPE2", seal<8, 2, 512, 2>},
  };
  const size_t ob = n * (L + 12);
  std::vector<uint8_t> ref(ob), got(ob);
  CK(hipMemcpy(ref.data(), d_ref, ob, hipMemcpyDeviceToHost));
  bool all = true;
  for (const V& v : vs) {
    CK(hipMemset(d_out, 0xA5, ob));
    v.run(b);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), d_out, ob, hipMemcpyDeviceToHost));
    const bool ok = got == ref;
    std::printf("check %-34s %s\n", v.name.c_str(), ok ? "IDENTICAL" : "DIFFERS");
    all = all && ok;
  }
  if (!all) return 2;
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  std::vector<std::vector<float>> ms(vs.size());
  for (int rd = 0; rd < rounds; ++rd)
    for (size_t i = 0; i < vs.size(); ++i) {
      vs[i].run(b);
      CK(hipEventRecord(t0, 0));
      for (int q = 0; q < reps; ++q) vs[i].run(b);
      CK(hipEventRecord(t1, 0));
      CK(hipEventSynchronize(t1));
      float m = 0;
      CK(hipEventElapsedTime(&m, t0, t1));
      ms[i].push_back(m / reps);
    }
  const double payload = (double)n * L;
  std::printf("\n%llu packets of %u + %u B, one key\n", (unsigned long long)n, H, L);
  for (size_t i = 0; i < vs.size(); ++i) {
    std::vector<float> s = ms[i];
    std::sort(s.begin(), s.end());
    const double med = s[s.size() / 2] * 1e-3;
    std::printf("%-36s median %8.3f ms  payload %7.1f GB/s\n", vs[i].name.c_str(), med * 1e3,
                payload / med / 1e9);
  }
  return 0;
}
