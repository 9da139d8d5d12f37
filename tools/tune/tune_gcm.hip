// tune_gcm.hip — AES-128-GCM-12 seal/open throughput on the headline packet
// shape (22-B header, 1350-B payload, one key: key-uniform waves), product
// kernel vs the first kernel (prev_gcm.inc), interleaved in one process.
// Also checks that the two produce identical ciphertext+tags (the first
// kernel is pinned against BoringSSL's vectors by tests/test_hip_gcm.py) for
// a key-uniform and a mixed-key batch, and that open(seal) verifies.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_gcm.hip -o tools/tune/build/tune_gcm
#include "../../libquic_amd/csrc/qpp_kernels.hip"
#include "prev_gcm.inc"

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

static std::vector<uint8_t> down(const uint8_t* d, size_t n) {
  std::vector<uint8_t> h(n);
  CK(hipMemcpy(h.data(), d, n, hipMemcpyDeviceToHost));
  return h;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 21);
  const int reps = argc > 2 ? atoi(argv[2]) : 3, rounds = 3;
  const uint32_t L = 1350, H = 22;
  constexpr uint32_t SC = 8;
  std::vector<uint64_t> ad_off(n), in_off(n), out_off(n), cad_off(n), cct_off(n), dout_off(n);
  std::vector<uint16_t> ad_len(n, H), in_len(n, L), ct_len(n, L + 12);
  for (uint64_t p = 0; p < n; ++p) {
    ad_off[p] = p * (H + L);
    in_off[p] = ad_off[p] + H;
    out_off[p] = p * (L + 12);
    cad_off[p] = p * (H + L + 12);
    cct_off[p] = cad_off[p] + H;
    dout_off[p] = p * L;
  }
  uint8_t *d_in, *d_out, *d_out_ref, *d_cat, *d_dec, *d_ok;
  CK(hipMalloc(&d_in, n * (H + L)));
  CK(hipMalloc(&d_out, n * (L + 12)));
  CK(hipMalloc(&d_out_ref, n * (L + 12)));
  CK(hipMalloc(&d_cat, n * (H + L + 12)));
  CK(hipMalloc(&d_dec, n * L));
  CK(hipMalloc(&d_ok, n));
  {
    std::vector<uint8_t> h(n * (H + L));
    uint64_t s = 0x243F6A8885A308D3ull;
    for (auto& b : h) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      b = (uint8_t)s;
    }
    CK(hipMemcpy(d_in, h.data(), h.size(), hipMemcpyHostToDevice));
  }
  const uint32_t nkeys = 7;
  std::vector<uint8_t> keys(16 * nkeys), pre(4 * nkeys);
  for (uint32_t i = 0; i < 16 * nkeys; ++i) keys[i] = (uint8_t)(i * 11 + 3);
  for (uint32_t i = 0; i < 4 * nkeys; ++i) pre[i] = (uint8_t)(0xA0 + i);
  std::vector<uint32_t> kidx_uni(n, 0), kidx_mix(n);
  std::vector<uint64_t> pns(n);
  for (uint64_t p = 0; p < n; ++p) {
    pns[p] = p + 1;
    kidx_mix[p] = (uint32_t)((p * 2654435761ull) % nkeys);
  }
  qfec::AeadArgs as{};
  as.io.bytes = d_in;
  as.io.ad_off = up(ad_off);
  as.io.ad_len = up(ad_len);
  as.io.in_off = up(in_off);
  as.io.in_len = up(in_len);
  as.io.out = d_out;
  as.io.out_off = up(out_off);
  as.io.n = n;
  as.keys = up(keys);
  as.prefixes = up(pre);
  as.key_idx = up(kidx_uni);
  as.packet_number = up(pns);
  as.path_id = nullptr;
  qfec::AeadArgs as_ref = as;
  as_ref.io.out = d_out_ref;
  qfec::AeadArgs ao{};
  ao.io.bytes = d_cat;
  ao.io.ad_off = up(cad_off);
  ao.io.ad_len = as.io.ad_len;
  ao.io.in_off = up(cct_off);
  ao.io.in_len = up(ct_len);
  ao.io.out = d_dec;
  ao.io.out_off = up(dout_off);
  ao.io.ok = d_ok;
  ao.io.n = n;
  ao.keys = as.keys;
  ao.prefixes = as.prefixes;
  ao.key_idx = as.key_idx;
  ao.packet_number = as.packet_number;
  const uint32_t grid = (uint32_t)((n + 255) / 256);
  const uint32_t gb = qfec::kGcmBlock, ggrid = (uint32_t)((n + gb - 1) / gb);
  auto seal_new = [&](const qfec::AeadArgs& a) {
    hipLaunchKernelGGL((qfec::aes128gcm_kernel<SC, false>), dim3(ggrid), dim3(gb), 0, 0, a);
  };
  auto seal_old = [&](const qfec::AeadArgs& a) {
    hipLaunchKernelGGL((qfec::gcm_v1::aes128gcm_kernel<SC, false>), dim3(grid), dim3(256), 0, 0, a);
  };
  auto open_new = [&](const qfec::AeadArgs& a) {
    hipLaunchKernelGGL((qfec::aes128gcm_kernel<SC, true>), dim3(ggrid), dim3(gb), 0, 0, a);
  };
  auto open_old = [&](const qfec::AeadArgs& a) {
    hipLaunchKernelGGL((qfec::gcm_v1::aes128gcm_kernel<SC, true>), dim3(grid), dim3(256), 0, 0, a);
  };
  int bad = 0;
  // correctness: new vs old seal, key-uniform and mixed-key; open(seal) ok
  for (int mix = 0; mix < 2; ++mix) {
    qfec::AeadArgs a = as, r = as_ref;
    uint32_t* kmix = mix ? up(kidx_mix) : nullptr;
    if (mix) a.key_idx = r.key_idx = kmix;
    CK(hipMemset(d_out, 0, n * (L + 12)));
    CK(hipMemset(d_out_ref, 0xFF, n * (L + 12)));
    seal_new(a);
    seal_old(r);
    CK(hipDeviceSynchronize());
    const auto x = down(d_out, n * (L + 12)), y = down(d_out_ref, n * (L + 12));
    uint64_t diff = 0;
    for (uint64_t p = 0; p < n; ++p)
      if (std::memcmp(&x[p * (L + 12)], &y[p * (L + 12)], L + 12) != 0) ++diff;
    std::printf("seal %s: packets differing new vs first kernel: %llu / %llu\n",
                mix ? "mixed-key" : "one-key", (unsigned long long)diff, (unsigned long long)n);
    bad |= diff != 0;
    CK(hipMemcpy2D(d_cat, H + L + 12, d_in, H + L, H, n, hipMemcpyDeviceToDevice));
    CK(hipMemcpy2D(d_cat + H, H + L + 12, d_out, L + 12, L + 12, n, hipMemcpyDeviceToDevice));
    qfec::AeadArgs o = ao;
    if (mix) o.key_idx = kmix;
    CK(hipMemset(d_ok, 0, n));
    open_new(o);
    CK(hipDeviceSynchronize());
    const auto ok = down(d_ok, n);
    uint64_t good = 0;
    for (auto v : ok) good += v;
    std::printf("open(seal) %s verified: %llu / %llu\n", mix ? "mixed-key" : "one-key",
                (unsigned long long)good, (unsigned long long)n);
    bad |= good != n;
    if (kmix) CK(hipFree(kmix));
  }
  // d_cat now holds the mixed-key ciphertexts: rebuild it for the one-key timing
  seal_new(as);
  CK(hipMemcpy2D(d_cat + H, H + L + 12, d_out, L + 12, L + 12, n, hipMemcpyDeviceToDevice));
  CK(hipDeviceSynchronize());
  struct V {
    std::string name;
    double bytes;
    std::function<void()> run;
  };
  const double enc_b = (double)n * (H + L + L + 12), dec_b = (double)n * (H + L + 12 + L);
  std::vector<V> vs = {
      {"seal product", enc_b, [&] { seal_new(as); }},
      {"seal first kernel", enc_b, [&] { seal_old(as); }},
      {"open product", dec_b, [&] { open_new(ao); }},
      {"open first kernel", dec_b, [&] { open_old(ao); }},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<double>> ms(vs.size());
  for (auto& v : vs) v.run();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(e0, 0));
      for (int q = 0; q < reps; ++q) vs[i].run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[i].push_back(t / reps);
    }
  std::printf("%-28s %10s %10s %12s\n", "variant", "ms", "HBM GB/s", "payload GB/s");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = ms[i];
    std::sort(v.begin(), v.end());
    const double t = v[v.size() / 2] * 1e-3;
    std::printf("%-28s %10.3f %10.1f %12.1f\n", vs[i].name.c_str(), t * 1e3, vs[i].bytes / t / 1e9,
                (double)n * L / t / 1e9);
  }
  return bad;
}
