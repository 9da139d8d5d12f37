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
  constexpr uint32_t SC = qfec::kGcmSC;
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
    hipLaunchKernelGGL((qfec::gcm_v1::aes128gcm_kernel<8, false>), dim3(grid), dim3(256), 0, 0, a);
  };
  auto open_new = [&](const qfec::AeadArgs& a) {
    hipLaunchKernelGGL((qfec::aes128gcm_kernel<SC, true>), dim3(ggrid), dim3(gb), 0, 0, a);
  };
  auto open_old = [&](const qfec::AeadArgs& a) {
    hipLaunchKernelGGL((qfec::gcm_v1::aes128gcm_kernel<8, true>), dim3(grid), dim3(256), 0, 0, a);
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
  {  // the 3-wave variant against the product, one key and mixed keys
    for (int mix = 0; mix < 2; ++mix) {
      qfec::AeadArgs a = as, r = as_ref;
      uint32_t* kmix = mix ? up(kidx_mix) : nullptr;
      if (mix) a.key_idx = r.key_idx = kmix;
      CK(hipMemset(d_out_ref, 0xFF, n * (L + 12)));
      seal_new(a);
      hipLaunchKernelGGL((qfec::aes128gcm_kernel<4, false, 4, 768, 3, true>),
                         dim3((uint32_t)((n + 767) / 768)), dim3(768), 0, 0, r);
      CK(hipDeviceSynchronize());
      const auto x = down(d_out, n * (L + 12)), y = down(d_out_ref, n * (L + 12));
      const bool same = x == y;
      std::printf("seal 768/wpe3 variant %s == product: %s\n", mix ? "mixed-key" : "one-key",
                  same ? "yes" : "NO");
      bad |= !same;
      if (kmix) CK(hipFree(kmix));
    }
  }
  {  // random lengths (payload 0..1452, header 0..59), 69 keys / 5 keys / 1 key:
     // every variant against the first kernel
    const uint64_t rn = 4096;
    std::vector<uint64_t> r_ad_off(rn), r_in_off(rn), r_out_off(rn);
    std::vector<uint16_t> r_ad_len(rn), r_in_len(rn);
    uint64_t pos = 0, opos = 0, st = 0x9E3779B97F4A7C15ull;
    auto rnd = [&](uint64_t m) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st % m; };
    for (uint64_t p = 0; p < rn; ++p) {
      r_ad_len[p] = (uint16_t)rnd(60);
      r_in_len[p] = (uint16_t)rnd(1453);
      r_ad_off[p] = pos;
      pos += r_ad_len[p] + rnd(9);
      r_in_off[p] = pos;
      pos += r_in_len[p] + rnd(9);
      r_out_off[p] = opos;
      opos += r_in_len[p] + 12;
    }
    qfec::AeadArgs ra = as;
    ra.io.ad_off = up(r_ad_off);
    ra.io.ad_len = up(r_ad_len);
    ra.io.in_off = up(r_in_off);
    ra.io.in_len = up(r_in_len);
    ra.io.out_off = up(r_out_off);
    ra.io.n = rn;
    for (uint32_t nk : {1u, 5u, 7u}) {
      std::vector<uint32_t> kk(rn);
      for (uint64_t p = 0; p < rn; ++p) kk[p] = nk == 1 ? 0u : (uint32_t)rnd(nk);
      uint32_t* dk = up(kk);
      ra.key_idx = dk;
      qfec::AeadArgs rr = ra;
      rr.io.out = d_out_ref;
      CK(hipMemset(d_out_ref, 0xFF, opos));
      hipLaunchKernelGGL((qfec::gcm_v1::aes128gcm_kernel<8, false>), dim3((uint32_t)((rn + 255) / 256)),
                         dim3(256), 0, 0, rr);
      CK(hipDeviceSynchronize());
      const auto want = down(d_out_ref, opos);
      struct RV { const char* name; std::function<void()> run; };
      std::vector<RV> rvs = {
          {"product", [&] { seal_new(ra); }},
          {"SC8 512 wpe2 uni", [&] { hipLaunchKernelGGL((qfec::aes128gcm_kernel<8, false, 4, 512, 2, true>), dim3((uint32_t)((rn + 511) / 512)), dim3(512), 0, 0, ra); }},
          {"SC8 512 wpe2 lane", [&] { hipLaunchKernelGGL((qfec::aes128gcm_kernel<8, false, 4, 512, 2, false>), dim3((uint32_t)((rn + 511) / 512)), dim3(512), 0, 0, ra); }},
          {"SC4 512 wpe2 uni", [&] { hipLaunchKernelGGL((qfec::aes128gcm_kernel<4, false, 4, 512, 2, true>), dim3((uint32_t)((rn + 511) / 512)), dim3(512), 0, 0, ra); }},
          {"SC4 768 wpe3 lane", [&] { hipLaunchKernelGGL((qfec::aes128gcm_kernel<4, false, 4, 768, 3, false>), dim3((uint32_t)((rn + 767) / 768)), dim3(768), 0, 0, ra); }},
          {"SC4 768 wpe3 NB2", [&] { hipLaunchKernelGGL((qfec::aes128gcm_kernel<4, false, 2, 768, 3, true>), dim3((uint32_t)((rn + 767) / 768)), dim3(768), 0, 0, ra); }},
      };
      for (auto& v : rvs) {
        CK(hipMemset(d_out, 0, opos));
        v.run();
        CK(hipDeviceSynchronize());
        const auto got = down(d_out, opos);
        uint64_t diff = 0, ctdiff = 0, shown = 0;
        for (uint64_t p = 0; p < rn; ++p)
          if (std::memcmp(&got[r_out_off[p]], &want[r_out_off[p]], r_in_len[p] + 12) != 0) {
            ++diff;
            uint32_t j = 0;
            while (got[r_out_off[p] + j] == want[r_out_off[p] + j]) ++j;
            if (j < r_in_len[p]) ++ctdiff;
            if (shown++ < 3)
              std::printf("   packet %llu len %u (nfull %u): first differing byte %u\n",
                          (unsigned long long)p, r_in_len[p], r_in_len[p] / 16u, j);
          }
        if (diff) std::printf("   %llu of them differ in the ciphertext\n", (unsigned long long)ctdiff);
        std::printf("random batch %u keys, %-20s differing packets: %llu / %llu\n", nk, v.name,
                    (unsigned long long)diff, (unsigned long long)rn);
      }
      CK(hipFree(dk));
    }
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
#define GCMV(NAME, BYTES, ARGS, SCV, OPENV, NBV, BLK, WPE, UNI)                             \
  {NAME, BYTES, [&] {                                                                      \
     hipLaunchKernelGGL((qfec::aes128gcm_kernel<SCV, OPENV, NBV, BLK, WPE, UNI>),          \
                        dim3((uint32_t)((n + BLK - 1) / BLK)), dim3(BLK), 0, 0, ARGS);     \
   }}
  std::vector<V> vs = {
      {"seal product", enc_b, [&] { seal_new(as); }},
      {"seal first kernel", enc_b, [&] { seal_old(as); }},
      {"open product", dec_b, [&] { open_new(ao); }},
      {"open first kernel", dec_b, [&] { open_old(ao); }},
      GCMV("seal SC8 512 wpe2 per-lane keys", enc_b, as, 8, false, 4, 512, 2, false),
      GCMV("seal SC8 512 wpe2 uniform keys", enc_b, as, 8, false, 4, 512, 2, true),
      GCMV("open SC8 512 wpe2 uniform keys", dec_b, ao, 8, true, 4, 512, 2, true),
      GCMV("open SC8 512 wpe2 per-lane keys", dec_b, ao, 8, true, 4, 512, 2, false),
      GCMV("seal SC4 768 wpe3 uniform keys", enc_b, as, 4, false, 4, 768, 3, true),
      GCMV("seal SC4 768 wpe3 NB2", enc_b, as, 4, false, 2, 768, 3, true),
      GCMV("open SC4 768 wpe3 uniform keys", dec_b, ao, 4, true, 4, 768, 3, true),
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
