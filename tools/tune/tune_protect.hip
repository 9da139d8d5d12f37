// tune_protect.hip — throughput of the NULL packet-protection kernels on the
// headline packet shape (1350-B payload, 22-B header), device-resident, and a
// VALU microbenchmark of the FNV-1a-128 byte step.  One process, interleaved.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_protect.hip -o tools/tune/build/tune_protect
#include "../../libquic_amd/csrc/qpp_kernels.hip"
#include "prev_protect.inc"

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

template <typename T>
static T* up(const std::vector<T>& v) {
  T* d;
  CK(hipMalloc(&d, v.size() * sizeof(T)));
  CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

// pure VALU: hash `bytes` synthetic bytes per lane from registers
__global__ void fnv_valu_kernel(uint32_t bytes, uint32_t* sink) {
  qfec::Fnv128 h = qfec::fnv_init();
  uint32_t w = threadIdx.x * 0x9E3779B9u;
  for (uint32_t i = 0; i < bytes; i += 4) {
    qfec::fnv_word(h, w);
    w = w * 1664525u + 1013904223u;
  }
  if ((h.x0 ^ h.x1 ^ h.x2 ^ h.x3) == 0x12345678u) sink[0] = h.x0;
}

// pure VALU, 16-byte chunks as the staged kernels hash them (R3 or byte-serial)
template <bool R3>
__global__ void fnv_valu_chunk_kernel(uint32_t bytes, uint32_t* sink) {
  qfec::Fnv128 h = qfec::fnv_init();
  uint32_t w = threadIdx.x * 0x9E3779B9u;
  for (uint32_t i = 0; i < bytes; i += 16) {
    const qfec::u32x4 v = {w, w ^ 0x5bd1e995u, w * 3u + 1u, w + 0x27d4eb2du};
    qfec::fnv_chunk<R3>(h, v);
    w = w * 1664525u + 1013904223u;
  }
  if ((h.x0 ^ h.x1 ^ h.x2 ^ h.x3) == 0x12345678u) sink[0] = h.x0;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 21);
  const uint32_t L = 1350, H = 22;
  const int reps = 5, rounds = 3;
  // packets: [header H | payload L] records back to back; outputs tag||payload
  std::vector<uint64_t> ad_off(n), in_off(n), out_off(n), dad_off(n), dct_off(n), dout_off(n);
  std::vector<uint16_t> ad_len(n, H), in_len(n, L), ct_len(n, L + 12);
  for (uint64_t p = 0; p < n; ++p) {
    ad_off[p] = p * (H + L);
    in_off[p] = p * (H + L) + H;
    out_off[p] = p * (L + 12);
    dout_off[p] = p * L;
  }
  uint8_t *d_in, *d_out, *d_out2, *d_ok;
  CK(hipMalloc(&d_in, n * (H + L)));
  CK(hipMalloc(&d_out, n * (L + 12)));
  CK(hipMalloc(&d_out2, n * L));
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
  qfec::ProtectArgs e{};
  e.bytes = d_in; e.ad_off = up(ad_off); e.ad_len = up(ad_len); e.in_off = up(in_off);
  e.in_len = up(in_len); e.out = d_out; e.out_off = up(out_off); e.n = n;
  CK(qfec::launch_null_protect(e, false, 0));
  CK(hipDeviceSynchronize());
  // decrypt input: [header | ciphertext] -> header from d_in, ciphertext in d_out
  // (two buffers: pass offsets relative to d_in? use one combined buffer instead)
  uint8_t* d_cat;
  CK(hipMalloc(&d_cat, n * (H + L + 12)));
  for (uint64_t p = 0; p < n; ++p) {
    dad_off[p] = p * (H + L + 12);
    dct_off[p] = dad_off[p] + H;
  }
  CK(hipMemcpy2D(d_cat, H + L + 12, d_in, H + L, H, n, hipMemcpyDeviceToDevice));
  CK(hipMemcpy2D(d_cat + H, H + L + 12, d_out, L + 12, L + 12, n, hipMemcpyDeviceToDevice));
  qfec::ProtectArgs d{};
  d.bytes = d_cat; d.ad_off = up(dad_off); d.ad_len = e.ad_len; d.in_off = up(dct_off);
  d.in_len = up(ct_len); d.out = d_out2; d.out_off = up(dout_off); d.ok = d_ok; d.n = n;
  CK(qfec::launch_null_protect(d, true, 0));
  CK(hipDeviceSynchronize());
  {
    std::vector<uint8_t> ok(n);
    CK(hipMemcpy(ok.data(), d_ok, n, hipMemcpyDeviceToHost));
    uint64_t good = 0;
    for (auto v : ok) good += v;
    std::printf("decrypt(encrypt) verified: %llu / %llu\n", (unsigned long long)good,
                (unsigned long long)n);
  }
  // ChaCha20-Poly1305: one key, packet numbers 1..n; seal out = ct || tag
  std::vector<uint8_t> key(32), pre(4);
  for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 7 + 1);
  for (int i = 0; i < 4; ++i) pre[i] = (uint8_t)(0xA0 + i);
  std::vector<uint32_t> kidx(n, 0);
  std::vector<uint64_t> pns(n);
  for (uint64_t p = 0; p < n; ++p) pns[p] = p + 1;
  qfec::AeadArgs as{};
  as.io = e;
  as.keys = up(key);
  as.prefixes = up(pre);
  as.key_idx = up(kidx);
  as.packet_number = up(pns);
  as.path_id = nullptr;
  CK(qfec::launch_chacha20poly1305(as, false, 0));
  CK(hipDeviceSynchronize());
  // open input: [header | ct || tag] records in a buffer of their own
  uint8_t* d_cat2;
  CK(hipMalloc(&d_cat2, n * (H + L + 12)));
  CK(hipMemcpy2D(d_cat2, H + L + 12, d_in, H + L, H, n, hipMemcpyDeviceToDevice));
  CK(hipMemcpy2D(d_cat2 + H, H + L + 12, d_out, L + 12, L + 12, n, hipMemcpyDeviceToDevice));
  qfec::AeadArgs ao = as;
  ao.io = d;
  ao.io.bytes = d_cat2;
  CK(qfec::launch_chacha20poly1305(ao, true, 0));
  CK(hipDeviceSynchronize());
  {
    std::vector<uint8_t> ok(n);
    CK(hipMemcpy(ok.data(), d_ok, n, hipMemcpyDeviceToHost));
    uint64_t good = 0;
    for (auto v : ok) good += v;
    std::printf("chacha20poly1305 open(seal) verified: %llu / %llu\n", (unsigned long long)good,
                (unsigned long long)n);
  }
  uint32_t* sink;
  CK(hipMalloc(&sink, 4));
  struct V {
    std::string name;
    double bytes;  // algorithmic bytes (HBM) per launch
    double hashed; // bytes run through FNV per launch
    std::function<void()> run;
  };
  const double enc_b = (double)n * (H + L + L + 12), dec_b = (double)n * (H + L + 12 + L);
  const double hashed = (double)n * (H + L);
  const uint32_t vb = 4096, vgrid = 256 * 8 * 4;  // 8 waves/SIMD worth of lanes... per CU
  std::vector<V> vs = {
      {"null encrypt staged (product)", enc_b, hashed, [&] { CK(qfec::launch_null_protect(e, false, 0)); }},
      {"null decrypt staged (product)", dec_b, hashed, [&] { CK(qfec::launch_null_protect(d, true, 0)); }},
      {"chacha20poly1305 seal (product)", enc_b, hashed, [&] { CK(qfec::launch_chacha20poly1305(as, false, 0)); }},
      {"chacha20poly1305 open (product)", dec_b, hashed, [&] { CK(qfec::launch_chacha20poly1305(ao, true, 0)); }},
      {"chacha20poly1305 seal SC=16", enc_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::c20p1305_seal_kernel<16>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, as); }},
      {"chacha20poly1305 open SC=16", dec_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::c20p1305_open_kernel<16>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, ao); }},
      {"chacha20poly1305 seal SC=8", enc_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::c20p1305_seal_kernel<8>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, as); }},
      {"chacha20poly1305 open SC=8", dec_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::c20p1305_open_kernel<8>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, ao); }},
      {"chacha20poly1305 seal SC=4", enc_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::c20p1305_seal_kernel<4>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, as); }},
      {"null encrypt staged SC=4", enc_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::null_encrypt_staged_kernel<4>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, e); }},
      {"null encrypt staged SC=8", enc_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::null_encrypt_staged_kernel<8>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, e); }},
      {"null encrypt direct (lane loads)", enc_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::null_encrypt_direct_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, e); }},
      {"null decrypt direct (lane loads)", dec_b, hashed, [&] {
         hipLaunchKernelGGL(qfec::null_decrypt_direct_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, d); }},
      {"FNV step VALU-only (4 KiB/lane)", 0.0, (double)vgrid * 256 * vb,
       [&] { hipLaunchKernelGGL(fnv_valu_kernel, dim3(vgrid), dim3(256), 0, 0, vb, sink); }},
      {"FNV chunk VALU-only R3", 0.0, (double)vgrid * 256 * vb,
       [&] { hipLaunchKernelGGL(fnv_valu_chunk_kernel<true>, dim3(vgrid), dim3(256), 0, 0, vb, sink); }},
      {"FNV chunk VALU-only serial", 0.0, (double)vgrid * 256 * vb,
       [&] { hipLaunchKernelGGL(fnv_valu_chunk_kernel<false>, dim3(vgrid), dim3(256), 0, 0, vb, sink); }},
      {"null encrypt staged serial FNV", enc_b, hashed, [&] {
         hipLaunchKernelGGL((qfec::null_encrypt_staged_kernel<16, false>), dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, e); }},
      {"null decrypt staged serial FNV", dec_b, hashed, [&] {
         hipLaunchKernelGGL((qfec::null_decrypt_staged_kernel<16, false>), dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, 0, d); }},
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
  std::printf("%-40s %10s %10s %12s\n", "variant", "ms", "HBM GB/s", "hashed GB/s");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = ms[i];
    std::sort(v.begin(), v.end());
    const double t = v[v.size() / 2] * 1e-3;
    std::printf("%-40s %10.3f %10.1f %12.1f\n", vs[i].name.c_str(), t * 1e3, vs[i].bytes / t / 1e9,
                vs[i].hashed / t / 1e9);
  }
  return 0;
}
