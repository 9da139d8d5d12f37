// ragged_variants.hip — correctness stress of the flat-window ragged kernel's
// build variants (unroll U, b32/b64 LDS XOR atomics, cache policy) on the
// GPU: bad-group counts over repeated encode + recover runs of 20,000 ragged
// groups against a host reference.  The b64 + U4 build fails ~1% of recover
// groups, nondeterministically (root cause not found; the product uses b32).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/debug/ragged_variants.hip -o tools/debug/build/ragged_variants
#include "../../libquic_amd/csrc/qfec_kernels.hip"
#include "../tune/ragged_legacy.inc"


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

int main(int argc, char** argv) {
  const int REPS = argc > 1 ? atoi(argv[1]) : 4;
  const uint64_t G = 20000;
  std::vector<uint32_t> ptr{0};
  std::vector<uint16_t> len;
  std::vector<uint64_t> off;
  std::vector<uint8_t> miss(G);
  uint64_t bytes = 0;
  for (uint64_t g = 0; g < G; ++g) {
    const uint32_t k = 5 + (uint32_t)(sm64(0x1234 ^ g) % 11);
    for (uint32_t i = 0; i < k; ++i) {
      const uint32_t l = 64 + (uint32_t)(sm64(0x5678 ^ (g * 256 + i)) % 1287);
      len.push_back((uint16_t)l);
      off.push_back(bytes);
      bytes += l;
    }
    ptr.push_back((uint32_t)len.size());
    miss[g] = (uint8_t)(sm64(0x9abc ^ g) % k);
  }
  std::vector<uint8_t> data(bytes);
  for (uint64_t j = 0; j < bytes; ++j) data[j] = (uint8_t)sm64(j * 7919);
  // host reference parity, plen and recovered rows
  std::vector<uint8_t> par(G * 1452, 0), rec(G * 1452, 0);
  std::vector<uint16_t> plen(G);
  for (uint64_t g = 0; g < G; ++g) {
    uint32_t mx = 0;
    for (uint32_t p = ptr[g]; p < ptr[g + 1]; ++p) {
      for (uint32_t j = 0; j < len[p]; ++j) par[g * 1452 + j] ^= data[off[p] + j];
      mx = std::max<uint32_t>(mx, len[p]);
    }
    plen[g] = (uint16_t)mx;
    for (uint32_t j = 0; j < mx; ++j) rec[g * 1452 + j] = par[g * 1452 + j];
    for (uint32_t p = ptr[g]; p < ptr[g + 1]; ++p) {
      if (p - ptr[g] == miss[g]) continue;
      for (uint32_t j = 0; j < len[p]; ++j) rec[g * 1452 + j] ^= data[off[p] + j];
    }
  }
  std::vector<uint64_t> poff(G);
  for (uint64_t g = 0; g < G; ++g) poff[g] = g * 1452;
  uint8_t* d_data = up(data);
  uint64_t* d_off = up(off);
  uint16_t* d_len = up(len);
  uint32_t* d_ptr = up(ptr);
  uint64_t* d_poff = up(poff);
  uint8_t* d_par = up(par);
  uint16_t* d_plen = up(plen);
  uint8_t* d_miss = up(miss);
  uint8_t *d_out, *d_enc;
  uint16_t* d_plen2;
  uint32_t* d_err;
  CK(hipMalloc(&d_out, G * 1452));
  CK(hipMalloc(&d_enc, G * 1452));
  CK(hipMalloc(&d_plen2, G * 2));
  CK(hipMalloc(&d_err, 4));
  CK(hipMemset(d_err, 0, 4));
  qfec::RaggedArgs a{};
  a.bytes = d_data;
  a.pkt_off = d_off;
  a.pkt_len = d_len;
  a.grp_ptr = d_ptr;
  a.n_groups = G;
  a.err = d_err;
  qfec::RaggedArgs ar = a, ae = a;
  ar.parity = d_par;
  ar.parity_off = d_poff;
  ar.parity_len = d_plen;
  ar.missing = d_miss;
  ar.out = d_out;
  ar.out_off = d_poff;
  ae.parity_off = d_poff;
  ae.parity_len_out = d_plen2;
  ae.out = d_enc;
  struct V {
    std::string name;
    std::function<void(bool)> run;  // arg: recover?
  };
  using namespace qfec;
  const dim3 grid((uint32_t)((G + 3) / 4)), blk(256);
#define QV(NAME, NT, U, ACC)                                                                    \
  {NAME, [&](bool r) {                                                                          \
     if (r) hipLaunchKernelGGL((ragged_xor_kernel<true, NT, U, 4, ACC>), grid, blk, 0, 0, ar);  \
     else hipLaunchKernelGGL((ragged_xor_kernel<false, NT, U, 4, ACC>), grid, blk, 0, 0, ae);   \
   }}
  std::vector<V> vs = {
      {"product", [&](bool r) { CK(launch_ragged(r ? ar : ae, r, 0)); }},
      QV("nt U2 b32", true, 2, 0),    QV("nt U4 b32", true, 4, 0),
      QV("nt U8 b32", true, 8, 0),    QV("def U4 b32", false, 4, 0),
      QV("nt U2 b32cm", true, 2, 1),  QV("nt U4 b32cm", true, 4, 1),
      QV("def U2 b32cm", false, 2, 1), QV("nt U1 b32cm", true, 1, 1),
      QV("nt U2 b64", true, 2, 2),    QV("nt U4 b64", true, 4, 2),
      QV("nt U8 b64", true, 8, 2),    QV("def U4 b64", false, 4, 2),
  };
#undef QV
  std::vector<uint8_t> h(G * 1452);
  for (auto& v : vs) {
    std::printf("%-24s", v.name.c_str());
    int tot[2] = {0, 0};
    for (int rep = 0; rep < REPS; ++rep) {
      for (int which = 0; which < 2; ++which) {
        const bool r = which == 1;
        uint8_t* dst = r ? d_out : d_enc;
        CK(hipMemset(dst, 0, G * 1452));
        v.run(r);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), dst, G * 1452, hipMemcpyDeviceToHost));
        const std::vector<uint8_t>& want = r ? rec : par;
        int bad = 0;
        for (uint64_t g = 0; g < G; ++g)
          bad += std::memcmp(&h[g * 1452], &want[g * 1452], plen[g]) != 0;
        if (bad) std::printf(" %s[%d]:%d", r ? "rec" : "enc", rep, bad);
        tot[r] += bad;
      }
    }
    uint32_t err;
    CK(hipMemcpy(&err, d_err, 4, hipMemcpyDeviceToHost));
    std::printf("  total bad enc %d rec %d over %d reps, err=%u\n", tot[0], tot[1], REPS, err);
  }
  return 0;
}
