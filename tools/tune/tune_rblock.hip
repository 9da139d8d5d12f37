// tune_rblock.hip — A/B of ragged_block_kernel forms on the configs[3] batch
// (2^20 groups, k 5-15, payloads 64-1350 B), one process,
// variants interleaved round by round; every variant's outputs (parity rows,
// parity lengths, revived rows) are compared byte for byte with the
// product's before it is timed.
//
//   tune_rblock [reps=10] [rounds=5] [palign=16] [slot=1536] [mode=0] [kmin kmax lmin lmax]
//     palign 16: payloads on 16-B boundaries (the payload arena's layout);
//     palign 1: byte-packed.  slot: parity / revived row stride per group.
//     mode 1: also the DIAG forms (whole-line stores; no stores; no tail);
//     mode 2: the block kernel against ragged_multi_kernel (two groups per
//     wave) on the given group shape (round 6's band table); mode 3: the
//     payload loads / parity stores through the caches instead of nontemporal;
//     mode 4: parity stores with explicit cache policies (sc1, sc0 sc1, nt sc1, ...).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_rblock.hip \
//          -o tools/tune/build/tune_rblock
#include "../../libquic_amd/csrc/qfec_kernels.hip"

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

using qfec::RaggedArgs;

static uint64_t sm64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
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

struct V {
  std::string name;
  bool rec;
  std::function<void(const RaggedArgs&)> run;
};

// (round 4: a TL template flag -- full windows only in the flat loop, each
// packet's partial last window by one lane after it -- measured exact and
// 0.59-0.62 against the product's 0.69-0.71: profiles/round4/ragged_tl/,
// commit ddd19fd; removed from the product)
#define BLK(REC, U, TL)                                                                    \
  [=](const RaggedArgs& a) {                                                               \
    static_assert(!TL, "TL variant removed");                                              \
    hipLaunchKernelGGL((qfec::ragged_block_kernel<REC, 4, 8, U, true, true, 0>),          \
                       dim3((uint32_t)((a.n_groups + 7) / 8)), dim3(256), 0, 0, a);        \
  }
// round 6: DIAG 1 (no stores), 2 (output rows stored as whole 128-B lines,
// zeros past the parity length: compared against the product's rows with the
// output buffers zeroed first, so the padding reads back as the product's),
// 4 (no tail logic: every window XORed whole), 5 (4 without stores)
#define BLKD(REC, D)                                                                       \
  [=](const RaggedArgs& a) {                                                               \
    hipLaunchKernelGGL((qfec::ragged_block_kernel<REC, 4, 8, 2, true, true, D>),          \
                       dim3((uint32_t)((a.n_groups + 7) / 8)), dim3(256), 0, 0, a);        \
  }

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const uint64_t G = 1 << 20;
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const uint64_t palign = argc > 3 ? (uint64_t)atoi(argv[3]) : 16u;
  const uint64_t slot = argc > 4 ? (uint64_t)atoi(argv[4]) : 1536u;
  const uint64_t seed = 0x51554944;
  std::vector<uint32_t> ptr{0};
  std::vector<uint16_t> len;
  std::vector<uint64_t> off, poff(G);
  std::vector<uint8_t> miss(G);
  uint64_t bytes = 0;
  double enc_alg = 0, rec_alg = 0;
  // round 6: the group shape (default configs[3]: k 5-15, 64-1350 B)
  const uint32_t kmin = argc > 6 ? (uint32_t)atoi(argv[6]) : 5u;
  const uint32_t kmax = argc > 7 ? (uint32_t)atoi(argv[7]) : 15u;
  const uint32_t lmin = argc > 8 ? (uint32_t)atoi(argv[8]) : 64u;
  const uint32_t lmax = argc > 9 ? (uint32_t)atoi(argv[9]) : 1350u;
  for (uint64_t g = 0; g < G; ++g) {
    const uint32_t k = kmin + (uint32_t)(sm64(seed ^ (0x6Bull << 56) ^ g) % (kmax - kmin + 1u));
    miss[g] = (uint8_t)(sm64(seed ^ (0x4Dull << 56) ^ g) % k);
    uint32_t mx = 0;
    double s = 0, sm = 0;
    for (uint32_t i = 0; i < k; ++i) {
      const uint32_t ln = lmin + (uint32_t)(sm64(seed ^ (0x4Cull << 56) ^ (g * 256 + i)) % (lmax - lmin + 1u));
      len.push_back((uint16_t)ln);
      off.push_back(bytes);
      bytes += (ln + palign - 1) / palign * palign;
      s += ln;
      if (i != miss[g]) sm += ln;
      mx = std::max(mx, ln);
    }
    enc_alg += s + mx;       // every packet read, the parity row written
    rec_alg += sm + 2.0 * mx;  // received packets + parity read, the revived row written
    ptr.push_back((uint32_t)len.size());
    poff[g] = g * slot;
  }
  uint8_t* data;
  CK(hipMalloc(&data, bytes + 4096));
  CK(hipMemset(data, 0x77, bytes + 4096));  // gaps between aligned payloads: not zero
  uint64_t* d_off = up(off);
  uint16_t* d_len = up(len);
  uint32_t* d_ptr = up(ptr);
  uint64_t* d_poff = up(poff);
  uint8_t* d_miss = up(miss);
  CK(qfec::launch_synth_ragged(data, d_off, d_len, d_ptr, 0, G, seed, 0));
  const uint64_t OB = G * slot;
  uint8_t *par_ref, *out_ref, *buf;
  uint16_t *plen_ref, *plen_v;
  uint32_t* err;
  CK(hipMalloc(&par_ref, OB));
  CK(hipMalloc(&out_ref, OB));
  CK(hipMalloc(&buf, OB));
  CK(hipMalloc(&plen_ref, G * 2));
  CK(hipMalloc(&plen_v, G * 2));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  CK(hipMemset(par_ref, 0, OB));  // (zero: the DIAG 2 rows' padding compares equal)
  CK(hipMemset(out_ref, 0, OB));

  RaggedArgs e{};
  e.bytes = data;
  e.pkt_off = d_off;
  e.pkt_len = d_len;
  e.grp_ptr = d_ptr;
  e.parity_off = d_poff;
  e.parity_len_out = plen_ref;
  e.out = par_ref;
  e.n_groups = G;
  e.err = err;
  RaggedArgs r = e;
  r.parity = par_ref;
  r.parity_len = plen_ref;
  r.missing = d_miss;
  r.out_off = d_poff;
  r.parity_len_out = nullptr;
  r.out = out_ref;
  BLK(false, 2, false)(e);  // the product's outputs: the reference of every variant
  BLK(true, 2, false)(r);
  CK(hipDeviceSynchronize());
  RaggedArgs ev = e, rv = r;  // variants write elsewhere
  ev.out = buf;
  ev.parity_len_out = plen_v;
  rv.out = buf;

  std::vector<V> vs;
  const int mode = argc > 5 ? atoi(argv[5]) : 0;
  if (mode == 2) {  // round 6 band table: the block kernel against two groups per wave
#define MULTI(REC)                                                                          \
  [=](const RaggedArgs& a) {                                                                \
    hipLaunchKernelGGL((qfec::ragged_multi_kernel<REC, true, 2, 2, 4>),                     \
                       dim3((uint32_t)((a.n_groups + 7) / 8)), dim3(256), 0, 0, a);         \
  }
    vs.push_back({"block encode", false, BLK(false, 2, false)});
    vs.push_back({"multi2 encode", false, MULTI(false)});
    vs.push_back({"block recover", true, BLK(true, 2, false)});
    vs.push_back({"multi2 recover", true, MULTI(true)});
  } else {
  vs.push_back({"product AL U2 encode", false, BLK(false, 2, false)});
  vs.push_back({"product AL U1 encode", false, BLK(false, 1, false)});
  vs.push_back({"product AL U2 encode (again)", false, BLK(false, 2, false)});
  vs.push_back({"product AL U2 recover", true, BLK(true, 2, false)});
  vs.push_back({"product AL U1 recover", true, BLK(true, 1, false)});
  if (mode == 3) {  // round 6: cache policy of the payload loads / parity stores
    vs.push_back({"cached stores encode", false, BLKD(false, 8)});
    vs.push_back({"cached stores recover", true, BLKD(true, 8)});
    vs.push_back({"cached loads encode", false, BLKD(false, 16)});
    vs.push_back({"cached loads recover", true, BLKD(true, 16)});
    vs.push_back({"cached both encode", false, BLKD(false, 24)});
    vs.push_back({"cached both recover", true, BLKD(true, 24)});
  }
  if (mode == 4) {  // round 6: explicit store policies (st16pol)
    vs.push_back({"stores sc1 encode", false, BLKD(false, 32)});
    vs.push_back({"stores sc0 sc1 encode", false, BLKD(false, 64)});
    vs.push_back({"stores nt sc1 encode", false, BLKD(false, 96)});
    vs.push_back({"stores nt sc0 sc1 encode", false, BLKD(false, 128)});
    vs.push_back({"stores sc1 recover", true, BLKD(true, 32)});
    vs.push_back({"stores nt sc1 recover", true, BLKD(true, 96)});
  }
  const bool diag = mode == 1;
  if (diag) {
    vs.push_back({"whole-line stores encode", false, BLKD(false, 2)});
    vs.push_back({"whole-line stores recover", true, BLKD(true, 2)});
    vs.push_back({"no stores encode (inexact)", false, BLKD(false, 1)});
    vs.push_back({"no stores recover (inexact)", true, BLKD(true, 1)});
    vs.push_back({"no tail logic encode (inexact)", false, BLKD(false, 4)});
    vs.push_back({"no tail, no stores enc (inexact)", false, BLKD(false, 5)});
  }
  }

  std::vector<uint8_t> h_ref(OB), h_v(OB);
  std::vector<uint16_t> hp_ref(G), hp_v(G);
  CK(hipMemcpy(hp_ref.data(), plen_ref, G * 2, hipMemcpyDeviceToHost));
  bool all_ok = true;
  for (const V& v : vs) {
    CK(hipMemset(buf, 0, OB));
    CK(hipMemset(plen_v, 0, G * 2));
    CK(hipMemset(err, 0, 4));
    v.run(v.rec ? rv : ev);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h_ref.data(), v.rec ? out_ref : par_ref, OB, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h_v.data(), buf, OB, hipMemcpyDeviceToHost));
    uint32_t e_h = 0;
    CK(hipMemcpy(&e_h, err, 4, hipMemcpyDeviceToHost));
    bool ok = h_ref == h_v && e_h == 0;
    if (!v.rec) {
      CK(hipMemcpy(hp_v.data(), plen_v, G * 2, hipMemcpyDeviceToHost));
      ok = ok && hp_ref == hp_v;
    }
    std::printf("check %-26s == product: %s (err %u)\n", v.name.c_str(), ok ? "yes" : "NO", e_h);
    if (v.name.find("inexact") == std::string::npos) all_ok = all_ok && ok;
  }
  if (!all_ok) return 2;

  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  std::vector<std::vector<float>> ms(vs.size());
  for (int rd = 0; rd < rounds; ++rd) {
    for (size_t i = 0; i < vs.size(); ++i) {
      const V& v = vs[i];
      v.run(v.rec ? rv : ev);  // warm
      CK(hipEventRecord(t0, 0));
      for (int q = 0; q < reps; ++q) v.run(v.rec ? rv : ev);
      CK(hipEventRecord(t1, 0));
      CK(hipEventSynchronize(t1));
      float m = 0;
      CK(hipEventElapsedTime(&m, t0, t1));
      ms[i].push_back(m / reps);
    }
  }
  std::printf("\n%llu groups, k %u-%u, len %u-%u (%.0f B per group), palign %llu, slot %llu; "
              "algorithmic GB: encode %.3f, recover %.3f\n",
              (unsigned long long)G, kmin, kmax, lmin, lmax, enc_alg / (double)G,
              (unsigned long long)palign, (unsigned long long)slot, enc_alg / 1e9, rec_alg / 1e9);
  for (size_t i = 0; i < vs.size(); ++i) {
    std::vector<float> s = ms[i];
    std::sort(s.begin(), s.end());
    const double med = s[s.size() / 2] * 1e-3;
    const double gbs = (vs[i].rec ? rec_alg : enc_alg) / med / 1e9;
    std::printf("%-26s median %8.1f us  min %8.1f us  %7.1f GB/s  %.4f of 8 TB/s\n",
                vs[i].name.c_str(), med * 1e6, s[0] * 1e3, gbs, gbs / 8000.0);
  }
  return 0;
}
