// tune_rchunk.hip — A/B of the chunk-phased ragged kernel (ragged_chunk_kernel,
// qfec_kernels.hip) against the product ragged_multi_kernel on the BASELINE
// configs[3] batch (2^20 groups, k 5-15, 64-1350 B, packed CSR), encode and
// recover, interleaved rounds in one process; every variant's bytes (and
// parity lengths) are compared with the product's.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_rchunk.hip -o tools/tune/build/tune_rchunk
// run:   tune_rchunk [reps] [rounds]
#include "../../libquic_amd/csrc/qfec_kernels.hip"
#include "ragged_legacy.inc"
#include "ragged_chunk.inc"

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

template <bool REC>
static void launch_multi(const RaggedArgs& a, uint64_t G) {
  hipLaunchKernelGGL((qfec::ragged_multi_kernel<REC, true, 2>), dim3((uint32_t)((G + 7) / 8)),
                     dim3(256), 0, 0, a);
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const uint64_t G = 1 << 20;
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int rounds = argc > 2 ? atoi(argv[2]) : 4;
  const uint64_t seed = 0x51554944;
  std::vector<uint32_t> ptr{0};
  std::vector<uint16_t> len;
  std::vector<uint64_t> off, poff(G);
  std::vector<uint8_t> miss(G);
  uint64_t bytes = 0;
  double enc_alg = 0, rec_alg = 0;
  for (uint64_t g = 0; g < G; ++g) {
    const uint32_t k = 5 + (uint32_t)(sm64(seed ^ (0x6Bull << 56) ^ g) % 11);
    miss[g] = (uint8_t)(sm64(seed ^ (0x4Dull << 56) ^ g) % k);
    uint32_t mx = 0;
    double s = 0, sm = 0;
    for (uint32_t i = 0; i < k; ++i) {
      const uint32_t ln = 64 + (uint32_t)(sm64(seed ^ (0x4Cull << 56) ^ (g * 256 + i)) % 1287);
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
    poff[g] = g * 1452;
  }
  uint8_t* data;
  CK(hipMalloc(&data, bytes + 4096));
  uint64_t* d_off = up(off);
  uint16_t* d_len = up(len);
  uint32_t* d_ptr = up(ptr);
  uint64_t* d_poff = up(poff);
  uint8_t* d_miss = up(miss);
  CK(qfec::launch_synth_ragged(data, d_off, d_len, d_ptr, 0, G, seed, 0));
  uint8_t *par, *out;
  uint16_t *plen, *plen2;
  uint32_t *err, *psync;
  CK(hipMalloc(&par, G * 1452));
  CK(hipMalloc(&out, G * 1452));
  CK(hipMalloc(&plen, G * 2));
  CK(hipMalloc(&plen2, G * 2));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&psync, 20 * 256));
  CK(hipMemset(err, 0, 4));
  CK(hipMemset(psync, 0, 20 * 256));
  CK(hipMemset(par, 0, G * 1452));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
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
  launch_multi<false>(e, G);  // reference parity (and lengths) for the recover runs
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
  vs.push_back({"multi2 encode", false, [=](const RaggedArgs& a) { launch_multi<false>(a, G); }});
#define RC(REC, U, GP, MEET)                                                                     \
  vs.push_back({std::string("chunk U" #U " GP" #GP " M" #MEET " ") + (REC ? "recover" : "encode"), REC, \
                [=](const RaggedArgs& a0) {                                                      \
                  const uint64_t per = (uint64_t)ncu * GP;                                       \
                  hipLaunchKernelGGL((qfec::ragged_chunk_kernel<REC, U, GP, false, MEET>), dim3(ncu), \
                                     dim3(qfec::kRcThreads), 0, 0, a0,                           \
                                     (uint32_t)((G + per - 1) / per), psync, nullptr);          \
                }})
#define RC2(REC, U, Q)                                                                          \
  vs.push_back({std::string("chunk2 U" #U " Q" #Q " ") + (REC ? "recover" : "encode"), REC,     \
                [=](const RaggedArgs& a0) {                                                      \
                  const uint64_t per = (uint64_t)ncu * 80;                                       \
                  hipLaunchKernelGGL((qfec::ragged_chunk2_kernel<REC, U, 80, false, Q>), dim3(ncu), \
                                     dim3(qfec::kRcThreads), 0, 0, a0,                           \
                                     (uint32_t)((G + per - 1) / per), psync, nullptr, nullptr); \
                }})
  RC(false, 2, 80, false);
  RC2(false, 2, 100);
  RC2(false, 2, 95);
  RC2(false, 2, 90);
  RC2(false, 2, 75);
  vs.push_back({"multi2 recover", true, [=](const RaggedArgs& a) { launch_multi<true>(a, G); }});
  RC2(true, 2, 100);
  RC2(true, 2, 90);
#undef RC

  std::vector<uint8_t> want_e(G * 1452), want_r(G * 1452), got(G * 1452);
  std::vector<uint16_t> want_pl(G), got_pl(G);
  CK(hipMemcpy(want_e.data(), par, G * 1452, hipMemcpyDeviceToHost));
  CK(hipMemcpy(want_pl.data(), plen, G * 2, hipMemcpyDeviceToHost));
  CK(hipMemset(out, 0, G * 1452));
  launch_multi<true>(r, G);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(want_r.data(), out, G * 1452, hipMemcpyDeviceToHost));
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
    uint64_t nbad = 0;
    if (!same)
      for (uint64_t g = 0; g < G; ++g)
        nbad += std::memcmp(&got[g * 1452], &(v.rec ? want_r : want_e)[g * 1452], 1452) != 0;
    std::printf("%-28s == product: %s (err %u, bad groups %llu)\n", v.name.c_str(),
                same ? "yes" : "NO", he, (unsigned long long)nbad);
    all_ok = all_ok && same;
  }
  std::vector<std::vector<float>> t(vs.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rd = 0; rd < rounds; ++rd) {
    for (size_t i = 0; i < vs.size(); ++i) {
      vs[i].run(vs[i].rec ? r : e2);  // warm
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < reps; ++k) vs[i].run(vs[i].rec ? r : e2);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms / reps);
    }
  }
  for (size_t i = 0; i < vs.size(); ++i) {
    std::vector<float> x = t[i];
    std::sort(x.begin(), x.end());
    const double ms = x[x.size() / 2];
    const double alg = vs[i].rec ? rec_alg : enc_alg;
    std::printf("%-28s median %.3f ms  %.1f GB/s  %.3f of 8 TB/s  (min %.3f max %.3f)\n",
                vs[i].name.c_str(), ms, alg / ms / 1e6, alg / ms / 1e6 / 8000.0, x.front(),
                x.back());
  }
  {  // per-phase breakdown (TIMED build, U2): setup / stream / meeting / stores, in us
    const uint64_t per = (uint64_t)ncu * 80;
    const uint32_t nph = (uint32_t)((G + per - 1) / per);
    uint64_t* d_ts;
    CK(hipMalloc(&d_ts, 8 * nph * 8));
    CK(hipMemset(d_ts, 0, 8 * nph * 8));
    for (int rec = 0; rec < 4; ++rec) {
      if (rec == 1)
        hipLaunchKernelGGL((qfec::ragged_chunk_kernel<true, 2, 80, true>), dim3(ncu),
                           dim3(qfec::kRcThreads), 0, 0, r, nph, psync, nullptr, d_ts);
      else if (rec == 0)
        hipLaunchKernelGGL((qfec::ragged_chunk_kernel<false, 2, 80, true>), dim3(ncu),
                           dim3(qfec::kRcThreads), 0, 0, e2, nph, psync, nullptr, d_ts);
      else if (rec == 2)
        hipLaunchKernelGGL((qfec::ragged_chunk2_kernel<false, 2, 80, true>), dim3(ncu),
                           dim3(qfec::kRcThreads), 0, 0, e2, nph, psync, nullptr, d_ts);
      else
        hipLaunchKernelGGL((qfec::ragged_chunk2_kernel<true, 2, 80, true>), dim3(ncu),
                           dim3(qfec::kRcThreads), 0, 0, r, nph, psync, nullptr, d_ts);
      CK(hipDeviceSynchronize());
      std::vector<uint64_t> ts(8 * nph);
      CK(hipMemcpy(ts.data(), d_ts, 8 * nph * 8, hipMemcpyDeviceToHost));
      for (int wgi = 0; wgi < 2; ++wgi) {
        double su = 0, st = 0, me = 0, sto = 0;
        for (uint32_t p = 1; p + 1 < nph; ++p) {
          const uint64_t* q = &ts[wgi * 4 * nph + 4 * p];
          su += (q[0] - q[-1]) / 100.0;  // 100 MHz ticks -> us
          st += (q[1] - q[0]) / 100.0;
          me += (q[2] - q[1]) / 100.0;
          sto += (q[3] - q[2]) / 100.0;
        }
        const double np_ = nph - 2;
        std::printf("%s %s wg %s per phase: setup %.2f us, stream %.2f us, meeting %.2f us, "
                    "stores %.2f us (%u phases)\n", rec >= 2 ? "chunk2" : "chunk",
                    (rec & 1) ? "recover" : "encode",
                    wgi ? "mid" : "0", su / np_, st / np_, me / np_, sto / np_, nph);
      }
    }
  }
  uint32_t ab = 0;
  CK(hipMemcpy(&ab, psync + 64 * 19, 4, hipMemcpyDeviceToHost));
  std::printf("abandoned phased launches: %u\n", ab);
  return all_ok ? 0 : 1;
}
