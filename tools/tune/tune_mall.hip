// tune_mall.hip — round 5 probe: can the 256 MiB Infinity Cache (MALL) hold a
// ragged phase's parity rows, so that the phase split the LDS cannot hold
// (DESIGN §4 "Round 5, ragged") happens in memory instead?
//
// Phase p of W groups: the product's ragged_block_kernel reads the phase's
// packets and writes its parity rows into a W-slot scratch ring that is
// rewritten every phase (small enough to stay in the MALL), then a scatter
// kernel copies the ring's rows to their output slots (the phase's HBM
// writes).  If the MALL absorbs the ring's writes, the HBM sees a read phase
// and a write phase per pair of launches — with the block kernel's read rate
// and no LDS capacity limit.
//
//   tune_mall [reps=5] [rounds=3] [palign=16] [slot=1536]
// Every phased variant is byte-compared with the one-pass product first.
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

namespace qfec {
namespace {

// One wave per group: copy row j of the scratch ring (slot stride `sslot`)
// to out + off[g0 + j], plen bytes (the last window as the 16 bytes ending at
// plen, as the kernels store it; plen >= 16 in this probe's batches).
__global__ __launch_bounds__(256) void scatter_rows_kernel(const uint8_t* __restrict__ ring,
                                                           uint32_t sslot, uint8_t* __restrict__ out,
                                                           const uint64_t* __restrict__ off,
                                                           const uint16_t* __restrict__ plen_v,
                                                           uint64_t g0, uint32_t W) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t j = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (j >= W) return;
  const uint32_t plen = plen_v[g0 + j];
  const uint8_t* src = ring + (uint64_t)j * sslot;
  uint8_t* dst = out + off[g0 + j];
  const uint32_t nw = (plen + 15u) >> 4;
  for (uint32_t t = lane; t < nw; t += 64u) {
    const uint32_t w = min(16u * t, plen - 16u);
    st16t<true>(dst + w, ld16(src + w));
  }
}

}  // namespace
}  // namespace qfec

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
  bool exact;  // byte-compared with the product
  std::function<void(const RaggedArgs&)> run;
};

template <bool REC, int DIAG = 0>
static void blk(const RaggedArgs& a) {
  hipLaunchKernelGGL((qfec::ragged_block_kernel<REC, 4, 8, 2, true, true, DIAG>),
                     dim3((uint32_t)((a.n_groups + 7) / 8)), dim3(256), 0, 0, a);
}

static uint8_t* g_ring = nullptr;
static uint64_t* g_ring_off = nullptr;  // j * slot
static uint32_t g_slot = 1536;

// one-pass into the ring only (parities overwrite each other: timing only)
template <bool REC>
static void blk_ring_only(const RaggedArgs& a0, uint32_t W) {
  for (uint64_t g0 = 0; g0 < a0.n_groups; g0 += W) {
    RaggedArgs a = a0;
    const uint32_t n = (uint32_t)std::min<uint64_t>(W, a0.n_groups - g0);
    a.grp_ptr = a0.grp_ptr + g0;
    a.n_groups = n;
    a.out = g_ring;
    if (REC) {
      a.missing = a0.missing + g0;
      a.parity_len = a0.parity_len + g0;
      a.parity_off = a0.parity_off + g0;
      a.out_off = g_ring_off;
    } else {
      a.parity_off = g_ring_off;
      a.parity_len_out = a0.parity_len_out + g0;
    }
    blk<REC>(a);
  }
}

// phased: per phase, the block kernel into the ring, then the ring's rows out
template <bool REC>
static void blk_mall_phased(const RaggedArgs& a0, uint32_t W, bool scatter = true) {
  for (uint64_t g0 = 0; g0 < a0.n_groups; g0 += W) {
    RaggedArgs a = a0;
    const uint32_t n = (uint32_t)std::min<uint64_t>(W, a0.n_groups - g0);
    a.grp_ptr = a0.grp_ptr + g0;
    a.n_groups = n;
    a.out = g_ring;
    if (REC) {
      a.missing = a0.missing + g0;
      a.parity_len = a0.parity_len + g0;
      a.parity_off = a0.parity_off + g0;
      a.out_off = g_ring_off;
    } else {
      a.parity_off = g_ring_off;
      a.parity_len_out = a0.parity_len_out + g0;
    }
    blk<REC>(a);
    if (scatter)
      hipLaunchKernelGGL(qfec::scatter_rows_kernel, dim3((n + 3) / 4), dim3(256), 0, 0,
                         (const uint8_t*)g_ring, g_slot, a0.out,
                         REC ? a0.out_off : a0.parity_off,
                         REC ? a0.parity_len : (const uint16_t*)a0.parity_len_out, g0, n);
  }
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const uint64_t G = 1 << 20;
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  const uint64_t palign = argc > 3 ? (uint64_t)atoi(argv[3]) : 16u;
  const uint64_t slot = argc > 4 ? (uint64_t)atoi(argv[4]) : 1536u;
  g_slot = (uint32_t)slot;
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
      bytes += (ln + palign - 1) / palign * palign;
      s += ln;
      if (i != miss[g]) sm += ln;
      mx = std::max(mx, ln);
    }
    enc_alg += s + mx;
    rec_alg += sm + 2.0 * mx;
    ptr.push_back((uint32_t)len.size());
    poff[g] = g * slot;
  }
  uint8_t* data;
  CK(hipMalloc(&data, bytes + 4096));
  CK(hipMemset(data, 0x77, bytes + 4096));
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
  const uint32_t WMAX = 1u << 17;
  CK(hipMalloc(&g_ring, (size_t)WMAX * slot));
  {
    std::vector<uint64_t> ro(WMAX);
    for (uint32_t j = 0; j < WMAX; ++j) ro[j] = (uint64_t)j * slot;
    g_ring_off = up(ro);
  }
  CK(hipMemset(err, 0, 4));
  CK(hipMemset(par_ref, 0xA5, OB));
  CK(hipMemset(out_ref, 0xA5, OB));

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
  blk<false>(e);
  blk<true>(r);
  CK(hipDeviceSynchronize());
  RaggedArgs ev = e, rv = r;
  ev.out = buf;
  ev.parity_len_out = plen_v;
  rv.out = buf;

  std::vector<V> vs;
  vs.push_back({"product block encode", false, true, [](const RaggedArgs& a) { blk<false>(a); }});
  for (uint32_t W : {16384u, 32768u, 65536u, 131072u}) {
    char nm[96];
    std::snprintf(nm, sizeof nm, "mall phased W%u encode", W);
    vs.push_back({nm, false, true, [W](const RaggedArgs& a) { blk_mall_phased<false>(a, W); }});
  }
  vs.push_back({"product block recover", true, true, [](const RaggedArgs& a) { blk<true>(a); }});
  for (uint32_t W : {32768u, 65536u}) {
    char nm[96];
    std::snprintf(nm, sizeof nm, "mall phased W%u recover", W);
    vs.push_back({nm, true, true, [W](const RaggedArgs& a) { blk_mall_phased<true>(a, W); }});
  }
  // timing-only diagnostics (not exact)
  vs.push_back({"block enc, no stores (DIAG 1)", false, false, [](const RaggedArgs& a) { blk<false, 1>(a); }});
  for (uint32_t W : {16384u, 65536u}) {
    char nm[96];
    std::snprintf(nm, sizeof nm, "block enc into ring W%u only", W);
    vs.push_back({nm, false, false, [W](const RaggedArgs& a) { blk_ring_only<false>(a, W); }});
    std::snprintf(nm, sizeof nm, "mall W%u enc, read phases only", W);
    vs.push_back({nm, false, false, [W](const RaggedArgs& a) { blk_mall_phased<false>(a, W, false); }});
  }

  std::vector<uint8_t> h_ref(OB), h_v(OB);
  std::vector<uint16_t> hp_ref(G), hp_v(G);
  CK(hipMemcpy(hp_ref.data(), plen_ref, G * 2, hipMemcpyDeviceToHost));
  bool all_ok = true;
  for (const V& v : vs) {
    if (!v.exact) continue;
    CK(hipMemset(buf, 0xA5, OB));
    CK(hipMemset(plen_v, 0, G * 2));
    CK(hipMemset(err, 0, 4));
    v.run(v.rec ? rv : ev);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h_ref.data(), v.rec ? out_ref : par_ref, OB, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h_v.data(), buf, OB, hipMemcpyDeviceToHost));
    uint32_t e_h = 0;
    CK(hipMemcpy(&e_h, err, 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < OB; ++i) bad += h_ref[i] != h_v[i];
    bool ok = bad == 0 && e_h == 0;
    if (!v.rec) {
      CK(hipMemcpy(hp_v.data(), plen_v, G * 2, hipMemcpyDeviceToHost));
      ok = ok && hp_ref == hp_v;
    }
    std::printf("check %-32s == product: %s (err %u, %zu bad bytes)\n", v.name.c_str(), ok ? "yes" : "NO",
                e_h, bad);
    all_ok = all_ok && ok;
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
  CK(hipDeviceSynchronize());
  std::printf("\nconfigs[3]: %llu groups, k 5-15, len 64-1350, palign %llu, slot %llu; algorithmic GB: "
              "encode %.3f, recover %.3f\n",
              (unsigned long long)G, (unsigned long long)palign, (unsigned long long)slot, enc_alg / 1e9,
              rec_alg / 1e9);
  for (size_t i = 0; i < vs.size(); ++i) {
    std::vector<float> s = ms[i];
    std::sort(s.begin(), s.end());
    const double med = s[s.size() / 2] * 1e-3;
    const double gbs = (vs[i].rec ? rec_alg : enc_alg) / med / 1e9;
    std::printf("%-34s median %8.1f us  min %8.1f us  %7.1f GB/s  %.4f of 8 TB/s\n", vs[i].name.c_str(),
                med * 1e6, s[0] * 1e3, gbs, gbs / 8000.0);
  }
  return 0;
}
