// tune_rw.hip — A/B of the ragged kernels: the parity-window form
// (ragged_window_kernel, PB load slots in flight) against the flat-window
// two-groups-per-wave kernel (ragged_multi_kernel), encode and recover on the
// BASELINE configs[3] batch (2^20 groups, k 5-15, 64-1350 B, packed CSR) or
// another k / length range.  Every variant's output bytes are compared with
// the multi kernel's, which is checked against a host XOR on a sample.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_rw.hip -o tools/tune/build/tune_rw
// run:   tune_rw [reps] [rounds] [kmin] [kspan] [lmin] [lspan] [packed_out]
#include "../../libquic_amd/csrc/qfec_kernels.hip"
#include "ragged_legacy.inc"
#include "ragged_exp.inc"

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

template <bool REC, int GPW, bool NT = true, int U = 2, bool ALIGN = false>
static void launch_multi(const RaggedArgs& a, uint64_t G) {
  const uint64_t per = (uint64_t)GPW * 4;
  if constexpr (ALIGN)
    hipLaunchKernelGGL((qfec::ragged_multi_align_kernel<REC, NT, GPW, U, 4, false, true>),
                       dim3((uint32_t)((G + per - 1) / per)), dim3(256), 0, 0, a);
  else
    hipLaunchKernelGGL((qfec::ragged_multi_kernel<REC, NT, GPW, U, 4, false>),
                     dim3((uint32_t)((G + per - 1) / per)), dim3(256), 0, 0, a);
}

// The product kernel at a given number of 4-wave blocks per CU (dynamic LDS
// padding; 160 KiB per CU): does it run faster with more waves in flight?
template <bool REC>
static void launch_multi_occ(const RaggedArgs& a, uint64_t G, int blocks_per_cu) {
  static size_t stat = 0;
  if (!stat) {
    hipFuncAttributes fa;
    CK(hipFuncGetAttributes(&fa, (const void*)qfec::ragged_multi_kernel<REC, true, 2, 2, 4, false>));
    stat = fa.sharedSizeBytes;
  }
  const size_t pad = (160u << 10) / blocks_per_cu - stat - 256;
  hipLaunchKernelGGL((qfec::ragged_multi_kernel<REC, true, 2, 2, 4, false>),
                     dim3((uint32_t)((G + 7) / 8)), dim3(256), pad, 0, a);
}

template <bool REC, int B, bool GATE, int FENCE = 0, int DBG = 0>
static void launch_flat(const RaggedArgs& a, uint64_t G, size_t pad_lds = 0) {
  // pad_lds: extra dynamic LDS per block (140 KiB: one block = 4 waves per CU)
  hipLaunchKernelGGL((qfec::ragged_flat_kernel<REC, true, B, GATE, FENCE, DBG>), dim3((uint32_t)((G + 3) / 4)),
                     dim3(256), pad_lds, 0, a);
}

template <bool REC, int PB, bool NT = true>
static void launch_win(const RaggedArgs& a, uint64_t G) {
  hipLaunchKernelGGL((qfec::ragged_window_kernel<REC, NT, PB>), dim3((uint32_t)((G + 3) / 4)),
                     dim3(256), 0, 0, a);
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);  // progress lines reach the log as they happen
  const uint64_t G = 1 << 20;
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const uint32_t kmin = argc > 3 ? atoi(argv[3]) : 5, kspan = argc > 4 ? atoi(argv[4]) : 11;
  const uint32_t lmin = argc > 5 ? atoi(argv[5]) : 64, lspan = argc > 6 ? atoi(argv[6]) : 1287;
  const bool packed_out = argc > 7 && atoi(argv[7]) != 0;
  // parity / revived slot stride when not packed (1452: kMaxPacketSize; 1472:
  // an ALIGNAS(64) char[kMaxPacketSize] slot; 1536: 128-B lines)
  const uint64_t slot = argc > 8 ? (uint64_t)atoi(argv[8]) : 1452u;
  const uint64_t SB = 1536;  // buffer bytes per group (any slot <= 1536)
  // TUNE_RW_PALIGN=16: payloads on 16-B boundaries (the payload arena's layout)
  const uint64_t palign = getenv("TUNE_RW_PALIGN") ? (uint64_t)atoi(getenv("TUNE_RW_PALIGN")) : 1u;
  // TUNE_RW_OUT16 (with packed_out): output rows back to back on 16-B boundaries
  const bool out16 = getenv("TUNE_RW_OUT16") != nullptr;
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
      const uint32_t ln = lmin + (uint32_t)(sm64(seed ^ (0x4Cull << 56) ^ (g * 256 + i)) % lspan);
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
    poff[g] = packed_out ? out_pos : g * slot;
    out_pos += out16 ? (mx + 15u) / 16u * 16u : mx;
  }
  uint8_t* data;
  CK(hipMalloc(&data, bytes + 4096));
  uint64_t* d_off = up(off);
  uint16_t* d_len = up(len);
  uint32_t* d_ptr = up(ptr);
  uint64_t* d_poff = up(poff);
  uint8_t* d_miss = up(miss);
  CK(hipMemset(data, 0, bytes + 4096));  // gaps between aligned payloads: zero (BLOCKZ)
  CK(qfec::launch_synth_ragged(data, d_off, d_len, d_ptr, 0, G, seed, 0));
  uint8_t *par, *out, *chk;
  uint16_t *plen, *plen2;
  uint32_t* err;
  CK(hipMalloc(&par, G * SB));
  CK(hipMalloc(&out, G * SB));
  CK(hipMalloc(&chk, G * SB));
  CK(hipMalloc(&plen, G * 2));
  CK(hipMalloc(&plen2, G * 2));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  CK(hipMemset(par, 0, G * SB));
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
  launch_multi<false, 2>(e, G);  // reference parity for the recover runs
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
    uint64_t stride = 0;  // != 0: output in slots of this stride (checked per group)
  };
  std::vector<V> vs;
  vs.push_back({"multi2 encode", false, [=](const RaggedArgs& a) { launch_multi<false, 2>(a, G); }});
  // store-cost diagnostic (ragged_multi_diag_kernel): MODE 0 product, 1 no
  // stores, 2 stores into a 4-MiB L2-resident window
#define RG_DIAG(REC, MODE, NAME)                                                                \
  vs.push_back({std::string(NAME) + (REC ? " recover" : " encode"), REC,                      \
                [=](const RaggedArgs& a0) {                                                    \
                  hipLaunchKernelGGL((qfec::ragged_multi_diag_kernel<REC, MODE>),              \
                                     dim3((uint32_t)((G + 7) / 8)), dim3(256), 0, 0, a0,       \
                                     0xA5A5F00Du);                                             \
                }})
  if (getenv("TUNE_RW_SPLIT")) {  // round 3: where the store tail's cost goes
    for (int rep = 0; rep < 2; ++rep) {
      RG_DIAG(false, 0, "diag0 product");
      RG_DIAG(false, 1, "diag1 nostore (not exact)");
      RG_DIAG(false, 11, "diag11 lds reads only (not exact)");
      RG_DIAG(false, 12, "diag12 stores only (not exact)");
      RG_DIAG(false, 2, "diag2 L2 store (not exact)");
    }
    RG_DIAG(true, 0, "diag0 product");
    RG_DIAG(true, 1, "diag1 nostore (not exact)");
    RG_DIAG(true, 11, "diag11 lds reads only (not exact)");
    RG_DIAG(true, 12, "diag12 stores only (not exact)");
  }
  if (getenv("TUNE_RW_DAL")) {  // round 3: destination-aligned stores, A/B twice each
    RG_DIAG(false, 0, "diag0 product");
    RG_DIAG(false, 10, "diag10 dst-aligned");
    RG_DIAG(false, 0, "diag0 product (again)");
    RG_DIAG(false, 10, "diag10 dst-aligned (again)");
    vs.push_back({"multi2 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2>(a, G); }});
    RG_DIAG(true, 0, "diag0 product");
    RG_DIAG(true, 10, "diag10 dst-aligned");
    RG_DIAG(true, 0, "diag0 product (again)");
    RG_DIAG(true, 10, "diag10 dst-aligned (again)");
  }
  if (getenv("TUNE_RW_DIAG")) {
    RG_DIAG(false, 0, "diag0 product");
    RG_DIAG(false, 1, "diag1 nostore (not exact)");
    RG_DIAG(false, 2, "diag2 L2 store (not exact)");
    vs.push_back({"multi2 U1 encode", false, [=](const RaggedArgs& a) { launch_multi<false, 2, true, 1>(a, G); }});
    vs.push_back({"multi2 U3 encode", false, [=](const RaggedArgs& a) { launch_multi<false, 2, true, 3>(a, G); }});
    vs.push_back({"multi2 U4 encode", false, [=](const RaggedArgs& a) { launch_multi<false, 2, true, 4>(a, G); }});
    RG_DIAG(false, 9, "diag9 bf xor loop");
    RG_DIAG(false, 7, "diag7 bf tail st");
    RG_DIAG(false, 6, "diag6 aligned st");
    RG_DIAG(false, 3, "diag3 wb stores");
    RG_DIAG(false, 4, "diag4 xcd order");
    RG_DIAG(false, 5, "diag5 xcd+wb");
    vs.push_back({"multi2 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2>(a, G); }});
    RG_DIAG(true, 0, "diag0 product");
    RG_DIAG(true, 1, "diag1 nostore (not exact)");
    RG_DIAG(true, 2, "diag2 L2 store (not exact)");
    vs.push_back({"multi2 U1 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2, true, 1>(a, G); }});
    vs.push_back({"multi2 U3 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2, true, 3>(a, G); }});
    vs.push_back({"multi2 U4 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2, true, 4>(a, G); }});
    RG_DIAG(true, 9, "diag9 bf xor loop");
    RG_DIAG(true, 8, "diag8 masked parity");
    RG_DIAG(true, 7, "diag7 bf tail st");
    RG_DIAG(true, 6, "diag6 aligned st");
    RG_DIAG(true, 3, "diag3 wb stores");
    RG_DIAG(true, 4, "diag4 xcd order");
    RG_DIAG(true, 5, "diag5 xcd+wb");
  }
#undef RG_DIAG
  // persistent waves over pairs (ragged_persist_kernel): a fresh zeroed
  // counter word per launch
  uint32_t* pctr;
  const uint32_t n_pctr = 1u << 20;
  CK(hipMalloc(&pctr, n_pctr * 4ull));
  CK(hipMemset(pctr, 0, n_pctr * 4ull));
  static uint32_t pctr_next = 0;
  int ncu0 = 0;
  CK(hipDeviceGetAttribute(&ncu0, hipDeviceAttributeMultiprocessorCount, 0));
#define RG_PERSIST(REC, DYN, BPC, NAME)                                                         \
  vs.push_back({std::string(NAME) + (REC ? " recover" : " encode"), REC,                      \
                [=](const RaggedArgs& a0) {                                                    \
                  if (pctr_next >= n_pctr) {                                                   \
                    std::fprintf(stderr, "out of counter words\n");                           \
                    std::exit(1);                                                              \
                  }                                                                            \
                  hipLaunchKernelGGL((qfec::ragged_persist_kernel<REC, DYN>),                  \
                                     dim3((uint32_t)(ncu0 * BPC)), dim3(256), 0, 0, a0,        \
                                     pctr + pctr_next++);                                      \
                }})
  if (getenv("TUNE_RW_PERSIST")) {
    RG_PERSIST(false, false, 8, "persist static x8");
    RG_PERSIST(false, true, 8, "persist dyn x8");
    vs.push_back({"multi2 encode (again)", false, [=](const RaggedArgs& a) { launch_multi<false, 2>(a, G); }});
    RG_PERSIST(false, true, 8, "persist dyn x8 (again)");
    RG_PERSIST(false, true, 7, "persist dyn x7");
    vs.push_back({"multi2 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2>(a, G); }});
    RG_PERSIST(true, false, 8, "persist static x8");
    RG_PERSIST(true, true, 8, "persist dyn x8");
    vs.push_back({"multi2 recover (again)", true, [=](const RaggedArgs& a) { launch_multi<true, 2>(a, G); }});
    RG_PERSIST(true, true, 8, "persist dyn x8 (again)");
  }
#define RG_PXCD(REC, C, BPC, NAME)                                                             \
  vs.push_back({std::string(NAME) + (REC ? " recover" : " encode"), REC,                      \
                [=](const RaggedArgs& a0) {                                                    \
                  if (pctr_next + 512u > n_pctr) {                                             \
                    std::fprintf(stderr, "out of counter words\n");                          \
                    std::exit(1);                                                              \
                  }                                                                            \
                  hipLaunchKernelGGL((qfec::ragged_persist_xcd_kernel<REC, C>),                \
                                     dim3((uint32_t)(ncu0 * BPC)), dim3(256), 0, 0, a0,        \
                                     pctr + pctr_next);                                        \
                  pctr_next += 512u;                                                           \
                }})
  if (getenv("TUNE_RW_PERSIST2")) {
    for (int rep = 0; rep < 2; ++rep) {
      vs.push_back({"multi2 encode (ref)", false, [=](const RaggedArgs& a) { launch_multi<false, 2>(a, G); }});
      RG_PXCD(false, 1, 8, "pxcd C1 x8");
      RG_PXCD(false, 2, 8, "pxcd C2 x8");
      RG_PXCD(false, 4, 8, "pxcd C4 x8");
      RG_PXCD(false, 2, 7, "pxcd C2 x7");
    }
    vs.push_back({"multi2 recover (ref)", true, [=](const RaggedArgs& a) { launch_multi<true, 2>(a, G); }});
    RG_PXCD(true, 2, 8, "pxcd C2 x8");
    RG_PXCD(true, 4, 8, "pxcd C4 x8");
  }
#undef RG_PXCD
#define RG_BLOCK(REC, WV, GPB, NAME) RG_BLOCKU(REC, WV, GPB, 2, NAME)
#define RG_BLOCKU(REC, WV, GPB, UU, NAME) RG_BLOCKX(REC, WV, GPB, UU, true, NAME)
#define RG_BLOCKX(REC, WV, GPB, UU, PF, NAME)                                                   \
  vs.push_back({std::string(NAME) + (REC ? " recover" : " encode"), REC,                      \
                [=](const RaggedArgs& a0) {                                                    \
                  hipLaunchKernelGGL((qfec::ragged_block_kernel<REC, WV, GPB, UU, PF>),        \
                                     dim3((uint32_t)((G + GPB - 1) / GPB)), dim3(64 * WV), 0, 0, \
                                     a0);                                                      \
                }})
#define RG_BLOCKA(REC, AL, NAME)                                                               \
  vs.push_back({std::string(NAME) + (REC ? " recover" : " encode"), REC,                      \
                [=](const RaggedArgs& a0) {                                                    \
                  hipLaunchKernelGGL((qfec::ragged_block_kernel<REC, 4, 8, 2, true, AL>),      \
                                     dim3((uint32_t)((G + 7) / 8)), dim3(256), 0, 0, a0);      \
                }})
#define RG_BLOCKD(REC, DG, NAME)                                                               \
  vs.push_back({std::string(NAME) + (REC ? " recover" : " encode"), REC,                      \
                [=](const RaggedArgs& a0) {                                                    \
                  hipLaunchKernelGGL((qfec::ragged_block_kernel<REC, 4, 8, 2, true, true, DG>), \
                                     dim3((uint32_t)((G + 7) / 8)), dim3(256), 0, 0, a0);      \
                }})
  // the block kernel at BPC blocks per CU (dynamic LDS padding; static LDS
  // ~19 KB allows 8)
#define RG_BLOCKO(REC, BPC, NAME)                                                              \
  vs.push_back({std::string(NAME) + (REC ? " recover" : " encode"), REC,                      \
                [=](const RaggedArgs& a0) {                                                    \
                  static size_t stat = 0;                                                      \
                  if (!stat) {                                                                 \
                    hipFuncAttributes fa;                                                      \
                    CK(hipFuncGetAttributes(&fa, (const void*)qfec::ragged_block_kernel<REC, 4, 8, 2, true, true, 0>)); \
                    stat = fa.sharedSizeBytes;                                                 \
                  }                                                                            \
                  const size_t pad = (160u << 10) / BPC - stat - 256;                          \
                  hipLaunchKernelGGL((qfec::ragged_block_kernel<REC, 4, 8, 2, true, true, 0>), \
                                     dim3((uint32_t)((G + 7) / 8)), dim3(256), pad, 0, a0);    \
                }})
  // TUNE_RW_BLOCKZ (round 3, profiles/round3/ragged_align/blockz.txt) ran a
  // DIAG 2 build of ragged_block_kernel (zero-padded 16-B payload slots, every
  // window loaded whole, no tail shift / mask): -1%, removed.
  if (getenv("TUNE_RW_WINAL")) {  // parity-window form (one wave per group) vs block, aligned payloads
    for (int rep = 0; rep < 2; ++rep) {
      RG_BLOCKD(false, 0, "block product");
      vs.push_back({"window PB16 encode", false, [=](const RaggedArgs& a) { launch_win<false, 16>(a, G); }});
      vs.push_back({"window PB8 encode", false, [=](const RaggedArgs& a) { launch_win<false, 8>(a, G); }});
    }
    for (int rep = 0; rep < 2; ++rep) {
      RG_BLOCKD(true, 0, "block product");
      vs.push_back({"window PB16 recover", true, [=](const RaggedArgs& a) { launch_win<true, 16>(a, G); }});
    }
  }
  if (getenv("TUNE_RW_BLOCKO")) {
    for (int rep = 0; rep < 2; ++rep) {
      RG_BLOCKD(false, 0, "block product");
      RG_BLOCKO(false, 7, "block 7/CU");
      RG_BLOCKO(false, 6, "block 6/CU");
      RG_BLOCKO(false, 5, "block 5/CU");
    }
    for (int rep = 0; rep < 2; ++rep) {
      RG_BLOCKD(true, 0, "block product");
      RG_BLOCKO(true, 7, "block 7/CU");
      RG_BLOCKO(true, 6, "block 6/CU");
    }
  }
  if (getenv("TUNE_RW_BLOCKD")) {  // the block kernel without its parity stores
    for (int rep = 0; rep < 2; ++rep) {
      RG_BLOCKD(false, 0, "block product");
      RG_BLOCKD(false, 1, "block nostore (not exact)");
    }
    for (int rep = 0; rep < 2; ++rep) {
      RG_BLOCKD(true, 0, "block product");
      RG_BLOCKD(true, 1, "block nostore (not exact)");
    }
  }
  if (getenv("TUNE_RW_BLOCKAL")) {  // aligned in-place tail loads (AL) on and off
    for (int rep = 0; rep < 2; ++rep) {
      RG_BLOCKA(false, false, "block AL0");
      RG_BLOCKA(false, true, "block AL1");
    }
    for (int rep = 0; rep < 2; ++rep) {
      RG_BLOCKA(true, false, "block AL0");
      RG_BLOCKA(true, true, "block AL1");
    }
  }
  if (getenv("TUNE_RW_BLOCK3")) {
    for (int rep = 0; rep < 2; ++rep) {
      vs.push_back({"multi2 recover (ref)", true, [=](const RaggedArgs& a) { launch_multi<true, 2>(a, G); }});
      RG_BLOCKX(true, 4, 8, 2, false, "block W4 G8 noPF");
      RG_BLOCKX(true, 4, 8, 2, true, "block W4 G8 PF");
    }
    for (int rep = 0; rep < 2; ++rep) {
      vs.push_back({"multi2 encode (ref)", false, [=](const RaggedArgs& a) { launch_multi<false, 2>(a, G); }});
      RG_BLOCKX(false, 4, 8, 2, true, "block W4 G8");
    }
  }
  if (getenv("TUNE_RW_BLOCK2")) {
    for (int rep = 0; rep < 2; ++rep) {
      vs.push_back({"multi2 encode (ref)", false, [=](const RaggedArgs& a) { launch_multi<false, 2>(a, G); }});
      RG_BLOCK(false, 4, 8, "block W4 G8");
      RG_BLOCK(false, 2, 4, "block W2 G4");
      RG_BLOCK(false, 2, 6, "block W2 G6");
      RG_BLOCK(false, 4, 6, "block W4 G6");
      RG_BLOCK(false, 4, 10, "block W4 G10");
      RG_BLOCKU(false, 4, 8, 1, "block W4 G8 U1");
      RG_BLOCKU(false, 4, 8, 3, "block W4 G8 U3");
    }
    for (int rep = 0; rep < 2; ++rep) {
      vs.push_back({"multi2 recover (ref)", true, [=](const RaggedArgs& a) { launch_multi<true, 2>(a, G); }});
      RG_BLOCK(true, 4, 8, "block W4 G8");
      RG_BLOCK(true, 2, 4, "block W2 G4");
      RG_BLOCK(true, 4, 6, "block W4 G6");
      RG_BLOCKU(true, 4, 8, 3, "block W4 G8 U3");
    }
  }
  if (getenv("TUNE_RW_BLOCK")) {
    for (int rep = 0; rep < 2; ++rep) {
      vs.push_back({"multi2 encode (ref)", false, [=](const RaggedArgs& a) { launch_multi<false, 2>(a, G); }});
      RG_BLOCK(false, 4, 8, "block W4 G8");
      RG_BLOCK(false, 4, 12, "block W4 G12");
      RG_BLOCK(false, 8, 16, "block W8 G16");
      RG_BLOCK(false, 16, 32, "block W16 G32");
    }
    vs.push_back({"multi2 recover (ref)", true, [=](const RaggedArgs& a) { launch_multi<true, 2>(a, G); }});
    RG_BLOCK(true, 4, 8, "block W4 G8");
    RG_BLOCK(true, 8, 16, "block W8 G16");
    RG_BLOCK(true, 16, 32, "block W16 G32");
  }
#undef RG_BLOCK
#undef RG_BLOCKU
#undef RG_BLOCKX
#undef RG_PERSIST
  // parity / revived slot strides in ONE process (the placement of the
  // buffers is per process): 1452, 1472 (ALIGNAS(64) char[kMaxPacketSize]),
  // 1536 (128-B lines), each twice
  if (getenv("TUNE_RW_SLOT")) {
    const uint64_t strides[3] = {1452, 1472, 1536};
    for (int rep = 0; rep < 2; ++rep)
      for (int rec = 0; rec < 2; ++rec)
        for (uint64_t st : strides) {
          std::vector<uint64_t> ps(G);
          for (uint64_t g = 0; g < G; ++g) ps[g] = g * st;
          uint64_t* d_ps = up(ps);
          uint8_t* par_s = nullptr;
          if (rec) {  // the parity in this stride's slots
            CK(hipMalloc(&par_s, G * SB));
            RaggedArgs es = e;
            es.out = par_s;
            es.parity_off = d_ps;
            es.parity_len_out = plen2;
            launch_multi<false, 2>(es, G);
            CK(hipDeviceSynchronize());
          }
          V v;
          v.name = "slot " + std::to_string(st) + (rec ? " recover" : " encode") + (rep ? " (again)" : "");
          v.rec = rec != 0;
          v.stride = st;
          v.run = [=](const RaggedArgs& a0) {
            RaggedArgs a = a0;
            a.parity_off = d_ps;
            if (rec) {
              a.parity = par_s;
              a.out_off = d_ps;
            }
            if (rec)
              launch_multi<true, 2>(a, G);
            else
              launch_multi<false, 2>(a, G);
          };
          vs.push_back(v);
        }
  }
  const bool diag_only = getenv("TUNE_RW_DIAG") != nullptr || getenv("TUNE_RW_DAL") != nullptr ||
                         getenv("TUNE_RW_PERSIST") != nullptr || getenv("TUNE_RW_SLOT") != nullptr ||
                         getenv("TUNE_RW_SPLIT") != nullptr ||
                         getenv("TUNE_RW_PERSIST2") != nullptr || getenv("TUNE_RW_BLOCK") != nullptr ||
                         getenv("TUNE_RW_BLOCK2") != nullptr ||
                         getenv("TUNE_RW_BLOCK3") != nullptr || getenv("TUNE_RW_BLOCKAL") != nullptr ||
                         getenv("TUNE_RW_BLOCKD") != nullptr || getenv("TUNE_RW_BLOCKO") != nullptr ||
                         getenv("TUNE_RW_WINAL") != nullptr;
  // phased (ragged_phase_kernel): waves per CU x slots per wave
  uint32_t* psync;
  CK(hipMalloc(&psync, 20 * 256));
  CK(hipMemset(psync, 0, 20 * 256));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
#define RG_PHASE(REC, W, S, BPC)                                                                \
  vs.push_back({std::string("phase W" #W " S" #S " x" #BPC " ") + (REC ? "recover" : "encode"), \
                REC, [=](const RaggedArgs& a0) {                                                \
                  const uint64_t per = (uint64_t)ncu * BPC * W * S * 2;                         \
                  hipLaunchKernelGGL((qfec::ragged_phase_kernel<REC, S, W>), dim3(ncu * BPC),   \
                                     dim3(64 * W), 0, 0, a0, (uint32_t)((G + per - 1) / per),  \
                                     psync);                                                    \
                }})
#define RG_PHASE2(REC, W, NP, DYN, U)                                                          \
  vs.push_back({std::string("phase2 W" #W " NP" #NP " U" #U " ") + (REC ? "recover" : "encode"),  \
                REC, [=](const RaggedArgs& a0) {                                               \
                  const uint64_t per = (uint64_t)ncu * NP * 2;                                 \
                  hipLaunchKernelGGL((qfec::ragged_phase2_kernel<REC, W, NP, DYN, U>), dim3(ncu), \
                                     dim3(64 * W), 0, 0, a0, (uint32_t)((G + per - 1) / per), \
                                     psync);                                                   \
                }})
  if (getenv("TUNE_RW_PHASE2")) {
    RG_PHASE2(false, 16, 40, true, 2);
    RG_PHASE2(false, 16, 40, true, 4);
    RG_PHASE2(false, 16, 40, true, 6);
    RG_PHASE2(false, 16, 40, true, 8);
    RG_PHASE2(false, 12, 42, true, 4);
    vs.push_back({"multi2 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2>(a, G); }});
    RG_PHASE2(true, 16, 40, true, 4);
    RG_PHASE2(true, 16, 40, true, 8);
  }
#undef RG_PHASE2
  if (!diag_only && !getenv("TUNE_RW_PHASE2")) {
    RG_PHASE(false, 4, 13, 1);
    RG_PHASE(false, 8, 6, 1);
    RG_PHASE(false, 12, 3, 1);
    RG_PHASE(false, 16, 2, 1);
    RG_PHASE(false, 16, 1, 2);
    RG_PHASE(false, 8, 2, 3);
    vs.push_back({"multi2 recover", true, [=](const RaggedArgs& a) { launch_multi<true, 2>(a, G); }});
    RG_PHASE(true, 16, 2, 1);
    RG_PHASE(true, 16, 1, 2);
  }
#undef RG_PHASE

  // correctness: each variant's output (and parity lengths) == the product's
  std::vector<uint8_t> want_e(G * SB), want_r(G * SB), got(G * SB);
  std::vector<uint16_t> want_pl(G), got_pl(G);
  CK(hipMemcpy(want_e.data(), par, G * SB, hipMemcpyDeviceToHost));
  CK(hipMemcpy(want_pl.data(), plen, G * 2, hipMemcpyDeviceToHost));
  CK(hipMemset(out, 0, G * SB));
  launch_multi<true, 2>(r, G);
  CK(hipMemcpy(want_r.data(), out, G * SB, hipMemcpyDeviceToHost));
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
    std::printf("multi2 vs host XOR: bad groups %d\n", bad);
  }
  std::vector<uint8_t> hdat(bytes);
  CK(hipMemcpy(hdat.data(), data, bytes, hipMemcpyDeviceToHost));
  bool all_ok = true;  // the d8 builds are KNOWN to differ: they do not fail the run
  for (auto& v : vs) {
    CK(hipMemset(out, 0, G * SB));
    CK(hipMemset(plen2, 0, G * 2));
    std::printf("check %s ...\n", v.name.c_str());
    v.run(v.rec ? r : e2);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), out, G * SB, hipMemcpyDeviceToHost));
    bool same = true;
    if (v.stride) {
      const std::vector<uint8_t>& want = v.rec ? want_r : want_e;
      for (uint64_t g = 0; g < G && same; ++g)
        same = std::memcmp(&got[g * v.stride], &want[poff[g]], want_pl[g]) == 0;
    } else {
      same = got == (v.rec ? want_r : want_e);
    }
    if (!v.rec) {
      CK(hipMemcpy(got_pl.data(), plen2, G * 2, hipMemcpyDeviceToHost));
      same = same && got_pl == want_pl;
    }
    uint32_t he;
    CK(hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost));
    std::printf("%-24s == multi2: %s (err %u)\n", v.name.c_str(), same ? "yes" : "NO", he);
    if (!same && !v.stride && v.name.find("not exact") == std::string::npos) {  // which groups, and where in them
      const std::vector<uint8_t>& want = v.rec ? want_r : want_e;
      uint64_t nbad = 0;
      for (uint64_t g = 0; g < G; ++g) {
        const uint8_t* x = &got[poff[g]];
        const uint8_t* y = &want[poff[g]];
        if (std::memcmp(x, y, want_pl[g]) == 0) continue;
        if (nbad++ < 4) {
          uint32_t j0 = 0, j1 = 0, W = 0;
          while (x[j0] == y[j0]) ++j0;
          j1 = want_pl[g] - 1;
          while (x[j1] == y[j1]) --j1;
          for (uint32_t p = ptr[g]; p < ptr[g + 1]; ++p)
            if (!v.rec || p - ptr[g] != miss[g]) W += (len[p] + 15) / 16;
          std::printf("   bad g %llu k %u plen %u W %u nit %u bytes [%u, %u]\n",
                      (unsigned long long)g, ptr[g + 1] - ptr[g], want_pl[g], W, (W + 63) / 64, j0, j1);
          // which 16-B parity windows differ, and does the difference equal
          // one packet's window (a lost or doubled XOR)?
          std::printf("     windows:");
          for (uint32_t t = 0; t < 91; ++t) {
            if (std::memcmp(x + 16 * t, y + 16 * t, 16) == 0) continue;
            std::printf(" %u", t);
            // find the packet q and flat index whose window t equals the difference
            for (uint32_t p = ptr[g], S = 0; p < ptr[g + 1]; ++p) {
              if (v.rec && p - ptr[g] == miss[g]) continue;
              const uint32_t n = (len[p] + 15) / 16;
              if (t < n) {
                uint8_t w[16] = {0};
                for (uint32_t b = 0; b < 16 && 16 * t + b < len[p]; ++b) w[b] = hdat[off[p] + 16 * t + b];
                bool eq = true;
                for (uint32_t b = 0; b < 16; ++b) eq = eq && ((uint8_t)(x[16 * t + b] ^ y[16 * t + b]) == w[b]);
                if (eq) std::printf("(=pkt%u f%u it%u)", p - ptr[g], S + t, (S + t) / 64);
              }
              S += n;
            }
          }
          std::printf("\n");
        }
      }
      std::printf("   bad groups %llu\n", (unsigned long long)nbad);
    }
    if (v.name.find("not exact") != std::string::npos) continue;  // not a FEC result
    if (v.name.find(" d8 ") == std::string::npos || v.name.find("1blk") != std::string::npos)  // NOLINT
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
  std::printf("k %u..%u, len %u..%u, %llu groups, %.3f GB packet buffer (payloads on %llu-B "
              "boundaries), parity slots %s %llu\n", kmin,
              kmin + kspan - 1, lmin, lmin + lspan - 1, (unsigned long long)G, bytes / 1e9,
              (unsigned long long)palign, packed_out ? (out16 ? "packed16" : "packed") : "stride",
              (unsigned long long)(packed_out ? 0 : slot));
  std::printf("%-24s %10s %10s %8s\n", "variant", "med GB/s", "max GB/s", "%8TB/s");
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = res[i];
    std::sort(v.begin(), v.end());
    std::printf("%-24s %10.1f %10.1f %7.1f%%\n", vs[i].name.c_str(), v[v.size() / 2], v.back(),
                v[v.size() / 2] / 80.0);
  }
  return all_ok ? 0 : 1;
}
