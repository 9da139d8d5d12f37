// tune_phase.hip — does separating the encode's read and write streams in TIME
// take the fixed kernel out of its slow placement modes (the
// modes are a property of the (rows, parity) buffer pair, i.e. of the read
// and write streams meeting in the DRAM)?
//
// A persistent grid (occupancy-sized) walks the batch in phases.  In phase p
// every workgroup XORs M x 3 groups (the product's 85 lanes x 16 B per group,
// 10 nt row loads per lane) into LDS, then all workgroups meet at a
// counter, then every workgroup stores its M x 3 parity rows (nt), then they
// meet again: the HBM sees phases of pure reads and pure writes.  The counter
// only shapes timing — no workgroup reads another's output — so every wait is
// bounded (kMaxSpin polls, then it goes on and counts a timeout); a stranded
// workgroup costs time, never a hang or a wrong result.
// SYNC 0 = same persistent walk without waiting, 1 = wait before the stores
// only, 2 = before and after.  Compared with the product kernel over 2 row
// buffers x 3 parity buffers, interleaved, one process; every variant's
// parity is compared with the product's.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_phase.hip -o tools/tune/build/tune_phase
#include "../../libquic_amd/csrc/qfec_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

using qfec::u32x4;
constexpr uint32_t kK = 10, kL = 1350, kC = 85, kGpb = 3;
constexpr uint32_t kMaxSpin = 4000;

// Barrier number `epoch` (1, 2, ...): a block adds to one of 16 sub-counters
// (256 B apart; ~B/16 adders each instead of B on one line — one counter for
// 1,024 blocks cost ~60 us per barrier); the last adder of a sub-counter in
// this epoch, told by the value its add returned, adds to the top counter,
// which everyone polls.
__device__ __forceinline__ void phase_wait(uint32_t* ctr, uint32_t epoch, uint32_t* timeouts) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t B = gridDim.x, sub = blockIdx.x & 15u, nsub = (B - sub + 15u) / 16u;
    const uint32_t old =
        __hip_atomic_fetch_add(ctr + 64u * (1u + sub), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1u == epoch * nsub)
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t target = epoch * min(B, 16u);
    uint32_t spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target &&
           ++spins < kMaxSpin)
      __builtin_amdgcn_s_sleep(1);
    if (spins >= kMaxSpin) __hip_atomic_fetch_add(timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
}

// PART: 0 the encode, 1 loads only (no parity stores), 2 stores only (no row
// loads) — the phases and waits unchanged, to split the time.
// A phase is S = R + M steps of 3 groups per block: the first R steps keep
// their parity in registers (static indices: fully unrolled), the other M in
// LDS (M <= 40: 160 KiB).  Bigger phases, fewer waits.
// FLAT: the row pointer passes through an empty asm (generic pointer: flat
// loads with immediate row offsets); RT: the row stride is a runtime value
// (kRtStride, as in the product) instead of the constant 1350.
__device__ uint32_t kRtStride = kL;
template <int M, int U, int SYNC, int PART = 0, int BS = 256, int R = 0, bool FLAT = true,
          bool RT = false>
__global__ __launch_bounds__(BS) void phase_kernel(const uint8_t* rows, uint8_t* out, uint64_t n,
                                                    uint32_t nphase, uint32_t* ctr,
                                                    uint32_t* timeouts) {
  const uint32_t rstride = RT ? kRtStride : kL;
  constexpr uint32_t kGpb = BS / kC;  // groups per step: 3 (256 lanes), 6, 12 (1,024)
  constexpr int S = R + M;
  static_assert(R % U == 0 && M % U == 0, "steps in units of U");
  const uint32_t tid = threadIdx.x, gl = tid / kC, t = tid - gl * kC;
  const bool lane_on = gl < kGpb;
  const uint32_t off = min(t * 16u, kL - 16u);
  const uint32_t B = gridDim.x;
  // the block's parity rows of one phase wait in LDS (own lane's slots only)
  __shared__ u32x4 s_acc[M][BS];
  u32x4 racc[R > 0 ? R : 1];
  for (uint32_t p = 0; p < nphase; ++p) {
    // steps i .. i+U-1 of phase p cover one contiguous window of B x 3U
    // groups (the product's sliding window), block b its 3U groups at 3Ub
    const uint64_t base = ((uint64_t)p * (S / U) * B + blockIdx.x) * (kGpb * U) + gl;
    auto step = [&](int i, u32x4 (&a)[U]) {
      u32x4 v[U][kK];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t g = base + (uint64_t)(i / U) * B * kGpb * U + (uint64_t)u * kGpb;
        const bool on = lane_on && g < n;
        const uint8_t* src = rows + (on ? g : 0) * (kK * rstride) + off;
        if constexpr (FLAT) asm volatile("" : "+v"(src) : : "memory");  // no hoisting across steps
#pragma unroll
        for (uint32_t r = 0; r < kK; ++r)
          v[u][r] = PART == 2 ? u32x4{(uint32_t)g, 0u, 0u, 0u} : qfec::ld16t<true>(src + r * rstride);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a[u] = v[u][0];
#pragma unroll
        for (uint32_t r = 1; r < kK; ++r) a[u] ^= v[u][r];
      }
    };
#pragma unroll
    for (int i = 0; i < R; i += U) {
      u32x4 a[U];
      step(i, a);
#pragma unroll
      for (int u = 0; u < U; ++u) racc[i + u] = a[u];
    }
#pragma unroll 1
    for (int i = R; i < S; i += U) {
      u32x4 a[U];
      step(i, a);
#pragma unroll
      for (int u = 0; u < U; ++u) s_acc[i - R + u][tid] = a[u];
    }
    if constexpr (SYNC >= 1) phase_wait(ctr, SYNC == 2 ? 2u * p + 1u : p + 1u, timeouts);
    auto gidx = [&](int i) {
      return base + (uint64_t)(i / U) * B * kGpb * U + (uint64_t)(i % U) * kGpb;
    };
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const uint64_t g = gidx(i);
      if (PART != 1 && lane_on && g < n) qfec::st16t<true>(out + g * kL + off, racc[i]);
    }
#pragma unroll 4
    for (int i = R; i < S; ++i) {
      const uint64_t g = gidx(i);
      if (PART != 1 && lane_on && g < n) qfec::st16t<true>(out + g * kL + off, s_acc[i - R][tid]);
    }
    if constexpr (SYNC == 2) phase_wait(ctr, 2u * p + 2u, timeouts);
  }
}

// Software-pipelined read phase: the next U steps' loads are issued before
// the current U steps are XORed and stored to LDS, so a wave never drains its
// loads between steps.
template <int M, int U, int SYNC, int PART = 0>
__global__ __launch_bounds__(256) void pipe_kernel(const uint8_t* rows, uint8_t* out, uint64_t n,
                                                   uint32_t nphase, uint32_t* ctr,
                                                   uint32_t* timeouts) {
  constexpr uint32_t kGpb = 3;
  static_assert(M % U == 0, "steps in units of U");
  const uint32_t tid = threadIdx.x, gl = tid / kC, t = tid - gl * kC;
  const bool lane_on = gl < kGpb;
  const uint32_t off = min(t * 16u, kL - 16u);
  const uint32_t B = gridDim.x;
  __shared__ u32x4 s_acc[M][256];
  for (uint32_t p = 0; p < nphase; ++p) {
    const uint64_t base = ((uint64_t)p * (M / U) * B + blockIdx.x) * (kGpb * U) + gl;
    auto issue = [&](int i, u32x4 (&v)[U][kK]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t g = base + (uint64_t)(i / U) * B * kGpb * U + (uint64_t)u * kGpb;
        const bool on = lane_on && g < n;
        const uint8_t* src = rows + (on ? g : 0) * (kK * kL) + off;
#pragma unroll
        for (uint32_t r = 0; r < kK; ++r) v[u][r] = qfec::ld16t<true>(src + r * kL);
      }
    };
    u32x4 cur[U][kK], nxt[U][kK];
    issue(0, cur);
#pragma unroll 1
    for (int i = 0; i < M; i += U) {
      if (i + U < M) issue(i + U, nxt);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        u32x4 a = cur[u][0];
#pragma unroll
        for (uint32_t r = 1; r < kK; ++r) a ^= cur[u][r];
        s_acc[i + u][tid] = a;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (uint32_t r = 0; r < kK; ++r) cur[u][r] = nxt[u][r];
    }
    if constexpr (SYNC >= 1) phase_wait(ctr, SYNC == 2 ? 2u * p + 1u : p + 1u, timeouts);
#pragma unroll 4
    for (int i = 0; i < M; ++i) {
      const uint64_t g = base + (uint64_t)(i / U) * B * kGpb * U + (uint64_t)(i % U) * kGpb;
      if (PART != 1 && lane_on && g < n) qfec::st16t<true>(out + g * kL + off, s_acc[i][tid]);
    }
    if constexpr (SYNC == 2) phase_wait(ctr, 2u * p + 2u, timeouts);
  }
}

__global__ void fill(uint8_t* p, uint64_t n, uint64_t salt) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8;
       i += (uint64_t)gridDim.x * blockDim.x)
    reinterpret_cast<uint64_t*>(p)[i] = (i ^ salt) * 0x9E3779B97F4A7C15ull;
}

__global__ void count_diff(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t* bad) {
  uint32_t c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8;
       i += (uint64_t)gridDim.x * blockDim.x)
    c += reinterpret_cast<const uint64_t*>(a)[i] != reinterpret_cast<const uint64_t*>(b)[i];
  if (c) atomicAdd(bad, c);
}

struct Var {
  std::string name;
  void (*k)(const uint8_t*, uint8_t*, uint64_t, uint32_t, uint32_t*, uint32_t*);
  int m, sync, part = 0, bs = 256;
  uint32_t grid = 0, nphase = 0;
};

int main(int argc, char** argv) {
  const uint64_t G = argc > 3 ? strtoull(argv[3], nullptr, 10) : (1 << 20);
  const uint64_t rows_b = G * kK * kL, par_b = G * kL;
  const int reps = argc > 1 ? atoi(argv[1]) : 5, rounds = argc > 2 ? atoi(argv[2]) : 3;
  const int NR = 2, NP = 3;
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<uint8_t*> rows(NR), par(NP);
  for (int i = 0; i < NR; ++i) {
    CK(hipMalloc(&rows[i], rows_b));
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, rows[i], rows_b, (uint64_t)i);
  }
  for (auto& p : par) CK(hipMalloc(&p, par_b + 4096));
  uint8_t* want;
  CK(hipMalloc(&want, par_b));
  uint32_t *d_err, *ctr, *tmo, *bad;
  CK(hipMalloc(&d_err, 4));
  CK(hipMalloc(&ctr, 17 * 256));
  CK(hipMalloc(&tmo, 4));
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(d_err, 0, 4));
  CK(hipMemset(tmo, 0, 4));
  CK(hipDeviceSynchronize());

  std::vector<Var> vs = {
  };
  for (auto& v : vs) {
    int bpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, reinterpret_cast<const void*>(v.k), v.bs, 0));
    bpc = std::min(bpc, 8);  // <= 5 here (LDS): the sgpr rule of 8-block residency is moot
    v.grid = (uint32_t)(bpc * ncu);
    const uint64_t per = (uint64_t)v.grid * v.m * (v.bs / kC);
    v.nphase = (uint32_t)((G + per - 1) / per);
    std::printf("%-24s blocks/CU %d grid %u phases %u\n", v.name.c_str(), bpc, v.grid, v.nphase);
  }
  auto product = [&](int i, int j) {
    qfec::FixedArgs a{};
    a.rows = rows[i];
    a.out = par[j];
    a.row_stride = kL;
    a.group_stride = kK * kL;
    a.parity_stride = kL;
    a.out_stride = kL;
    a.n_groups = G;
    a.k = kK;
    a.L = kL;
    a.err = d_err;
    CK(qfec::launch_fixed(a, true, 0));
  };
  uint32_t* psync;
  CK(hipMalloc(&psync, 20 * 256));
  CK(hipMemset(psync, 0, 20 * 256));
  auto product_phased = [&](int i, int j) {
    qfec::FixedArgs a{};
    a.rows = rows[i];
    a.out = par[j];
    a.row_stride = kL;
    a.group_stride = kK * kL;
    a.parity_stride = kL;
    a.out_stride = kL;
    a.n_groups = G;
    a.k = kK;
    a.L = kL;
    a.err = d_err;
    a.phase_sync = psync;
    a.ncu = (uint32_t)ncu;
    CK(qfec::launch_fixed(a, true, 0));
  };
  // the product's phase_xor_kernel instantiated directly: MEET2 x FLAT
  using PK = void (*)(qfec::FixedArgs, uint32_t, uint32_t, uint32_t);
  std::vector<std::pair<std::string, PK>> pks = {
      {"prod (256 x 40)", qfec::phase_xor_kernel<10, false>},
      {"prod recover (256 x 40)", qfec::phase_xor_kernel<10, true>},
      {"prod recover parity-first", qfec::phase_xor_kernel<10, true, false, false, 1, 40, 256, false, true>},
      {"prod dflt-load", qfec::phase_xor_kernel<10, false, false, false, 1, 40, 256, false, true, false>},
      {"prod recover dflt-load", qfec::phase_xor_kernel<10, true, false, false, 1, 40, 256, false, true, false>},
      {"prod edge-dflt", qfec::phase_xor_kernel<10, false, false, false, 1, 40, 256, false, true, true, true>},
      {"prod recover compact", qfec::phase_xor_kernel<10, true, false, false, 1, 40, 256, false, true, true, false, true>},
      {"prod recover masked", qfec::phase_xor_kernel<10, true, false, false, 1, 40, 256, false, true, true, false, false>},
      {"prod 256 x 40+32", qfec::phase_xor_kernel<10, false, false, false, 1, 40, 256, false, true, true, false, true, 32>},
      {"prod recover 40+32", qfec::phase_xor_kernel<10, true, false, false, 1, 40, 256, false, true, true, false, true, 32>},
      {"prod recover 40+32 rpf", qfec::phase_xor_kernel<10, true, false, false, 1, 40, 256, false, true, true, false, true, 32, true>},
      {"prod recover 40+48 rpf", qfec::phase_xor_kernel<10, true, false, false, 1, 40, 256, false, true, true, false, true, 48, true>},
      // round 4: recover with fewer / other register steps
      {"prod recover 40+32 rpf early", qfec::phase_xor_kernel<10, true, false, false, 1, 40, 256, false, true, true, false, true, 32, true, true>},
      {"prod recover 40+32 rpf again", qfec::phase_xor_kernel<10, true, false, false, 1, 40, 256, false, true, true, false, true, 32, true>},
      {"prod recover 40+32 rpf early again", qfec::phase_xor_kernel<10, true, false, false, 1, 40, 256, false, true, true, false, true, 32, true, true>},
      {"prod 256 x 40+56", qfec::phase_xor_kernel<10, false, false, false, 1, 40, 256, false, true, true, false, true, 56>},
      {"prod 256 x 40+48", qfec::phase_xor_kernel<10, false, false, false, 1, 40, 256, false, true, true, false, true, 48>},
  };
  pks.push_back({"prod recover one-pass", nullptr});
  uint8_t* d_miss;
  CK(hipMalloc(&d_miss, G));
  {
    std::vector<uint8_t> hm(G);
    for (uint64_t g = 0; g < G; ++g) hm[g] = (uint8_t)((g * 2654435761u >> 7) % kK);
    CK(hipMemcpy(d_miss, hm.data(), G, hipMemcpyHostToDevice));
  }
  const uint32_t pnph = (uint32_t)((G + (uint64_t)ncu * 40 * 3 - 1) / ((uint64_t)ncu * 40 * 3));
  auto prod_variant = [&](int w, int i, int j) {
    qfec::FixedArgs a{};
    a.rows = rows[i];
    a.out = par[j];
    a.row_stride = kL;
    a.group_stride = kK * kL;
    a.parity_stride = kL;
    a.out_stride = kL;
    a.n_groups = G;
    a.k = kK;
    a.L = kL;
    a.err = d_err;
    a.phase_sync = psync;
    a.ncu = (uint32_t)ncu;
    if (pks[w].first.find("recover") != std::string::npos) {
      a.parity = par[(j + 1) % NP];
      a.missing = d_miss;
    }
    if (!pks[w].second) a.phase_sync = nullptr;
    // geometry from the name: threads x steps, blocks per CU
    uint32_t nt = 256, st = 40, bpc = 1;
    if (pks[w].first.find("512 x 20") != std::string::npos) nt = 512, st = 20;
    if (pks[w].first.find("1024 x 10") != std::string::npos) nt = 1024, st = 10;
    if (pks[w].first.find("256 x 20") != std::string::npos) st = 20, bpc = 2;
    if (pks[w].first.find("256 x 32") != std::string::npos) st = 32;
    if (pks[w].first.find("128 x 80") != std::string::npos) nt = 128, st = 80;
    if (pks[w].first.find("192 x 53") != std::string::npos) nt = 192, st = 53;
    if (pks[w].first.find("40+32") != std::string::npos) st = 72;
    if (pks[w].first.find("40+56") != std::string::npos) st = 96;
    if (pks[w].first.find("40+40") != std::string::npos) st = 80;
    if (pks[w].first.find("40+48") != std::string::npos) st = 88;
    if (pks[w].first.find("40+64") != std::string::npos) st = 104;
    if (pks[w].first.find("40+24") != std::string::npos) st = 64;
    if (pks[w].first.find("40+16") != std::string::npos) st = 56;
    if (pks[w].first.find("32+32") != std::string::npos) st = 64;
    const uint32_t gpb = nt / 85u, grid = ncu * bpc;
    const uint64_t per = (uint64_t)grid * st * gpb;
    const uint32_t nph = (uint32_t)((G + per - 1) / per);
    (void)pnph;
    // the product spreads the batch evenly over its phases (launch_fixed)
    a.phase_steps = (uint32_t)((G + (uint64_t)grid * gpb * nph - 1) / ((uint64_t)grid * gpb * nph));
    if (pks[w].second)
      hipLaunchKernelGGL(pks[w].second, dim3(grid), dim3(nt), 0, 0, a, 85u, gpb, nph);
    else
      CK(qfec::launch_fixed(a, true, 0));  // one-pass (no phase_sync)
  };
  auto launch = [&](const Var& v, int i, int j) {
    CK(hipMemsetAsync(ctr, 0, 17 * 256, 0));
    hipLaunchKernelGGL(v.k, dim3(v.grid), dim3(v.bs), 0, 0, rows[i], par[j], G, v.nphase, ctr, tmo);
  };
  // exactness against the product on rows0
  for (int i = 0; i < NR; ++i) {
    product(i, 0);
    CK(hipMemcpy(want, par[0], par_b, hipMemcpyDeviceToDevice));
    for (auto& v : vs) {
      if (v.part) continue;
      CK(hipMemset(par[1], 0, par_b));
      launch(v, i, 1);
      CK(hipMemset(bad, 0, 4));
      hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, 0, par[1], want, par_b, bad);
      uint32_t h = 0;
      CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
      if (h) std::printf("%s rows%d: %u differing words\n", v.name.c_str(), i, h);
    }
  }
  for (int i = 0; i < NR; ++i) {
    product(i, 0);
    CK(hipMemcpy(want, par[0], par_b, hipMemcpyDeviceToDevice));
    for (int w = 0; w < (int)pks.size(); ++w) {
      if (pks[w].first.find("recover") != std::string::npos) continue;  // tests/test_hip_phase.py
      CK(hipMemset(par[1], 0, par_b));
      prod_variant(w, i, 1);
      CK(hipMemset(bad, 0, 4));
      hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, 0, par[1], want, par_b, bad);
      uint32_t h = 0;
      CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
      if (h) std::printf("%s rows%d: %u differing words\n", pks[w].first.c_str(), i, h);
    }
  }
  {  // recover variants against the product's recover on the same buffers
    int w0 = -1;
    for (int w = 0; w < (int)pks.size(); ++w)
      if (pks[w].first == "prod recover (256 x 40)") w0 = w;
    for (int i = 0; i < NR; ++i) {
      CK(hipMemset(par[1], 0, par_b));
      prod_variant(w0, i, 1);
      CK(hipMemcpy(want, par[1], par_b, hipMemcpyDeviceToDevice));
      for (int w = 0; w < (int)pks.size(); ++w) {
        if (w == w0 || pks[w].first.find("recover") == std::string::npos || !pks[w].second) continue;
        CK(hipMemset(par[1], 0, par_b));
        prod_variant(w, i, 1);
        CK(hipMemset(bad, 0, 4));
        hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, 0, par[1], want, par_b, bad);
        uint32_t h = 0;
        CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
        if (h) std::printf("%s rows%d: %u differing words\n", pks[w].first.c_str(), i, h);
      }
    }
  }
  std::printf("exactness checked (silence = every variant equals the product)\n");
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int NV = (int)vs.size() + 2 + (int)pks.size();
  std::vector<std::vector<double>> res(NV * NR * NP);
  for (int r = 0; r < rounds; ++r)
    for (int i = 0; i < NR; ++i)
      for (int j = 0; j < NP; ++j)
        for (int v = 0; v < NV; ++v) {
          double tot = 0;
          for (int q = 0; q <= reps; ++q) {
            if (v < (int)vs.size()) CK(hipMemsetAsync(ctr, 0, 17 * 256, 0));
            CK(hipEventRecord(e0, 0));
            if (v < (int)vs.size())
              hipLaunchKernelGGL(vs[v].k, dim3(vs[v].grid), dim3(vs[v].bs), 0, 0, rows[i], par[j], G,
                                 vs[v].nphase, ctr, tmo);
            else if (v == (int)vs.size())
              product(i, j);
            else if (v == (int)vs.size() + 1)
              product_phased(i, j);
            else
              prod_variant(v - (int)vs.size() - 2, i, j);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (q) tot += ms;  // first launch = warm-up
          }
          res[(v * NR + i) * NP + j].push_back((double)(rows_b + par_b) / (tot / reps * 1e-3) / 8e12);
        }
  uint32_t h_tmo = 0;
  CK(hipMemcpy(&h_tmo, tmo, 4, hipMemcpyDeviceToHost));
  std::printf("\nfrac of 8 TB/s (median of %d rounds x %d launches)\n%-24s", rounds, reps, "variant");
  for (int i = 0; i < NR; ++i)
    for (int j = 0; j < NP; ++j) std::printf("  r%d/p%d", i, j);
  std::printf("\n");
  for (int v = 0; v < NV; ++v) {
    std::printf("%-24s", v < (int)vs.size()        ? vs[v].name.c_str()
                         : v == (int)vs.size()     ? "product one-pass"
                         : v == (int)vs.size() + 1 ? "product phased"
                                                   : pks[v - vs.size() - 2].first.c_str());
    for (int i = 0; i < NR; ++i)
      for (int j = 0; j < NP; ++j) {
        auto x = res[(v * NR + i) * NP + j];
        std::sort(x.begin(), x.end());
        std::printf(" %.4f", x[x.size() / 2]);
      }
    std::printf("\n");
  }
  std::printf("phase-wait timeouts (all variants, all launches): %u\n", h_tmo);
  return 0;
}
