// null_phased.hip — a grid-phased NULL encrypt (VERDICT r3 item 6 experiment).
// phased_copy.hip showed a copy whose reads and writes are split in time
// across the grid (one meeting per phase) runs 0.707 of 8 TB/s against the
// streaming copy's 0.634.  NULL encrypt is a copy plus an FNV-1a-128 hash
// (0.513 in the product, 0.81 of the streaming copy).  Here: a persistent
// grid of two 4-wave blocks per CU; each wave owns 64 packets per batch (as
// the product's staged kernel); per phase every wave LOADS HS 256-B slabs of
// its packets into VGPRs (coalesced, chunk-major), the grid meets, then each
// slab is transposed through LDS, hashed (the lane's own packet) and STORED
// from the VGPRs.  Reads and writes are separated in time; the FNV work runs
// in the write phases.  Waves whose batch writes over its own payload (in
// place) take the product's staged schedule and only attend the meetings.
// Every variant's output (tags + payload copies) is compared byte for byte
// with the product kernel's before it is timed.
//
//   null_phased [packets=10485760] [reps=5] [rounds=3]
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/null_phased.hip \
//          -o tools/tune/build/null_phased
#include "../../libquic_amd/csrc/qpp_kernels.hip"

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

namespace qfec {
namespace {

constexpr uint64_t kMeetTimeout = 20000;  // s_memrealtime ticks (100 MHz): 200 us

__device__ __forceinline__ uint32_t* mw(uint32_t* ps, uint32_t i) { return ps + 64u * i; }
__device__ __forceinline__ uint32_t mload(uint32_t* w) {
  return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// grid-wide meeting number `epoch` (16 sub-counters + a top counter; word 18
// = abandoned: a meeting that times out lets everyone through from then on)
__device__ __forceinline__ void meet(uint32_t* ps, uint32_t epoch) {
  __syncthreads();
  if (threadIdx.x == 0 && mload(mw(ps, 18)) == 0u) {
    const uint32_t B = gridDim.x, sub = blockIdx.x & 15u, nsub = (B - sub + 15u) / 16u;
    const uint32_t old =
        __hip_atomic_fetch_add(mw(ps, 1u + sub), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1u == epoch * nsub)
      __hip_atomic_fetch_add(mw(ps, 0), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t target = epoch * min(B, 16u);
    const uint64_t t0 = wall_clock64();
    while (mload(mw(ps, 0)) < target) {
      if (wall_clock64() - t0 > kMeetTimeout) {
        __hip_atomic_fetch_or(mw(ps, 18), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      if (mload(mw(ps, 18)) != 0u) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// the last block out resets the words (word 19 counts abandoned launches)
__device__ __forceinline__ void meet_exit(uint32_t* ps) {
  __syncthreads();
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(mw(ps, 17), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
          gridDim.x - 1u) {
    if (mload(mw(ps, 18)) != 0u)
      __hip_atomic_fetch_add(mw(ps, 19), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t i = 0; i < 19u; ++i)
      __hip_atomic_store(mw(ps, i), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <uint32_t SC, uint32_t HS, int MINW>
__global__ __launch_bounds__(kBlock, MINW) void null_encrypt_phased_kernel(ProtectArgs a, uint32_t* ps,
                                                                          uint32_t nbatch,
                                                                          uint32_t nph) {
  __shared__ u32x4 s_rows[kWaves][64 * (SC + 1u)];
  __shared__ StageMeta s_meta[kWaves][64];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint32_t epoch = 0;
  for (uint32_t j = 0; j < nbatch; ++j) {
    const uint64_t p = (((uint64_t)j * gridDim.x + blockIdx.x) * kWaves + wv) * 64u + lane;
    const bool valid = p < a.n;
    const uint8_t* ad = nullptr;
    const uint8_t* pt = nullptr;
    uint8_t* o = nullptr;
    uint32_t alen = 0, plen = 0;
    if (valid) {
      ad = a.bytes + a.ad_off[p];
      pt = a.bytes + a.in_off[p];
      alen = a.ad_len[p];
      plen = a.in_len[p];
      o = a.out + a.out_off[p];
    }
    const DstSplit sp = dst_split(o + kTag, plen);
    const StageMeta m = line_meta(pt + sp.hd, o + kTag + sp.hd, sp.nmid, o + kTag + sp.hd);
    s_meta[wv][lane] = m;
    const u32x4 head = valid ? load_head(pt, plen) : u32x4{0u, 0u, 0u, 0u};
    const u32x4 tail = valid ? load_tail(pt, plen) : u32x4{0u, 0u, 0u, 0u};
    Fnv128 h = fnv_init();
    if (valid) {
      fnv_span<true>(h, ad, alen);
      fnv_bytes(h, head, 0u, sp.hd);
    }
    const bool overlap = valid && o + kTag < pt + plen && pt < o + kTag + plen;
    if (wave_any_qpp(overlap)) {
      // in place: the product's schedule now, then only the meetings
      stage_hash<true, SC, true, true, kNullNT>(h, s_meta[wv], s_rows[wv], lane, m.nfull, m.lo);
      for (uint32_t q = 0; q < nph; ++q) meet(ps, ++epoch);
    } else {
      const uint32_t nslab = (wave_max_u32(m.nfull) + SC - 1) / SC;
      for (uint32_t q = 0; q < nph; ++q) {
        u32x4 v[HS][SC];
#pragma unroll
        for (uint32_t s = 0; s < HS; ++s) {
          const uint32_t sl = q * HS + s;
          if (sl < nslab) stage_load<SC, true, false>(s_meta[wv], lane, sl, v[s]);
        }
        meet(ps, ++epoch);
#pragma unroll
        for (uint32_t s = 0; s < HS; ++s) {
          const uint32_t sl = q * HS + s;
          if (sl < nslab) {
            stage_to_lds<SC>(s_rows[wv], lane, v[s]);
#pragma unroll
            for (uint32_t c = 0; c < SC; ++c)
              if (sl * SC + c >= m.lo && sl * SC + c < m.nfull)
                fnv_chunk<true>(h, s_rows[wv][lane * (SC + 1u) + c]);
            stage_store<SC, true, true>(s_meta[wv], lane, sl, v[s]);
          }
        }
      }
    }
    if (valid) {
      const uint32_t t0 = tail_pos(sp.hd + 16u * sp.nmid, plen);
      fnv_bytes(h, tail, t0, sp.tl);
      store_from_aligned_start(o + kTag + sp.hd + 16u * sp.nmid, tail, t0, sp.tl);
      store_to_aligned_end(o + kTag, head, 0u, sp.hd);
      const uint32_t tag[3] = {h.x0, h.x1, h.x2};
      __builtin_memcpy(o, tag, kTag);
    }
  }
  meet_exit(ps);
}

}  // namespace
}  // namespace qfec

__global__ void fill_bytes(uint8_t* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 29)) * 0xBF58476D1CE4E5B9ull;
    p[i] = (uint8_t)(z >> 40);
  }
}

template <typename T>
static T* up(const std::vector<T>& v) {
  T* d;
  CK(hipMalloc(&d, v.size() * sizeof(T)));
  CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 10485760ull;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int rounds = argc > 3 ? atoi(argv[3]) : 3;
  const uint32_t L = 1350, H = 22;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  // the bench's packed layout: [header H | payload L] back to back; out tag||payload
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
  hipLaunchKernelGGL(fill_bytes, dim3(4096), dim3(256), 0, 0, d_in, n * (H + L));
  CK(hipGetLastError());
  qfec::ProtectArgs e{};
  e.bytes = d_in;
  e.ad_off = up(ad_off);
  e.ad_len = up(ad_len);
  e.in_off = up(in_off);
  e.in_len = up(in_len);
  e.out = d_ref;
  e.out_off = up(out_off);
  e.n = n;
  uint32_t* ps;
  CK(hipMalloc(&ps, 64 * 4 * 32));
  CK(hipMemset(ps, 0, 64 * 4 * 32));
  CK(qfec::launch_null_protect(e, false, 0));  // the product's output: the reference
  CK(hipDeviceSynchronize());
  qfec::ProtectArgs ev = e;
  ev.out = d_out;

  const uint32_t grid = 2u * (uint32_t)ncu;  // two 4-wave blocks per CU (LDS: 2 x 78 KiB)
  const uint32_t nbatch = (uint32_t)((n + (uint64_t)grid * 256u - 1) / ((uint64_t)grid * 256u));
  const uint32_t slabs = (7u + (L + 15u) / 16u + 15u) / 16u;  // line grid shift <= 7 chunks
  struct V {
    std::string name;
    bool product;
    std::function<void()> run;
  };
  std::vector<V> vs = {
      {"product (staged)", true, [&] { CK(qfec::launch_null_protect(ev, false, 0)); }},
      {"phased HS=2", false,
       [&] {
         hipLaunchKernelGGL((qfec::null_encrypt_phased_kernel<16, 2, 2>), dim3(grid), dim3(256), 0,
                            0, ev, ps, nbatch, (slabs + 1u) / 2u);
       }},
      {"phased HS=3", false,
       [&] {
         hipLaunchKernelGGL((qfec::null_encrypt_phased_kernel<16, 3, 2>), dim3(grid), dim3(256), 0,
                            0, ev, ps, nbatch, (slabs + 2u) / 3u);
       }},
      {"product (staged) again", true, [&] { CK(qfec::launch_null_protect(ev, false, 0)); }},
  };
  const uint64_t OB = n * (L + 12);
  std::vector<uint8_t> h_ref(OB), h_v(OB);
  CK(hipMemcpy(h_ref.data(), d_ref, OB, hipMemcpyDeviceToHost));
  bool ok = true;
  for (const V& v : vs) {
    CK(hipMemset(d_out, 0xA5, OB));
    v.run();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h_v.data(), d_out, OB, hipMemcpyDeviceToHost));
    const bool same = h_v == h_ref;
    std::printf("check %-24s %s\n", v.name.c_str(), same ? "== product" : "MISMATCH");
    ok = ok && same;
  }
  if (!ok) return 2;
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < vs.size(); ++i) {
      vs[i].run();
      CK(hipEventRecord(t0, 0));
      for (int q = 0; q < reps; ++q) vs[i].run();
      CK(hipEventRecord(t1, 0));
      CK(hipEventSynchronize(t1));
      float m = 0;
      CK(hipEventElapsedTime(&m, t0, t1));
      ms[i].push_back(m / reps);
    }
  uint32_t h_ps[64 * 20];
  CK(hipMemcpy(h_ps, ps, sizeof(h_ps), hipMemcpyDeviceToHost));
  // algorithmic bytes: header + payload read, tag + payload written
  const double bytes = (double)n * (H + L + 12 + L);
  std::printf("\n%llu packets x (%u + %u) B, %d CUs, grid %u, %u batches; bytes = read + written\n",
              (unsigned long long)n, H, L, ncu, grid, nbatch);
  for (size_t i = 0; i < vs.size(); ++i) {
    std::vector<float> s = ms[i];
    std::sort(s.begin(), s.end());
    const double sec = s[s.size() / 2] * 1e-3;
    std::printf("%-26s %9.1f us  %8.1f GB/s  %.4f of 8 TB/s\n", vs[i].name.c_str(), sec * 1e6,
                bytes / sec / 1e9, bytes / sec / 8e12);
  }
  std::printf("abandoned phased launches: %u\n", h_ps[64 * 19]);
  return 0;
}
