// tune_hostlat.hip — round 5: what the small-batch service's one-group
// flush (12.7 us, profiles/round5/service/stamps_svc5c.txt: first group
// 5.6 us, fence 1.3 us) is made of, one PCIe access shape at a time.  One
// wave, timed in the kernel with the 100-MHz wall clock (10-ns ticks):
//   A  one 8-B load (lane 0) of mapped host memory
//   B  1 KiB: 16 B per lane (the service's poll look)
//   C  a 10 x 1350 B group: 20 16-B buffer loads per lane, all in flight
//      (window_group's trip: packets back to back)
//   D  C with every packet 64 KiB apart (one 4-KiB page each)
//   E  C as two dependent trips of 10 loads
//   F  1350 B stored to host memory + a system-scope fence (the output and
//      the fence before the token)
//   G  C then F (one group's whole device-side work)
// each warm (the same bytes every rep) and cold (a new 1-MiB window of a
// 512-MiB buffer every rep).  Host-measured ping-pong through a resident
// wave (the host stores a word, the wave's poll sees it and stores an
// answer, the host spins on it) with the poll reading 8 B or 1 KiB per look
// and with or without s_sleep between looks.  Medians of 400.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_hostlat.hip -o tools/tune/build/tune_hostlat
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void use(uint32_t v) { asm volatile("" ::"v"(v)); }

__device__ __forceinline__ u32x4 bload(const uint8_t* base, uint32_t off) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7FFFFFFF, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 2);
}

// 20 loads of one group: packet r at base + r * pstride, windows w0 / w1
template <int NL>
__device__ __forceinline__ uint32_t group_loads(const uint8_t* base, uint64_t pstride, uint32_t lane,
                                                int first) {
  u32x4 v[NL];
  const uint32_t w0 = min(16u * lane, 1334u), w1 = min(16u * (lane + 64u), 1334u);
#pragma unroll
  for (int u = 0; u < NL; ++u) {
    const int j = first + u;
    v[u] = bload(base + (uint64_t)(j % 10) * pstride, j < 10 ? w0 : w1);
  }
  uint32_t x = 0;
#pragma unroll
  for (int u = 0; u < NL; ++u) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  return x;
}

__global__ __launch_bounds__(64) void probe(const uint8_t* host, uint8_t* hout, uint64_t* res,
                                            int mode, uint64_t off) {
  const uint32_t lane = threadIdx.x;
  const uint8_t* b = host + off;
  uint32_t x = 0;
  const uint64_t t0 = wall_clock64();
  if (mode == 0) {
    if (lane == 0) x = (uint32_t)__hip_atomic_load(reinterpret_cast<const uint64_t*>(b),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else if (mode == 1) {
    const u32x4 v = bload(b, 16u * lane);
    x = v.x ^ v.w;
  } else if (mode == 2) {
    x = group_loads<20>(b, 1350, lane, 0);
  } else if (mode == 3) {
    x = group_loads<20>(b, 65536, lane, 0);
  } else if (mode == 4) {
    x = group_loads<10>(b, 1350, lane, 0);
    use(x);
    uint32_t z;  // 0, but only once the first trip's bytes are in
    asm volatile("v_and_b32 %0, 0, %1" : "=v"(z) : "v"(x));
    x ^= group_loads<10>(b + z, 1350, lane, 10);
  }
  use(x);
  const uint64_t t1 = wall_clock64();
  if (mode == 5 || mode == 6) {
    if (mode == 6) x = group_loads<20>(b, 1350, lane, 0);
    u32x4 o = {x, lane, 3u, 4u};
    uint8_t* d = hout + off;
    if (lane < 85u) *reinterpret_cast<u32x4*>(d + 16u * lane) = o;
    if (lane + 64u < 85u) *reinterpret_cast<u32x4*>(d + 16u * (lane + 64u)) = o;
    __threadfence_system();
  }
  const uint64_t t2 = wall_clock64();
  if (lane == 0) {
    res[0] = mode >= 5 ? t2 - t0 : t1 - t0;
    res[1] = x;
  }
}

// resident ping-pong: look at ping (8 B, or 1 KiB with the word in lane 0's
// first 8 B), answer on pong; n rounds
__global__ __launch_bounds__(64) void pingpong(const uint64_t* ping, uint64_t* pong, uint32_t n,
                                               int wide, int sleep) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = 1; i <= n; ++i) {
    for (;;) {
      uint64_t v;
      if (wide) {
        const uint64_t a = __hip_atomic_load(ping + 2u * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t c = __hip_atomic_load(ping + 2u * lane + 1u, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
        use((uint32_t)c);
        v = (uint64_t)__shfl((unsigned long long)a, 0, 64);
      } else {
        v = __hip_atomic_load(ping, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (v >= i) break;
      if (sleep) __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) __hip_atomic_store(pong, (uint64_t)i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// the same with four 8-B looks in flight: each pass waits for the oldest
// look only and issues the next (a look lands every quarter round trip)
__device__ __forceinline__ uint64_t lk(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(64) void pingpong_pipe(const uint64_t* ping, uint64_t* pong, uint32_t n) {
  const uint32_t lane = threadIdx.x;
  uint32_t i = 1;
  uint64_t a = lk(ping), b = lk(ping), c = lk(ping), d = lk(ping);
  auto step = [&](uint64_t& x) {
    if (x >= i) {
      if (lane == 0) __hip_atomic_store(pong, (uint64_t)i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      ++i;
    }
    x = lk(ping);
  };
  while (i <= n) {
    step(a);
    step(b);
    step(c);
    step(d);
  }
  use((uint32_t)(a ^ b ^ c ^ d));
}

using Clock = std::chrono::steady_clock;

int main() {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const size_t HB = 512ull << 20;
  uint8_t *h_in, *h_out;
  const unsigned fl = hipHostMallocMapped | hipHostMallocPortable;
  CK(hipHostMalloc(&h_in, HB, fl));
  CK(hipHostMalloc(&h_out, HB, fl));
  for (size_t i = 0; i < HB; i += 4096) std::memset(h_in + i, (int)(i >> 12), 4096);
  std::memset(h_out, 0, HB);
  uint8_t *d_in, *d_out;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_in), h_in, 0));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_out), h_out, 0));
  uint64_t* d_res;
  CK(hipMalloc(&d_res, 64));
  const char* names[] = {"A 8 B", "B 1 KiB (16 B/lane)", "C group 10x1350 B, 20 loads",
                         "D group, packets 64 KiB apart", "E group as 2 dependent trips",
                         "F 1350 B store + system fence", "G C then F"};
  const int R = 400;
  for (int mode = 0; mode < 7; ++mode)
    for (int cold = 0; cold < 2; ++cold) {
      std::vector<double> t;
      for (int r = 0; r < R + 20; ++r) {
        // cold: a new 1-MiB window each rep (D spans 640 KiB)
        const uint64_t off = cold ? ((uint64_t)(r % 500) << 20) : 0;
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_in, d_out, d_res, mode, off);
        CK(hipDeviceSynchronize());
        uint64_t h[2];
        CK(hipMemcpy(h, d_res, 16, hipMemcpyDeviceToHost));
        if (r >= 20) t.push_back(h[0] * 0.01);
      }
      std::sort(t.begin(), t.end());
      std::printf("%-34s %-4s median %6.2f us  p10 %6.2f  p90 %6.2f\n", names[mode],
                  cold ? "cold" : "warm", t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10]);
    }
  // ping-pong
  uint64_t* ping = reinterpret_cast<uint64_t*>(h_in);
  uint64_t* pong = reinterpret_cast<uint64_t*>(h_out);
  for (int wide = 0; wide < 3; ++wide)
    for (int sleep = 0; sleep < (wide == 2 ? 1 : 2); ++sleep) {
      const uint32_t n = 2000;
      __atomic_store_n(ping, 0ull, __ATOMIC_SEQ_CST);
      __atomic_store_n(pong, 0ull, __ATOMIC_SEQ_CST);
      if (wide == 2)
        hipLaunchKernelGGL(pingpong_pipe, dim3(1), dim3(64), 0, 0,
                           reinterpret_cast<const uint64_t*>(d_in), reinterpret_cast<uint64_t*>(d_out), n);
      else
        hipLaunchKernelGGL(pingpong, dim3(1), dim3(64), 0, 0, reinterpret_cast<const uint64_t*>(d_in),
                           reinterpret_cast<uint64_t*>(d_out), n, wide, sleep);
      std::vector<double> t;
      bool ok = true;
      for (uint32_t i = 1; i <= n; ++i) {
        const auto c0 = Clock::now();
        __atomic_store_n(ping, (uint64_t)i, __ATOMIC_RELEASE);
        const auto lim = c0 + std::chrono::seconds(2);
        while (__atomic_load_n(pong, __ATOMIC_ACQUIRE) != i) {
          if (Clock::now() > lim) {
            ok = false;
            break;
          }
        }
        if (!ok) break;
        const auto c1 = Clock::now();
        // a gap, as between flushes
        while (std::chrono::duration<double, std::micro>(Clock::now() - c1).count() < 20.0) {
        }
        if (i > 50) t.push_back(std::chrono::duration<double, std::micro>(c1 - c0).count());
      }
      if (!ok) {
        // let the kernel finish: publish the last round
        __atomic_store_n(ping, (uint64_t)n, __ATOMIC_RELEASE);
        CK(hipDeviceSynchronize());
        std::printf("ping-pong wide=%d sleep=%d: no answer within 2 s\n", wide, sleep);
        return 2;
      }
      CK(hipDeviceSynchronize());
      std::sort(t.begin(), t.end());
      std::printf("ping-pong %-6s look, %-8s median %6.2f us  p10 %6.2f  p90 %6.2f\n",
                  wide == 2 ? "4x8 B" : wide ? "1 KiB" : "8 B",
                  wide == 2 ? "pipelined" : sleep ? "s_sleep2" : "spin", t[t.size() / 2],
                  t[t.size() / 10], t[t.size() * 9 / 10]);
    }
  return 0;
}
