// probe_vram_host.hip — round 6: can the host write the
// small-batch service's job entries straight into device memory?  The
// worker's poll and entry copy are PCIe round trips today (host-mapped
// ring: ~1.4 us per trip); with the ring in VRAM the worker would poll local
// HBM and the host's stores would cross the link as posted writes.
//
// 1. fine-grained device memory (hipExtMallocWithFlags hipDeviceMallocFinegrained)
//    -- its pointer attributes: is it host-accessible (a host pointer)?
// 2. only if so: host writes a pattern, a kernel checks it; a ping-pong
//    (host stores a word in VRAM, a wave spinning on it locally answers in
//    host-mapped memory) against the same ping-pong through host memory.
//
//   probe_vram_host [reps=2000]
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/probe_vram_host.hip \
//          -o tools/tune/build/probe_vram_host
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

__global__ void check_kernel(const uint32_t* p, uint32_t n, uint32_t* bad) {
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    if (p[i] != i * 2654435761u) atomicAdd(bad, 1u);
}

// one wave: wait for ping == i (volatile, system scope), answer pong = i, reps times;
// bounded: gives up after ~0.2 s without a new ping
__global__ void pong_kernel(uint32_t* ping, uint32_t* pong, uint32_t reps, uint32_t* stuck) {
  if (threadIdx.x != 0) return;
  for (uint32_t i = 1; i <= reps; ++i) {
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(ping, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != i) {
      if (wall_clock64() - t0 > 20000000ull) {  // 100-MHz ticks: 0.2 s
        *stuck = i;
        return;
      }
    }
    __hip_atomic_store(pong, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static double pingpong_us(uint32_t* ping_host_view, uint32_t* ping_dev, uint32_t* pong_host,
                          uint32_t* pong_dev, uint32_t* stuck, int reps) {
  __atomic_store_n(ping_host_view, 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(pong_host, 0u, __ATOMIC_SEQ_CST);
  hipLaunchKernelGGL(pong_kernel, dim3(1), dim3(64), 0, 0, ping_dev, pong_dev, (uint32_t)reps, stuck);
  std::vector<double> t;
  for (int i = 1; i <= reps; ++i) {
    const auto a = std::chrono::steady_clock::now();
    __atomic_store_n(ping_host_view, (uint32_t)i, __ATOMIC_SEQ_CST);
    const auto limit = a + std::chrono::milliseconds(200);
    while (__atomic_load_n(pong_host, __ATOMIC_ACQUIRE) != (uint32_t)i)
      if (std::chrono::steady_clock::now() > limit) {
        std::printf("  ping-pong: no answer to ping %d\n", i);
        CK(hipDeviceSynchronize());
        return -1;
      }
    t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
  }
  CK(hipDeviceSynchronize());
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const int reps = argc > 1 ? atoi(argv[1]) : 2000;
  uint32_t* stuck;
  CK(hipMalloc(&stuck, 4));
  CK(hipMemset(stuck, 0, 4));
  // the host-memory reference: ping and pong both in host-mapped memory
  uint32_t *hping, *hpong;
  CK(hipHostMalloc(&hping, 4096, hipHostMallocMapped | hipHostMallocPortable));
  CK(hipHostMalloc(&hpong, 4096, hipHostMallocMapped | hipHostMallocPortable));
  uint32_t *hping_d, *hpong_d;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hping_d), hping, 0));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hpong_d), hpong, 0));
  std::printf("ping-pong through host memory: median %.2f us\n",
              pingpong_us(hping, hping_d, hpong, hpong_d, stuck, reps));

  const size_t bytes = 1 << 20;
  uint32_t* v = nullptr;
  hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&v), bytes, hipDeviceMallocFinegrained);
  std::printf("fine-grained device memory: %s\n", hipGetErrorString(e));
  if (e != hipSuccess) return 0;
  hipPointerAttribute_t at;
  CK(hipPointerGetAttributes(&at, v));
  std::printf("  attributes: type %d, device %d, devicePointer %p, hostPointer %p, isManaged %d\n",
              (int)at.type, at.device, at.devicePointer, at.hostPointer, (int)at.isManaged);
  if (!at.hostPointer) {
    std::printf("  not host-accessible: a VRAM ring needs the host to reach it another way\n");
    return 0;
  }
  uint32_t* hv = static_cast<uint32_t*>(at.hostPointer);
  const uint32_t n = (uint32_t)(bytes / 4);
  const auto a = std::chrono::steady_clock::now();
  for (uint32_t i = 0; i < n; ++i) hv[i] = i * 2654435761u;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  const double wus = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
  uint32_t* bad;
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(check_kernel, dim3(1), dim3(1024), 0, 0, v, n, bad);
  CK(hipDeviceSynchronize());
  uint32_t hb = 0;
  CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  std::printf("  host wrote 1 MiB into VRAM in %.1f us (%.2f GB/s); device check: %u wrong words\n",
              wus, bytes / wus / 1e3, hb);
  // 8 KB (a 64-group entry) host write time
  std::vector<double> t8;
  for (int r = 0; r < 200; ++r) {
    const auto b = std::chrono::steady_clock::now();
    std::memcpy(hv, hping, 4096);
    std::memcpy(hv + 1024, hping, 4096);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    t8.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - b).count());
  }
  std::sort(t8.begin(), t8.end());
  std::printf("  host memcpy of 8 KiB into VRAM: median %.2f us\n", t8[t8.size() / 2]);
  std::printf("ping-pong, ping in VRAM (host stores, the wave polls locally), pong in host memory: "
              "median %.2f us\n",
              pingpong_us(hv + 4096, v + 4096, hpong, hpong_d, stuck, reps));
  uint32_t hs = 0;
  CK(hipMemcpy(&hs, stuck, 4, hipMemcpyDeviceToHost));
  if (hs) std::printf("  (the wave gave up at ping %u)\n", hs);
  return 0;
}
