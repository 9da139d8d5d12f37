// tune_latency.hip — what one small flush's ~29 us is made of
// (QuicFecReviveBatch::Flush of one group, bench_connection): round-trip of
// a tiny kernel on a non-blocking stream, host-measured, by completion method:
//   A: launch + hipEventRecord + hipEventSynchronize
//   B: launch + hipEventRecord + spin on hipEventQuery
//   C: launch + hipStreamSynchronize
//   D: launch; the kernel's last store is a flag in mapped pinned memory
//      (system-scope release), the host spins on it
//   E: A, with the kernel reading 16 B from mapped host memory (one PCIe read)
//   F: A, with the kernel reading 3 dependent 8-B values from mapped host
//      memory (the ragged kernel's grp_ptr -> table -> payload chain)
//   G: launch + hipStreamWriteValue32 of a mapped flag, host spins on it
//   H: launch + a second 1-thread kernel storing the mapped flag, host spins
//   I: hipPointerGetAttributes on a pinned pointer (host cost only)
//   J: hipSetDevice (host cost only)
// Median of 2,000 round trips each.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/tune/tune_latency.hip -o tools/tune/build/tune_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

__global__ void tiny(uint32_t* out, uint32_t v) {
  if (threadIdx.x == 0) out[0] = v;
}
__global__ void flag_kernel(uint32_t* dev_out, uint32_t* host_flag, uint32_t v) {
  if (threadIdx.x == 0) {
    dev_out[0] = v;
    __hip_atomic_store(host_flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
__global__ void read1(const uint64_t* host, uint64_t* out) {
  if (threadIdx.x == 0) out[0] = host[0] + host[1];
}
__global__ void chain3(const uint64_t* host, uint64_t* out) {
  if (threadIdx.x == 0) {
    const uint64_t a = host[0];
    const uint64_t b = host[a];
    out[0] = host[b];
  }
}

using Clock = std::chrono::steady_clock;

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  uint32_t* d;
  CK(hipMalloc(&d, 64));
  uint32_t* hflag;
  CK(hipHostMalloc(&hflag, 64, hipHostMallocMapped | hipHostMallocPortable));
  uint32_t* hflag_dev;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hflag_dev), hflag, 0));
  uint64_t* htab;
  CK(hipHostMalloc(&htab, 4096, hipHostMallocMapped | hipHostMallocPortable));
  htab[0] = 5;
  htab[5] = 9;
  htab[9] = 42;
  htab[1] = 7;
  uint64_t* htab_dev;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&htab_dev), htab, 0));
  const int N = 2000;
  const char* names[] = {"A event sync",       "B event query spin",     "C stream sync",
                         "D mapped flag spin", "E A + one PCIe read",    "F A + 3 dependent reads",
                         "G write-value flag", "H flag kernel after",    "I pointer attributes",
                         "J hipSetDevice"};
  for (int m = 0; m < 10; ++m) {
    std::vector<double> t;
    for (int i = 0; i < N + 50; ++i) {
      const uint32_t v = (uint32_t)(i + 1) * 8 + (uint32_t)m;
      const auto t0 = Clock::now();
      if (m == 3) {
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, d, hflag_dev, v);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != v) {
        }
      } else if (m == 6) {
        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, v);
        CK(hipStreamWriteValue32(s, hflag_dev, v, 0));
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != v) {
        }
      } else if (m == 7) {
        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, v);
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, s, d + 4, hflag_dev, v);
        while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != v) {
        }
      } else if (m == 8) {
        hipPointerAttribute_t attr;
        CK(hipPointerGetAttributes(&attr, htab));
      } else if (m == 9) {
        CK(hipSetDevice(0));
      } else {
        if (m == 4)
          hipLaunchKernelGGL(read1, dim3(1), dim3(64), 0, s, htab_dev, (uint64_t*)d);
        else if (m == 5)
          hipLaunchKernelGGL(chain3, dim3(1), dim3(64), 0, s, htab_dev, (uint64_t*)d);
        else
          hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d, v);
        if (m == 2) {
          CK(hipStreamSynchronize(s));
        } else {
          CK(hipEventRecord(ev, s));
          if (m == 1) {
            hipError_t e;
            while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
            }
            CK(e);
          } else {
            CK(hipEventSynchronize(ev));
          }
        }
      }
      const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
      if (i >= 50) t.push_back(us);
    }
    std::sort(t.begin(), t.end());
    std::printf("%-26s median %7.1f us  p10 %7.1f  p90 %7.1f\n", names[m], t[t.size() / 2],
                t[t.size() / 10], t[t.size() * 9 / 10]);
  }
  CK(hipStreamSynchronize(s));
  return 0;
}
