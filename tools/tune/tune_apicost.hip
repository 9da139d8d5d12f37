// tune_apicost.hip — round 6: what the HIP runtime calls on the connection
// thread's path cost (ns per call, median of 5 runs of 200,000 calls):
// hipGetDevice, hipSetDevice (same device), hipStreamQuery / hipEventQuery on
// an idle stream / event, and the steady clock for scale.
//   build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/tune/tune_apicost.hip \
//            -o tools/probe_bin/tune_apicost
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

template <class F>
static double per_call_ns(F f) {
  constexpr int kN = 200000;
  std::vector<double> r;
  for (int rep = 0; rep < 5; ++rep) {
    const auto a = std::chrono::steady_clock::now();
    for (int i = 0; i < kN; ++i) f();
    r.push_back(std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - a).count() / kN);
  }
  std::sort(r.begin(), r.end());
  return r[2];
}

int main() {
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventRecord(ev, s));
  CK(hipStreamSynchronize(s));
  int cur = -1;
  std::printf("hipGetDevice      %7.1f ns\n", per_call_ns([&] { (void)hipGetDevice(&cur); }));
  std::printf("hipSetDevice(0)   %7.1f ns\n", per_call_ns([&] { (void)hipSetDevice(0); }));
  std::printf("hipStreamQuery    %7.1f ns\n", per_call_ns([&] { (void)hipStreamQuery(s); }));
  std::printf("hipEventQuery     %7.1f ns\n", per_call_ns([&] { (void)hipEventQuery(ev); }));
  std::printf("steady_clock      %7.1f ns\n",
              per_call_ns([&] { (void)std::chrono::steady_clock::now(); }));
  CK(hipEventDestroy(ev));
  CK(hipStreamDestroy(s));
  return 0;
}
