// svc_host_cost.cc — round 5: the connection thread's cost of one small
// QFEC_ASYNC batch on the small-batch service (connection_e2e at one
// connection: ~0.64 us per C-ABI call, 1.3 groups a call).  One group of
// 10 x 1350 B in qfec_host_alloc memory, per repetition:
//   call      qfec_encode_ragged(QFEC_PTR_MAPPED | QFEC_ASYNC)
//   complete  qfec_complete(wait) minus the time blocked on the device
//             (measured as the spin until the flag; reported apart)
// with a gap of `gap_us` between repetitions (the loop turn's other work),
// medians over 2,000 calls; also hipSetDevice alone.  Needs a GPU.
// build: g++ -O2 -std=c++17 -I include tools/tune/svc_host_cost.cc -L libquic_amd -lqfec
//          -Wl,-rpath,$PWD/libquic_amd -o tools/tune/build/svc_host_cost
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "qfec.h"

using Clock = std::chrono::steady_clock;
static double us(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}
static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(q * (v.size() - 1))];
}

int main(int argc, char** argv) {
  const double gap_us = argc > 1 ? std::atof(argv[1]) : 20.0;
  const int k = 10;
  const uint32_t L = 1350;
  qfec_ctx* ctx = qfec_create(0);
  if (!ctx) {
    std::fprintf(stderr, "qfec_create: %s\n", qfec_last_error(nullptr));
    return 2;
  }
  uint8_t* bytes = static_cast<uint8_t*>(qfec_host_alloc(1 << 20));
  uint8_t* par = static_cast<uint8_t*>(qfec_host_alloc(1 << 16));
  if (!bytes || !par) return 3;
  for (int i = 0; i < (1 << 20); ++i) bytes[i] = (uint8_t)(i * 131 + 7);
  std::vector<uint64_t> off(k);
  std::vector<uint16_t> len(k, (uint16_t)L);
  for (int i = 0; i < k; ++i) off[i] = 4096 + (uint64_t)i * L;
  const uint32_t ptr[2] = {0, (uint32_t)k};
  const uint64_t poff = 0;
  uint16_t plen = 0;
  const int N = 2000, W = 100;
  std::vector<double> t_call, t_done;
  for (int r = 0; r < N + W; ++r) {
    const auto a0 = Clock::now();
    int rc = qfec_encode_ragged(ctx, bytes, off.data(), len.data(), ptr, 1, par, &poff, &plen,
                                QFEC_PTR_MAPPED | QFEC_ASYNC);
    const auto a1 = Clock::now();
    rc = rc ? rc : qfec_complete(ctx, 1);
    const auto a2 = Clock::now();
    if (rc != QFEC_OK) {
      std::fprintf(stderr, "rep %d: %s\n", r, qfec_last_error(ctx));
      return 4;
    }
    if (r >= W) {
      t_call.push_back(us(a0, a1));
      t_done.push_back(us(a1, a2));
    }
    const auto g0 = Clock::now();
    while (us(g0, Clock::now()) < gap_us) {
    }
  }
  uint64_t st[3] = {0, 0, 0};
  qfec_debug_service(ctx, -1, st);
  std::printf("{\"gap_us\": %.0f, \"call_us_p50\": %.3f, \"call_us_p10\": %.3f, \"call_us_p90\": %.3f, "
              "\"complete_wait_us_p50\": %.3f, \"service_launches\": %llu, \"service_jobs\": %llu}\n",
              gap_us, pct(t_call, 0.5), pct(t_call, 0.1), pct(t_call, 0.9), pct(t_done, 0.5),
              (unsigned long long)st[0], (unsigned long long)st[1]);
  qfec_destroy(ctx);
  return 0;
}
