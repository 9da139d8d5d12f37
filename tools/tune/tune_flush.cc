// tune_flush.cc — where one small connection flush's time goes
// (bench_connection: QuicFecEncodeBatch::Flush of ONE group of 10 x 1350 B).
// Medians of 2,000 repetitions, host clock:
//   flush:    QuicFecEncodeBatch::Flush (ComputeAll + views), as the bench
//   abi:      qfec_encode_ragged(QFEC_PTR_MAPPED) alone on prebuilt tables over
//             the same kind of pinned payloads (qfec_host_alloc)
//   abi_n64:  the same for 64 groups
//   sync:     qfec_sync on an idle context (one D2H of the error word + sync)
// build: g++ -O2 -std=c++17 -Iinclude -Ilibquic_amd/csrc tools/tune/tune_flush.cc \
//          -Llibquic_amd -lqfec -Wl,-rpath,$PWD/libquic_amd -Wl,-rpath-link,/opt/rocm/lib \
//          -o tools/tune/build/tune_flush
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "qfec.h"
#include "quic_fec_connection.h"

using namespace net;
using Clock = std::chrono::steady_clock;

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const int k = 10, reps = 2000;
  const uint32_t L = 1350;
  qfec_ctx* ctx = qfec_create(0);
  if (!ctx) return 2;
  std::vector<std::string> pays(k, std::string(L, '\0'));
  for (int i = 0; i < k; ++i)
    for (uint32_t j = 0; j < L; ++j) pays[i][j] = (char)(i * 31 + j * 7);
  // 1: the bench's Flush
  std::vector<double> t;
  for (int r = 0; r < reps + 20; ++r) {
    QuicFecEncodeBatch batch;
    QuicFecSender s(k);
    for (int i = 0; i < k; ++i) s.OnDataPacket(1 + i, pays[i], false, nullptr);
    s.CloseFecGroup(1 + k, &batch);
    const auto t0 = Clock::now();
    if (batch.Flush(ctx) != QFEC_OK) return 1;
    t.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
  }
  std::printf("flush (1 group)          %7.1f us\n", median(t));
  // 2: the C-ABI call alone
  for (int G : {1, 64}) {
    uint8_t* bytes = static_cast<uint8_t*>(qfec_host_alloc((size_t)G * k * L));
    uint8_t* par = static_cast<uint8_t*>(qfec_host_alloc((size_t)G * L));
    std::vector<uint64_t> off(G * k), poff(G);
    std::vector<uint16_t> len(G * k, L), plen(G);
    std::vector<uint32_t> ptr(G + 1);
    for (int g = 0; g < G; ++g) {
      ptr[g] = g * k;
      poff[g] = (uint64_t)g * L;
      for (int i = 0; i < k; ++i) {
        off[g * k + i] = ((uint64_t)g * k + i) * L;
        std::memcpy(bytes + off[g * k + i], pays[i].data(), L);
      }
    }
    ptr[G] = G * k;
    t.clear();
    for (int r = 0; r < reps + 20; ++r) {
      const auto t0 = Clock::now();
      if (qfec_encode_ragged(ctx, bytes, off.data(), len.data(), ptr.data(), G, par, poff.data(),
                             plen.data(), QFEC_PTR_MAPPED) != QFEC_OK)
        return 1;
      t.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
    std::printf("abi (%2d groups)          %7.1f us\n", G, median(t));
    qfec_host_free(bytes);
    qfec_host_free(par);
  }
  t.clear();
  for (int r = 0; r < reps; ++r) {
    const auto t0 = Clock::now();
    qfec_sync(ctx);
    t.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
  }
  std::printf("qfec_sync (idle)         %7.1f us\n", median(t));
  qfec_destroy(ctx);
  return 0;
}
