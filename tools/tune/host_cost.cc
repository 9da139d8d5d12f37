// host_cost.cc — where the connection thread's time goes in one batched FEC
// launch (QuicFecBatcher::Launch at 4,096 connections
// cost 0.44 us per group against 0.24 at 64).  N groups of 10 x 1350 B are
// folded round-robin over the groups (QuicFecGroup::Update: the payloads
// copied into the pinned payload arena, untimed), the caches swept, then per
// repetition:
//   launch   QuicFecGroup::Launch(async): CSR tables over the arena
//            payloads + qfec_encode_ragged(QFEC_PTR_MAPPED | QFEC_ASYNC)
//   finish   QuicFecGroup::Finish(wait), of which `wait` is blocked on the GPU
//   tables   of launch: the CSR table build (QuicFecGroup::launch_profile)
//   capi     of launch: the qfec_encode_ragged call (the C-ABI's own share)
// Median microseconds per group; one JSON line per N.  Needs a GPU.
//
// build: g++ -O2 -std=c++17 -I include -I libquic_amd/csrc tools/tune/host_cost.cc \
//          -L libquic_amd -lqfec -Wl,-rpath,$PWD/libquic_amd -o tools/tune/build/host_cost
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "quic_fec_group.h"

using namespace net;
using Clock = std::chrono::steady_clock;

static double us(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}
static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int k = 10;
  const size_t L = 1350;
  std::vector<size_t> sizes = {64, 1024, 4096, 16384};
  if (argc > 1) {
    sizes.clear();
    for (int i = 1; i < argc; ++i) sizes.push_back(std::strtoull(argv[i], nullptr, 10));
  }
  qfec_ctx* ctx = qfec_create(0);
  if (!ctx) {
    std::fprintf(stderr, "qfec_create: %s\n", qfec_last_error(nullptr));
    return 2;
  }
  std::string pay(L, '\0');
  std::vector<uint8_t> sweep(64u << 20);
  for (size_t i = 0; i < L; ++i) pay[i] = static_cast<char>(i * 131 + 7);
  for (size_t N : sizes) {
    const int reps = N >= 16384 ? 8 : 30;
    std::vector<double> t_launch, t_finish, t_wait, t_tables, t_capi;
    for (int r = 0; r < reps + 2; ++r) {
      std::vector<std::unique_ptr<QuicFecGroup>> gs;
      std::vector<QuicFecGroup*> raw;
      gs.reserve(N);
      for (size_t g = 0; g < N; ++g) {
        gs.emplace_back(new QuicFecGroup(1000 + 20 * g, ctx));
        raw.push_back(gs.back().get());
      }
      // packets arrive round-robin over the connections (as in a server loop:
      // every group's payloads interleaved with every other group's in the
      // arena), then the thread does other work (a 64-MiB sweep evicts the
      // groups from the caches) before the loop turn's launch
      for (int i = 0; i < k; ++i)
        for (size_t g = 0; g < N; ++g) {
          QuicPacketHeader h;
          h.packet_number = 1000 + 20 * g + i;
          h.is_in_fec_group = IN_FEC_GROUP;
          h.fec_group = 1000 + 20 * g;
          pay[0] = static_cast<char>(g + i);
          gs[g]->Update(ENCRYPTION_FORWARD_SECURE, h, StringPiece(pay));
        }
      for (size_t i = 0; i < sweep.size(); i += 64) sweep[i] += 1;
      QuicFecGroup::Pending p;
      const QuicFecGroup::LaunchProfile before = QuicFecGroup::launch_profile();
      const auto a0 = Clock::now();
      int rc = QuicFecGroup::Launch(ctx, raw, &p, /*async=*/true);
      const auto a1 = Clock::now();
      rc = rc ? rc : QuicFecGroup::Finish(&p, /*wait=*/false);
      const auto a2 = Clock::now();
      if (rc == QFEC_PENDING) rc = QuicFecGroup::Finish(&p, /*wait=*/true);
      const auto a3 = Clock::now();
      if (rc != QFEC_OK) {
        std::fprintf(stderr, "N=%zu: %s\n", N, qfec_last_error(ctx));
        return 3;
      }
      if (r < 2) continue;  // warm-up: staging slots, arena slabs
      const QuicFecGroup::LaunchProfile& after = QuicFecGroup::launch_profile();
      t_launch.push_back(us(a0, a1) / N);
      t_finish.push_back(us(a1, a3) / N);
      t_wait.push_back(us(a2, a3) / N);
      t_tables.push_back((after.tables_us - before.tables_us) / N);
      t_capi.push_back((after.call_us - before.call_us) / N);
    }
    std::printf("{\"groups\": %zu, \"k\": %d, \"L\": %zu, \"launch_us_per_group\": %.4f, "
                "\"finish_us_per_group\": %.4f, \"wait_us_per_group\": %.4f, "
                "\"tables_us_per_group\": %.4f, \"capi_us_per_group\": %.4f}\n",
                N, k, L, med(t_launch), med(t_finish), med(t_wait), med(t_tables), med(t_capi));
    std::fflush(stdout);
  }
  qfec_destroy(ctx);
  return 0;
}
