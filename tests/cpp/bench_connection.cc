// bench_connection.cc — connection-layer FEC latency and throughput
// (bench.py's "connection" leg).
//
// What a QUIC server thread does with the GPU path: N connections each close
// one FEC group of 10 data packets x 1350 B (QuicFecSender -> one shared
// QuicFecEncodeBatch), or each have one group with exactly one lost packet and
// the FEC packet received (QuicFecReceiver -> one shared QuicFecReviveBatch).
// Timed: ONE Flush of the batch — CSR build, one ragged launch reading the
// payloads in place from the groups' pinned payload arena (QFEC_PTR_MAPPED)
// and writing the accumulators back into it (up to 256 groups the index
// tables are read in place as well and completion is a host-mapped flag;
// above that they are staged to the device), the redundancy /
// revived-payload views — for N = 1, 64, 4096, 65536 groups.
// Beside it the CPU FEC path the reference ran on the connection thread:
// every payload XORed into the group accumulator (the oracle's
// qo_group_encode / qo_group_recover, word-wise XorBuffers), one core.
// Outputs are checked against the oracle (bench-side checker only).
//
// Prints one JSON object on stdout.  Needs a GPU.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "qfec_oracle.h"
#include "quic_fec_connection.h"

using namespace net;
using Clock = std::chrono::steady_clock;

static double us_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int k = 10;
  const uint32_t L = 1350;
  std::vector<size_t> sizes = {1, 64, 4096, 65536};
  if (argc > 1) {
    sizes.clear();
    for (int i = 1; i < argc; ++i) sizes.push_back(std::strtoull(argv[i], nullptr, 10));
  }
  qfec_ctx* ctx = qfec_create(0);
  if (!ctx) {
    std::fprintf(stderr, "qfec_create: %s\n", qfec_last_error(nullptr));
    return 2;
  }
  std::printf("{\"k\": %d, \"L\": %u, \"legs\": [", k, L);
  bool first = true, all_ok = true;
  for (size_t N : sizes) {
    // payloads of connection g, packet i: counter-based bytes
    std::vector<std::string> pays(N * k, std::string(L, '\0'));
    for (size_t g = 0; g < N; ++g)
      for (int i = 0; i < k; ++i)
        qo_synth_row(0x51554943, g, i, L, reinterpret_cast<uint8_t*>(&pays[g * k + i][0]));
    // the oracle's redundancy per group (checker + the received FEC packets)
    std::vector<std::string> red(N, std::string(L, '\0'));
    for (size_t g = 0; g < N; ++g) {
      const uint8_t* p[16];
      uint32_t l[16];
      for (int i = 0; i < k; ++i) {
        p[i] = reinterpret_cast<const uint8_t*>(pays[g * k + i].data());
        l[i] = L;
      }
      qo_group_encode(p, l, k, reinterpret_cast<uint8_t*>(&red[g][0]));
    }
    const int reps = N >= 65536 ? 5 : N >= 4096 ? 20 : 200;
    std::vector<double> t_enc, t_rev, t_build;  // t_build: the batch's assembly between flushes
    bool ok = true;
    for (int r = 0; r < reps + 1; ++r) {  // rep 0 warms the context's staging
      const auto b0 = Clock::now();
      // the loop turn starts: the small-batch service's worker runs by the
      // flush (QuicFecBatcher does this on its first group)
      qfec_service_warm(ctx);
      QuicFecEncodeBatch batch;
      for (size_t g = 0; g < N; ++g) {
        QuicFecSender s(k);
        for (int i = 0; i < k; ++i) s.OnDataPacket(1 + i, pays[g * k + i], false, nullptr);
        s.CloseFecGroup(1 + k, &batch);
      }
      if (r > 0) t_build.push_back(us_since(b0));
      auto t0 = Clock::now();
      const int rc = batch.Flush(ctx);
      const double us = us_since(t0);
      if (rc != QFEC_OK) {
        std::fprintf(stderr, "encode flush: %s\n", qfec_last_error(ctx));
        return 1;
      }
      if (r > 0) t_enc.push_back(us);
      if (r == 1) {
        for (size_t g = 0; g < N; ++g) {
          const StringPiece rd = batch.entries()[g].redundancy;
          ok &= rd.size() == L && std::memcmp(rd.data(), red[g].data(), L) == 0;
        }
      }
    }
    for (int r = 0; r < reps + 1; ++r) {
      qfec_service_warm(ctx);  // (the loop turn starts, as above)
      QuicFecReviveBatch rb;
      for (size_t g = 0; g < N; ++g) {
        QuicFecReceiver rx;
        const int lost = static_cast<int>(g % k);
        for (int i = 0; i < k; ++i) {
          if (i == lost) continue;
          QuicPacketHeader h;
          h.packet_number = 1 + i;
          h.is_in_fec_group = IN_FEC_GROUP;
          h.fec_group = 1;
          rx.OnPacket(ENCRYPTION_FORWARD_SECURE, h, pays[g * k + i]);
        }
        QuicPacketHeader fh;
        fh.packet_number = 1 + k;
        fh.is_in_fec_group = IN_FEC_GROUP;
        fh.fec_group = 1;
        fh.fec_flag = true;
        rx.OnPacket(ENCRYPTION_FORWARD_SECURE, fh, red[g]);
        rx.CollectRevivable(&rb, reinterpret_cast<void*>(g));
      }
      std::vector<QuicFecReviveBatch::Revived> out;
      out.reserve(N);
      auto t0 = Clock::now();
      const int rc = rb.Flush(ctx, &out);
      const double us = us_since(t0);
      if (rc != QFEC_OK) {
        std::fprintf(stderr, "revive flush: %s\n", qfec_last_error(ctx));
        return 1;
      }
      if (r > 0) t_rev.push_back(us);
      if (r == 1) {
        ok &= out.size() == N;
        for (const auto& rv : out) {
          const size_t g = reinterpret_cast<size_t>(rv.tag);
          const int lost = static_cast<int>(g % k);
          ok &= rv.header.packet_number == static_cast<QuicPacketNumber>(1 + lost) &&
                rv.payload.size() == L &&
                std::memcmp(rv.payload.data(), pays[g * k + lost].data(), L) == 0;
        }
      }
    }
    // the CPU FEC path on one core (the connection thread): accumulate every
    // payload into the group's parity / revive from the received ones
    std::vector<uint8_t> acc(QO_MAX_PACKET_SIZE);
    std::vector<double> c_enc, c_rev;
    for (int r = 0; r < reps; ++r) {
      auto t0 = Clock::now();
      for (size_t g = 0; g < N; ++g) {
        const uint8_t* p[16];
        uint32_t l[16];
        for (int i = 0; i < k; ++i) {
          p[i] = reinterpret_cast<const uint8_t*>(pays[g * k + i].data());
          l[i] = L;
        }
        qo_group_encode(p, l, k, acc.data());
      }
      c_enc.push_back(us_since(t0));
      t0 = Clock::now();
      for (size_t g = 0; g < N; ++g) {
        const uint8_t* p[16];
        uint32_t l[16];
        for (int i = 0; i < k; ++i) {
          p[i] = reinterpret_cast<const uint8_t*>(pays[g * k + i].data());
          l[i] = L;
        }
        qo_group_recover(p, l, k, reinterpret_cast<const uint8_t*>(red[g].data()), L,
                         static_cast<uint32_t>(g % k), acc.data());
      }
      c_rev.push_back(us_since(t0));
    }
    const double me = median(t_enc), mr = median(t_rev);
    const double ce = median(c_enc), cr = median(c_rev);
    all_ok &= ok;
    std::printf("%s{\"groups\": %zu, \"reps\": %d, \"encode_flush_us\": %.1f, "
                "\"encode_Mgroups_per_s\": %.4f, \"revive_flush_us\": %.1f, "
                "\"revive_Mgroups_per_s\": %.4f, \"cpu_1core_encode_us\": %.1f, "
                "\"cpu_1core_revive_us\": %.1f, \"encode_build_us\": %.1f, \"verified\": %s}",
                first ? "" : ", ", N, reps, me, N / me, mr, N / mr, ce, cr, median(t_build),
                ok ? "true" : "false");
    first = false;
  }
  std::printf("], \"verified\": %s}\n", all_ok ? "true" : "false");
  qfec_destroy(ctx);
  return all_ok ? 0 : 1;
}
