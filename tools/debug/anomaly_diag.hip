// anomaly_diag.hip — what exactly is wrong in the groups the round-1 ragged
// build gets wrong ("a build-dependent wrong result")?
//
// Runs the failing round-1 instance ragged_xor_kernel<recover, nt, U = 4,
// 4 waves, ACC = 2 (2 x ds_xor_b64)> from commit 9ecab67 (the kernel source is
// taken from git history, not copied here) on the same 20,000 ragged groups
// as tools/debug/ragged_variants.hip, and for every wrong group explains the
// difference d = got ^ want (over the group's parity length) in terms of the
// kernel's work items: a received packet's 16-B window t lands at accumulator
// bytes [16t, 16t+16) and was handled by wave-iteration f/64, lane f%64,
// unroll slot (f/64) % U, where f = S + t is its flat window index.  A d equal
// to one window's contribution = that window's XOR was lost (or applied
// twice); anything else is printed raw.
//
// build:
//   git worktree add --detach /tmp/wt_9ecab67 9ecab67
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 \
//     -DQFEC_KERNELS='"/tmp/wt_9ecab67/libquic_amd/csrc/qfec_kernels.hip"' \
//     tools/debug/anomaly_diag.hip -o tools/debug/build/anomaly_diag
#include QFEC_KERNELS

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

static uint64_t sm64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
template <typename T>
static T* up(const std::vector<T>& v) {
  T* d;
  CK(hipMalloc(&d, v.size() * sizeof(T)));
  CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  const int REPS = argc > 1 ? atoi(argv[1]) : 2;
  const int U = 4;
  const uint64_t G = 20000, SL = 1452;
  std::vector<uint32_t> ptr{0};
  std::vector<uint16_t> len;
  std::vector<uint64_t> off;
  std::vector<uint8_t> miss(G);
  uint64_t bytes = 0;
  for (uint64_t g = 0; g < G; ++g) {
    const uint32_t k = 5 + (uint32_t)(sm64(0x1234 ^ g) % 11);
    for (uint32_t i = 0; i < k; ++i) {
      const uint32_t l = 64 + (uint32_t)(sm64(0x5678 ^ (g * 256 + i)) % 1287);
      len.push_back((uint16_t)l);
      off.push_back(bytes);
      bytes += l;
    }
    ptr.push_back((uint32_t)len.size());
    miss[g] = (uint8_t)(sm64(0x9abc ^ g) % k);
  }
  std::vector<uint8_t> data(bytes);
  for (uint64_t j = 0; j < bytes; ++j) data[j] = (uint8_t)sm64(j * 7919);
  std::vector<uint8_t> par(G * SL, 0), rec(G * SL, 0);
  std::vector<uint16_t> plen(G);
  for (uint64_t g = 0; g < G; ++g) {
    uint32_t mx = 0;
    for (uint32_t p = ptr[g]; p < ptr[g + 1]; ++p) {
      for (uint32_t j = 0; j < len[p]; ++j) par[g * SL + j] ^= data[off[p] + j];
      mx = std::max<uint32_t>(mx, len[p]);
    }
    plen[g] = (uint16_t)mx;
    for (uint32_t j = 0; j < mx; ++j) rec[g * SL + j] = par[g * SL + j];
    for (uint32_t p = ptr[g]; p < ptr[g + 1]; ++p) {
      if (p - ptr[g] == miss[g]) continue;
      for (uint32_t j = 0; j < len[p]; ++j) rec[g * SL + j] ^= data[off[p] + j];
    }
  }
  std::vector<uint64_t> poff(G);
  for (uint64_t g = 0; g < G; ++g) poff[g] = g * SL;
  qfec::RaggedArgs a{};
  a.bytes = up(data);
  a.pkt_off = up(off);
  a.pkt_len = up(len);
  a.grp_ptr = up(ptr);
  a.n_groups = G;
  CK(hipMalloc(&a.err, 4));
  CK(hipMemset(a.err, 0, 4));
  a.parity = up(par);
  a.parity_off = up(poff);
  a.parity_len = up(plen);
  a.missing = up(miss);
  uint8_t* d_out;
  CK(hipMalloc(&d_out, G * SL));
  a.out = d_out;
  a.out_off = a.parity_off;

  std::vector<uint8_t> h(G * SL);
  std::map<int, int> by_slot, by_lane_mod, by_kind, by_wave;
  std::map<int, int> by_it;
  int shown = 0, bad_groups = 0, explained = 0;
  for (int rep = 0; rep < REPS; ++rep) {
    CK(hipMemset(d_out, 0, G * SL));
    hipLaunchKernelGGL((qfec::ragged_xor_kernel<true, true, 4, 4, 2>), dim3((uint32_t)(G / 4)),
                       dim3(256), 0, 0, a);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d_out, G * SL, hipMemcpyDeviceToHost));
    for (uint64_t g = 0; g < G; ++g) {
      const uint8_t* got = &h[g * SL];
      const uint8_t* want = &rec[g * SL];
      if (!std::memcmp(got, want, plen[g])) continue;
      ++bad_groups;
      std::vector<uint8_t> d(plen[g]);
      for (uint32_t j = 0; j < plen[g]; ++j) d[j] = got[j] ^ want[j];
      // the received packets in kernel order, their flat window starts
      std::vector<uint32_t> rp, S;
      uint32_t s = 0;
      for (uint32_t i = 0; i < ptr[g + 1] - ptr[g]; ++i) {
        if (i == miss[g]) continue;
        rp.push_back(ptr[g] + i);
        S.push_back(s);
        s += (len[ptr[g] + i] + 15u) / 16u;
      }
      const uint32_t W = s;
      // every window's contribution (16 B at 16t, the last one zero-padded)
      int hits = 0;
      std::vector<std::pair<uint32_t, uint32_t>> which;  // (packet r, window t)
      for (uint32_t r = 0; r < rp.size(); ++r) {
        const uint32_t l = len[rp[r]];
        for (uint32_t t = 0; 16u * t < l; ++t) {
          bool eq = true;
          for (uint32_t j = 0; j < plen[g] && eq; ++j) {
            const bool in = j >= 16u * t && j < 16u * t + 16u && j < l;
            const uint8_t c = in ? data[off[rp[r]] + j] : 0;
            eq = d[j] == c;
          }
          if (eq) {
            ++hits;
            which.push_back({r, t});
          }
        }
      }
      uint32_t first = plen[g], last = 0;
      for (uint32_t j = 0; j < plen[g]; ++j)
        if (d[j]) {
          first = std::min(first, j);
          last = j;
        }
      if (hits == 1) {
        ++explained;
        const uint32_t r = which[0].first, t = which[0].second;
        const uint32_t f = S[r] + t, it = f / 64u, lane = f % 64u;
        by_slot[it % U]++;
        by_lane_mod[lane]++;
        by_it[it]++;
        by_kind[t == 0 ? 0 : (16u * t + 16u > len[rp[r]] ? 2 : 1)]++;
        by_wave[(int)(g % 4)]++;
        if (shown < 25) {
          ++shown;
          std::printf("g %llu k %u W %u: window (r %u, t %u, len %u) f %u it %u lane %u slot %u "
                      "nit %u wave %llu\n",
                      (unsigned long long)g, (unsigned)(ptr[g + 1] - ptr[g]), W, r, t,
                      len[rp[r]], f, it, lane, it % U, (W + 63) / 64,
                      (unsigned long long)(g % 4));
        }
      } else if (shown < 40) {
        ++shown;
        int nz = 0;
        for (uint8_t c : d) nz += c != 0;
        std::printf("g %llu: unexplained (%d single-window matches), %d nonzero bytes in "
                    "[%u, %u], plen %u W %u\n",
                    (unsigned long long)g, hits, nz, first, last, plen[g], W);
        // Hypothesis: the low dword of one window's first ds_xor_b64 was
        // replaced by the value the next instruction writes into that data
        // register (the high half's LDS address = base + 16t + 8).  For each
        // window t whose low dword differs, find packets r with
        // delta ^ data_dw(r, t) == C + 16t for one C.
        std::map<uint32_t, int> cands;
        int ndw = 0;
        for (uint32_t t = 0; 16u * t + 4u <= plen[g]; ++t) {
          uint32_t dd;
          std::memcpy(&dd, &d[16u * t], 4);
          if (!dd) continue;
          ++ndw;
          for (uint32_t r = 0; r < rp.size(); ++r) {
            const uint32_t l = len[rp[r]];
            if (16u * t >= l) continue;
            uint8_t b[4];
            for (int j = 0; j < 4; ++j)
              b[j] = 16u * t + j < l ? data[off[rp[r]] + 16u * t + j] : 0;
            uint32_t dw;
            std::memcpy(&dw, b, 4);
            cands[(dd ^ dw) - 16u * t]++;
          }
        }
        uint32_t bestC = 0;
        int best = 0;
        for (auto& kv : cands)
          if (kv.second > best) best = kv.second, bestC = kv.first;
        std::printf("   %d windows with a wrong low dword; delta ^ data - 16t = 0x%x for %d of them\n",
                    ndw, bestC, best);
        if (shown <= 6) {  // machine-readable dump: window contributions, parity, got, want
          for (uint32_t t = 0; 16u * t < plen[g]; ++t) {
            std::printf("W g %llu t %u got ", (unsigned long long)g, t);
            for (uint32_t j = 16u * t; j < 16u * t + 16u; ++j)
              std::printf("%02x", j < plen[g] ? got[j] : 0);
            std::printf(" want ");
            for (uint32_t j = 16u * t; j < 16u * t + 16u; ++j)
              std::printf("%02x", j < plen[g] ? want[j] : 0);
            std::printf(" par ");
            for (uint32_t j = 16u * t; j < 16u * t + 16u; ++j)
              std::printf("%02x", j < plen[g] ? par[g * SL + j] : 0);
            for (uint32_t r = 0; r < rp.size(); ++r) {
              const uint32_t l = len[rp[r]];
              if (16u * t >= l) continue;
              std::printf(" c%u:%u:", r, S[r] + t);
              for (uint32_t j = 16u * t; j < 16u * t + 16u; ++j)
                std::printf("%02x", j < l ? data[off[rp[r]] + j] : 0);
            }
            std::printf("\n");
          }
        }
        if (shown <= 2) {  // full dump of the first two
          for (uint32_t t = 0; 16u * t < plen[g]; ++t) {
            bool any = false;
            for (uint32_t j = 16u * t; j < std::min<uint32_t>(16u * t + 16u, plen[g]); ++j)
              any |= d[j] != 0;
            if (!any) continue;
            std::printf("   t %3u delta ", t);
            for (uint32_t j = 16u * t; j < 16u * t + 16u; ++j)
              std::printf("%02x", j < plen[g] ? d[j] : 0);
            for (uint32_t r = 0; r < rp.size(); ++r) {
              const uint32_t l = len[rp[r]];
              if (16u * t >= l) continue;
              std::printf(" | r%u(f%u) ", r, S[r] + t);
              for (uint32_t j = 16u * t; j < 16u * t + 8u; ++j)
                std::printf("%02x", j < l ? data[off[rp[r]] + j] : 0);
            }
            std::printf("\n");
          }
        }
        // 8-B halves: which accumulator words differ
        std::printf("   differing 8-B words:");
        for (uint32_t w = 0; 8u * w < plen[g]; ++w) {
          bool any = false;
          for (uint32_t j = 8u * w; j < std::min<uint32_t>(8u * w + 8u, plen[g]); ++j)
            any |= d[j] != 0;
          if (any) std::printf(" %u", w);
        }
        std::printf("\n");
      }
    }
  }
  std::printf("\n%d bad groups over %d reps, %d explained as exactly one window's XOR\n",
              bad_groups, REPS, explained);
  std::printf("by unroll slot:");
  for (auto& kv : by_slot) std::printf(" u%d=%d", kv.first, kv.second);
  std::printf("\nby window kind (0 first, 1 middle, 2 last/partial):");
  for (auto& kv : by_kind) std::printf(" %d=%d", kv.first, kv.second);
  std::printf("\nby wave in block:");
  for (auto& kv : by_wave) std::printf(" w%d=%d", kv.first, kv.second);
  std::printf("\nby wave-iteration:");
  for (auto& kv : by_it) std::printf(" it%d=%d", kv.first, kv.second);
  std::printf("\nby lane:");
  for (auto& kv : by_lane_mod) std::printf(" %d:%d", kv.first, kv.second);
  std::printf("\n");
  return 0;
}
