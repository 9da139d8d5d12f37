// test_quic_fec_group.cc — tests of the C++ QuicFecGroup host mirror
// (libquic_amd/csrc/quic_fec_group.h), GPU-backed, checked against the C
// oracle (oracle/qfec_oracle.c — test infrastructure).
//
// Cases follow the historical QuicFecGroup behaviour (SURVEY.md §8(a) a1/a2,
// Appendix A): revive every lost position with the FEC packet arriving before,
// between and after the data; duplicates refused; out-of-range packets refused;
// oversize payload refused ("Illegal payload size", kMaxPacketSize
// quic_protocol.h:66); revived payload zero-padded (PADDING_FRAME = 0,
// quic_framer.cc:1224-1231); effective encryption level is the minimum seen;
// many groups in one ComputeAll launch.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "qfec_oracle.h"
#include "quic_fec_group.h"
#include "quic_fec_wire.h"

using namespace net;

static int g_fail = 0, g_checks = 0;
#define EXPECT(cond)                                                         \
  do {                                                                       \
    ++g_checks;                                                              \
    if (!(cond)) {                                                           \
      ++g_fail;                                                              \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);   \
    }                                                                        \
  } while (0)

// Payloads of unequal length (so parity_len > the shortest).
static std::vector<std::string> MakePayloads(int n, uint64_t seed) {
  std::vector<std::string> v;
  for (int i = 0; i < n; ++i) {
    uint32_t len = qo_ragged_len(seed, 1, i, 1, 1350);
    std::string s(len, '\0');
    qo_synth_row(seed, 1, i, len, reinterpret_cast<uint8_t*>(&s[0]));
    v.push_back(s);
  }
  return v;
}

static std::string OracleParity(const std::vector<std::string>& p) {
  std::vector<const uint8_t*> ptr;
  std::vector<uint32_t> len;
  for (auto& s : p) {
    ptr.push_back(reinterpret_cast<const uint8_t*>(s.data()));
    len.push_back(s.size());
  }
  std::string out(kMaxPacketSize, '\0');
  int n = qo_group_encode(ptr.data(), len.data(), p.size(), reinterpret_cast<uint8_t*>(&out[0]));
  out.resize(n > 0 ? n : 0);
  return out;
}

static QuicPacketHeader Header(QuicPacketNumber n, QuicFecGroupNumber grp, bool fec) {
  QuicPacketHeader h;
  h.packet_number = n;
  h.fec_flag = fec;
  h.is_in_fec_group = IN_FEC_GROUP;
  h.fec_group = grp;
  return h;
}

// FEC arrives at position `fec_pos` among the k-1 received data packets.
static void ReviveCase(qfec_ctx* ctx, int k, int lost, int fec_pos) {
  const QuicFecGroupNumber first = 100;
  auto pays = MakePayloads(k, 0x51554944);
  std::string redundancy = OracleParity(pays);
  QuicFecGroup group(first, ctx);
  int seen = 0;
  bool fec_done = false;
  for (int i = 0; i < k; ++i) {
    if (!fec_done && seen == fec_pos) {
      EXPECT(group.UpdateFec(ENCRYPTION_FORWARD_SECURE, Header(first + k, first, true),
                             redundancy));
      fec_done = true;
    }
    if (i == lost) continue;
    EXPECT(!group.CanRevive() || fec_done);
    EXPECT(group.Update(ENCRYPTION_FORWARD_SECURE, Header(first + i, first, false), pays[i]));
    ++seen;
  }
  if (!fec_done)
    EXPECT(group.UpdateFec(ENCRYPTION_FORWARD_SECURE, Header(first + k, first, true), redundancy));
  EXPECT(group.CanRevive());
  EXPECT(!group.IsFinished());
  char buf[kMaxPacketSize];
  QuicPacketHeader out;
  size_t n = group.Revive(&out, buf, sizeof(buf));
  EXPECT(n == redundancy.size());
  EXPECT(out.packet_number == first + lost);
  EXPECT(!out.fec_flag);
  EXPECT(std::memcmp(buf, pays[lost].data(), pays[lost].size()) == 0);
  bool zero_tail = true;
  for (size_t j = pays[lost].size(); j < n; ++j) zero_tail &= buf[j] == 0;
  EXPECT(zero_tail);
  EXPECT(group.IsFinished());
  EXPECT(!group.CanRevive());
}

int main() {
  qfec_ctx* ctx = qfec_create(0);
  if (!ctx) {
    std::fprintf(stderr, "qfec_create failed: %s\n", qfec_last_error(nullptr));
    return 2;
  }
  // every lost position x every FEC arrival position
  for (int k : {1, 2, 5, 10}) {
    for (int lost = 0; lost < k; ++lost)
      for (int fec_pos = 0; fec_pos < k; ++fec_pos) ReviveCase(ctx, k, lost, fec_pos);
  }
  // send side: PayloadParity == oracle parity; duplicate refused
  {
    auto pays = MakePayloads(7, 0x51554943);
    QuicFecGroup group(1, ctx);
    for (int i = 0; i < 7; ++i)
      EXPECT(group.Update(ENCRYPTION_INITIAL, Header(1 + i, 1, false), pays[i]));
    EXPECT(!group.Update(ENCRYPTION_INITIAL, Header(3, 1, false), pays[2]));  // duplicate
    StringPiece par = group.PayloadParity();
    std::string want = OracleParity(pays);
    EXPECT(par.size() == want.size());
    EXPECT(std::memcmp(par.data(), want.data(), want.size()) == 0);
    EXPECT(group.NumReceivedPackets() == 7);
    EXPECT(group.EffectiveEncryptionLevel() == ENCRYPTION_INITIAL);
    EXPECT(!group.CanRevive());  // no redundancy yet
  }
  // zero-copy capture (UpdateInPlace): payloads serialized into arena packet
  // buffers after a header, adopted by the group -> the same parity; a
  // refused packet (duplicate) leaves its buffer with the caller; a buffer
  // range outside the buffer is refused
  {
    auto pays = MakePayloads(9, 0x51554951);
    QuicFecGroup group(1, ctx);
    const QuicFecGroup::LaunchProfile p0 = QuicFecGroup::launch_profile();
    for (int i = 0; i < 9; ++i) {
      const size_t hdr = 9 + i % 4;  // the packet header before the payload
      QuicFecGroup::PacketBuffer b = QuicFecGroup::AllocPacketBuffer(hdr + pays[i].size());
      EXPECT(!b.empty());
      std::memset(b.data(), 0xEE, hdr);
      std::memcpy(b.data() + hdr, pays[i].data(), pays[i].size());
      EXPECT(group.UpdateInPlace(ENCRYPTION_FORWARD_SECURE, Header(1 + i, 1, false), &b, hdr,
                                 pays[i].size()));
      EXPECT(b.empty());  // adopted
    }
    EXPECT(QuicFecGroup::launch_profile().payloads_adopted - p0.payloads_adopted == 9);
    EXPECT(QuicFecGroup::launch_profile().payloads_copied == p0.payloads_copied);
    QuicFecGroup::PacketBuffer dup = QuicFecGroup::AllocPacketBuffer(64);
    EXPECT(!group.UpdateInPlace(ENCRYPTION_FORWARD_SECURE, Header(3, 1, false), &dup, 0, 64));
    EXPECT(!dup.empty());  // not adopted: the caller still owns it
    EXPECT(!group.UpdateInPlace(ENCRYPTION_FORWARD_SECURE, Header(20, 1, false), &dup, 60, 5));
    StringPiece par = group.PayloadParity();
    std::string want = OracleParity(pays);
    EXPECT(par.size() == want.size() && std::memcmp(par.data(), want.data(), want.size()) == 0);
  }
  // oversize payload refused; 1452 accepted
  {
    QuicFecGroup group(1, ctx);
    std::string big(kMaxPacketSize + 1, 'x');
    EXPECT(!group.Update(ENCRYPTION_NONE, Header(1, 1, false), big));
    std::string max(kMaxPacketSize, 'y');
    EXPECT(group.Update(ENCRYPTION_NONE, Header(1, 1, false), max));
    EXPECT(group.PayloadParity().size() == kMaxPacketSize);
  }
  // FEC claims a range that excludes a received packet; second FEC refused
  {
    QuicFecGroup group(10, ctx);
    EXPECT(group.Update(ENCRYPTION_NONE, Header(15, 10, false), std::string("abc")));
    EXPECT(!group.UpdateFec(ENCRYPTION_NONE, Header(14, 10, true), std::string("abc")));
    EXPECT(group.UpdateFec(ENCRYPTION_NONE, Header(16, 10, true), std::string("abc")));
    EXPECT(!group.UpdateFec(ENCRYPTION_NONE, Header(16, 10, true), std::string("abc")));
    // after the range is known, packets outside it are refused
    EXPECT(!group.Update(ENCRYPTION_NONE, Header(9, 10, false), std::string("zz")));
    EXPECT(!group.Update(ENCRYPTION_NONE, Header(16, 10, false), std::string("zz")));
  }
  // effective encryption level = minimum; IsWaitingForPacketBefore
  {
    QuicFecGroup group(50, ctx);
    EXPECT(group.EffectiveEncryptionLevel() == NUM_ENCRYPTION_LEVELS);
    EXPECT(group.Update(ENCRYPTION_FORWARD_SECURE, Header(51, 50, false), std::string("q")));
    EXPECT(group.Update(ENCRYPTION_INITIAL, Header(52, 50, false), std::string("r")));
    EXPECT(group.EffectiveEncryptionLevel() == ENCRYPTION_INITIAL);
    EXPECT(group.IsWaitingForPacketBefore(60));
    EXPECT(!group.IsWaitingForPacketBefore(50));
    EXPECT(group.UpdateFec(ENCRYPTION_NONE, Header(54, 50, true), std::string("s")));
    EXPECT(group.EffectiveEncryptionLevel() == ENCRYPTION_NONE);
    EXPECT(!group.IsWaitingForPacketBefore(50));
    EXPECT(group.IsWaitingForPacketBefore(51));
  }
  // revive buffer too small -> 0
  {
    auto pays = MakePayloads(3, 0x51554945);
    QuicFecGroup group(1, ctx);
    EXPECT(group.Update(ENCRYPTION_NONE, Header(1, 1, false), pays[0]));
    EXPECT(group.Update(ENCRYPTION_NONE, Header(2, 1, false), pays[1]));
    EXPECT(group.UpdateFec(ENCRYPTION_NONE, Header(4, 1, true), OracleParity(pays)));
    char small[8];
    QuicPacketHeader h;
    EXPECT(group.Revive(&h, small, sizeof(small)) == 0);
  }
  // many groups, one launch
  {
    const int G = 300;
    std::vector<std::vector<std::string>> all;
    std::vector<QuicFecGroup*> groups;
    for (int g = 0; g < G; ++g) {
      int k = 1 + g % 17;
      auto pays = MakePayloads(k, 0x1000 + g);
      auto* grp = new QuicFecGroup(1000 * g + 1, ctx);
      for (int i = 0; i < k; ++i)
        grp->Update(ENCRYPTION_NONE, Header(1000 * g + 1 + i, 1000 * g + 1, false), pays[i]);
      all.push_back(pays);
      groups.push_back(grp);
    }
    EXPECT(QuicFecGroup::ComputeAll(ctx, groups) == QFEC_OK);
    for (int g = 0; g < G; ++g) {
      std::string want = OracleParity(all[g]);
      StringPiece got = groups[g]->PayloadParity();
      EXPECT(got.size() == want.size() && std::memcmp(got.data(), want.data(), want.size()) == 0);
      delete groups[g];
    }
  }
  // payload arena across threads: groups filled on worker threads outlive
  // them (a thread's slabs go to the process-wide pool when it exits), are
  // computed and destroyed here; the second round's threads take the drained
  // slabs back from the pool
  for (int round = 0; round < 3; ++round) {
    const int T = 6, k = 5;
    std::vector<std::unique_ptr<QuicFecGroup>> made(T);
    std::vector<std::vector<std::string>> pays(T);
    std::vector<std::thread> ts;
    for (int t = 0; t < T; ++t)
      ts.emplace_back([&, t] {
        pays[t] = MakePayloads(k, 0x7000 + 16 * round + t);
        made[t].reset(new QuicFecGroup(1));  // the thread's default context
        for (int i = 0; i < k; ++i)
          made[t]->Update(ENCRYPTION_NONE, Header(1 + i, 1, false), pays[t][i]);
      });
    for (auto& th : ts) th.join();
    std::vector<QuicFecGroup*> gs;
    for (auto& g : made) gs.push_back(g.get());
    EXPECT(QuicFecGroup::ComputeAll(ctx, gs) == QFEC_OK);
    for (int t = 0; t < T; ++t) {
      const std::string want = OracleParity(pays[t]);
      const StringPiece got = made[t]->PayloadParity();
      EXPECT(got.size() == want.size() && std::memcmp(got.data(), want.data(), want.size()) == 0);
    }
  }
  // wire format: FEC packet header round trip (v<=31 private flags + offset)
  {
    uint8_t buf[8];
    FecHeaderFields f;
    f.entropy_flag = true;
    f.fec_flag = true;
    f.in_fec_group = true;
    f.fec_group_offset = 9;
    size_t n = WriteFecPrivateHeader(f, buf, sizeof(buf));
    EXPECT(n == 2);
    EXPECT(buf[0] == (PACKET_PRIVATE_FLAGS_ENTROPY | PACKET_PRIVATE_FLAGS_FEC_GROUP |
                      PACKET_PRIVATE_FLAGS_FEC));
    FecHeaderFields back;
    std::string err;
    EXPECT(ParseFecPrivateHeader(buf, n, 31, 20, &back, &err) == n);
    EXPECT(back.fec_flag && back.in_fec_group && back.entropy_flag && back.fec_group_offset == 9);
    EXPECT(ParseFecPrivateHeader(buf, n, 32, 20, &back, &err) == 0);  // v32: illegal flags
    EXPECT(ParseFecPrivateHeader(buf, n, 31, 9, &back, &err) == 0);   // offset >= packet number
  }
  qfec_destroy(ctx);
  std::printf("%d checks, %d failures\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
