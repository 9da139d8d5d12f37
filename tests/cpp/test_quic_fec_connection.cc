// test_quic_fec_connection.cc — connection-level FEC (quic_fec_connection.h):
// send-side groups of the historical QuicPacketCreator, the receive-side group
// map of the historical QuicConnection, and cross-connection batches (one
// ragged launch per flush).
//
//   --cpu   bookkeeping only (no device needed: nothing is flushed)
//   (none)  also a lossy multi-connection simulation on the GPU: every packet
//           goes through the v<=31 private header (quic_fec_wire.h), random
//           loss and reordering; every group with exactly one lost data packet
//           and a received FEC packet must be revived bit-exactly (payload
//           zero padded to the redundancy length), no other group revived.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "qfec_oracle.h"
#include "quic_fec_connection.h"
#include "quic_fec_wire.h"

using namespace net;

static int g_fail = 0, g_checks = 0;
#define EXPECT(cond)                                                       \
  do {                                                                     \
    ++g_checks;                                                            \
    if (!(cond)) {                                                         \
      ++g_fail;                                                            \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                      \
  } while (0)

static std::string Payload(uint64_t conn, uint64_t pn, uint32_t len) {
  std::string s(len, '\0');
  qo_synth_row(0x51554943, conn, static_cast<uint32_t>(pn & 0xFF) ^ static_cast<uint32_t>(pn >> 8),
               len, reinterpret_cast<uint8_t*>(&s[0]));
  return s;
}

static QuicPacketHeader DataHeader(QuicPacketNumber pn, QuicFecGroupNumber grp) {
  QuicPacketHeader h;
  h.packet_number = pn;
  h.is_in_fec_group = IN_FEC_GROUP;
  h.fec_group = grp;
  return h;
}

// ---------------------------------------------------------------------------
// CPU: bookkeeping
// ---------------------------------------------------------------------------
static void SenderBookkeeping() {
  QuicFecSender s(3);
  EXPECT(!s.IsFecGroupOpen());
  EXPECT(!s.ShouldSendFec(true));
  FecHeaderFields f;
  EXPECT(s.OnDataPacket(10, Payload(1, 10, 100), false, &f));
  EXPECT(f.in_fec_group && f.fec_group_offset == 0);
  EXPECT(s.IsFecGroupOpen() && s.NumPacketsInGroup() == 1);
  EXPECT(!s.ShouldSendFec(false) && s.ShouldSendFec(true));
  EXPECT(s.OnDataPacket(12, Payload(1, 12, 50), true, &f));  // numbers may skip
  EXPECT(f.in_fec_group && f.fec_group_offset == 2 && f.entropy_flag);
  EXPECT(!s.OnDataPacket(12, Payload(1, 12, 50), false, &f));  // not increasing
  EXPECT(!s.OnDataPacket(13, std::string(kMaxPacketSize + 1, 'x'), false, &f));  // oversize
  EXPECT(s.OnDataPacket(13, Payload(1, 13, 1350), false, &f));
  EXPECT(s.ShouldSendFec(false));
  QuicFecEncodeBatch batch;
  EXPECT(!s.CloseFecGroup(13, &batch));  // FEC packet must follow the data
  EXPECT(s.CloseFecGroup(14, &batch, &s));
  EXPECT(!s.IsFecGroupOpen() && batch.size() == 1);
  EXPECT(batch.entries()[0].fec_group == 10 && batch.entries()[0].fec_packet_number == 14);
  EXPECT(batch.entries()[0].group->NumReceivedPackets() == 3);
  // protection off: packets are not grouped
  s.StopFecProtection();
  EXPECT(s.OnDataPacket(15, Payload(1, 15, 10), false, &f));
  EXPECT(!f.in_fec_group && !s.IsFecGroupOpen());
  // group size clamps to the uint8 offset range
  s.set_max_packets_per_fec_group(1000);
  EXPECT(s.max_packets_per_fec_group() == 255);
  s.set_max_packets_per_fec_group(0);
  EXPECT(s.max_packets_per_fec_group() == 1);
  // a group cannot span more than 255 packet numbers
  QuicFecSender t(255);
  EXPECT(t.OnDataPacket(1, Payload(2, 1, 10), false, &f));
  // offset 255 is the FEC packet's: a data packet there would leave the group
  // unclosable, so it is refused and the group stays usable
  EXPECT(!t.OnDataPacket(256, Payload(2, 256, 10), false, &f));
  EXPECT(t.OnDataPacket(255, Payload(2, 255, 10), false, &f) && f.fec_group_offset == 254);
  EXPECT(!t.CloseFecGroup(257, &batch));  // offset 256: beyond uint8
  EXPECT(t.CloseFecGroup(256, &batch) && !t.IsFecGroupOpen());
}

static void ReceiverBookkeeping() {
  QuicFecReceiver r;  // kMaxFecGroups = 2
  QuicPacketHeader h = DataHeader(5, 5);
  EXPECT(r.OnPacket(ENCRYPTION_FORWARD_SECURE, h, Payload(1, 5, 20)));
  EXPECT(r.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(9, 9), Payload(1, 9, 20)));
  EXPECT(r.NumGroups() == 2);
  // a third group evicts the lowest; the evicted group is not recreated
  EXPECT(r.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(13, 13), Payload(1, 13, 20)));
  EXPECT(r.NumGroups() == 2 && r.GetGroup(5) == nullptr && r.GetGroup(9) && r.GetGroup(13));
  EXPECT(!r.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(6, 5), Payload(1, 6, 20)));
  // a group older than every kept group is not created when the map is full
  EXPECT(!r.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(8, 7), Payload(1, 8, 20)));
  // duplicates refused; not-in-group refused
  EXPECT(!r.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(9, 9), Payload(1, 9, 20)));
  QuicPacketHeader plain;
  plain.packet_number = 30;
  EXPECT(!r.OnPacket(ENCRYPTION_FORWARD_SECURE, plain, Payload(1, 30, 20)));
  // group 9 = packets 9..11, FEC = 12: 10 received, 11 lost -> revivable
  EXPECT(r.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(10, 9), Payload(1, 10, 20)));
  QuicPacketHeader fec = DataHeader(12, 9);
  fec.fec_flag = true;
  EXPECT(r.OnPacket(ENCRYPTION_FORWARD_SECURE, fec, std::string(20, '\0')));
  EXPECT(r.GetGroup(9)->CanRevive());
  QuicFecReviveBatch rb;
  EXPECT(r.CollectRevivable(&rb, &r) == 1 && rb.size() == 1 && r.GetGroup(9) == nullptr);
  // a late packet of a collected group does not reopen it
  EXPECT(!r.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(11, 9), Payload(1, 11, 20)));
  // a finished group (nothing lost) leaves the map
  QuicFecReceiver r2(4);
  EXPECT(r2.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(1, 1), Payload(1, 1, 20)));
  EXPECT(r2.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(2, 1), Payload(1, 2, 20)));
  QuicPacketHeader fec2 = DataHeader(3, 1);
  fec2.fec_flag = true;
  EXPECT(r2.OnPacket(ENCRYPTION_FORWARD_SECURE, fec2, std::string(20, '\0')));
  EXPECT(r2.NumGroups() == 0);
  // CloseFecGroupsBefore drops groups waiting for older packets
  EXPECT(r2.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(20, 20), Payload(1, 20, 20)));
  EXPECT(r2.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(31, 30), Payload(1, 31, 20)));
  r2.CloseFecGroupsBefore(25);
  EXPECT(r2.GetGroup(20) == nullptr && r2.GetGroup(30) != nullptr);
  r2.CloseFecGroupsBefore(31);
  EXPECT(r2.GetGroup(30) == nullptr && r2.NumGroups() == 0);
}

// Zero-copy receive (OnPacketInPlace): the packet is "decrypted" into a
// payload-arena buffer after a header; the group adopts the buffer (left
// empty), a refused packet leaves it with the caller, and a group dropped
// while its packet is still being parsed (a STOP_WAITING frame in that very
// packet: CloseFecGroupsBefore) keeps the adopted bytes readable until the
// next packet (under AddressSanitizer, released arena bytes are poisoned).
static void ReceiverInPlace() {
  QuicFecReceiver r(4);
  auto decrypt = [](const std::string& payload, size_t hdr) {
    QuicFecGroup::PacketBuffer b = QuicFecGroup::AllocPacketBuffer(kMaxPacketSize);
    std::memset(b.data(), 0x33, hdr);
    std::memcpy(b.data() + hdr, payload.data(), payload.size());
    return b;
  };
  const std::string p1 = Payload(3, 41, 700), p2 = Payload(3, 42, 900);
  QuicFecGroup::PacketBuffer b1 = decrypt(p1, 11);
  EXPECT(r.OnPacketInPlace(ENCRYPTION_FORWARD_SECURE, DataHeader(41, 41), &b1, 11, p1.size()));
  EXPECT(b1.empty());
  QuicFecGroup::PacketBuffer dup = decrypt(p1, 11);
  EXPECT(!r.OnPacketInPlace(ENCRYPTION_FORWARD_SECURE, DataHeader(41, 41), &dup, 11, p1.size()));
  EXPECT(!dup.empty());
  EXPECT(!r.OnPacketInPlace(ENCRYPTION_FORWARD_SECURE, DataHeader(42, 41), &dup, 1400, 100));
  QuicFecGroup::PacketBuffer b2 = decrypt(p2, 9);
  const char* view = b2.data() + 9;  // what the framer goes on parsing
  EXPECT(r.OnPacketInPlace(ENCRYPTION_FORWARD_SECURE, DataHeader(42, 41), &b2, 9, p2.size()));
  r.CloseFecGroupsBefore(43);  // the packet's own STOP_WAITING drops the group
  EXPECT(r.GetGroup(41) == nullptr);
  EXPECT(std::memcmp(view, p2.data(), p2.size()) == 0);  // still readable
  // the next packet retires it
  QuicFecGroup::PacketBuffer b3 = decrypt(p1, 8);
  EXPECT(r.OnPacketInPlace(ENCRYPTION_FORWARD_SECURE, DataHeader(50, 50), &b3, 8, p1.size()));
  EXPECT(r.GetGroup(50) != nullptr && r.NumGroups() == 1);
}

// Zero-copy send (OnDataPacketInPlace): each packet serialized into an arena
// buffer after a header of its own length; the group adopts the buffers and
// its parity is the XOR of the payloads at their BUFFER offsets -- not at the
// packets' FEC-group offsets (round 4: a local group offset shadowed the
// buffer offset, and only the first packet of a group, at offset 0 both ways
// when its header was empty, came out right).  The parity is compared where
// the group can compute it (the CPU stub build, or a device).
static void SenderInPlace() {
  QuicFecSender s(4);
  const size_t hdr[3] = {11, 9, 14};
  std::string want(1200, '\0');
  FecHeaderFields f;
  for (int i = 0; i < 3; ++i) {
    const std::string p = Payload(5, 70 + i, 1000 + 100 * i);
    QuicFecGroup::PacketBuffer b = QuicFecGroup::AllocPacketBuffer(kMaxPacketSize);
    std::memset(b.data(), 0x5A, hdr[i]);  // the packet header: not protected
    std::memcpy(b.data() + hdr[i], p.data(), p.size());
    std::memset(b.data() + hdr[i] + p.size(), 0x77, 16);  // beyond the payload
    EXPECT(s.OnDataPacketInPlace(70 + i, &b, hdr[i], p.size(), false, &f));
    EXPECT(b.empty() && f.fec_group_offset == i);
    for (size_t j = 0; j < p.size(); ++j) want[j] ^= p[j];
  }
  QuicFecGroup::PacketBuffer bad = QuicFecGroup::AllocPacketBuffer(100);
  EXPECT(!s.OnDataPacketInPlace(80, &bad, 50, 60, false, &f));  // outside its buffer
  QuicFecEncodeBatch batch;
  EXPECT(s.CloseFecGroup(73, &batch, &s) && batch.size() == 1);
  StringPiece par = batch.entries()[0].group->PayloadParity();
  if (!par.empty()) {
    EXPECT(par.size() == want.size());
    EXPECT(par.size() == want.size() && std::memcmp(par.data(), want.data(), want.size()) == 0);
  }
}

// ---------------------------------------------------------------------------
// GPU: lossy multi-connection simulation
// ---------------------------------------------------------------------------
struct Wire {  // one packet on the wire: private header + payload (header fields alongside)
  int conn;
  QuicPacketNumber pn;
  std::vector<uint8_t> bytes;
};

struct GroupTruth {
  std::vector<QuicPacketNumber> data;
  QuicPacketNumber fec_pn = 0;
  std::map<QuicPacketNumber, bool> lost;
  bool fec_lost = false;
};

// A full-width group: 255 data packets (offsets 0..254) + the FEC packet at
// offset 255 = 256 payloads.  Lossless, the receiver takes every packet and the
// group finishes (the 256th payload completes it and is not kept); with one
// loss it folds 255 payloads and can revive.
static void FullWidthGroup() {
  QuicFecSender s(1000);  // clamps to 255
  EXPECT(s.max_packets_per_fec_group() == 255);
  FecHeaderFields f;
  for (QuicPacketNumber pn = 1; pn <= 255; ++pn)
    EXPECT(s.OnDataPacket(pn, Payload(7, pn, 40 + pn % 50), false, &f) &&
           f.fec_group_offset == pn - 1);
  EXPECT(s.ShouldSendFec(false));
  QuicFecEncodeBatch batch;
  EXPECT(s.CloseFecGroup(256, &batch));
  for (int lost : {-1, 0, 254}) {
    QuicFecReceiver r;
    for (QuicPacketNumber pn = 1; pn <= 255; ++pn) {
      if ((int)pn - 1 == lost) continue;
      EXPECT(r.OnPacket(ENCRYPTION_FORWARD_SECURE, DataHeader(pn, 1),
                        Payload(7, pn, 40 + pn % 50)));
    }
    QuicPacketHeader fh = DataHeader(256, 1);
    fh.fec_flag = true;
    EXPECT(r.OnPacket(ENCRYPTION_FORWARD_SECURE, fh, std::string(90, 'r')));
    const QuicFecGroup* g = r.GetGroup(1);
    if (lost < 0) {
      EXPECT(g == nullptr || g->IsFinished());  // finished groups leave the map
    } else {
      EXPECT(g != nullptr && g->CanRevive());
    }
  }
  // the group object itself: 256 payloads only when the last one completes it
  QuicFecGroup grp(1);
  for (QuicPacketNumber pn = 1; pn <= 255; ++pn)
    EXPECT(grp.Update(ENCRYPTION_NONE, DataHeader(pn, 1), Payload(8, pn, 30)));
  QuicPacketHeader fh = DataHeader(256, 1);
  fh.fec_flag = true;
  EXPECT(grp.UpdateFec(ENCRYPTION_NONE, fh, std::string(30, 'z')));
  EXPECT(grp.IsFinished() && !grp.CanRevive());
  EXPECT(grp.PayloadParity().empty() && !grp.detailed_error().empty());
  // an entry outside the uint8 group-offset range: Flush refuses the whole
  // batch before any launch (FecPacketBody could not serialise it)
  for (QuicPacketNumber fec_pn : {QuicPacketNumber(1 + 256), QuicPacketNumber(0)}) {
    QuicFecEncodeBatch bad;
    QuicFecEncodeBatch::Entry e;
    e.fec_group = 1;
    e.fec_packet_number = fec_pn;
    e.group.reset(new QuicFecGroup(1));
    EXPECT(e.group->Update(ENCRYPTION_NONE, DataHeader(1, 1), Payload(9, 1, 20)));
    bad.Add(std::move(e));
    EXPECT(bad.Flush(nullptr) == QFEC_ERR_INVALID_FEC_DATA);
    EXPECT(bad.entries().back().FecPacketBody().empty());
  }
}

static void Simulation(qfec_ctx* ctx, int conns, int packets_per_conn, double loss,
                       uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::vector<std::unique_ptr<QuicFecSender>> senders;
  std::vector<std::unique_ptr<QuicFecReceiver>> receivers;
  std::vector<QuicPacketNumber> next_pn(conns, 1);
  std::vector<int> sent(conns, 0);
  std::map<std::pair<int, QuicPacketNumber>, std::string> payloads;  // truth
  std::map<std::pair<int, QuicFecGroupNumber>, GroupTruth> truth;
  for (int c = 0; c < conns; ++c) {
    senders.emplace_back(new QuicFecSender(2 + (c * 7) % 19));  // group sizes 2..20
    receivers.emplace_back(new QuicFecReceiver(16));
  }
  senders[0]->set_max_packets_per_fec_group(255);
  size_t revived_total = 0, flushes = 0, batched_groups = 0;
  std::vector<QuicFecReviveBatch::Revived> revived;
  std::vector<std::string> revived_bytes;  // owned copies (the views end with their batch)
  bool done = false;
  while (!done) {
    done = true;
    std::vector<Wire> wire;
    QuicFecEncodeBatch enc;
    for (int c = 0; c < conns; ++c) {
      const int burst = 1 + static_cast<int>(rng() % 4);
      for (int b = 0; b < burst && sent[c] < packets_per_conn; ++b, ++sent[c]) {
        const QuicPacketNumber pn = next_pn[c]++;
        const uint32_t len = 1 + static_cast<uint32_t>(rng() % QFEC_DEFAULT_MAX_PACKET_SIZE);
        std::string p = Payload(c, pn, len);
        FecHeaderFields f;
        EXPECT(senders[c]->OnDataPacket(pn, p, false, &f));
        payloads[{c, pn}] = p;
        const QuicFecGroupNumber grp = pn - f.fec_group_offset;
        truth[{c, grp}].data.push_back(pn);
        Wire w{c, pn, std::vector<uint8_t>(2 + len)};
        const size_t hn = WriteFecPrivateHeader(f, w.bytes.data(), w.bytes.size());
        EXPECT(hn == 2);
        std::memcpy(w.bytes.data() + hn, p.data(), len);
        w.bytes.resize(hn + len);
        wire.push_back(std::move(w));
        const bool last = sent[c] + 1 == packets_per_conn;
        if (senders[c]->ShouldSendFec(last)) {
          const QuicPacketNumber fpn = next_pn[c]++;
          truth[{c, grp}].fec_pn = fpn;
          EXPECT(senders[c]->CloseFecGroup(fpn, &enc, reinterpret_cast<void*>(static_cast<intptr_t>(c))));
        }
      }
      if (sent[c] < packets_per_conn) done = false;
    }
    // every closed group of every connection: one encode launch
    if (enc.size()) {
      EXPECT(enc.Flush(ctx) == QFEC_OK);
      ++flushes;
      batched_groups += enc.size();
      for (auto& e : enc.entries()) {
        const int c = static_cast<int>(reinterpret_cast<intptr_t>(e.tag));
        const std::vector<uint8_t> body = e.FecPacketBody();
        // the body parses back: FEC | FEC_GROUP, offset to the group's first packet
        FecHeaderFields pf;
        std::string err;
        EXPECT(ParseFecPrivateHeader(body.data(), body.size(),
                                     kQuicVersion31, e.fec_packet_number, &pf, &err) == 2);
        EXPECT(pf.fec_flag && pf.in_fec_group &&
               e.fec_packet_number - pf.fec_group_offset == e.fec_group);
        // redundancy == oracle XOR of the group's payloads
        std::vector<const uint8_t*> ptr;
        std::vector<uint32_t> len;
        for (QuicPacketNumber pn : truth[{c, e.fec_group}].data) {
          const std::string& s = payloads[{c, pn}];
          ptr.push_back(reinterpret_cast<const uint8_t*>(s.data()));
          len.push_back(static_cast<uint32_t>(s.size()));
        }
        std::vector<uint8_t> want(kMaxPacketSize);
        const int wl = qo_group_encode(ptr.data(), len.data(), ptr.size(), want.data());
        EXPECT(wl == static_cast<int>(body.size()) - 2);
        EXPECT(std::memcmp(want.data(), body.data() + 2, wl) == 0);
        wire.push_back(Wire{c, e.fec_packet_number, body});
      }
    }
    // lossy, reordering network
    std::shuffle(wire.begin(), wire.end(), rng);
    for (Wire& w : wire) {
      FecHeaderFields pf;
      std::string err;
      const size_t hn = ParseFecPrivateHeader(w.bytes.data(), w.bytes.size(), kQuicVersion31,
                                              w.pn, &pf, &err);
      EXPECT(hn == 2);
      const QuicFecGroupNumber grp = w.pn - pf.fec_group_offset;
      const bool drop = std::uniform_real_distribution<double>(0, 1)(rng) < loss;
      if (pf.fec_flag) {
        truth[{w.conn, grp}].fec_lost = drop;
      } else {
        truth[{w.conn, grp}].lost[w.pn] = drop;
      }
      if (drop) continue;
      QuicPacketHeader h;
      h.packet_number = w.pn;
      ApplyFecHeader(pf, &h);
      EXPECT(h.fec_group == grp);
      EXPECT(receivers[w.conn]->OnPacket(
          ENCRYPTION_FORWARD_SECURE, h,
          StringPiece(reinterpret_cast<const char*>(w.bytes.data()) + hn, w.bytes.size() - hn)));
    }
    // every revivable group of every connection: one recover launch
    QuicFecReviveBatch rb;
    for (int c = 0; c < conns; ++c)
      receivers[c]->CollectRevivable(&rb, reinterpret_cast<void*>(static_cast<intptr_t>(c)));
    if (rb.size()) {
      const size_t before = revived.size();
      EXPECT(rb.Flush(ctx, &revived) == QFEC_OK);
      revived_total += revived.size() - before;
      // the payload views live as long as rb's groups: copy them out
      for (size_t i = before; i < revived.size(); ++i)
        revived_bytes.emplace_back(revived[i].payload.data(), revived[i].payload.size());
    }
  }
  // expected revivals: exactly one data packet lost and the FEC packet received
  size_t expect = 0;
  std::map<std::pair<int, QuicPacketNumber>, bool> want_revived;
  for (auto& kv : truth) {
    const GroupTruth& g = kv.second;
    int nlost = 0;
    QuicPacketNumber lost_pn = 0;
    for (auto& l : g.lost)
      if (l.second) {
        ++nlost;
        lost_pn = l.first;
      }
    if (g.fec_pn && !g.fec_lost && nlost == 1) {
      ++expect;
      want_revived[{kv.first.first, lost_pn}] = true;
    }
  }
  EXPECT(revived_total == expect);
  size_t exact = 0;
  for (size_t k = 0; k < revived.size(); ++k) {
    const auto& r = revived[k];
    const std::string& rp = revived_bytes[k];
    const int c = static_cast<int>(reinterpret_cast<intptr_t>(r.tag));
    EXPECT(want_revived.count({c, r.header.packet_number}) == 1);
    const std::string& p = payloads[{c, r.header.packet_number}];
    // revived payload = original, zero padded to the redundancy length
    bool ok = rp.size() >= p.size() && std::memcmp(rp.data(), p.data(), p.size()) == 0;
    for (size_t i = p.size(); ok && i < rp.size(); ++i) ok = rp[i] == '\0';
    EXPECT(ok);
    exact += ok;
  }
  std::printf("simulation: %d connections x %d packets, loss %.2f: %zu groups flushed in %zu "
              "encode launches, %zu revived (%zu expected, %zu bit-exact)\n",
              conns, packets_per_conn, loss, batched_groups, flushes, revived_total, expect,
              exact);
}

int main(int argc, char** argv) {
  const bool cpu_only = argc > 1 && std::strcmp(argv[1], "--cpu") == 0;
  SenderBookkeeping();
  ReceiverBookkeeping();
  ReceiverInPlace();
  SenderInPlace();
  FullWidthGroup();
  if (!cpu_only) {
    qfec_ctx* ctx = qfec_create(0);
    EXPECT(ctx != nullptr);
    if (ctx) {
      Simulation(ctx, 48, 400, 0.08, 1);
      Simulation(ctx, 8, 2000, 0.02, 2);
      qfec_destroy(ctx);
    }
  }
  std::printf("%d checks, %d failures\n", g_checks, g_fail);
  return g_fail == 0 ? 0 : 1;
}
