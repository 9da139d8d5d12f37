// ref_framer_shim.cc — a C API over the REFERENCE's QuicFramer, compiled from
// /root/reference by oracle/ref/Makefile into oracle/_ref/libref_framer.so.
//
// TEST INFRASTRUCTURE ONLY (the checker of the v<=31 FEC wire rows, SURVEY.md
// §8(a) a3/a4/a6, §8(f) rank 1).  The product never links or loads it.
//
// Every QUIC function used here is the reference's own, unmodified:
//   QuicFramer::AppendPacketHeader      quic_framer.cc:720-775  (public header,
//                                                                 packet number)
//   QuicFramer::BuildDataPacket         quic_framer.cc:356-459  (ack / ping /
//                                                                 padding frames)
//   QuicFramer::EncryptInPlace          quic_framer.cc:1820-1839 (NullEncrypter)
//   QuicFramer::ProcessPacket           quic_framer.cc:537-585
//     -> ProcessAuthenticatedHeader     quic_framer.cc:1102-1141 (FEC bits, offset)
//     -> ProcessAckFrame (v<=31 revived packets list) quic_framer.cc:1477-1493
// The visitor records what the framer reports and, like the reference's
// QuicConnection::ProcessValidatedPacket ("Drop any FEC packet.",
// quic_connection.cc:1388-1392), stops processing at an FEC packet's header.
// Built with -DNDEBUG (a release build): DCHECKs off, and BoringSSL's error
// strings (Go-generated err_data.c) are unreachable and dropped by
// --gc-sections; -z defs proves nothing is left undefined.
#include <cstring>
#include <string>

#include "net/quic/core/quic_framer.h"
#include "net/quic/core/quic_data_writer.h"

using namespace net;

extern "C" {

struct ref_parse_result {
  int32_t accepted;     // ProcessPacket's return value
  int32_t error;        // framer.error() (QuicErrorCode)
  int32_t header_seen;  // OnPacketHeader reached: the private header parsed
  int32_t entropy_flag;
  int32_t fec_flag;
  int32_t n_ack;
  int32_t n_ping;
  int32_t n_padding;
  int32_t n_stream;
  int32_t complete;     // OnPacketComplete
  uint64_t packet_number;
  uint64_t ack_largest_observed;
  uint64_t ack_missing_count;
  char detailed_error[256];
};

}  // extern "C"

namespace {

class RecordingVisitor : public QuicFramerVisitorInterface {
 public:
  explicit RecordingVisitor(ref_parse_result* r) : r_(r) {}
  void OnError(QuicFramer*) override {}
  bool OnProtocolVersionMismatch(QuicVersion) override { return false; }
  void OnPacket() override {}
  void OnPublicResetPacket(const QuicPublicResetPacket&) override {}
  void OnVersionNegotiationPacket(const QuicVersionNegotiationPacket&) override {}
  bool OnUnauthenticatedPublicHeader(const QuicPacketPublicHeader&) override { return true; }
  bool OnUnauthenticatedHeader(const QuicPacketHeader&) override { return true; }
  void OnDecryptedPacket(EncryptionLevel) override {}
  bool OnPacketHeader(const QuicPacketHeader& h) override {
    r_->header_seen = 1;
    r_->packet_number = h.packet_number;
    r_->entropy_flag = h.entropy_flag;
    r_->fec_flag = h.fec_flag;
    return !h.fec_flag;  // QuicConnection drops FEC packets here
  }
  bool OnStreamFrame(const QuicStreamFrame&) override {
    ++r_->n_stream;
    return true;
  }
  bool OnAckFrame(const QuicAckFrame& f) override {
    ++r_->n_ack;
    r_->ack_largest_observed = f.largest_observed;
    r_->ack_missing_count = f.packets.NumPacketsSlow();
    return true;
  }
  bool OnStopWaitingFrame(const QuicStopWaitingFrame&) override { return true; }
  bool OnPaddingFrame(const QuicPaddingFrame&) override {
    ++r_->n_padding;
    return true;
  }
  bool OnPingFrame(const QuicPingFrame&) override {
    ++r_->n_ping;
    return true;
  }
  bool OnRstStreamFrame(const QuicRstStreamFrame&) override { return true; }
  bool OnConnectionCloseFrame(const QuicConnectionCloseFrame&) override { return true; }
  bool OnGoAwayFrame(const QuicGoAwayFrame&) override { return true; }
  bool OnWindowUpdateFrame(const QuicWindowUpdateFrame&) override { return true; }
  bool OnBlockedFrame(const QuicBlockedFrame&) override { return true; }
  bool OnPathCloseFrame(const QuicPathCloseFrame&) override { return true; }
  void OnPacketComplete() override { r_->complete = 1; }

 private:
  ref_parse_result* r_;
};

QuicPacketNumberLength PnLength(int n) {
  switch (n) {
    case 1: return PACKET_1BYTE_PACKET_NUMBER;
    case 2: return PACKET_2BYTE_PACKET_NUMBER;
    case 4: return PACKET_4BYTE_PACKET_NUMBER;
    default: return PACKET_6BYTE_PACKET_NUMBER;
  }
}

QuicPacketHeader MakeHeader(uint64_t pn, int pn_len, bool entropy) {
  QuicPacketHeader h;
  h.public_header.connection_id = 0x0102030405060708ull;
  h.public_header.connection_id_length = PACKET_8BYTE_CONNECTION_ID;
  h.public_header.reset_flag = false;
  h.public_header.version_flag = false;
  h.public_header.packet_number_length = PnLength(pn_len);
  h.packet_number = pn;
  h.entropy_flag = entropy;
  return h;
}

}  // namespace

#define REF_API extern "C" __attribute__((visibility("default")))

// Parse one (NULL-encrypted) packet with a server-side QuicFramer at `version`.
REF_API int ref_framer_parse(int version, const uint8_t* pkt, size_t len, ref_parse_result* r) {
  std::memset(r, 0, sizeof(*r));
  QuicFramer framer(AllSupportedVersions(), QuicTime::Zero(), Perspective::IS_SERVER);
  framer.set_version(static_cast<QuicVersion>(version));
  RecordingVisitor visitor(r);
  framer.set_visitor(&visitor);
  QuicEncryptedPacket packet(reinterpret_cast<const char*>(pkt), len, false);
  r->accepted = framer.ProcessPacket(packet) ? 1 : 0;
  r->error = framer.error();
  std::strncpy(r->detailed_error, framer.detailed_error().c_str(), sizeof(r->detailed_error) - 1);
  return r->accepted;
}

// The public header + packet number the reference writes for a data packet
// (AppendPacketHeader without the v<=33 private flags byte it appends last).
// Returns the byte count (= the AEAD associated data length), 0 on failure.
REF_API size_t ref_framer_public_header(int version, uint64_t pn, int pn_len, uint8_t* out,
                                        size_t cap) {
  QuicFramer framer(AllSupportedVersions(), QuicTime::Zero(), Perspective::IS_CLIENT);
  framer.set_version(static_cast<QuicVersion>(version));
  char buf[64];
  QuicDataWriter writer(sizeof(buf), buf);
  if (!framer.AppendPacketHeader(MakeHeader(pn, pn_len, false), &writer)) return 0;
  size_t n = writer.length();
  if (version <= QUIC_VERSION_33) n -= 1;  // the private flags byte
  if (n > cap) return 0;
  std::memcpy(out, buf, n);
  return n;
}

// A complete plaintext data packet built by the reference framer: kind 0 = one
// ack frame (largest_observed, missing packets [miss_lo[i], miss_hi[i])), kind
// 1 = one ping frame.  *ad_len receives the associated-data length.
REF_API size_t ref_framer_build(int version, uint64_t pn, int pn_len, int entropy, int kind,
                                uint64_t largest_observed, const uint64_t* miss_lo,
                                const uint64_t* miss_hi, size_t n_miss, uint8_t* out, size_t cap,
                                size_t* ad_len) {
  QuicFramer framer(AllSupportedVersions(), QuicTime::Zero(), Perspective::IS_CLIENT);
  framer.set_version(static_cast<QuicVersion>(version));
  QuicPacketHeader header = MakeHeader(pn, pn_len, entropy != 0);
  QuicAckFrame ack;
  QuicFrames frames;
  if (kind == 0) {
    ack.largest_observed = largest_observed;
    ack.missing = true;
    for (size_t i = 0; i < n_miss; ++i) ack.packets.Add(miss_lo[i], miss_hi[i]);
    frames.push_back(QuicFrame(&ack));
  } else {
    frames.push_back(QuicFrame(QuicPingFrame()));
  }
  const size_t n = framer.BuildDataPacket(header, frames, reinterpret_cast<char*>(out), cap);
  *ad_len = GetStartOfEncryptedData(framer.version(), PACKET_8BYTE_CONNECTION_ID, false, false,
                                    false, PnLength(pn_len));
  return n;
}

// NullEncrypter over buf[ad_len, total) in place (QuicFramer::EncryptInPlace).
REF_API size_t ref_framer_encrypt(int version, uint64_t pn, uint8_t* buf, size_t ad_len,
                                  size_t total, size_t cap) {
  QuicFramer framer(AllSupportedVersions(), QuicTime::Zero(), Perspective::IS_CLIENT);
  framer.set_version(static_cast<QuicVersion>(version));
  return framer.EncryptInPlace(ENCRYPTION_NONE, kDefaultPathId, pn, ad_len, total, cap,
                               reinterpret_cast<char*>(buf));
}
