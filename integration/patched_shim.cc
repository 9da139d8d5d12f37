// patched_shim.cc — end-to-end drop-in check of integration/libquic_fec.patch:
// the REFERENCE's QuicPacketCreator and QuicFramer, patched, sending and
// receiving a FEC-protected QUIC_VERSION_31 stream through the MI355X FEC path.
//
// Built by integration/build.py into integration/_build/libquic_fec_patched.so
// together with the patched reference sources and the FEC host code
// (-DQFEC_WITH_LIBQUIC); the XOR runs in libqfec.so on the GPU.
//
//   send:    QuicPacketCreator (patched SerializePacket: FEC encode hook,
//            MaybeSendFecPacketAndCloseGroup: FEC packets via BuildFecPacket)
//            with a QuicFecSender, NULL encryption, a delegate that keeps the
//            encrypted packets;
//   channel: one data packet in `drop_every` dropped (never an FEC packet);
//   receive: QuicFramer (patched ProcessAuthenticatedHeader / ProcessDataPacket
//            -> OnFecProtectedPayload / OnFecData) with a visitor that feeds a
//            QuicFecReceiver, as the patched QuicConnection does; after every
//            packet, revivable groups are revived in one launch and re-injected
//            through QuicFramer::ProcessRevivedPacket; the visitor reassembles
//            the stream from received AND revived stream frames.
// The stream must come out byte-identical with every dropped packet revived.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "net/quic/core/crypto/null_encrypter.h"
#include "net/quic/core/crypto/quic_random.h"
#include "net/quic/core/quic_fec_connection.h"
#include "net/quic/core/quic_framer.h"
#include "net/quic/core/quic_packet_creator.h"
#include "net/quic/core/quic_simple_buffer_allocator.h"
#include "net/quic/core/quic_utils.h"

using namespace net;

extern "C" {
struct fec_e2e_result {
  uint64_t data_packets_sent;
  uint64_t fec_packets_sent;
  uint64_t dropped;
  uint64_t revived;
  uint64_t stream_bytes;
  int32_t stream_ok;      // reassembled stream == sent stream
  int32_t framer_errors;  // packets the receiving framer refused
  int32_t fec_header_ok;  // every received data packet carried in_fec_group + group
  int32_t status;         // 0 ok, else a failure code
  char detail[256];
};
}

namespace {

class CollectingDelegate : public QuicPacketCreator::DelegateInterface {
 public:
  struct Sent {
    QuicPacketNumber number;
    std::string bytes;
  };
  void OnSerializedPacket(SerializedPacket* p) override {
    sent.push_back({p->packet_number, std::string(p->encrypted_buffer, p->encrypted_length)});
    QuicUtils::DeleteFrames(&p->retransmittable_frames);
  }
  void OnUnrecoverableError(QuicErrorCode error, const std::string& details,
                            ConnectionCloseSource) override {
    this->error = details.empty() ? "unrecoverable error" : details;
  }
  std::vector<Sent> sent;
  std::string error;
};

class ReceiverVisitor : public QuicFramerVisitorInterface {
 public:
  explicit ReceiverVisitor(size_t stream_len) : stream(stream_len, '\0'), have(stream_len, 0) {}
  void OnError(QuicFramer*) override {}
  bool OnProtocolVersionMismatch(QuicVersion) override { return false; }
  void OnPacket() override {}
  void OnPublicResetPacket(const QuicPublicResetPacket&) override {}
  void OnVersionNegotiationPacket(const QuicVersionNegotiationPacket&) override {}
  bool OnUnauthenticatedPublicHeader(const QuicPacketPublicHeader&) override { return true; }
  bool OnUnauthenticatedHeader(const QuicPacketHeader&) override { return true; }
  void OnDecryptedPacket(EncryptionLevel level) override { level_ = level; }
  bool OnPacketHeader(const QuicPacketHeader& h) override {
    last_header = h;
    if (!h.fec_flag && h.is_in_fec_group != IN_FEC_GROUP) header_ok = false;
    return true;
  }
  bool OnStreamFrame(const QuicStreamFrame& f) override {
    if (f.offset + f.data_length > stream.size()) return false;
    std::memcpy(&stream[f.offset], f.data_buffer, f.data_length);
    std::memset(&have[f.offset], 1, f.data_length);
    return true;
  }
  bool OnAckFrame(const QuicAckFrame&) override { return true; }
  bool OnStopWaitingFrame(const QuicStopWaitingFrame&) override { return true; }
  bool OnPaddingFrame(const QuicPaddingFrame&) override { return true; }
  bool OnPingFrame(const QuicPingFrame&) override { return true; }
  bool OnRstStreamFrame(const QuicRstStreamFrame&) override { return true; }
  bool OnConnectionCloseFrame(const QuicConnectionCloseFrame&) override { return true; }
  bool OnGoAwayFrame(const QuicGoAwayFrame&) override { return true; }
  bool OnWindowUpdateFrame(const QuicWindowUpdateFrame&) override { return true; }
  bool OnBlockedFrame(const QuicBlockedFrame&) override { return true; }
  bool OnPathCloseFrame(const QuicPathCloseFrame&) override { return true; }
  void OnPacketComplete() override {}
  // the patched framer's FEC callbacks -> the receiver's group map
  void OnFecProtectedPayload(base::StringPiece payload) override {
    fec_receiver.OnPacket(level_, last_header, payload);
  }
  bool OnFecData(base::StringPiece redundancy) override {
    fec_receiver.OnPacket(level_, last_header, redundancy);
    return true;
  }

  QuicFecReceiver fec_receiver;
  QuicPacketHeader last_header;
  std::string stream;
  std::vector<uint8_t> have;
  bool header_ok = true;

 private:
  EncryptionLevel level_ = ENCRYPTION_NONE;
};

}  // namespace

#define SHIM_API extern "C" __attribute__((visibility("default")))

namespace {
// A crash inside the patched stack prints the native frames (addresses are
// resolved offline with addr2line against this .so) before the default action.
void crash_trace(int sig) {
  void* f[64];
  const int n = backtrace(f, 64);
  backtrace_symbols_fd(f, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
}  // namespace

SHIM_API int fec_e2e_run(int version, int group_size, uint64_t stream_len, int drop_every,
                         fec_e2e_result* r) {
  std::memset(r, 0, sizeof(*r));
  signal(SIGSEGV, crash_trace);
  const QuicVersion v = static_cast<QuicVersion>(version);
  const QuicStreamId kStream = 5;
  // the stream: counter bytes
  std::string data(stream_len, '\0');
  for (uint64_t i = 0; i < stream_len; ++i)
    data[i] = static_cast<char>((i * 2654435761u) >> 13);

  // ---- send
  QuicFramer client(AllSupportedVersions(), QuicTime::Zero(), Perspective::IS_CLIENT);
  client.set_version(v);
  SimpleBufferAllocator allocator;
  CollectingDelegate delegate;
  QuicPacketCreator creator(0x1122334455667788ull, &client, QuicRandom::GetInstance(), &allocator,
                            &delegate);
  creator.StopSendingVersion();
  // stream data needs a non-NONE encryption level (QuicPacketCreator::AddFrame
  // refuses it otherwise); NullEncrypter at FORWARD_SECURE keeps the bytes
  // readable by the server framer's default NullDecrypter
  client.SetEncrypter(ENCRYPTION_FORWARD_SECURE, new NullEncrypter());
  creator.set_encryption_level(ENCRYPTION_FORWARD_SECURE);
  QuicFecSender fec_sender(group_size);
  creator.set_fec_sender(&fec_sender);
  struct iovec iov;
  QuicIOVector io = MakeIOVector(data, &iov);
  uint64_t off = 0;
  while (off < stream_len) {
    QuicFrame frame;
    if (!creator.ConsumeData(kStream, io, off, off, false, false, &frame)) {
      std::snprintf(r->detail, sizeof(r->detail), "ConsumeData failed at %llu",
                    (unsigned long long)off);
      r->status = 1;
      return r->status;
    }
    off += frame.stream_frame->data_length;
    creator.Flush();  // one stream frame per packet; FEC packet when a group fills
  }
  const size_t sent_before_close = delegate.sent.size();
  const bool open_before_close = fec_sender.IsFecGroupOpen();
  creator.MaybeSendFecPacketAndCloseGroup(/*force_close=*/true);
  std::snprintf(r->detail, sizeof(r->detail),
                "sent %zu packets before the final close (group open: %d), %zu after",
                sent_before_close, (int)open_before_close, delegate.sent.size());
  if (!delegate.error.empty()) {
    std::snprintf(r->detail, sizeof(r->detail), "sender: %s", delegate.error.c_str());
    r->status = 2;
    return r->status;
  }

  // ---- receive (drop one data packet in drop_every)
  QuicFramer server(AllSupportedVersions(), QuicTime::Zero(), Perspective::IS_SERVER);
  server.set_version(v);
  ReceiverVisitor visitor(stream_len);
  server.set_visitor(&visitor);
  qfec_ctx* ctx = qfec_create(0);
  if (!ctx) {
    std::snprintf(r->detail, sizeof(r->detail), "qfec_create: %s", qfec_last_error(nullptr));
    r->status = 3;
    return r->status;
  }
  uint64_t data_index = 0;
  // The sender knows which packets it sent as FEC packets; here they are
  // recognised by parsing every sent packet, in send order, with one probe
  // framer (it must see the whole sequence: a 1-byte packet number is
  // expanded against the last one it saw).
  QuicFramer probe(AllSupportedVersions(), QuicTime::Zero(), Perspective::IS_SERVER);
  probe.set_version(v);
  ReceiverVisitor pv(stream_len);
  probe.set_visitor(&pv);
  for (const auto& p : delegate.sent) {
    QuicEncryptedPacket pkt(p.bytes.data(), p.bytes.size(), false);
    pv.last_header = QuicPacketHeader();
    probe.ProcessPacket(pkt);
    const bool is_fec = pv.last_header.fec_flag;
    if (is_fec) {
      ++r->fec_packets_sent;
    } else {
      ++r->data_packets_sent;
      if (drop_every > 0 && data_index++ % drop_every == static_cast<uint64_t>(drop_every / 2)) {
        ++r->dropped;
        continue;
      }
    }
    if (!server.ProcessPacket(pkt)) ++r->framer_errors;
    // the patched QuicConnection's MaybeProcessRevivedPackets
    QuicFecReviveBatch batch;
    if (visitor.fec_receiver.CollectRevivable(&batch) > 0) {
      std::vector<QuicFecReviveBatch::Revived> revived;
      if (batch.Flush(ctx, &revived) != QFEC_OK) {
        std::snprintf(r->detail, sizeof(r->detail), "revive flush: %s", qfec_last_error(ctx));
        r->status = 4;
        break;
      }
      for (auto& rv : revived) {
        QuicPacketHeader h(visitor.last_header.public_header);
        h.packet_number = rv.header.packet_number;
        h.is_in_fec_group = IN_FEC_GROUP;
        h.fec_group = rv.header.fec_group;
        if (server.ProcessRevivedPacket(&h, rv.payload))
          ++r->revived;
        else
          ++r->framer_errors;
      }
    }
  }
  qfec_destroy(ctx);
  r->stream_bytes = stream_len;
  bool all = true;
  for (uint8_t b : visitor.have) all &= b != 0;
  r->stream_ok = all && visitor.stream == data;
  r->fec_header_ok = visitor.header_ok;
  return r->status;
}

// ---------------------------------------------------------------------------
// The v<=31 ack's revived-packets list as the PATCHED framer writes and reads
// it (quic_framer.cc AppendAckFrameAndTypeByte / ProcessAckFrame): the tests
// parse what fec_ack_build writes with the UNPATCHED reference framer
// (oracle/_ref), which reads the list's count and numbers and discards them.
// ---------------------------------------------------------------------------
namespace {

QuicPacketHeader AckHeader(uint64_t pn) {
  QuicPacketHeader h;
  h.public_header.connection_id = 0x0102030405060708ull;  // as oracle/ref/ref_framer_shim.cc
  h.public_header.connection_id_length = PACKET_8BYTE_CONNECTION_ID;
  h.public_header.version_flag = false;
  h.public_header.packet_number_length = PACKET_6BYTE_PACKET_NUMBER;
  h.packet_number = pn;
  return h;
}

class AckCollector : public QuicFramerVisitorInterface {
 public:
  void OnError(QuicFramer*) override {}
  bool OnProtocolVersionMismatch(QuicVersion) override { return false; }
  void OnPacket() override {}
  void OnPublicResetPacket(const QuicPublicResetPacket&) override {}
  void OnVersionNegotiationPacket(const QuicVersionNegotiationPacket&) override {}
  bool OnUnauthenticatedPublicHeader(const QuicPacketPublicHeader&) override { return true; }
  bool OnUnauthenticatedHeader(const QuicPacketHeader&) override { return true; }
  void OnDecryptedPacket(EncryptionLevel) override {}
  bool OnPacketHeader(const QuicPacketHeader&) override { return true; }
  bool OnStreamFrame(const QuicStreamFrame&) override { return true; }
  bool OnAckFrame(const QuicAckFrame& f) override {
    ++acks;
    ack = f;
    return true;
  }
  bool OnStopWaitingFrame(const QuicStopWaitingFrame&) override { return true; }
  bool OnPaddingFrame(const QuicPaddingFrame&) override { return true; }
  bool OnPingFrame(const QuicPingFrame&) override {
    ++pings;
    return true;
  }
  bool OnRstStreamFrame(const QuicRstStreamFrame&) override { return true; }
  bool OnConnectionCloseFrame(const QuicConnectionCloseFrame&) override { return true; }
  bool OnGoAwayFrame(const QuicGoAwayFrame&) override { return true; }
  bool OnWindowUpdateFrame(const QuicWindowUpdateFrame&) override { return true; }
  bool OnBlockedFrame(const QuicBlockedFrame&) override { return true; }
  bool OnPathCloseFrame(const QuicPathCloseFrame&) override { return true; }
  void OnPacketComplete() override { complete = true; }
  QuicAckFrame ack;
  int acks = 0, pings = 0;
  bool complete = false;
};

}  // namespace

// A v<=31 packet (8-byte connection id, 6-byte packet number, no version)
// carrying one ack -- largest_observed, missing ranges [lo, hi), the revived
// list -- and, if with_ping, a PING after it; NULL-encrypted at ENCRYPTION_NONE.
// Returns the packet length (0 on failure).
SHIM_API size_t fec_ack_build(int version, uint64_t pn, uint64_t largest_observed,
                              const uint64_t* miss_lo, const uint64_t* miss_hi, size_t n_miss,
                              const uint64_t* revived, size_t n_revived, int with_ping,
                              uint8_t* out, size_t cap) {
  QuicFramer framer(AllSupportedVersions(), QuicTime::Zero(), Perspective::IS_CLIENT);
  framer.set_version(static_cast<QuicVersion>(version));
  const QuicPacketHeader header = AckHeader(pn);
  QuicAckFrame ack;
  ack.largest_observed = largest_observed;
  ack.missing = true;
  for (size_t i = 0; i < n_miss; ++i) ack.packets.Add(miss_lo[i], miss_hi[i]);
  ack.revived_packets.insert(revived, revived + n_revived);
  QuicFrames frames;
  frames.push_back(QuicFrame(&ack));
  if (with_ping) frames.push_back(QuicFrame(QuicPingFrame()));
  char* buf = reinterpret_cast<char*>(out);
  // room for the NULL encrypter's 12-byte hash (as the creator's
  // max_plaintext_size_)
  const size_t n =
      framer.BuildDataPacket(header, frames, buf, framer.GetMaxPlaintextSize(cap));
  if (n == 0) return 0;
  return framer.EncryptInPlace(ENCRYPTION_NONE, kDefaultPathId, pn,
                               GetStartOfEncryptedData(framer.version(), header), n, cap, buf);
}

// Parses a packet with the PATCHED framer: the ack's revived list into
// revived[0 .. return) (at most cap), -1 if the packet was refused or held no
// ack; *pings = PING frames seen after it, *largest = the ack's largest observed.
SHIM_API int fec_ack_parse(int version, const uint8_t* buf, size_t len, uint64_t* revived,
                           size_t cap, int* pings, uint64_t* largest) {
  QuicFramer framer(AllSupportedVersions(), QuicTime::Zero(), Perspective::IS_SERVER);
  framer.set_version(static_cast<QuicVersion>(version));
  AckCollector v;
  framer.set_visitor(&v);
  QuicEncryptedPacket p(reinterpret_cast<const char*>(buf), len, false);
  if (!framer.ProcessPacket(p) || v.acks != 1 || !v.complete) return -1;
  size_t i = 0;
  for (QuicPacketNumber r : v.ack.revived_packets) {
    if (i == cap) break;
    revived[i++] = r;
  }
  *pings = v.pings;
  *largest = v.ack.largest_observed;
  return static_cast<int>(i);
}
