// connection_shim.cc — end-to-end drop-in check of integration/libquic_fec.patch
// through the REFERENCE's QuicConnection (patched): the real
// ProcessUdpPacket -> ProcessValidatedPacket -> MaybeProcessRevivedPackets
// receive path (quic_connection.cc:1286-1392) and the real send path
// (SendStreamData -> QuicPacketGenerator -> QuicPacketCreator::SerializePacket
// -> the FEC hooks -> SendOrQueuePacket -> QuicPacketWriter), with the XOR on
// the GPU (libqfec.so).
//
// Built by integration/build.py into integration/_build/libquic_fec_patched.so
// with quic_connection.cc and everything it reaches compiled from
// /root/reference (no stand-ins).  What the harness supplies is what a
// libquic embedder supplies (quic_connection.h:275-287, quic_alarm_factory.h,
// quic_packet_writer.h:36-67): a simulated clock, an alarm factory whose
// alarms the loop fires, and an in-memory packet writer per direction that
// drops chosen client->server data packets (at most one per FEC group, never
// an FEC packet).
//
//   n_pairs client/server connection pairs at QUIC_VERSION_31; every client
//   sends stream 5 (stream_len bytes, FEC groups of group_size packets) with
//   NULL encryption at ENCRYPTION_FORWARD_SECURE; every server reassembles it.
//   Loop turn: complete the previous turn's batched FEC work (emits FEC
//   packets, re-injects revived packets) -> deliver the packets written last
//   turn -> fire due alarms -> launch this turn's FEC work (one encode + one
//   revive GPU launch for every connection) -> advance the clock 1 ms.
//   batched = 0 leaves the batcher out: each connection flushes one group per
//   launch, synchronously (the latency path).
//
// The historical connection-thread cost of the same FEC work is timed beside
// it: every FEC-protected packet the clients write is XORed into its group's
// 1452-byte accumulator word by word (QuicFecGroupInterface::XorBuffers, the
// removed reference code: SURVEY.md Appendix A), on this thread.
#include <execinfo.h>
#include <signal.h>
#include <time.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "net/base/ip_address.h"
#include "net/base/ip_endpoint.h"
#include "net/quic/core/crypto/null_decrypter.h"
#include "net/quic/core/crypto/null_encrypter.h"
#include "net/quic/core/crypto/quic_random.h"
#include "net/quic/core/quic_alarm.h"
#include "net/quic/core/quic_alarm_factory.h"
#include "net/quic/core/quic_clock.h"
#include "net/quic/core/quic_connection.h"
#include "net/quic/core/crypto/crypto_handshake_message.h"
#include "net/quic/core/quic_config.h"
#include "net/quic/core/quic_fec_connection.h"
#include "net/quic/core/quic_flags.h"
#include "net/quic/core/quic_framer.h"
#include "net/quic/core/quic_packet_writer.h"
#include "net/quic/core/quic_simple_buffer_allocator.h"

using namespace net;

extern "C" {
struct fec_conn_params {
  int32_t version;      // QuicVersion (31)
  int32_t n_pairs;      // client/server connection pairs
  int32_t group_size;   // packets per FEC group (EnableFecSending); 0: FEC off
  int32_t drop_every;   // drop one data packet in about one group of drop_every; 0: none
  uint64_t stream_len;  // bytes each client sends on stream 5
  int32_t batched;      // 1: one QuicFecBatcher for all connections
  int32_t max_turns;
  int32_t fail_encode;  // 1: every FEC launch fails (GPU failure path)
  int32_t require_gpu;  // 1: fail (status 3) without a HIP device
  int32_t no_end_flush; // 1: no SendFecPacketNow at the end (partial groups: FEC alarm only)
  int32_t reorder;       // R > 0: client->server packets reordered (adjacent pairs
                         // swapped, about one in R held back a turn)
  int32_t inject_unencrypted_fec;  // 1: client 0 also sends an FEC packet at ENCRYPTION_NONE
  int32_t close_mid_batch;  // T > 0: from turn T, client 0 closes its connection while
                            // one of its FEC packets is pending in the batcher
  int32_t fec_option;       // 1 / 2: the client sends FEC connection option kFSTR / kFHDR
                            // (the session's FEC policy; negotiated through QuicConfig and
                            // applied by SetFromConfig at both ends -- no EnableFecSending)
};

struct fec_conn_result {
  uint64_t data_packets_sent;   // client->server FEC-protected data packets written
  uint64_t fec_packets_sent;    // client FEC packets written (clients' stats agree)
  uint64_t dropped;             // data packets the channel dropped
  uint64_t revived;             // servers' packets_revived
  uint64_t groups_one_loss;     // groups that lost exactly one data packet
  uint64_t fec_groups_skipped;  // clients' fec_groups_skipped
  uint64_t retransmitted;       // clients' packets_retransmitted
  uint64_t stream_bytes;        // per connection
  uint64_t turns;
  uint64_t launches;            // batcher launches (0 unbatched)
  uint64_t groups_encoded;      // batcher deliveries
  uint64_t groups_revived;
  double fec_wall_us;           // wall time inside the batcher's Launch + Complete (with callbacks)
  double fec_host_us;           // of which the FEC work itself (batcher launch_us + complete_us)
  double cpu_xor_us;            // the historical per-packet XOR of the same packets, one core
  uint64_t cpu_xor_groups;      // groups XORed by it
  int32_t streams_ok;           // connections whose stream arrived complete and identical
  int32_t connected;            // connections still connected at the end
  int32_t status;               // 0 ok, else a failure code
  char detail[256];
  double fec_wait_us;           // of fec_host_us: blocked waiting for the device (Complete(true))
  double fec_launch_us;         // of fec_host_us: the batcher's Launch (tables + queueing)
  uint64_t debug_revived;       // QuicConnectionDebugVisitor::OnRevivedPacket calls (servers)
  // the v<=31 ack's revived-packets list and the packets' entropy bits
  uint64_t revived_reported;    // distinct packets clients saw listed as revived in acks
  uint64_t acks_with_revived;   // acks (clients received) listing any revived packet
  uint64_t retransmitted_after_report;  // retransmissions of a packet already reported revived
  uint64_t retransmitted_of_revived;    // retransmissions of packets the servers revived
  uint64_t protected_entropy_set;       // FEC-protected data packets sent with entropy bit 1
  int32_t server_close_error;   // first server's QuicErrorCode if it closed, else 0
  int32_t client_close_error;   // first client's QuicErrorCode if it closed, else 0
  int32_t peer_saw_close;       // server 0 closed by the peer (close_mid_batch)
  int32_t closed_with_pending;  // client 0 had a pending FEC packet when it closed
  double fec_tables_us;         // of fec_launch_us: CSR tables
  double fec_call_us;           // of fec_launch_us: the C-ABI calls queueing the launches
  double fec_launch_us_max;     // the slowest single batcher Launch
  uint64_t payloads_adopted;    // FEC payloads captured without a copy (both sides)
  uint64_t payloads_copied;     // FEC payloads copied into the arena
  uint64_t slabs_allocated;     // payload-arena slabs allocated during the run
};
}

namespace {

double now_us() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

class SimClock : public QuicClock {
 public:
  QuicTime ApproximateNow() const override { return now_; }
  QuicTime Now() const override { return now_; }
  QuicWallTime WallNow() const override {
    return QuicWallTime::FromUNIXMicroseconds((now_ - QuicTime::Zero()).ToMicroseconds());
  }
  void Advance(QuicTime::Delta d) { now_ = now_ + d; }

 private:
  QuicTime now_ = QuicTime::Zero() + QuicTime::Delta::FromMilliseconds(1000);
};

class SimAlarm;

class SimAlarmFactory : public QuicAlarmFactory {
 public:
  QuicAlarm* CreateAlarm(QuicAlarm::Delegate* delegate) override;
  QuicArenaScopedPtr<QuicAlarm> CreateAlarm(QuicArenaScopedPtr<QuicAlarm::Delegate> delegate,
                                            QuicConnectionArena* arena) override;
  // Fires every alarm due at `now` (alarms set while firing wait for the next call).
  int FireDue(QuicTime now);
  std::vector<SimAlarm*> alarms;
};

class SimAlarm : public QuicAlarm {
 public:
  SimAlarm(QuicArenaScopedPtr<Delegate> d, SimAlarmFactory* f) : QuicAlarm(std::move(d)), f_(f) {
    f_->alarms.push_back(this);
  }
  ~SimAlarm() override {
    auto& v = f_->alarms;
    v.erase(std::remove(v.begin(), v.end(), this), v.end());
  }
  void FireNow() { Fire(); }

 protected:
  void SetImpl() override {}
  void CancelImpl() override {}

 private:
  SimAlarmFactory* f_;
};

QuicAlarm* SimAlarmFactory::CreateAlarm(QuicAlarm::Delegate* delegate) {
  return new SimAlarm(QuicArenaScopedPtr<QuicAlarm::Delegate>(delegate), this);
}

QuicArenaScopedPtr<QuicAlarm> SimAlarmFactory::CreateAlarm(
    QuicArenaScopedPtr<QuicAlarm::Delegate> delegate, QuicConnectionArena* arena) {
  if (arena != nullptr) return arena->New<SimAlarm>(std::move(delegate), this);
  return QuicArenaScopedPtr<QuicAlarm>(new SimAlarm(std::move(delegate), this));
}

int SimAlarmFactory::FireDue(QuicTime now) {
  std::vector<SimAlarm*> due;
  for (SimAlarm* a : alarms)
    if (a->IsSet() && a->deadline() <= now) due.push_back(a);
  int n = 0;
  for (SimAlarm* a : due) {
    // an earlier alarm's callback may have cancelled or deleted this one
    if (std::find(alarms.begin(), alarms.end(), a) == alarms.end()) continue;
    if (!a->IsSet() || a->deadline() > now) continue;
    a->FireNow();
    ++n;
  }
  return n;
}

class SimHelper : public QuicConnectionHelperInterface {
 public:
  explicit SimHelper(const SimClock* clock) : clock_(clock) {}
  const QuicClock* GetClock() const override { return clock_; }
  QuicRandom* GetRandomGenerator() override { return QuicRandom::GetInstance(); }
  QuicBufferAllocator* GetBufferAllocator() override { return &allocator_; }

 private:
  const SimClock* clock_;
  SimpleBufferAllocator allocator_;
};

// Parses the packets one direction writes (in write order: the framer expands
// truncated packet numbers against the last one it saw) for the drop policy.
class HeaderProbe : public QuicFramerVisitorInterface {
 public:
  explicit HeaderProbe(QuicVersion v)
      : framer_(QuicVersionVector{v}, QuicTime::Zero(), Perspective::IS_SERVER) {
    framer_.set_version(v);
    framer_.set_visitor(this);
    framer_.SetDecrypter(ENCRYPTION_FORWARD_SECURE, new NullDecrypter());
  }
  // false if the packet could not be parsed (header is then invalid)
  bool Parse(const char* p, size_t n, QuicPacketHeader* h, std::string* payload) {
    ok_ = false;
    payload_ = payload;
    QuicEncryptedPacket pkt(p, n, false);
    framer_.ProcessPacket(pkt);
    if (ok_) *h = header_;
    return ok_;
  }

  void OnError(QuicFramer*) override {}
  bool OnProtocolVersionMismatch(QuicVersion) override { return false; }
  void OnPacket() override {}
  void OnPublicResetPacket(const QuicPublicResetPacket&) override {}
  void OnVersionNegotiationPacket(const QuicVersionNegotiationPacket&) override {}
  bool OnUnauthenticatedPublicHeader(const QuicPacketPublicHeader&) override { return true; }
  bool OnUnauthenticatedHeader(const QuicPacketHeader&) override { return true; }
  void OnDecryptedPacket(EncryptionLevel) override {}
  bool OnPacketHeader(const QuicPacketHeader& h) override {
    header_ = h;
    ok_ = true;
    return true;  // go on: the FEC callbacks hand over the protected payload
  }
  bool OnStreamFrame(const QuicStreamFrame&) override { return true; }
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
  void OnFecProtectedPayload(base::StringPiece payload) override {
    if (payload_) payload_->assign(payload.data(), payload.size());
  }

 private:
  QuicFramer framer_;
  QuicPacketHeader header_;
  std::string* payload_ = nullptr;
  bool ok_ = false;
};

struct Wire {
  std::vector<std::string> now, next;  // packets in flight (delivered next turn)
};

struct Run;

class SimWriter : public QuicPacketWriter {
 public:
  SimWriter(Run* run, Wire* wire, bool client, QuicVersion v)
      : run_(run), wire_(wire), client_(client), probe_(v) {}
  WriteResult WritePacket(const char* buffer, size_t buf_len, const IPAddress&,
                          const IPEndPoint&, PerPacketOptions*) override;
  bool IsWriteBlockedDataBuffered() const override { return false; }
  bool IsWriteBlocked() const override { return false; }
  void SetWritable() override {}
  QuicByteCount GetMaxPacketSize(const IPEndPoint&) const override { return kMaxPacketSize; }

  // historical connection-thread XOR state per open group
  std::map<QuicFecGroupNumber, std::vector<uint64_t>> xor_acc;
  std::map<QuicFecGroupNumber, int> dropped_in_group;

 private:
  Run* run_;
  Wire* wire_;
  bool client_;
  HeaderProbe probe_;
  std::string payload_;
};

// Where Chromium's QuicConnectionLogger would emit NetLog's
// QUIC_SESSION_PACKET_HEADER_REVIVED (net_log_event_type_list.h:1834): the
// debug visitor's OnRevivedPacket, which the patch restores.  libquic ships no
// logger, so the harness counts the calls.
class RevivalCounter : public QuicConnectionDebugVisitor {
 public:
  void OnRevivedPacket(const QuicPacketHeader& header, base::StringPiece payload) override {
    ++count;
    bytes += payload.size();
    revived.insert(header.packet_number);
  }
  uint64_t count = 0, bytes = 0;
  std::set<QuicPacketNumber> revived;  // this server's revived packet numbers
};

// The sender's view of the revived-packets list (one per client): every
// revived packet an ack reported, and every retransmission it sent after
// that report (MarkPacketNotRetransmittable should leave none).
class AckWatch : public QuicConnectionDebugVisitor {
 public:
  void OnAckFrame(const QuicAckFrame& frame) override {
    if (!frame.revived_packets.empty()) ++acks_with_revived;
    reported.insert(frame.revived_packets.begin(), frame.revived_packets.end());
  }
  void OnPacketSent(const SerializedPacket&, QuicPathId, QuicPacketNumber original_packet_number,
                    TransmissionType, QuicTime) override {
    if (original_packet_number == 0) return;
    retransmitted_originals.push_back(original_packet_number);
    if (reported.count(original_packet_number)) ++after_report;
  }
  std::set<QuicPacketNumber> reported;
  std::vector<QuicPacketNumber> retransmitted_originals;
  uint64_t acks_with_revived = 0, after_report = 0;
};

class Endpoint : public QuicConnectionVisitorInterface {
 public:
  Endpoint(Run* run, bool client, size_t stream_len) : run_(run), client_(client) {
    if (!client) {
      received.assign(stream_len, '\0');
      have.assign(stream_len, 0);
    }
  }
  // client: push stream data while the connection takes it
  void Pump();

  void OnStreamFrame(const QuicStreamFrame& f) override {
    if (client_ || f.stream_id != 5) return;
    if (f.offset + f.data_length > received.size()) {
      bad_frame = true;
      return;
    }
    std::memcpy(&received[f.offset], f.data_buffer, f.data_length);
    std::memset(&have[f.offset], 1, f.data_length);
    if (f.fin) fin = true;
  }
  void OnWindowUpdateFrame(const QuicWindowUpdateFrame&) override {}
  void OnBlockedFrame(const QuicBlockedFrame&) override {}
  void OnRstStream(const QuicRstStreamFrame&) override {}
  void OnGoAway(const QuicGoAwayFrame&) override {}
  void OnConnectionClosed(QuicErrorCode error, const std::string& details,
                          ConnectionCloseSource source) override {
    closed = true;
    close_error = error;
    close_details = details;
    close_from_peer = source == ConnectionCloseSource::FROM_PEER;
  }
  void OnWriteBlocked() override {}
  void OnSuccessfulVersionNegotiation(const QuicVersion&) override {}
  void OnCanWrite() override { Pump(); }
  void OnCongestionWindowChange(QuicTime) override {}
  void OnConnectionMigration(PeerAddressChangeType) override {}
  void OnPathDegrading() override {}
  void PostProcessAfterData() override {}
  bool WillingAndAbleToWrite() const override { return client_ && sent < run_data_len(); }
  bool HasPendingHandshake() const override { return false; }
  bool HasOpenDynamicStreams() const override { return WillingAndAbleToWrite(); }

  size_t run_data_len() const;

  QuicConnection* conn = nullptr;
  uint64_t sent = 0;  // client: stream bytes consumed
  std::string received;
  std::vector<uint8_t> have;
  bool fin = false, bad_frame = false, closed = false, close_from_peer = false;
  QuicErrorCode close_error = QUIC_NO_ERROR;
  std::string close_details;

 private:
  Run* run_;
  bool client_;
};

struct Run {
  fec_conn_params p;
  fec_conn_result* r;
  std::string data;  // the stream every client sends
  QuicVersion version;
};

size_t Endpoint::run_data_len() const { return run_->data.size(); }

void Endpoint::Pump() {
  if (!client_ || closed) return;
  while (sent < run_->data.size() && conn->CanWriteStreamData()) {
    struct iovec iov;
    iov.iov_base = const_cast<char*>(run_->data.data() + sent);
    iov.iov_len = run_->data.size() - sent;
    QuicIOVector io(&iov, 1, iov.iov_len);
    const QuicConsumedData c = conn->SendStreamData(5, io, sent, /*fin=*/true, nullptr);
    sent += c.bytes_consumed;
    if (c.bytes_consumed == 0) break;
  }
}

// About one group in drop_every loses the data packet at a per-group offset.
uint64_t Mix(uint64_t z) {  // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

bool DropPolicy(const fec_conn_params& p, QuicFecGroupNumber g, QuicPacketNumber pn) {
  if (p.drop_every <= 0) return false;
  const uint64_t h = (g + 0x9E3779B97F4A7C15ull) * 0xBF58476D1CE4E5B9ull;
  if ((h >> 33) % (uint64_t)p.drop_every != 0) return false;
  // one of the group's first 8 packets (a short last group has them too)
  return pn - g == (h >> 17) % (uint64_t)std::min(8, std::max(1, p.group_size));
}

WriteResult SimWriter::WritePacket(const char* buffer, size_t buf_len, const IPAddress&,
                                   const IPEndPoint&, PerPacketOptions*) {
  if (client_) {
    QuicPacketHeader h;
    payload_.clear();
    const bool parsed = probe_.Parse(buffer, buf_len, &h, &payload_);
    if (parsed && h.is_in_fec_group != IN_FEC_GROUP && run_->p.group_size <= 0 &&
        DropPolicy(run_->p, h.packet_number & ~uint64_t(7), h.packet_number)) {
      ++run_->r->dropped;  // FEC off: the reference's loss recovery alone
      return WriteResult(WRITE_STATUS_OK, static_cast<int>(buf_len));
    }
    if (parsed && h.is_in_fec_group == IN_FEC_GROUP) {
      if (h.fec_flag) {
        ++run_->r->fec_packets_sent;
        if (dropped_in_group[h.fec_group] == 1) ++run_->r->groups_one_loss;
        dropped_in_group.erase(h.fec_group);
        auto it = xor_acc.find(h.fec_group);
        if (it != xor_acc.end()) {
          ++run_->r->cpu_xor_groups;
          xor_acc.erase(it);
        }
      } else {
        ++run_->r->data_packets_sent;
        if (h.entropy_flag) ++run_->r->protected_entropy_set;
        // the historical sender: XorBuffers of this packet's protected
        // plaintext into the group's accumulator, on the connection thread
        std::vector<uint64_t>& acc = xor_acc[h.fec_group];
        if (acc.empty()) acc.assign(kMaxPacketSize / 8 + 1, 0);  // the group's accumulator
        const double t0 = now_us();
        const size_t nw = payload_.size() / 8;
        const uint64_t* w = reinterpret_cast<const uint64_t*>(payload_.data());
        uint64_t* a = acc.data();
        for (size_t i = 0; i < nw; ++i) a[i] ^= w[i];
        uint8_t* ab = reinterpret_cast<uint8_t*>(a);
        for (size_t i = nw * 8; i < payload_.size(); ++i) ab[i] ^= (uint8_t)payload_[i];
        run_->r->cpu_xor_us += now_us() - t0;
        if (DropPolicy(run_->p, h.fec_group, h.packet_number) &&
            dropped_in_group[h.fec_group] == 0) {
          ++dropped_in_group[h.fec_group];
          ++run_->r->dropped;
          return WriteResult(WRITE_STATUS_OK, static_cast<int>(buf_len));
        }
      }
    }
  }
  wire_->next.emplace_back(buffer, buf_len);
  return WriteResult(WRITE_STATUS_OK, static_cast<int>(buf_len));
}

// A reordering link (deterministic): adjacent packets of a turn swap places
// with probability 1/2, and about one packet in R waits for the next turn
// (it then arrives after packets sent after it, FEC packets included).
void Reorder(std::vector<std::string>* now, std::vector<std::string>* later, int R, int turn,
             int conn) {
  std::vector<std::string> keep;
  keep.reserve(now->size());
  for (size_t j = 0; j < now->size(); ++j) {
    const uint64_t h = Mix(((uint64_t)turn << 40) ^ ((uint64_t)conn << 20) ^ j);
    if (h % (uint64_t)R == 0) later->push_back(std::move((*now)[j]));
    else keep.push_back(std::move((*now)[j]));
  }
  for (size_t j = 0; j + 1 < keep.size(); j += 2)
    if (Mix(((uint64_t)turn << 40) ^ ((uint64_t)conn << 20) ^ (j + 0x55555)) & 1)
      std::swap(keep[j], keep[j + 1]);
  now->swap(keep);
}

void crash_trace(int sig) {
  void* f[64];
  const int n = backtrace(f, 64);
  backtrace_symbols_fd(f, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

}  // namespace

#define SHIM_API extern "C" __attribute__((visibility("default")))

SHIM_API int fec_conn_run(const fec_conn_params* params, fec_conn_result* r) {
  std::memset(r, 0, sizeof(*r));
  const QuicFecGroup::LaunchProfile prof0 = QuicFecGroup::launch_profile();
  signal(SIGSEGV, crash_trace);
  signal(SIGABRT, crash_trace);
  FLAGS_quic_disable_pre_32 = false;  // QUIC_VERSION_31 carries FEC
  Run run;
  run.p = *params;
  run.r = r;
  run.version = static_cast<QuicVersion>(params->version);
  run.data.resize(params->stream_len);
  for (uint64_t i = 0; i < params->stream_len; ++i)
    run.data[i] = static_cast<char>((i * 2654435761u) >> 13);
  const int n = params->n_pairs;
  const QuicVersionVector versions{run.version};

  SimClock clock;
  SimHelper helper(&clock);
  SimAlarmFactory alarms;
  // Without a device every FEC launch fails (QuicFecGroup has no CPU path):
  // the groups go without FEC and the reference's loss recovery delivers the
  // stream — the GPU-failure path, runnable on the CPU.  fail_encode forces
  // that path on a GPU (qfec_debug_fail_launches on the batcher's context).
  qfec_ctx* ctx = (params->group_size > 0 || params->fec_option) ? qfec_create(0) : nullptr;
  if (!ctx && params->require_gpu) {
    std::snprintf(r->detail, sizeof(r->detail), "qfec_create: %s", qfec_last_error(nullptr));
    return r->status = 3;
  }
  if (ctx && !params->fail_encode) {
    // one untimed mapped async launch first: the context's staging slots are
    // allocated at its first launch, once per context, not per group (the
    // batcher's stats then time steady-state work)
    uint8_t* w = static_cast<uint8_t*>(qfec_host_alloc(4096));
    if (w) {
      std::memset(w, 0x5A, 4096);
      const uint64_t off[1] = {0}, poff[1] = {2048};
      const uint16_t len[1] = {64};
      const uint32_t ptr[2] = {0, 1};
      uint16_t plen[1] = {0};
      if (qfec_encode_ragged(ctx, w, off, len, ptr, 1, w, poff, plen,
                             QFEC_PTR_MAPPED | QFEC_ASYNC) == QFEC_OK)
        qfec_complete(ctx, 1);
      qfec_host_free(w);
    }
  }
  if (ctx && params->fail_encode) qfec_debug_fail_launches(ctx, 1);
  std::unique_ptr<QuicFecBatcher> batcher;
  if (params->batched) batcher.reset(new QuicFecBatcher(ctx));
  if (!params->batched && params->fail_encode) {
    std::snprintf(r->detail, sizeof(r->detail), "fail_encode needs batched (the batcher's context)");
    return r->status = 4;
  }

  std::vector<std::unique_ptr<Wire>> c2s(n), s2c(n);
  std::vector<std::unique_ptr<SimWriter>> cw(n), sw(n);
  std::vector<std::unique_ptr<Endpoint>> ce(n), se(n);
  std::vector<std::unique_ptr<RevivalCounter>> slog(n);
  std::vector<std::unique_ptr<AckWatch>> cwatch(n);
  std::vector<std::unique_ptr<QuicConnection>> cc(n), sc(n);
  const IPEndPoint client_addr(IPAddress(10, 0, 0, 1), 4433);
  for (int i = 0; i < n; ++i) {
    c2s[i].reset(new Wire());
    s2c[i].reset(new Wire());
    cw[i].reset(new SimWriter(&run, c2s[i].get(), true, run.version));
    sw[i].reset(new SimWriter(&run, s2c[i].get(), false, run.version));
    ce[i].reset(new Endpoint(&run, true, params->stream_len));
    se[i].reset(new Endpoint(&run, false, params->stream_len));
    const QuicConnectionId cid = 0x5100000000ull + i;
    const IPEndPoint server_addr(IPAddress(10, 0, 1, (uint8_t)(1 + i % 250)), 443);
    cc[i].reset(new QuicConnection(cid, server_addr, &helper, &alarms, cw[i].get(), false,
                                   Perspective::IS_CLIENT, versions));
    sc[i].reset(new QuicConnection(cid, client_addr, &helper, &alarms, sw[i].get(), false,
                                   Perspective::IS_SERVER, versions));
    for (QuicConnection* c : {cc[i].get(), sc[i].get()}) {
      c->SetEncrypter(ENCRYPTION_FORWARD_SECURE, new NullEncrypter());
      c->SetDefaultEncryptionLevel(ENCRYPTION_FORWARD_SECURE);
      // (inject_unencrypted_fec: server 0 keeps only the ENCRYPTION_NONE
      // decrypter, so what it decrypts first is at ENCRYPTION_NONE -- NULL
      // encryption is the same at every level)
      if (!(params->inject_unencrypted_fec && i == 0 && c == sc[i].get()))
        c->SetDecrypter(ENCRYPTION_FORWARD_SECURE, new NullDecrypter());
      if (batcher) c->set_fec_batcher(batcher.get());
    }
    slog[i].reset(new RevivalCounter());
    cwatch[i].reset(new AckWatch());
    cc[i]->set_visitor(ce[i].get());
    sc[i]->set_visitor(se[i].get());
    sc[i]->set_debug_visitor(slog[i].get());
    cc[i]->set_debug_visitor(cwatch[i].get());
    ce[i]->conn = cc[i].get();
    se[i]->conn = sc[i].get();
    if (params->fec_option) {
      // the session's FEC policy as a client connection option: the client's
      // QuicConfig sends it in its CHLO, the server's QuicConfig processes that
      // hello, and each connection gets its negotiated config as
      // QuicSession::OnConfigNegotiated hands it over (SetFromConfig)
      QuicConfig ccfg, scfg;
      QuicTagVector opts;
      opts.push_back(params->fec_option == 2 ? kFHDR : kFSTR);
      ccfg.SetConnectionOptionsToSend(opts);
      CryptoHandshakeMessage chlo;
      ccfg.ToHandshakeMessage(&chlo);
      std::string details;
      if (scfg.ProcessPeerHello(chlo, CLIENT, &details) != QUIC_NO_ERROR) {
        std::snprintf(r->detail, sizeof(r->detail), "server config: %s", details.c_str());
        return r->status = 6;
      }
      cc[i]->SetFromConfig(ccfg);
      sc[i]->SetFromConfig(scfg);
    }
    if (params->group_size > 0) cc[i]->EnableFecSending(params->group_size);
  }
  if (params->inject_unencrypted_fec && n > 0) {
    // an FEC packet for group 1 at ENCRYPTION_NONE, ahead of client 0's
    // first packets: server 0 must close with QUIC_UNENCRYPTED_FEC_DATA
    QuicFramer f(versions, clock.Now(), Perspective::IS_CLIENT);
    f.set_version(run.version);
    QuicPacketHeader h;
    h.public_header.connection_id = 0x5100000000ull;
    h.public_header.connection_id_length = PACKET_8BYTE_CONNECTION_ID;
    h.public_header.version_flag = true;
    h.public_header.versions = versions;
    h.public_header.packet_number_length = PACKET_6BYTE_PACKET_NUMBER;
    h.packet_number = 3;
    h.fec_flag = true;
    h.is_in_fec_group = IN_FEC_GROUP;
    h.fec_group = 1;
    const std::string redundancy(100, '\x5A');
    char buf[kMaxPacketSize];
    const size_t len = f.BuildFecPacket(h, redundancy, buf, sizeof(buf));
    const size_t enc = len == 0 ? 0
                                : f.EncryptInPlace(ENCRYPTION_NONE, kDefaultPathId, h.packet_number,
                                                   GetStartOfEncryptedData(run.version, h), len,
                                                   sizeof(buf), buf);
    if (enc == 0) {
      std::snprintf(r->detail, sizeof(r->detail), "could not build the unencrypted FEC packet");
      return r->status = 5;
    }
    c2s[0]->next.emplace_back(buf, enc);
  }
  for (int i = 0; i < n; ++i) ce[i]->Pump();

  const IPEndPoint server_self(IPAddress(10, 0, 1, 1), 443);
  int turn = 0;
  bool flushed = false;
  for (; turn < params->max_turns; ++turn) {
    if (batcher) {
      const double t0 = now_us();
      batcher->Complete(true);  // emits FEC packets, re-injects revived ones
      r->fec_wall_us += now_us() - t0;
    }
    bool in_flight = false;
    for (int i = 0; i < n; ++i) {
      c2s[i]->now.swap(c2s[i]->next);
      s2c[i]->now.swap(s2c[i]->next);
      if (params->reorder > 0) Reorder(&c2s[i]->now, &c2s[i]->next, params->reorder, turn, i);
      for (const std::string& pk : c2s[i]->now)
        sc[i]->ProcessUdpPacket(server_self, client_addr,
                                QuicReceivedPacket(pk.data(), pk.size(), clock.Now()));
      for (const std::string& pk : s2c[i]->now)
        cc[i]->ProcessUdpPacket(client_addr, server_self,
                                QuicReceivedPacket(pk.data(), pk.size(), clock.Now()));
      in_flight = in_flight || !c2s[i]->now.empty() || !s2c[i]->now.empty();
      c2s[i]->now.clear();
      s2c[i]->now.clear();
    }
    alarms.FireDue(clock.Now());
    if (batcher) {
      const double t0 = now_us();
      batcher->Launch();  // the GPU works while the next turn starts
      r->fec_wall_us += now_us() - t0;
    }
    if (params->close_mid_batch > 0 && turn >= params->close_mid_batch && n > 0 &&
        cc[0]->connected() && cc[0]->NumPendingFecPackets() > 0) {
      // a batched group of client 0 is in flight: close now (the close frame
      // must leave although packets after the pending FEC packet are held)
      r->closed_with_pending = 1;
      cc[0]->CloseConnection(QUIC_PEER_GOING_AWAY, "closed while FEC is pending",
                             ConnectionCloseBehavior::SEND_CONNECTION_CLOSE_PACKET);
    }
    clock.Advance(QuicTime::Delta::FromMilliseconds(1));
    bool done = true;
    for (int i = 0; i < n && done; ++i) {
      const bool complete = se[i]->fin && std::all_of(se[i]->have.begin(), se[i]->have.end(),
                                                      [](uint8_t b) { return b != 0; });
      done = (complete || ce[i]->closed || se[i]->closed) && !cc[i]->HasQueuedData() &&
             !(params->no_end_flush && cc[i]->connected() && cc[i]->IsFecGroupOpen());
    }
    bool wire_busy = false;
    for (int i = 0; i < n; ++i)
      wire_busy = wire_busy || !c2s[i]->next.empty() || !s2c[i]->next.empty();
    if (done && !wire_busy && !(batcher && (batcher->InFlight() || batcher->NumQueued()))) {
      // the end of the data: close every partial group now (as the FEC alarm
      // would), so that every group's FEC packet is sent and counted
      if (!flushed && params->group_size > 0 && !params->no_end_flush) {
        flushed = true;
        for (int i = 0; i < n; ++i)
          if (cc[i]->connected()) cc[i]->SendFecPacketNow();
        continue;
      }
      break;
    }
    (void)in_flight;
  }
  if (batcher) {
    batcher->Complete(true);
    r->launches = batcher->stats().launches;
    r->groups_encoded = batcher->stats().groups_encoded;
    r->groups_revived = batcher->stats().groups_revived;
    r->fec_host_us = batcher->stats().launch_us + batcher->stats().complete_us;
    r->fec_wait_us = batcher->stats().wait_us;
    r->fec_launch_us = batcher->stats().launch_us;
    r->fec_tables_us = batcher->stats().tables_us;
    r->fec_call_us = batcher->stats().call_us;
    r->fec_launch_us_max = batcher->stats().launch_us_max;
  }
  r->turns = turn;
  r->payloads_adopted = QuicFecGroup::launch_profile().payloads_adopted - prof0.payloads_adopted;
  r->payloads_copied = QuicFecGroup::launch_profile().payloads_copied - prof0.payloads_copied;
  r->slabs_allocated = QuicFecGroup::launch_profile().slabs_allocated - prof0.slabs_allocated;
  r->stream_bytes = params->stream_len;
  for (int i = 0; i < n; ++i) {
    r->debug_revived += slog[i]->count;
    r->revived_reported += cwatch[i]->reported.size();
    r->acks_with_revived += cwatch[i]->acks_with_revived;
    r->retransmitted_after_report += cwatch[i]->after_report;
    for (QuicPacketNumber p : cwatch[i]->retransmitted_originals)
      r->retransmitted_of_revived += slog[i]->revived.count(p);
    if (!r->server_close_error && se[i]->closed) r->server_close_error = se[i]->close_error;
    if (!r->client_close_error && ce[i]->closed) r->client_close_error = ce[i]->close_error;
  }
  if (n > 0)
    r->peer_saw_close = se[0]->closed && se[0]->close_from_peer &&
                        se[0]->close_error == QUIC_PEER_GOING_AWAY;
  std::string first_close;
  for (int i = 0; i < n; ++i) {
    const QuicConnectionStats& cs = cc[i]->GetStats();
    const QuicConnectionStats& ss = sc[i]->GetStats();
    r->revived += ss.packets_revived;
    r->fec_groups_skipped += cs.fec_groups_skipped;
    r->retransmitted += cs.packets_retransmitted;
    const bool ok = se[i]->fin && !se[i]->bad_frame && se[i]->received == run.data;
    r->streams_ok += ok ? 1 : 0;
    r->connected += (cc[i]->connected() && sc[i]->connected()) ? 1 : 0;
    if (first_close.empty() && (ce[i]->closed || se[i]->closed))
      first_close = (ce[i]->closed ? "client " + ce[i]->close_details
                                   : "server " + se[i]->close_details);
  }
  if (!first_close.empty())
    std::snprintf(r->detail, sizeof(r->detail), "closed: %s", first_close.c_str());
  // connections before the batcher (they Forget themselves), the batcher
  // before its contexts
  cc.clear();
  sc.clear();
  batcher.reset();
  if (ctx) qfec_destroy(ctx);
  return r->status;
}
