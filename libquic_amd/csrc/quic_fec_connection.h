// quic_fec_connection.h — connection-level FEC on top of the GPU-backed
// QuicFecGroup: the send-side group state of the historical QuicPacketCreator
// and the receive-side group map of the historical QuicConnection, with the
// XOR work of many connections batched into ONE ragged kernel launch
// (SURVEY.md §8(f) rank 2).
//
// The reference snapshot no longer has this code (FEC was removed at
// QUIC_VERSION_32, src/net/quic/core/quic_protocol.h:373); what remains are
// the two hook sites and the v<=31 wire vestiges:
//   send:    QuicPacketCreator::SerializePacket (quic_packet_creator.cc:517-563)
//            between BuildDataPacket (:530) and EncryptInPlace (:549) —
//            QuicFecSender::OnDataPacket takes the plaintext after the header;
//            when ShouldSendFec() the creator closes the group and serializes an
//            FEC packet whose body comes from QuicFecEncodeBatch::Flush.
//   receive: QuicConnection::ProcessValidatedPacket (quic_connection.cc:1388-1392,
//            today "Drop any FEC packet") — QuicFecReceiver::OnPacket takes the
//            decrypted payload of a packet in a group (or the redundancy of an
//            FEC packet); revivable groups go to a QuicFecReviveBatch whose
//            Flush returns the revived packets for QuicFramer's revived-packet
//            path (the v<=31 ack frame lists them, quic_fec_wire.h).
// Member names and semantics follow the historical classes [no in-container
// source]: max_packets_per_fec_group (<= 255: uint8 offset,
// quic_framer.cc:1126-1136), ShouldSendFec(force_close), IsFecGroupOpen,
// kMaxFecGroups = 2 groups kept on receive with the lowest evicted,
// CloseFecGroupsBefore(packet_number).
//
// Threading: like QuicConnection (quic_connection.h:14), not thread-safe; a
// batch may collect from many connections of one thread.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <map>
#include <set>
#include <memory>
#include <string>
#include <vector>

#include "quic_fec_group.h"
#include "quic_fec_wire.h"

namespace net {

const size_t kMaxFecGroups = 2;                   // receive-side groups kept open
const size_t kDefaultMaxPacketsPerFecGroup = 10;  // send-side group size

class QuicFecEncodeBatch;
class QuicFecReviveBatch;

// ---------------------------------------------------------------------------
// Send side (one per connection).
// ---------------------------------------------------------------------------
class QuicFecSender {
 public:
  explicit QuicFecSender(size_t max_packets_per_fec_group = kDefaultMaxPacketsPerFecGroup);
  ~QuicFecSender();

  // Clamped to [1, 255] (uint8 group offset).  Takes effect for the next group.
  void set_max_packets_per_fec_group(size_t n);
  size_t max_packets_per_fec_group() const { return max_packets_per_fec_group_; }

  // FEC protection on/off for subsequent data packets (historical
  // StartFecProtection / StopFecProtection); stopping does not close an open
  // group — the caller sends its FEC packet first (ShouldSendFec(true)).
  void StartFecProtection() { fec_protect_ = true; }
  void StopFecProtection() { fec_protect_ = false; }
  bool fec_protection() const { return fec_protect_; }

  // A data packet was built (plaintext payload after the header).  When
  // protection is on it joins the open group (opening one at this packet
  // number if none is open); the return value holds the FEC header fields
  // to write in front of it (in_fec_group + offset; WriteFecPrivateHeader).
  // Fails (returns false) on a payload above kMaxPacketSize or a packet number
  // that does not increase; *fields is then unchanged.
  bool OnDataPacket(QuicPacketNumber packet_number, StringPiece payload, bool entropy_flag,
                    FecHeaderFields* fields);
  // The same without a copy: the payload is buf->data() + [offset, offset +
  // len) and the open group adopts *buf (QuicFecGroup::UpdateInPlace; the
  // packet creator serialized the packet into a QuicFecGroup::AllocPacketBuffer
  // and encrypts it out of place).  With protection off nothing is adopted.
  bool OnDataPacketInPlace(QuicPacketNumber packet_number, QuicFecGroup::PacketBuffer* buf,
                           size_t offset, size_t len, bool entropy_flag, FecHeaderFields* fields);

  bool IsFecGroupOpen() const { return group_ != nullptr; }
  // The open group's number (its first packet), 0 when none is open.
  QuicFecGroupNumber FecGroupNumber() const { return group_ ? group_->FecGroupNumber() : 0; }
  size_t NumPacketsInGroup() const { return group_ ? group_->NumReceivedPackets() : 0; }
  // The open group is full, or force_close and it holds at least one packet.
  bool ShouldSendFec(bool force_close) const;

  // Close the open group; its FEC packet will be packet `fec_packet_number`
  // (> every packet of the group, at most 255 above the group's first).  The
  // group moves into `batch`; its redundancy and serialized FEC packet body
  // come from the batch's Flush.  `tag` identifies the connection there.
  bool CloseFecGroup(QuicPacketNumber fec_packet_number, QuicFecEncodeBatch* batch,
                     void* tag = nullptr);
  // The same, handing the closed group to the caller (e.g. for a
  // QuicFecBatcher): its redundancy is group->PayloadParity() once computed.
  bool CloseFecGroup(QuicPacketNumber fec_packet_number, std::unique_ptr<QuicFecGroup>* group);

  const std::string& detailed_error() const { return detailed_error_; }

 private:
  bool OnData(QuicPacketNumber packet_number, StringPiece payload,
              QuicFecGroup::PacketBuffer* buf, size_t offset, bool entropy_flag,
              FecHeaderFields* fields);

  size_t max_packets_per_fec_group_;
  bool fec_protect_ = true;
  std::unique_ptr<QuicFecGroup> group_;
  QuicPacketNumber last_packet_number_ = kInvalidPacketNumber;
  std::string detailed_error_;
};

// Closed send-side groups of any number of connections.
class QuicFecEncodeBatch {
 public:
  struct Entry {
    void* tag = nullptr;
    QuicPacketNumber fec_packet_number = kInvalidPacketNumber;
    QuicFecGroupNumber fec_group = 0;
    bool entropy_flag = false;
    std::unique_ptr<QuicFecGroup> group;
    // After Flush: the FEC packet's redundancy, a view of the group's
    // accumulator (payload arena memory the kernel wrote in place), valid
    // while the entry lives.  QuicFramer::BuildFecPacket writes the header.
    StringPiece redundancy;
    // The v<=31 FEC packet body: private header + redundancy
    // (SerializeFecPacketBody); empty before Flush.  Flush refuses a batch
    // with an entry outside the uint8 group-offset range
    // (QFEC_ERR_INVALID_FEC_DATA), so after a successful Flush it is never
    // empty.
    std::vector<uint8_t> FecPacketBody() const;
  };

  // ONE ragged encode launch for every entry (QuicFecGroup::ComputeAll); then
  // every entry's redundancy is set.  Returns a qfec_* code; on failure no
  // redundancy is set.
  int Flush(qfec_ctx* ctx);
  std::vector<Entry>& entries() { return entries_; }
  size_t size() const { return entries_.size(); }
  void Clear() { entries_.clear(); }
  void Add(Entry e) { entries_.push_back(std::move(e)); }

 private:
  std::vector<Entry> entries_;
};

// ---------------------------------------------------------------------------
// Receive side (one per connection): the group map.
// ---------------------------------------------------------------------------
class QuicFecReceiver {
 public:
  explicit QuicFecReceiver(size_t max_fec_groups = kMaxFecGroups);
  ~QuicFecReceiver();

  // A decrypted packet that belongs to an FEC group: a data packet
  // (header.is_in_fec_group, payload = plaintext after the header) or an FEC
  // packet (header.fec_flag, payload = redundancy).  Returns false if it was
  // not taken: not in a group, its group was already evicted, or the group
  // refused it (duplicate, outside the protected range, oversize).
  bool OnPacket(EncryptionLevel level, const QuicPacketHeader& header, StringPiece payload);
  // The same without a copy: the payload is buf->data() + [offset, offset +
  // len) -- the framer decrypted the packet into this payload-arena buffer --
  // and its group adopts *buf (left empty) when it takes the packet.
  bool OnPacketInPlace(EncryptionLevel level, const QuicPacketHeader& header,
                       QuicFecGroup::PacketBuffer* buf, size_t offset, size_t len);

  // Drop every group still waiting for a packet below `packet_number` (the
  // peer stopped waiting for them: STOP_WAITING / least unacked).
  void CloseFecGroupsBefore(QuicPacketNumber packet_number);

  // Move every group that can revive now into `batch` (they leave the map;
  // later packets of a revived group are ignored as finished).
  size_t CollectRevivable(QuicFecReviveBatch* batch, void* tag = nullptr);
  // The same, appending the groups to `groups` (e.g. for a QuicFecBatcher).
  size_t CollectRevivable(std::vector<std::unique_ptr<QuicFecGroup>>* groups);

  size_t NumGroups() const { return group_map_.size(); }
  const QuicFecGroup* GetGroup(QuicFecGroupNumber n) const;
  const std::string& detailed_error() const { return detailed_error_; }

 private:
  bool OnPacketImpl(EncryptionLevel level, const QuicPacketHeader& header, StringPiece payload,
                    QuicFecGroup::PacketBuffer* buf, size_t offset);
  // A dropped group is kept until the next packet: it may hold (adopted) the
  // buffer the packet being processed was decrypted into, whose frames the
  // framer is still parsing (a STOP_WAITING frame closes groups mid-packet).
  void Retire(std::unique_ptr<QuicFecGroup> g);
  QuicFecGroup* GetFecGroup(QuicFecGroupNumber n);
  void MarkClosed(QuicFecGroupNumber n);

  // Recently finished / revived / evicted groups, so a late packet does not
  // reopen them (bounded; CloseFecGroupsBefore prunes below its threshold).
  static const size_t kClosedGroupMemory = 256;

  size_t max_fec_groups_;
  std::map<QuicFecGroupNumber, std::unique_ptr<QuicFecGroup>> group_map_;
  std::set<QuicFecGroupNumber> closed_;
  std::vector<std::unique_ptr<QuicFecGroup>> retired_;
  std::string detailed_error_;
};

// Revivable groups of any number of connections.
class QuicFecReviveBatch {
 public:
  struct Revived {
    void* tag = nullptr;
    QuicPacketHeader header;  // packet_number of the lost packet, fec_group set
    // redundancy length, zero padded (PADDING frames): a view of the group's
    // accumulator, valid until this batch's next Flush / Clear / destruction
    StringPiece payload;
    // the lowest decryption level of the packets the payload was rebuilt
    // from (QuicFecGroup::EffectiveEncryptionLevel): the revived packet is
    // processed at this level, as the historical connection did
    EncryptionLevel level = NUM_ENCRYPTION_LEVELS;
  };

  void Add(void* tag, std::unique_ptr<QuicFecGroup> group);
  size_t size() const { return groups_.size(); }
  // ONE ragged launch for every collected group, then each group's revived
  // packet, in collection order.  The revived groups are kept (their
  // accumulators back the payload views) until the next Flush or Clear.
  // Returns a qfec_* code.
  int Flush(qfec_ctx* ctx, std::vector<Revived>* revived);
  void Clear() { flushed_.clear(); }

 private:
  std::vector<std::pair<void*, std::unique_ptr<QuicFecGroup>>> groups_;
  std::vector<std::pair<void*, std::unique_ptr<QuicFecGroup>>> flushed_;
};

// ---------------------------------------------------------------------------
// Event-loop batching across connections (embedder-owned, one per thread).
// ---------------------------------------------------------------------------
// The connections of one event loop hand it their closed send-side groups
// (with the FEC packet's header, whose number they reserved) and their
// revivable receive-side groups; once per loop turn the embedder calls
// Launch() — ONE encode and ONE revive ragged launch for everything collected,
// queued asynchronously (QFEC_ASYNC: the payloads are read in place from the
// mapped arena) — goes on serving sockets, and calls Complete() (next turn,
// or when it polls done), which hands every result to its connection:
// OnFecRedundancy emits the FEC packet, OnRevivedPackets re-injects the
// revived packets.  A failed launch is reported per group (ok == false): the
// group then goes without FEC and loss recovery retransmits as without FEC.
class QuicFecBatcher {
 public:
  class Visitor {  // a connection
   public:
    virtual ~Visitor() {}
    // The redundancy of a group handed over with AddClosedGroup (a view valid
    // during the call), or ok == false and an empty view.
    virtual void OnFecRedundancy(const QuicPacketHeader& fec_header, StringPiece redundancy,
                                 bool ok) = 0;
    // The packets revived from this visitor's groups, in the order added
    // (payload views valid during the call).
    virtual void OnRevivedPackets(const std::vector<QuicFecReviveBatch::Revived>& revived) = 0;
  };

  struct Stats {
    uint64_t launches = 0;         // Launch() calls that queued GPU work
    uint64_t groups_encoded = 0;   // FEC redundancies delivered
    uint64_t groups_revived = 0;   // revived packets delivered
    uint64_t groups_failed = 0;    // groups whose GPU work failed
    // connection-thread time spent on the FEC work itself: building the index
    // tables and queueing the launches (Launch), and completing them
    // (Complete: waiting, if the GPU is not done yet, plus the parity
    // lengths) — not the visitors' callbacks
    double launch_us = 0;
    double complete_us = 0;
    // of complete_us: blocked in a waiting Complete(true) until the device
    // finished (a connection thread that polls with Complete(false) skips it)
    double wait_us = 0;
    // of launch_us: the CSR tables over the payloads, and the C-ABI calls
    // that queue the two launches (QuicFecGroup::launch_profile); the
    // slowest single Launch
    double tables_us = 0;
    double call_us = 0;
    double launch_us_max = 0;
  };

  explicit QuicFecBatcher(qfec_ctx* ctx = nullptr) : ctx_(ctx) {}
  // Waits for launched work; delivers nothing.
  ~QuicFecBatcher();
  QuicFecBatcher(const QuicFecBatcher&) = delete;
  QuicFecBatcher& operator=(const QuicFecBatcher&) = delete;

  void AddClosedGroup(Visitor* v, const QuicPacketHeader& fec_header,
                      std::unique_ptr<QuicFecGroup> group);
  void AddRevivable(Visitor* v, std::unique_ptr<QuicFecGroup> group);
  // A visitor going away: its queued groups are dropped and its launched
  // ones complete without a callback.
  void Forget(Visitor* v);

  size_t NumQueued() const { return enc_.size() + rev_.size(); }
  bool InFlight() const { return !enc_live_.empty() || !rev_live_.empty(); }
  // Queue the collected work as one encode + one revive launch (completing a
  // previous launch first).  Returns a qfec_* code (a failure is also
  // delivered per group by the next Complete).
  int Launch();
  // Deliver the launched work to the visitors: wait blocks; otherwise
  // QFEC_PENDING while the GPU is still on it.
  int Complete(bool wait);
  // Launch + Complete(true).
  int Flush();
  const Stats& stats() const { return stats_; }

 private:
  struct EncodeItem {
    Visitor* v;
    QuicPacketHeader header;
    std::unique_ptr<QuicFecGroup> group;
  };
  struct ReviveItem {
    Visitor* v;
    std::unique_ptr<QuicFecGroup> group;
  };
  qfec_ctx* ctx_;
  std::vector<EncodeItem> enc_, enc_live_;
  std::vector<ReviveItem> rev_, rev_live_;
  QuicFecGroup::Pending enc_pending_, rev_pending_;
  std::vector<QuicFecGroup*> launch_groups_;  // Launch's group list
  // the last Launch sent a batch the small-batch service takes (1..64 groups
  // of one kind): only then does the next turn warm the worker
  bool last_turn_small_ = true;
  Stats stats_;
};

}  // namespace net
