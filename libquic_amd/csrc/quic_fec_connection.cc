// quic_fec_connection.cc — see quic_fec_connection.h.
#include "quic_fec_connection.h"

#include <algorithm>
#include <chrono>

namespace net {

// ---------------------------------------------------------------------------
// QuicFecSender
// ---------------------------------------------------------------------------
QuicFecSender::QuicFecSender(size_t max_packets_per_fec_group) {
  set_max_packets_per_fec_group(max_packets_per_fec_group);
}

QuicFecSender::~QuicFecSender() = default;

void QuicFecSender::set_max_packets_per_fec_group(size_t n) {
  max_packets_per_fec_group_ = std::min<size_t>(std::max<size_t>(n, 1), QFEC_MAX_GROUP_PACKETS);
}

bool QuicFecSender::OnDataPacket(QuicPacketNumber packet_number, StringPiece payload,
                                 bool entropy_flag, FecHeaderFields* fields) {
  return OnData(packet_number, payload, nullptr, 0, entropy_flag, fields);
}

bool QuicFecSender::OnDataPacketInPlace(QuicPacketNumber packet_number,
                                        QuicFecGroup::PacketBuffer* buf, size_t offset,
                                        size_t len, bool entropy_flag, FecHeaderFields* fields) {
  if (buf == nullptr || buf->empty() || offset > buf->size() || len > buf->size() - offset) {
    detailed_error_ = "payload outside its packet buffer";
    return false;
  }
  return OnData(packet_number, StringPiece(buf->data() + offset, len), buf, offset, entropy_flag,
                fields);
}

bool QuicFecSender::OnData(QuicPacketNumber packet_number, StringPiece payload,
                           QuicFecGroup::PacketBuffer* buf, size_t offset, bool entropy_flag,
                           FecHeaderFields* fields) {
  if (last_packet_number_ != kInvalidPacketNumber && packet_number <= last_packet_number_) {
    detailed_error_ = "packet number does not increase: " + std::to_string(packet_number);
    return false;
  }
  if (payload.size() > kMaxPacketSize) {
    detailed_error_ = "Illegal payload size: " + std::to_string(payload.size());
    return false;
  }
  FecHeaderFields f;
  f.entropy_flag = entropy_flag;
  if (fec_protect_) {
    if (!group_) group_.reset(new QuicFecGroup(packet_number));
    const QuicPacketNumber group_offset = packet_number - group_->FecGroupNumber();
    // uint8 first_fec_protected_packet_offset: the FEC packet needs an offset
    // above every data packet's, so data packets stop at offset 254.
    if (group_offset >= 0xFF) {
      detailed_error_ = "data packet at FEC group offset " + std::to_string(group_offset) +
                        ": no room left for the FEC packet (close the group first)";
      return false;
    }
    QuicPacketHeader h;
    h.packet_number = packet_number;
    h.entropy_flag = entropy_flag;
    h.is_in_fec_group = IN_FEC_GROUP;
    h.fec_group = group_->FecGroupNumber();
    const bool ok = buf ? group_->UpdateInPlace(ENCRYPTION_FORWARD_SECURE, h, buf, offset,
                                                payload.size())
                        : group_->Update(ENCRYPTION_FORWARD_SECURE, h, payload);
    if (!ok) {
      detailed_error_ = group_->detailed_error();
      return false;
    }
    f.in_fec_group = true;
    f.fec_group_offset = static_cast<uint8_t>(group_offset);
  }
  last_packet_number_ = packet_number;
  if (fields) *fields = f;
  return true;
}

bool QuicFecSender::ShouldSendFec(bool force_close) const {
  if (!group_) return false;
  const size_t n = group_->NumReceivedPackets();
  return n >= max_packets_per_fec_group_ || (force_close && n > 0);
}

bool QuicFecSender::CloseFecGroup(QuicPacketNumber fec_packet_number, QuicFecEncodeBatch* batch,
                                  void* tag) {
  if (!group_ || !batch) return false;
  if (fec_packet_number <= last_packet_number_ ||
      fec_packet_number - group_->FecGroupNumber() > 0xFF) {
    detailed_error_ = "FEC packet number outside the group's offset range";
    return false;
  }
  QuicFecEncodeBatch::Entry e;
  e.tag = tag;
  e.fec_packet_number = fec_packet_number;
  e.fec_group = group_->FecGroupNumber();
  e.group = std::move(group_);
  batch->Add(std::move(e));
  last_packet_number_ = fec_packet_number;
  return true;
}

bool QuicFecSender::CloseFecGroup(QuicPacketNumber fec_packet_number,
                                  std::unique_ptr<QuicFecGroup>* group) {
  QuicFecEncodeBatch batch;
  if (!group || !CloseFecGroup(fec_packet_number, &batch)) return false;
  *group = std::move(batch.entries().back().group);
  return true;
}

// ---------------------------------------------------------------------------
// QuicFecEncodeBatch
// ---------------------------------------------------------------------------
int QuicFecEncodeBatch::Flush(qfec_ctx* ctx) {
  // every entry must fit the v<=31 FEC header (uint8 group offset,
  // quic_framer.cc:1126-1136) before anything is launched: FecPacketBody()
  // then cannot fail after a successful Flush
  for (const Entry& e : entries_)
    if (!e.group || e.fec_group == 0 || e.fec_group > e.fec_packet_number ||
        e.fec_packet_number - e.fec_group > 0xFF)
      return QFEC_ERR_INVALID_FEC_DATA;
  std::vector<QuicFecGroup*> groups;
  groups.reserve(entries_.size());
  for (Entry& e : entries_) groups.push_back(e.group.get());
  const int rc = QuicFecGroup::ComputeAll(ctx, groups);  // one launch
  if (rc != QFEC_OK) return rc;
  for (Entry& e : entries_) e.redundancy = e.group->PayloadParity();
  return QFEC_OK;
}

std::vector<uint8_t> QuicFecEncodeBatch::Entry::FecPacketBody() const {
  std::vector<uint8_t> body(2 + redundancy.size());
  const size_t n = SerializeFecPacketBody(fec_packet_number, fec_group, entropy_flag, redundancy,
                                          body.data(), body.size());
  body.resize(n);
  return body;
}

// ---------------------------------------------------------------------------
// QuicFecReceiver
// ---------------------------------------------------------------------------
QuicFecReceiver::QuicFecReceiver(size_t max_fec_groups)
    : max_fec_groups_(std::max<size_t>(max_fec_groups, 1)) {}

QuicFecReceiver::~QuicFecReceiver() = default;

QuicFecGroup* QuicFecReceiver::GetFecGroup(QuicFecGroupNumber n) {
  auto it = group_map_.find(n);
  if (it != group_map_.end()) return it->second.get();
  if (closed_.count(n) != 0) return nullptr;  // finished / revived / closed: not recreated
  if (group_map_.size() >= max_fec_groups_) {
    // Too many groups: a group older than all kept ones was dropped before
    // and is not recreated; otherwise the lowest group is dropped.
    if (n < group_map_.begin()->first) return nullptr;
    MarkClosed(group_map_.begin()->first);
    Retire(std::move(group_map_.begin()->second));
    group_map_.erase(group_map_.begin());
  }
  QuicFecGroup* g = new QuicFecGroup(n);
  group_map_[n].reset(g);
  return g;
}

bool QuicFecReceiver::OnPacket(EncryptionLevel level, const QuicPacketHeader& header,
                               StringPiece payload) {
  return OnPacketImpl(level, header, payload, nullptr, 0);
}

bool QuicFecReceiver::OnPacketInPlace(EncryptionLevel level, const QuicPacketHeader& header,
                                      QuicFecGroup::PacketBuffer* buf, size_t offset, size_t len) {
  if (buf == nullptr || buf->empty() || offset > buf->size() || len > buf->size() - offset) {
    detailed_error_ = "payload outside its packet buffer";
    return false;
  }
  return OnPacketImpl(level, header, StringPiece(buf->data() + offset, len), buf, offset);
}

void QuicFecReceiver::Retire(std::unique_ptr<QuicFecGroup> g) {
  retired_.push_back(std::move(g));
}

bool QuicFecReceiver::OnPacketImpl(EncryptionLevel level, const QuicPacketHeader& header,
                                   StringPiece payload, QuicFecGroup::PacketBuffer* buf,
                                   size_t offset) {
  // groups dropped while an earlier packet was processed: its frames have
  // been parsed by now, so the payloads they adopted can go
  retired_.clear();
  if (header.is_in_fec_group != IN_FEC_GROUP || header.fec_group == 0) {
    detailed_error_ = "packet is not in an FEC group";
    return false;
  }
  QuicFecGroup* g = GetFecGroup(header.fec_group);
  if (!g) {
    detailed_error_ = "FEC group already closed";
    return false;
  }
  bool ok;
  if (buf)
    ok = header.fec_flag ? g->UpdateFecInPlace(level, header, buf, offset, payload.size())
                         : g->UpdateInPlace(level, header, buf, offset, payload.size());
  else
    ok = header.fec_flag ? g->UpdateFec(level, header, payload)
                         : g->Update(level, header, payload);
  if (!ok) {
    detailed_error_ = g->detailed_error();
    return false;
  }
  if (g->IsFinished()) {  // nothing lost: no revival needed, stop tracking
    MarkClosed(header.fec_group);
    auto it = group_map_.find(header.fec_group);
    Retire(std::move(it->second));
    group_map_.erase(it);
  }
  return true;
}

void QuicFecReceiver::MarkClosed(QuicFecGroupNumber n) {
  closed_.insert(n);
  while (closed_.size() > kClosedGroupMemory) closed_.erase(closed_.begin());
}

void QuicFecReceiver::CloseFecGroupsBefore(QuicPacketNumber packet_number) {
  // groups that start below the threshold can never be useful again
  closed_.erase(closed_.begin(), closed_.lower_bound(packet_number));
  for (auto it = group_map_.begin(); it != group_map_.end();) {
    if (it->second->IsWaitingForPacketBefore(packet_number)) {
      MarkClosed(it->first);
      Retire(std::move(it->second));
      it = group_map_.erase(it);
    } else {
      ++it;
    }
  }
}

size_t QuicFecReceiver::CollectRevivable(QuicFecReviveBatch* batch, void* tag) {
  size_t n = 0;
  for (auto it = group_map_.begin(); it != group_map_.end();) {
    if (it->second->CanRevive()) {
      MarkClosed(it->first);
      batch->Add(tag, std::move(it->second));
      it = group_map_.erase(it);
      ++n;
    } else {
      ++it;
    }
  }
  return n;
}

size_t QuicFecReceiver::CollectRevivable(std::vector<std::unique_ptr<QuicFecGroup>>* groups) {
  size_t n = 0;
  for (auto it = group_map_.begin(); it != group_map_.end();) {
    if (it->second->CanRevive()) {
      MarkClosed(it->first);
      groups->push_back(std::move(it->second));
      it = group_map_.erase(it);
      ++n;
    } else {
      ++it;
    }
  }
  return n;
}

const QuicFecGroup* QuicFecReceiver::GetGroup(QuicFecGroupNumber n) const {
  auto it = group_map_.find(n);
  return it == group_map_.end() ? nullptr : it->second.get();
}

// ---------------------------------------------------------------------------
// QuicFecReviveBatch
// ---------------------------------------------------------------------------
void QuicFecReviveBatch::Add(void* tag, std::unique_ptr<QuicFecGroup> group) {
  groups_.emplace_back(tag, std::move(group));
}

int QuicFecReviveBatch::Flush(qfec_ctx* ctx, std::vector<Revived>* revived) {
  flushed_.clear();  // the previous Flush's payload views end here
  std::vector<QuicFecGroup*> gs;
  gs.reserve(groups_.size());
  for (auto& g : groups_) gs.push_back(g.second.get());
  const int rc = QuicFecGroup::ComputeAll(ctx, gs);  // one launch
  if (rc != QFEC_OK) return rc;
  if (revived) revived->reserve(revived->size() + groups_.size());
  for (auto& g : groups_) {
    Revived r;
    r.tag = g.first;
    if (g.second->ReviveInPlace(&r.header, &r.payload) == 0) continue;  // not for CanRevive() groups
    r.level = g.second->EffectiveEncryptionLevel();
    if (revived) revived->push_back(r);
  }
  flushed_.swap(groups_);
  groups_.clear();
  return QFEC_OK;
}

// ---------------------------------------------------------------------------
// QuicFecBatcher
// ---------------------------------------------------------------------------
QuicFecBatcher::~QuicFecBatcher() {
  QuicFecGroup::Finish(&enc_pending_, true);
  QuicFecGroup::Finish(&rev_pending_, true);
}

// The turn's first group warms the small-batch service (qfec_service_warm):
// the worker is then resident by the turn's Launch instead of relaunched
// there.  Only after a turn whose batch the service took: a loop
// that flushes hundreds of groups a turn never uses the worker, and a warm
// one would hold 8 CUs and poll the host for its 100-us idle time for
// nothing.  Best effort: a failure shows at Launch as before.
void QuicFecBatcher::AddClosedGroup(Visitor* v, const QuicPacketHeader& fec_header,
                                    std::unique_ptr<QuicFecGroup> group) {
  if (ctx_ && last_turn_small_ && NumQueued() == 0) (void)qfec_service_warm(ctx_);
  enc_.push_back(EncodeItem{v, fec_header, std::move(group)});
}

void QuicFecBatcher::AddRevivable(Visitor* v, std::unique_ptr<QuicFecGroup> group) {
  if (ctx_ && last_turn_small_ && NumQueued() == 0) (void)qfec_service_warm(ctx_);
  rev_.push_back(ReviveItem{v, std::move(group)});
}

void QuicFecBatcher::Forget(Visitor* v) {
  enc_.erase(std::remove_if(enc_.begin(), enc_.end(),
                            [v](const EncodeItem& e) { return e.v == v; }),
             enc_.end());
  rev_.erase(std::remove_if(rev_.begin(), rev_.end(),
                            [v](const ReviveItem& e) { return e.v == v; }),
             rev_.end());
  for (EncodeItem& e : enc_live_)  // launched: the groups stay until completion
    if (e.v == v) e.v = nullptr;
  for (ReviveItem& e : rev_live_)
    if (e.v == v) e.v = nullptr;
}

int QuicFecBatcher::Launch() {
  int rc = QFEC_OK;
  if (InFlight()) rc = Complete(true);
  if (enc_.empty() && rev_.empty()) return rc;
  const auto t0 = std::chrono::steady_clock::now();
  const QuicFecGroup::LaunchProfile before = QuicFecGroup::launch_profile();
  enc_live_.swap(enc_);
  rev_live_.swap(rev_);
  // (the service takes a mapped batch of up to 64 groups: qfec_capi.cpp kSvcGroups)
  last_turn_small_ = (enc_live_.size() >= 1u && enc_live_.size() <= 64u) ||
                     (rev_live_.size() >= 1u && rev_live_.size() <= 64u);
  std::vector<QuicFecGroup*>& gs = launch_groups_;  // keeps its capacity
  gs.clear();
  for (EncodeItem& e : enc_live_) gs.push_back(e.group.get());
  const int erc = QuicFecGroup::Launch(ctx_, gs, &enc_pending_, /*async=*/true);
  gs.clear();
  for (ReviveItem& e : rev_live_) gs.push_back(e.group.get());
  const int rrc = QuicFecGroup::Launch(ctx_, gs, &rev_pending_, /*async=*/true);
  ++stats_.launches;
  const double us =
      std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  stats_.launch_us += us;
  stats_.launch_us_max = std::max(stats_.launch_us_max, us);
  const QuicFecGroup::LaunchProfile& after = QuicFecGroup::launch_profile();
  stats_.tables_us += after.tables_us - before.tables_us;
  stats_.call_us += after.call_us - before.call_us;
  return erc ? erc : rrc;
}

int QuicFecBatcher::Complete(bool wait) {
  if (!InFlight()) return QFEC_OK;
  // each launch completes on its own ticket (its own code)
  const auto t0 = std::chrono::steady_clock::now();
  auto spent = [&] {
    stats_.complete_us += std::chrono::duration<double, std::micro>(
                              std::chrono::steady_clock::now() - t0).count();
  };
  // poll first; a blocking wait for the device is timed on its own (wait_us:
  // the GPU's latency, not connection-thread work)
  auto finish = [&](QuicFecGroup::Pending* p) {
    int r = QuicFecGroup::Finish(p, false);
    if (r == QFEC_PENDING && wait) {
      const auto w0 = std::chrono::steady_clock::now();
      r = QuicFecGroup::Finish(p, true);
      stats_.wait_us += std::chrono::duration<double, std::micro>(
                            std::chrono::steady_clock::now() - w0).count();
    }
    return r;
  };
  const int erc = finish(&enc_pending_);
  if (erc == QFEC_PENDING) return spent(), QFEC_PENDING;
  const int rrc = finish(&rev_pending_);
  if (rrc == QFEC_PENDING) return spent(), QFEC_PENDING;  // enc_pending_ keeps its result
  spent();
  // callbacks may add new work (an emitted FEC packet lets the next packets
  // out, which may close the next group): hand over local copies
  std::vector<EncodeItem> enc;
  std::vector<ReviveItem> rev;
  enc.swap(enc_live_);
  rev.swap(rev_live_);
  for (EncodeItem& e : enc) {
    if (!e.v) continue;
    StringPiece red;
    const bool ok = erc == QFEC_OK;
    if (ok) red = e.group->PayloadParity();
    ok ? ++stats_.groups_encoded : ++stats_.groups_failed;
    e.v->OnFecRedundancy(e.header, red, ok);
  }
  // revived packets, grouped per visitor in the order added
  std::vector<QuicFecReviveBatch::Revived> out;
  for (size_t i = 0; i < rev.size();) {
    Visitor* v = rev[i].v;
    size_t j = i;
    out.clear();
    for (; j < rev.size() && rev[j].v == v; ++j) {
      if (rrc != QFEC_OK) {
        ++stats_.groups_failed;
        continue;
      }
      QuicFecReviveBatch::Revived r;
      r.tag = v;
      if (rev[j].group->ReviveInPlace(&r.header, &r.payload) == 0) continue;
      r.level = rev[j].group->EffectiveEncryptionLevel();
      out.push_back(r);
      ++stats_.groups_revived;
    }
    if (v && !out.empty()) v->OnRevivedPackets(out);
    i = j;
  }
  return erc ? erc : rrc;
}

int QuicFecBatcher::Flush() {
  const int lrc = Launch();
  const int crc = Complete(true);
  return lrc ? lrc : crc;
}

}  // namespace net
