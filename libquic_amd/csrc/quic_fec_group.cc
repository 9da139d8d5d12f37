// quic_fec_group.cc — GPU-backed QuicFecGroup (see quic_fec_group.h).
//
// Group bookkeeping follows the historical QuicFecGroup contract (SURVEY.md
// §8(a) rows a1/a2, Appendix A); all payload XOR runs in the gfx950 ragged
// kernel through qfec_encode_ragged (one launch for one group, or for every
// group handed to ComputeAll).
#include "quic_fec_group.h"

#include <algorithm>
#include <cstring>
#include <limits>

namespace net {
namespace {

struct ThreadCtx {
  qfec_ctx* ctx = nullptr;
  ~ThreadCtx() {
    if (ctx) qfec_destroy(ctx);
  }
};

qfec_ctx* thread_default_ctx() {
  static thread_local ThreadCtx t;
  if (!t.ctx) t.ctx = qfec_create(0);
  return t.ctx;
}

}  // namespace

QuicFecGroup::QuicFecGroup(QuicFecGroupNumber fec_group_number, qfec_ctx* ctx)
    : fec_group_number_(fec_group_number), ctx_(ctx) {}

QuicFecGroup::~QuicFecGroup() = default;

qfec_ctx* QuicFecGroup::context() const { return ctx_ ? ctx_ : thread_default_ctx(); }

bool QuicFecGroup::Fold(StringPiece payload, bool completes_group) {
  if (payload.size() > kMaxPacketSize) {
    detailed_error_ = "Illegal payload size: " + std::to_string(payload.size());
    return false;
  }
  if (payload.empty()) return true;  // XOR of nothing
  if (lens_.size() >= QFEC_MAX_GROUP_PACKETS) {
    // A group spans 256 packet numbers (uint8 offset 0..255): 255 data
    // packets + the FEC packet.  The 256th payload can only arrive when it
    // completes the group, which then has nothing to revive; it is not kept.
    if (completes_group) {
      unkept_payload_ = true;
      return true;
    }
    detailed_error_ = "FEC group holds more than 255 payloads";
    return false;
  }
  bytes_.insert(bytes_.end(), payload.data(), payload.data() + payload.size());
  lens_.push_back(static_cast<uint16_t>(payload.size()));
  dirty_ = true;
  return true;
}

bool QuicFecGroup::Update(EncryptionLevel encryption_level, const QuicPacketHeader& header,
                          StringPiece decrypted_payload) {
  if (received_packets_.count(header.packet_number) != 0) return false;
  if (min_protected_packet_ != kInvalidPacketNumber &&
      max_protected_packet_ != kInvalidPacketNumber &&
      (header.packet_number < min_protected_packet_ ||
       header.packet_number > max_protected_packet_)) {
    detailed_error_ = "FEC group does not cover received packet: " +
                      std::to_string(header.packet_number);
    return false;
  }
  const bool completes = min_protected_packet_ != kInvalidPacketNumber &&
                         received_packets_.size() + 1 ==
                             max_protected_packet_ - min_protected_packet_ + 1;
  if (!Fold(decrypted_payload, completes)) return false;
  received_packets_.insert(header.packet_number);
  if (encryption_level < effective_encryption_level_)
    effective_encryption_level_ = encryption_level;
  return true;
}

bool QuicFecGroup::UpdateFec(EncryptionLevel encryption_level, const QuicPacketHeader& header,
                             StringPiece redundancy) {
  if (min_protected_packet_ != kInvalidPacketNumber) return false;  // redundancy already seen
  const QuicPacketNumber fec_packet_number = header.packet_number;
  if (fec_packet_number <= fec_group_number_ ||
      fec_packet_number - fec_group_number_ > QFEC_MAX_GROUP_PACKETS) {
    detailed_error_ = "FEC packet number outside the group's uint8 offset range";
    return false;
  }
  for (QuicPacketNumber p : received_packets_) {
    if (p < fec_group_number_ || p >= fec_packet_number) {
      detailed_error_ = "FEC group does not cover received packet: " + std::to_string(p);
      return false;
    }
  }
  const bool completes = received_packets_.size() == fec_packet_number - fec_group_number_;
  if (!Fold(redundancy, completes)) return false;
  min_protected_packet_ = fec_group_number_;
  max_protected_packet_ = fec_packet_number - 1;
  if (encryption_level < effective_encryption_level_)
    effective_encryption_level_ = encryption_level;
  return true;
}

QuicPacketCount QuicFecGroup::NumMissingPackets() const {
  if (min_protected_packet_ == kInvalidPacketNumber)
    return std::numeric_limits<QuicPacketCount>::max();
  return (max_protected_packet_ - min_protected_packet_ + 1) - received_packets_.size();
}

bool QuicFecGroup::CanRevive() const { return NumMissingPackets() == 1; }

bool QuicFecGroup::IsFinished() const { return NumMissingPackets() == 0; }

bool QuicFecGroup::IsWaitingForPacketBefore(QuicPacketNumber num) const {
  // Entire range is larger than the threshold.
  if (min_protected_packet_ != kInvalidPacketNumber && min_protected_packet_ >= num) return false;
  // The group is anchored at fec_group_number_: nothing below it is protected.
  if (fec_group_number_ >= num) return false;
  return true;
}

int QuicFecGroup::EnsureParity() const {
  if (!dirty_) return QFEC_OK;
  std::vector<QuicFecGroup*> one{const_cast<QuicFecGroup*>(this)};
  return ComputeAll(context(), one);
}

StringPiece QuicFecGroup::PayloadParity() const {
  if (unkept_payload_) {
    detailed_error_ = "finished group of 256 payloads: its accumulator was not kept";
    return StringPiece();
  }
  if (EnsureParity() != QFEC_OK) return StringPiece();
  return StringPiece(reinterpret_cast<const char*>(parity_.data()), payload_parity_len_);
}

size_t QuicFecGroup::Revive(QuicPacketHeader* header, char* decrypted_payload, size_t len) {
  if (!CanRevive()) return 0;
  QuicPacketNumber missing = kInvalidPacketNumber;
  for (QuicPacketNumber i = min_protected_packet_; i <= max_protected_packet_; ++i) {
    if (received_packets_.count(i) == 0) {
      missing = i;
      break;
    }
  }
  if (missing == kInvalidPacketNumber) return 0;
  if (EnsureParity() != QFEC_OK) return 0;
  if (payload_parity_len_ > len) {
    detailed_error_ = "revive buffer smaller than the redundancy";
    return 0;
  }
  std::memcpy(decrypted_payload, parity_.data(), payload_parity_len_);
  header->packet_number = missing;
  header->entropy_flag = false;  // unknown entropy
  header->fec_flag = false;
  header->is_in_fec_group = IN_FEC_GROUP;
  header->fec_group = fec_group_number_;
  received_packets_.insert(missing);
  return payload_parity_len_;
}

int QuicFecGroup::ComputeAll(qfec_ctx* ctx, const std::vector<QuicFecGroup*>& groups) {
  std::vector<QuicFecGroup*> work;
  for (QuicFecGroup* g : groups)
    if (g && g->dirty_) work.push_back(g);
  if (work.empty()) return QFEC_OK;
  if (!ctx) ctx = thread_default_ctx();
  if (!ctx) {
    for (QuicFecGroup* g : work) g->detailed_error_ = qfec_last_error(nullptr);
    return QFEC_ERR_INTERNAL;
  }
  // Ragged CSR over every folded payload of every group, addressed IN PLACE:
  // the C-ABI takes one base pointer plus 64-bit offsets, so the base is the
  // lowest of the groups' payload buffers and each packet's offset is its
  // distance from it (likewise for the parity accumulators).  The host path
  // of qfec_encode_ragged gathers straight from the groups into its pinned
  // staging — no intermediate copy here.
  size_t npk = 0;
  std::vector<QuicFecGroup*> launched;
  launched.reserve(work.size());
  uintptr_t in_base = UINTPTR_MAX, out_base = UINTPTR_MAX;
  for (QuicFecGroup* g : work) {
    if (g->lens_.empty()) {  // only empty payloads folded: parity is empty
      g->payload_parity_len_ = 0;
      g->parity_.clear();
      g->dirty_ = false;
      continue;
    }
    g->parity_.resize(kMaxPacketSize);
    in_base = std::min(in_base, reinterpret_cast<uintptr_t>(g->bytes_.data()));
    out_base = std::min(out_base, reinterpret_cast<uintptr_t>(g->parity_.data()));
    npk += g->lens_.size();
    launched.push_back(g);
  }
  if (launched.empty()) return QFEC_OK;
  std::vector<uint64_t> pkt_off;
  pkt_off.reserve(npk);
  std::vector<uint16_t> pkt_len;
  pkt_len.reserve(npk);
  std::vector<uint32_t> grp_ptr(1, 0);
  grp_ptr.reserve(launched.size() + 1);
  std::vector<uint64_t> parity_off;
  parity_off.reserve(launched.size());
  for (QuicFecGroup* g : launched) {
    uint64_t o = reinterpret_cast<uintptr_t>(g->bytes_.data()) - in_base;
    for (uint16_t l : g->lens_) {
      pkt_off.push_back(o);
      pkt_len.push_back(l);
      o += l;
    }
    grp_ptr.push_back(static_cast<uint32_t>(pkt_len.size()));
    parity_off.push_back(reinterpret_cast<uintptr_t>(g->parity_.data()) - out_base);
  }
  std::vector<uint16_t> plen(launched.size(), 0);
  int rc = qfec_encode_ragged(ctx, reinterpret_cast<const uint8_t*>(in_base), pkt_off.data(),
                              pkt_len.data(), grp_ptr.data(), launched.size(),
                              reinterpret_cast<uint8_t*>(out_base), parity_off.data(),
                              plen.data(), QFEC_PTR_HOST);
  if (rc != QFEC_OK) {
    for (QuicFecGroup* g : launched) g->detailed_error_ = qfec_last_error(ctx);
    return rc;
  }
  for (size_t i = 0; i < launched.size(); ++i) {
    QuicFecGroup* g = launched[i];
    g->payload_parity_len_ = plen[i];
    g->parity_.resize(plen[i]);
    g->dirty_ = false;
  }
  return QFEC_OK;
}

}  // namespace net
