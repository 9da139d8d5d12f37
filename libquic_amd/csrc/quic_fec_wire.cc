// quic_fec_wire.cc — see quic_fec_wire.h.
#include "quic_fec_wire.h"

#include <cstring>

namespace net {

size_t WriteFecPrivateHeader(const FecHeaderFields& f, uint8_t* buf, size_t cap) {
  if (f.fec_flag && !f.in_fec_group) return 0;  // an FEC packet always names its group
  const size_t need = f.in_fec_group ? 2 : 1;
  if (cap < need) return 0;
  uint8_t flags = PACKET_PRIVATE_FLAGS_NONE;
  if (f.entropy_flag) flags |= PACKET_PRIVATE_FLAGS_ENTROPY;
  if (f.in_fec_group) flags |= PACKET_PRIVATE_FLAGS_FEC_GROUP;
  if (f.fec_flag) flags |= PACKET_PRIVATE_FLAGS_FEC;
  buf[0] = flags;
  if (f.in_fec_group) buf[1] = f.fec_group_offset;
  return need;
}

size_t ParseFecPrivateHeader(const uint8_t* buf, size_t len, int quic_version,
                             QuicPacketNumber packet_number, FecHeaderFields* out,
                             std::string* detailed_error) {
  if (len < 1) {
    *detailed_error = "Unable to read private flags.";
    return 0;
  }
  const uint8_t flags = buf[0];
  const uint8_t max =
      quic_version > kQuicVersion31 ? PACKET_PRIVATE_FLAGS_MAX_VERSION_32 : PACKET_PRIVATE_FLAGS_MAX;
  if (flags > max) {
    *detailed_error = "Illegal private flags value.";
    return 0;
  }
  FecHeaderFields f;
  f.entropy_flag = (flags & PACKET_PRIVATE_FLAGS_ENTROPY) != 0;
  f.fec_flag = (flags & PACKET_PRIVATE_FLAGS_FEC) != 0;
  f.in_fec_group = (flags & PACKET_PRIVATE_FLAGS_FEC_GROUP) != 0;
  size_t used = 1;
  if (f.in_fec_group) {
    if (len < 2) {
      *detailed_error = "Unable to read first fec protected packet offset.";
      return 0;
    }
    f.fec_group_offset = buf[1];
    if (f.fec_group_offset >= packet_number) {
      *detailed_error =
          "First fec protected packet offset must be less than the packet number.";
      return 0;
    }
    used = 2;
  }
  *out = f;
  return used;
}

void ApplyFecHeader(const FecHeaderFields& f, QuicPacketHeader* header) {
  header->entropy_flag = f.entropy_flag;
  header->fec_flag = f.fec_flag;
  header->is_in_fec_group = f.in_fec_group ? IN_FEC_GROUP : NOT_IN_FEC_GROUP;
  header->fec_group = f.in_fec_group ? header->packet_number - f.fec_group_offset : 0;
}

size_t WriteRevivedPackets(const std::vector<QuicPacketNumber>& revived,
                           size_t packet_number_length, uint8_t* buf, size_t cap) {
  if (revived.size() > 255 || packet_number_length < 1 || packet_number_length > 8) return 0;
  const size_t need = kNumberOfRevivedPacketsSize + revived.size() * packet_number_length;
  if (cap < need) return 0;
  buf[0] = static_cast<uint8_t>(revived.size());
  size_t o = 1;
  for (QuicPacketNumber p : revived) {
    if (packet_number_length < 8 && (p >> (8 * packet_number_length)) != 0) return 0;
    for (size_t b = 0; b < packet_number_length; ++b) buf[o++] = static_cast<uint8_t>(p >> (8 * b));
  }
  return o;
}

size_t ParseRevivedPackets(const uint8_t* buf, size_t len, size_t packet_number_length,
                           std::vector<QuicPacketNumber>* revived, std::string* detailed_error) {
  if (len < kNumberOfRevivedPacketsSize) {
    *detailed_error = "Unable to read num revived packets.";
    return 0;
  }
  const size_t n = buf[0];
  size_t o = 1;
  revived->clear();
  for (size_t i = 0; i < n; ++i) {
    if (o + packet_number_length > len) {
      *detailed_error = "Unable to read revived packet.";
      return 0;
    }
    QuicPacketNumber p = 0;
    for (size_t b = 0; b < packet_number_length; ++b)
      p |= static_cast<QuicPacketNumber>(buf[o++]) << (8 * b);
    revived->push_back(p);
  }
  return o;
}

size_t SerializeFecPacketBody(QuicPacketNumber packet_number, QuicFecGroupNumber fec_group,
                              bool entropy_flag, StringPiece redundancy, uint8_t* buf,
                              size_t cap) {
  if (fec_group == 0 || fec_group > packet_number || packet_number - fec_group > 255) return 0;
  if (redundancy.size() > kMaxPacketSize) return 0;
  FecHeaderFields f;
  f.entropy_flag = entropy_flag;
  f.fec_flag = true;
  f.in_fec_group = true;
  f.fec_group_offset = static_cast<uint8_t>(packet_number - fec_group);
  const size_t h = WriteFecPrivateHeader(f, buf, cap);
  if (h == 0 || cap - h < redundancy.size()) return 0;
  std::memcpy(buf + h, redundancy.data(), redundancy.size());
  return h + redundancy.size();
}

}  // namespace net
