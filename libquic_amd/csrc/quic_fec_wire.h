// quic_fec_wire.h — the v<=31 FEC wire vestiges of libquic, restated so FEC
// packets produced by the GPU path can be framed and parsed (SURVEY.md §8(f)
// rank 1).  Host C++; no payload bytes are touched here.
//
//   * Private flags byte + 1-byte first_fec_protected_packet_offset:
//     write mirrors the v<=31 header that QuicFramer::ProcessAuthenticatedHeader
//     parses (quic_framer.cc:1102-1141); flag values quic_protocol.h:343-358.
//   * Ack-frame revived-packets list (v<=31): count byte + N packet numbers of
//     the largest-observed length, little-endian (quic_framer.cc:1477-1493
//     parse, :2307-2317 write; kNumberOfRevivedPacketsSize quic_framer.h:64-65).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "quic_fec_group.h"
#ifdef QFEC_WITH_LIBQUIC
#include "net/quic/core/quic_framer.h"
#endif

namespace net {

#ifndef QFEC_WITH_LIBQUIC
// Standalone build: the reference's values (a libquic build takes them from
// quic_protocol.h / quic_framer.h).
enum QuicPacketPrivateFlags : uint8_t {  // quic_protocol.h:343-358
  PACKET_PRIVATE_FLAGS_NONE = 0,
  PACKET_PRIVATE_FLAGS_ENTROPY = 1 << 0,
  PACKET_PRIVATE_FLAGS_FEC_GROUP = 1 << 1,
  PACKET_PRIVATE_FLAGS_FEC = 1 << 2,
  PACKET_PRIVATE_FLAGS_MAX = (1 << 3) - 1,
  PACKET_PRIVATE_FLAGS_MAX_VERSION_32 = (1 << 1) - 1,
};

const size_t kNumberOfRevivedPacketsSize = 1;  // quic_framer.h:64-65
#endif

const int kQuicVersion31 = 31;  // last version with FEC (quic_protocol.h:371-373)

struct FecHeaderFields {
  bool entropy_flag = false;
  bool fec_flag = false;      // payload is redundancy, not frames
  bool in_fec_group = false;  // payload is protected by a group
  uint8_t fec_group_offset = 0;  // packet_number - fec_group (first protected packet)
};

// Writes the private flags byte (+ offset byte when in a group).  Returns the
// bytes written, 0 if `cap` is too small or the fields are inconsistent
// (fec_flag without a group).
size_t WriteFecPrivateHeader(const FecHeaderFields& f, uint8_t* buf, size_t cap);

// Parses what WriteFecPrivateHeader wrote, with QuicFramer's checks: flags
// above the version's maximum are illegal (v > 31: only the entropy bit), the
// offset must be < packet_number.  Returns bytes consumed or 0 and sets
// *detailed_error (QUIC_INVALID_PACKET_HEADER in the framer).
size_t ParseFecPrivateHeader(const uint8_t* buf, size_t len, int quic_version,
                             QuicPacketNumber packet_number, FecHeaderFields* out,
                             std::string* detailed_error);

// Fills a QuicPacketHeader's FEC fields from parsed private flags.
void ApplyFecHeader(const FecHeaderFields& f, QuicPacketHeader* header);

// Ack-frame revived packets list.
size_t WriteRevivedPackets(const std::vector<QuicPacketNumber>& revived,
                           size_t packet_number_length, uint8_t* buf, size_t cap);
size_t ParseRevivedPackets(const uint8_t* buf, size_t len, size_t packet_number_length,
                           std::vector<QuicPacketNumber>* revived, std::string* detailed_error);

// Serialise a complete FEC packet body for the send side: private header
// (FEC | FEC_GROUP, offset = packet_number - fec_group) followed by the
// redundancy (QuicFecGroup::PayloadParity()).  Returns bytes written or 0.
size_t SerializeFecPacketBody(QuicPacketNumber packet_number, QuicFecGroupNumber fec_group,
                              bool entropy_flag, StringPiece redundancy, uint8_t* buf,
                              size_t cap);

}  // namespace net
