// quic_fec_group.h — C++ host mirror of libquic's (removed) QuicFecGroup,
// backed by the MI355X C-ABI (include/qfec.h).
//
// The reference snapshot no longer ships src/net/quic/quic_fec_group.{h,cc} or
// quic_fec_group_interface.{h,cc} (named only by /root/reference/Makefile:5332-5384);
// the surface below keeps the historical member names and meanings
//  so the two hook sites can call it unchanged:
//   send:    QuicPacketCreator::SerializePacket, after BuildDataPacket
//            (quic_packet_creator.cc:530) and before EncryptInPlace (:549):
//              group.Update(level, header, plaintext_after_header);
//              ... PayloadParity() when the group closes.
//   receive: QuicConnection::ProcessValidatedPacket (quic_connection.cc:1388-1392),
//            which today drops FEC packets:
//              header.fec_flag ? group.UpdateFec(level, header, redundancy)
//                              : group.Update(level, header, decrypted_payload);
//              if (group.CanRevive()) group.Revive(&header, buf, kMaxPacketSize);
//
// Difference in *where* the XOR runs: the historical class XORed every payload
// into a 1452-byte accumulator on the connection thread.  Here a group only
// keeps the payload bytes; the XOR runs on the GPU, either for one group when
// PayloadParity()/Revive() is asked, or for many groups (across connections)
// in ONE ragged kernel launch via QuicFecGroup::ComputeAll().  Results are
// byte-identical; there is no CPU fallback — without a
// device the group reports failure.
//
// Where the payloads live: a per-thread arena of pinned, device-mapped host
// slabs (qfec_host_alloc), so ComputeAll hands the kernel the packets where
// Update() put them (QFEC_PTR_MAPPED: read in place over PCIe, no gather, no
// staging copy); the accumulators are written back into the same arena.  A
// slab is reused once every payload in it has been released.  Without mapped
// memory (no device) the arena falls back to ordinary heap slabs and
// ComputeAll stages through the context (QFEC_PTR_HOST).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <set>
#include <string>
#include <vector>

#include "qfec.h"  // include/qfec.h

#ifdef QFEC_WITH_LIBQUIC
// Built inside libquic, with integration/libquic_fec.patch applied: the
// reference's own types.  The patch restores the v<=31 group fields of
// QuicPacketHeader (is_in_fec_group, fec_group) and the QuicFecGroupNumber /
// InFecGroup declarations in quic_protocol.h.
#include "base/strings/string_piece.h"
#include "net/quic/core/quic_bandwidth.h"
#include "net/quic/core/quic_protocol.h"

namespace net {
using base::StringPiece;
#else
namespace net {

// Standalone build (no libquic headers): mirrors of the reference's types in
// quic_protocol.h, same names and values.  Never compiled together with the
// reference headers — a libquic build defines QFEC_WITH_LIBQUIC instead.
typedef uint64_t QuicPacketNumber;                 // quic_protocol.h:44
typedef QuicPacketNumber QuicFecGroupNumber;       // historical v<=31 header field
typedef uint64_t QuicPacketCount;                  // quic_bandwidth.h:21
const QuicPacketNumber kInvalidPacketNumber = 0;   // quic_protocol.h:752-753
const size_t kMaxPacketSize = QFEC_MAX_PACKET_SIZE;  // quic_protocol.h:66

enum EncryptionLevel : int8_t {  // quic_protocol.h:1173-1179
  ENCRYPTION_NONE = 0,
  ENCRYPTION_INITIAL = 1,
  ENCRYPTION_FORWARD_SECURE = 2,
  NUM_ENCRYPTION_LEVELS,
};

enum InFecGroup { NOT_IN_FEC_GROUP, IN_FEC_GROUP };  // historical v<=31 header field

// The FEC-relevant part of QuicPacketHeader (quic_protocol.h:756-770) plus the
// v<=31 group fields parsed by QuicFramer::ProcessAuthenticatedHeader
// (quic_framer.cc:1122-1137: fec_group = packet_number - offset).
struct QuicPacketHeader {
  QuicPacketNumber packet_number = 0;
  bool entropy_flag = false;
  bool fec_flag = false;
  InFecGroup is_in_fec_group = NOT_IN_FEC_GROUP;
  QuicFecGroupNumber fec_group = 0;
};

// Non-owning byte view (base::StringPiece).
struct StringPiece {
  const char* ptr = nullptr;
  size_t len = 0;
  StringPiece() = default;
  StringPiece(const char* p, size_t n) : ptr(p), len(n) {}
  StringPiece(const std::string& s) : ptr(s.data()), len(s.size()) {}  // NOLINT
  const char* data() const { return ptr; }
  size_t size() const { return len; }
  bool empty() const { return len == 0; }
};
#endif  // QFEC_WITH_LIBQUIC

// A vector whose first N elements live inside the object (trivially
// copyable T): a group's payload tables take no heap allocation up to N
// packets.  Thousands of groups are created and destroyed per event-loop turn
// at thousands of connections, and their small vector blocks, once freed,
// made the allocator consolidate for milliseconds at an unrelated later free
// (measured inside QuicFecBatcher::Launch, round 4).
template <typename T, size_t N>
class QfecSmallVec {
 public:
  QfecSmallVec() = default;
  QfecSmallVec(const QfecSmallVec&) = delete;
  QfecSmallVec& operator=(const QfecSmallVec&) = delete;
  ~QfecSmallVec() {
    if (p_ != in_) delete[] p_;
  }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T* data() { return p_; }
  const T* data() const { return p_; }
  T* begin() { return p_; }
  T* end() { return p_ + n_; }
  const T* begin() const { return p_; }
  const T* end() const { return p_ + n_; }
  T& operator[](size_t i) { return p_[i]; }
  const T& operator[](size_t i) const { return p_[i]; }
  void push_back(const T& v) {
    if (n_ == cap_) {
      const size_t c = cap_ * 2;
      T* q = new T[c];
      for (size_t i = 0; i < n_; ++i) q[i] = p_[i];
      if (p_ != in_) delete[] p_;
      p_ = q;
      cap_ = c;
    }
    p_[n_++] = v;
  }

 private:
  T in_[N];
  T* p_ = in_;
  size_t n_ = 0, cap_ = N;
};

// Layout guard.  QuicFecGroup and the structs a caller
// hands it are C++ objects exported from libqfec.so: a caller compiled against
// an older quic_fec_group.h allocates them with its own size and offsets, and
// the library's code then writes past them (round 4: a stale tool build
// corrupted its heap).  The caller's inline constructors store a tag of the
// layout THEY were compiled with as the objects' first word (offset 0 in any
// version); every library entry point compares it with the library's own tag
// and refuses a mismatch -- false / 0 / QFEC_ERR_INTERNAL, nothing touched,
// one line on stderr -- instead of corrupting memory.  Bump the version with
// any change to these classes' members.
#define QFEC_FEC_GROUP_LAYOUT_VERSION 5u
#define QFEC_FEC_GROUP_LAYOUT_TAG                                                        \
  ((uint64_t)sizeof(::net::QuicFecGroup) |                                             \
   ((uint64_t)alignof(::net::QuicFecGroup) << 20) |                                    \
   ((uint64_t)(sizeof(::net::QuicFecGroup::Pending) & 1023u) << 26) |                  \
   ((uint64_t)(sizeof(::net::QuicFecGroup::LaunchTables) & 1023u) << 36) |             \
   ((uint64_t)(sizeof(::net::QuicFecGroup::PacketBuffer) & 1023u) << 46) |             \
   ((uint64_t)QFEC_FEC_GROUP_LAYOUT_VERSION << 56))

class QuicFecGroup {
 public:
  // `ctx` may be null: a per-thread context on device 0 is created on first use.
  // Inline (caller-compiled): every member is initialised with the caller's
  // own layout, and the layout tag recorded first.
  explicit QuicFecGroup(QuicFecGroupNumber fec_group_number, qfec_ctx* ctx = nullptr)
      : layout_tag_(QFEC_FEC_GROUP_LAYOUT_TAG), fec_group_number_(fec_group_number), ctx_(ctx) {}
  // Inline too: the library releases the payloads only for a matching layout;
  // the members' destructors then run with the caller's layout.
  ~QuicFecGroup() { ReleaseStorage(); }
  QuicFecGroup(const QuicFecGroup&) = delete;
  QuicFecGroup& operator=(const QuicFecGroup&) = delete;

  // A data packet decrypted at `encryption_level`.  False if the packet was
  // already seen, lies outside the protected range, or its payload is longer
  // than kMaxPacketSize ("Illegal payload size").  The payload is copied into
  // the group's pinned payload arena.
  bool Update(EncryptionLevel encryption_level, const QuicPacketHeader& header,
              StringPiece decrypted_payload);

  // Zero-copy capture (send side): a buffer in the calling thread's pinned
  // payload arena, into which the packet creator serializes the whole packet
  // (header + frames) and from which it encrypts out of place; the group then
  // ADOPTS the buffer (UpdateInPlace) instead of copying the payload: the
  // connection thread's per-packet FEC cost is no longer a 1,350-B memcpy (or,
  // historically, a 1,350-B XOR) but a table entry.  Move-only; a buffer that
  // is not adopted is released on destruction.
  class PacketBuffer {
   public:
    PacketBuffer() = default;
    ~PacketBuffer();
    PacketBuffer(PacketBuffer&& o) noexcept;
    PacketBuffer& operator=(PacketBuffer&& o) noexcept;
    PacketBuffer(const PacketBuffer&) = delete;
    PacketBuffer& operator=(const PacketBuffer&) = delete;
    char* data() const { return reinterpret_cast<char*>(p_); }
    size_t size() const { return n_; }
    bool empty() const { return p_ == nullptr; }

   private:
    friend class QuicFecGroup;
    uint8_t* p_ = nullptr;
    void* slab_ = nullptr;
    size_t n_ = 0;
  };
  // n <= the arena slab size; an empty buffer when no arena memory is left
  // (or the caller's layout does not match the library's).
  static PacketBuffer AllocPacketBuffer(size_t n) {
    PacketBuffer b;
    AllocPacketBufferInto(n, QFEC_FEC_GROUP_LAYOUT_TAG, &b);
    return b;
  }
  // Update() for a payload at buf->data() + [offset, offset + len): on
  // success the group owns *buf (it is left empty), the payload is not copied.
  bool UpdateInPlace(EncryptionLevel encryption_level, const QuicPacketHeader& header,
                     PacketBuffer* buf, size_t offset, size_t len);
  // UpdateFec() for a redundancy at buf->data() + [offset, offset + len)
  // (receive side: the framer decrypted the packet into the arena buffer).
  bool UpdateFecInPlace(EncryptionLevel encryption_level, const QuicPacketHeader& header,
                        PacketBuffer* buf, size_t offset, size_t len);
  // The FEC packet: protects [fec_group_number, header.packet_number).  False if
  // a redundancy was already seen or a received packet is outside that range.
  bool UpdateFec(EncryptionLevel encryption_level, const QuicPacketHeader& header,
                 StringPiece redundancy);
  // Exactly one protected packet is missing and the redundancy is present.
  bool CanRevive() const;
  // Every protected packet has been received or revived.
  bool IsFinished() const;
  // Writes the missing packet (zero padded to the redundancy length) and
  // returns its length; 0 if it cannot be revived or `len` is too small.
  size_t Revive(QuicPacketHeader* header, char* decrypted_payload, size_t len);
  // Revive without a copy: *payload views the group's accumulator, valid while
  // the group lives and takes no further packets.  Same header and return
  // value as Revive().
  size_t ReviveInPlace(QuicPacketHeader* header, StringPiece* payload);
  // True if this group protects packets with numbers below `num`.
  bool IsWaitingForPacketBefore(QuicPacketNumber num) const;
  // XOR of every payload folded in so far (data and redundancy), zero padded;
  // on the send side this is the FEC packet's redundancy.  Computed on the GPU.
  StringPiece PayloadParity() const;
  QuicPacketCount NumReceivedPackets() const { return num_received_; }
  EncryptionLevel EffectiveEncryptionLevel() const { return effective_encryption_level_; }
  QuicFecGroupNumber FecGroupNumber() const { return fec_group_number_; }

  // Compute the accumulators of many groups in ONE ragged launch (the batch
  // path the GPU wants: groups from many connections).  Returns a qfec_*
  // code; afterwards PayloadParity()/Revive() of every group are free.
  static int ComputeAll(qfec_ctx* ctx, const std::vector<QuicFecGroup*>& groups);

  // ComputeAll in two halves, for an event loop that overlaps the GPU work
  // with its other work: Launch queues the ONE ragged launch (QFEC_ASYNC when
  // every payload sits in mapped arena memory, else it completes at once) and
  // Finish completes THAT launch (qfec_complete_ticket: its own code, not
  // another op's of the same context) and sets every group's parity.  The
  // groups must stay alive and take no packets in between.
  struct Pending {
    uint64_t layout_tag = QFEC_FEC_GROUP_LAYOUT_TAG;  // first: the layout guard
    qfec_ctx* ctx = nullptr;
    std::vector<QuicFecGroup*> launched;
    std::vector<uint16_t> plen;  // parity_len_out, filled at completion
    int rc = QFEC_OK;            // a synchronous failure at launch
    bool live = false;
    uint64_t ticket = 0;         // the queued launch (qfec_async_ticket)
  };
  static int Launch(qfec_ctx* ctx, const std::vector<QuicFecGroup*>& groups, Pending* p,
                    bool async);

  // The launch's index tables, built in Launch one group at a time (Append)
  // in one pass over the groups; reused across launches (cleared, capacity
  // kept).  A group must take no packets once appended (closed / collected
  // groups).
  struct LaunchTables {
    uint64_t layout_tag = QFEC_FEC_GROUP_LAYOUT_TAG;  // first: the layout guard
    std::vector<QuicFecGroup*> groups;
    std::vector<uint64_t> pkt_off;     // absolute payload addresses until the launch
    std::vector<uint16_t> pkt_len;
    std::vector<uint32_t> grp_ptr{0};
    std::vector<uint64_t> parity_off;  // absolute accumulator addresses until the launch
    uintptr_t in_base = UINTPTR_MAX, out_base = UINTPTR_MAX;
    bool mapped = true;
    int rc = QFEC_OK;  // an append failed (out of payload memory)
    void Clear();
    // false (and rc set) when the group's accumulator cannot be allocated;
    // a group with nothing to compute is finished here and not added
    bool Append(QuicFecGroup* g);
  };
  // Launch over prebuilt tables (cleared on return: the call stages them).
  static int Launch(qfec_ctx* ctx, LaunchTables* t, Pending* p, bool async);
  // wait: block; otherwise QFEC_PENDING while the work runs.  Returns the
  // launch's qfec_* code (also in every launched group's detailed_error).
  static int Finish(Pending* p, bool wait);

  // This thread's Launch time split (microseconds, accumulated): building the
  // CSR tables over the payloads, and the qfec_*_ragged call that queues the
  // launch (measurement: bench.py connection legs, tools/tune/host_cost.cc);
  // and its payload captures.
  struct LaunchProfile {
    double tables_us = 0;
    double call_us = 0;
    uint64_t launches = 0;
    uint64_t groups = 0;
    uint64_t packets = 0;
    // payload capture (Update / UpdateInPlace): copied into the arena, or
    // adopted in place (zero-copy send side)
    uint64_t payloads_copied = 0;
    uint64_t payload_bytes_copied = 0;
    uint64_t payloads_adopted = 0;
    // 32-MiB payload-arena slabs this thread allocated (pinned: a
    // hipHostMalloc each, milliseconds) -- growth inside a timed loop shows here
    uint64_t slabs_allocated = 0;
  };
  static LaunchProfile& launch_profile();

  // Detailed reason of the last failure (QuicFramer::detailed_error style).
  const std::string& detailed_error() const { return detailed_error_; }

 private:
  // Layout guard: true (and one line on stderr) when `tag` -- an object's
  // first word, written by the caller's inline constructor -- is not the
  // library's own layout tag.
  static bool StaleLayout(uint64_t tag);
  bool StaleLayout() const { return StaleLayout(layout_tag_); }
  static void AllocPacketBufferInto(size_t n, uint64_t caller_tag, PacketBuffer* out);
  void ReleaseStorage();
  bool Fold(StringPiece payload, bool completes_group, PacketBuffer* adopt = nullptr,
            size_t adopt_offset = 0);
  bool UpdateImpl(EncryptionLevel encryption_level, const QuicPacketHeader& header,
                  StringPiece payload, PacketBuffer* adopt, size_t adopt_offset);
  bool UpdateFecImpl(EncryptionLevel encryption_level, const QuicPacketHeader& header,
                     StringPiece redundancy, PacketBuffer* adopt, size_t adopt_offset);
  int EnsureParity() const;
  QuicPacketCount NumMissingPackets() const;
  qfec_ctx* context() const;

  // FIRST data member, at offset 0 in every layout version (the guard reads it
  // before trusting any other offset)
  uint64_t layout_tag_;
#ifdef QFEC_TEST_STALE_LAYOUT
  // test only (tests/cpp/test_layout_guard.cc): a caller whose header differs
  char stale_test_pad_[64] = {};
#endif
  QuicFecGroupNumber fec_group_number_;
  qfec_ctx* ctx_;
  // Received packet numbers: the 256 a group can span (uint8 offset from
  // fec_group_number_) as a bitmap; any other (only a malformed peer sends
  // one, refused later by UpdateFec as the historical class did) in a set.
  bool HasReceived(QuicPacketNumber n) const;
  void MarkReceived(QuicPacketNumber n);
  uint64_t recv_bits_[4] = {0, 0, 0, 0};
  std::set<QuicPacketNumber> recv_other_;
  size_t num_received_ = 0;
  QuicPacketNumber min_protected_packet_ = kInvalidPacketNumber;
  QuicPacketNumber max_protected_packet_ = kInvalidPacketNumber;
  EncryptionLevel effective_encryption_level_ = NUM_ENCRYPTION_LEVELS;
  // Folded payloads (data packets and redundancy) in the payload arena, with
  // their lengths; the GPU-computed accumulator (kMaxPacketSize bytes of arena,
  // valid when !dirty_).
  struct Span {
    uint8_t* p = nullptr;  // the arena allocation
    void* slab = nullptr;  // the arena slab holding p (released on destruction)
    size_t n = 0;
    uint8_t* data = nullptr;  // the payload: p, or inside p for an adopted packet buffer
  };
  static Span ArenaAlloc(size_t n);
  static void ArenaFree(Span* s);
  // up to kInlinePayloads payloads without a heap allocation (QfecSmallVec)
  static constexpr size_t kInlinePayloads = 16;
  QfecSmallVec<Span, kInlinePayloads> payloads_;
  QfecSmallVec<uint16_t, kInlinePayloads> lens_;
  // kept as payloads are folded, for Launch's table build
  QfecSmallVec<uint64_t, kInlinePayloads> addrs_;  // payload addresses (payloads_[i].data)
  uintptr_t min_data_ = UINTPTR_MAX;  // lowest payload address
  bool payloads_mapped_ = true;       // every payload in a device-mapped slab
  mutable Span parity_;
  mutable size_t payload_parity_len_ = 0;
  mutable bool dirty_ = false;
  bool unkept_payload_ = false;  // a 256th payload completed the group (Fold)
  mutable std::string detailed_error_;
};

}  // namespace net
