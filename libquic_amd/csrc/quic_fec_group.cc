// quic_fec_group.cc — GPU-backed QuicFecGroup (see quic_fec_group.h).
//
// Group bookkeeping follows the historical QuicFecGroup contract (SURVEY.md
// §8(a) rows a1/a2, Appendix A); all payload XOR runs in the gfx950 ragged
// kernel through qfec_encode_ragged (one launch for one group, or for every
// group handed to ComputeAll).
#include "quic_fec_group.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>

#if defined(__SANITIZE_ADDRESS__)
#include <sanitizer/asan_interface.h>
#define QFEC_POISON(p, n) ASAN_POISON_MEMORY_REGION((p), (n))
#define QFEC_UNPOISON(p, n) ASAN_UNPOISON_MEMORY_REGION((p), (n))
#else
#define QFEC_POISON(p, n) ((void)(p), (void)(n))
#define QFEC_UNPOISON(p, n) ((void)(p), (void)(n))
#endif

namespace net {
namespace {

// Per-thread bump allocator over slabs of pinned, device-mapped host memory
// (heap slabs when no device is present).  A slab is reused once everything
// allocated in it has been released; a thread's slabs go to a process-wide
// pool when the thread exits (its payloads may still be alive), and any
// thread takes a drained slab from the pool before allocating a new one, so
// the pinned footprint is bounded by the peak of live payloads, not by the
// number of threads that ever ran.  Under AddressSanitizer the free parts of
// a slab are poisoned: an access past a payload's own bytes is reported.
struct ArenaSlab {
  uint8_t* base = nullptr;
  size_t used = 0;
  std::atomic<size_t> live{0};  // bytes handed out and not yet released
  bool mapped = false;
};

class SlabPool {
 public:
  static SlabPool& Get() {
    static SlabPool* p = new SlabPool();  // never destroyed: outlives thread exits
    return *p;
  }
  void Put(std::vector<ArenaSlab*>* slabs) {
    std::lock_guard<std::mutex> l(mu_);
    slabs_.insert(slabs_.end(), slabs->begin(), slabs->end());
    slabs->clear();
  }
  ArenaSlab* TakeDrained() {
    std::lock_guard<std::mutex> l(mu_);
    for (size_t i = 0; i < slabs_.size(); ++i) {
      if (slabs_[i]->live.load(std::memory_order_acquire) == 0) {
        ArenaSlab* s = slabs_[i];
        slabs_[i] = slabs_.back();
        slabs_.pop_back();
        return s;
      }
    }
    return nullptr;
  }

 private:
  std::mutex mu_;
  std::vector<ArenaSlab*> slabs_;
};

class PayloadArena {
 public:
  static constexpr size_t kSlabBytes = 32u << 20;

  static PayloadArena& ForThread() {
    static thread_local PayloadArena a;
    return a;
  }

  ~PayloadArena() { SlabPool::Get().Put(&slabs_); }

  // n <= kSlabBytes; returns 16-byte aligned storage.
  uint8_t* Alloc(size_t n, ArenaSlab** slab) {
    const size_t r = (n + 15) & ~size_t(15);
    if (!cur_ || cur_->used + r > kSlabBytes) cur_ = NextSlab();
    if (!cur_) return nullptr;
    uint8_t* p = cur_->base + cur_->used;
    cur_->used += r;
    cur_->live.fetch_add(r, std::memory_order_relaxed);
    QFEC_UNPOISON(p, n);
    *slab = cur_;
    return p;
  }

  static void Release(ArenaSlab* slab, uint8_t* p, size_t n) {
    QFEC_POISON(p, n);
    slab->live.fetch_sub((n + 15) & ~size_t(15), std::memory_order_acq_rel);
  }

 private:
  ArenaSlab* NextSlab() {
    for (ArenaSlab* s : slabs_) {
      if (s != cur_ && s->live.load(std::memory_order_acquire) == 0) {
        s->used = 0;
        return s;
      }
    }
    if (ArenaSlab* s = SlabPool::Get().TakeDrained()) {
      s->used = 0;
      slabs_.push_back(s);
      return s;
    }
    ArenaSlab* s = new ArenaSlab();
    ++QuicFecGroup::launch_profile().slabs_allocated;
    if (mapped_ok_) {
      s->base = static_cast<uint8_t*>(qfec_host_alloc(kSlabBytes));
      s->mapped = s->base != nullptr;
      mapped_ok_ = s->mapped;  // no device: stop asking
    }
    if (!s->base) s->base = static_cast<uint8_t*>(std::malloc(kSlabBytes));
    if (!s->base) {
      delete s;
      return nullptr;
    }
    QFEC_POISON(s->base, kSlabBytes);
    slabs_.push_back(s);
    return s;
  }

  std::vector<ArenaSlab*> slabs_;
  ArenaSlab* cur_ = nullptr;
  bool mapped_ok_ = true;
};

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

// Layout guard (quic_fec_group.h): the caller's tag against this library's.
bool QuicFecGroup::StaleLayout(uint64_t tag) {
  constexpr uint64_t kMine = QFEC_FEC_GROUP_LAYOUT_TAG;
  if (tag == kMine) return false;
  static std::atomic<bool> said{false};
  if (!said.exchange(true))
    std::fprintf(stderr,
                 "libqfec: QuicFecGroup used by code built against a different "
                 "quic_fec_group.h (layout tag %016llx, library %016llx): refused "
                 "(QUIC_INTERNAL_ERROR); rebuild the caller\n",
                 (unsigned long long)tag, (unsigned long long)kMine);
  return true;
}

void QuicFecGroup::ReleaseStorage() {
  if (StaleLayout()) return;  // nothing of a foreign layout is touched
  for (Span& sp : payloads_) ArenaFree(&sp);
  ArenaFree(&parity_);
}

QuicFecGroup::Span QuicFecGroup::ArenaAlloc(size_t n) {
  Span sp;
  ArenaSlab* slab = nullptr;
  sp.p = PayloadArena::ForThread().Alloc(n, &slab);
  if (sp.p) {
    sp.slab = slab;
    sp.n = n;
    sp.data = sp.p;
  }
  return sp;
}

void QuicFecGroup::ArenaFree(Span* sp) {
  if (sp->p) PayloadArena::Release(static_cast<ArenaSlab*>(sp->slab), sp->p, sp->n);
  *sp = Span();
}

qfec_ctx* QuicFecGroup::context() const { return ctx_ ? ctx_ : thread_default_ctx(); }

QuicFecGroup::PacketBuffer::~PacketBuffer() {
  if (p_) PayloadArena::Release(static_cast<ArenaSlab*>(slab_), p_, n_);
}

QuicFecGroup::PacketBuffer::PacketBuffer(PacketBuffer&& o) noexcept
    : p_(o.p_), slab_(o.slab_), n_(o.n_) {
  o.p_ = nullptr;
  o.slab_ = nullptr;
  o.n_ = 0;
}

QuicFecGroup::PacketBuffer& QuicFecGroup::PacketBuffer::operator=(PacketBuffer&& o) noexcept {
  if (this != &o) {
    if (p_) PayloadArena::Release(static_cast<ArenaSlab*>(slab_), p_, n_);
    p_ = o.p_;
    slab_ = o.slab_;
    n_ = o.n_;
    o.p_ = nullptr;
    o.slab_ = nullptr;
    o.n_ = 0;
  }
  return *this;
}

void QuicFecGroup::AllocPacketBufferInto(size_t n, uint64_t caller_tag, PacketBuffer* b) {
  if (StaleLayout(caller_tag) || b == nullptr) return;
  const Span sp = ArenaAlloc(n);
  b->p_ = sp.p;
  b->slab_ = sp.slab;
  b->n_ = sp.p ? n : 0;
}

bool QuicFecGroup::Fold(StringPiece payload, bool completes_group, PacketBuffer* adopt,
                        size_t adopt_offset) {
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
  Span sp;
  if (adopt) {  // zero-copy: the payload already sits in arena memory
    sp.p = adopt->p_;
    sp.slab = adopt->slab_;
    sp.n = adopt->n_;
    sp.data = adopt->p_ + adopt_offset;
    adopt->p_ = nullptr;
    adopt->slab_ = nullptr;
    adopt->n_ = 0;
    ++launch_profile().payloads_adopted;
  } else {
    sp = ArenaAlloc(payload.size());
    if (!sp.p) {
      detailed_error_ = "out of payload memory";
      return false;
    }
    std::memcpy(sp.p, payload.data(), payload.size());
    LaunchProfile& prof = launch_profile();
    ++prof.payloads_copied;
    prof.payload_bytes_copied += payload.size();
  }
  payloads_.push_back(sp);
  lens_.push_back(static_cast<uint16_t>(payload.size()));
  addrs_.push_back(reinterpret_cast<uintptr_t>(sp.data));
  min_data_ = std::min(min_data_, reinterpret_cast<uintptr_t>(sp.data));
  payloads_mapped_ = payloads_mapped_ && static_cast<ArenaSlab*>(sp.slab)->mapped;
  dirty_ = true;
  return true;
}

bool QuicFecGroup::HasReceived(QuicPacketNumber n) const {
  const QuicPacketNumber d = n - fec_group_number_;
  if (n >= fec_group_number_ && d < 256) return (recv_bits_[d >> 6] >> (d & 63)) & 1;
  return recv_other_.count(n) != 0;
}

void QuicFecGroup::MarkReceived(QuicPacketNumber n) {
  const QuicPacketNumber d = n - fec_group_number_;
  if (n >= fec_group_number_ && d < 256)
    recv_bits_[d >> 6] |= 1ull << (d & 63);
  else
    recv_other_.insert(n);
  ++num_received_;
}

bool QuicFecGroup::Update(EncryptionLevel encryption_level, const QuicPacketHeader& header,
                          StringPiece decrypted_payload) {
  if (StaleLayout()) return false;
  return UpdateImpl(encryption_level, header, decrypted_payload, nullptr, 0);
}

bool QuicFecGroup::UpdateInPlace(EncryptionLevel encryption_level, const QuicPacketHeader& header,
                                 PacketBuffer* buf, size_t offset, size_t len) {
  if (StaleLayout()) return false;
  if (buf == nullptr || buf->empty() || offset > buf->size() || len > buf->size() - offset) {
    detailed_error_ = "payload outside its packet buffer";
    return false;
  }
  return UpdateImpl(encryption_level, header, StringPiece(buf->data() + offset, len), buf,
                    offset);
}

bool QuicFecGroup::UpdateImpl(EncryptionLevel encryption_level, const QuicPacketHeader& header,
                              StringPiece decrypted_payload, PacketBuffer* adopt,
                              size_t adopt_offset) {
  if (HasReceived(header.packet_number)) return false;
  if (min_protected_packet_ != kInvalidPacketNumber &&
      max_protected_packet_ != kInvalidPacketNumber &&
      (header.packet_number < min_protected_packet_ ||
       header.packet_number > max_protected_packet_)) {
    detailed_error_ = "FEC group does not cover received packet: " +
                      std::to_string(header.packet_number);
    return false;
  }
  const bool completes = min_protected_packet_ != kInvalidPacketNumber &&
                         num_received_ + 1 ==
                             max_protected_packet_ - min_protected_packet_ + 1;
  if (!Fold(decrypted_payload, completes, adopt, adopt_offset)) return false;
  MarkReceived(header.packet_number);
  if (encryption_level < effective_encryption_level_)
    effective_encryption_level_ = encryption_level;
  return true;
}

bool QuicFecGroup::UpdateFec(EncryptionLevel encryption_level, const QuicPacketHeader& header,
                             StringPiece redundancy) {
  if (StaleLayout()) return false;
  return UpdateFecImpl(encryption_level, header, redundancy, nullptr, 0);
}

bool QuicFecGroup::UpdateFecInPlace(EncryptionLevel encryption_level,
                                    const QuicPacketHeader& header, PacketBuffer* buf,
                                    size_t offset, size_t len) {
  if (StaleLayout()) return false;
  if (buf == nullptr || buf->empty() || offset > buf->size() || len > buf->size() - offset) {
    detailed_error_ = "redundancy outside its packet buffer";
    return false;
  }
  return UpdateFecImpl(encryption_level, header, StringPiece(buf->data() + offset, len), buf,
                       offset);
}

bool QuicFecGroup::UpdateFecImpl(EncryptionLevel encryption_level,
                                 const QuicPacketHeader& header, StringPiece redundancy,
                                 PacketBuffer* adopt, size_t adopt_offset) {
  if (min_protected_packet_ != kInvalidPacketNumber) return false;  // redundancy already seen
  const QuicPacketNumber fec_packet_number = header.packet_number;
  if (fec_packet_number <= fec_group_number_ ||
      fec_packet_number - fec_group_number_ > QFEC_MAX_GROUP_PACKETS) {
    detailed_error_ = "FEC packet number outside the group's uint8 offset range";
    return false;
  }
  // every received packet must lie in [fec_group_number_, fec_packet_number)
  QuicPacketNumber outside = kInvalidPacketNumber;
  if (!recv_other_.empty()) outside = *recv_other_.begin();
  const uint64_t span = fec_packet_number - fec_group_number_;  // 1..255
  for (uint64_t w = span >> 6; w < 4 && outside == kInvalidPacketNumber; ++w) {
    const uint64_t lo = w == (span >> 6) ? (span & 63) : 0;
    const uint64_t bits = lo == 64 ? 0 : recv_bits_[w] & (~0ull << lo);
    if (bits) outside = fec_group_number_ + 64 * w + __builtin_ctzll(bits);
  }
  if (outside != kInvalidPacketNumber) {
    detailed_error_ = "FEC group does not cover received packet: " + std::to_string(outside);
    return false;
  }
  const bool completes = num_received_ == span;
  if (!Fold(redundancy, completes, adopt, adopt_offset)) return false;
  min_protected_packet_ = fec_group_number_;
  max_protected_packet_ = fec_packet_number - 1;
  if (encryption_level < effective_encryption_level_)
    effective_encryption_level_ = encryption_level;
  return true;
}

QuicPacketCount QuicFecGroup::NumMissingPackets() const {
  if (min_protected_packet_ == kInvalidPacketNumber)
    return std::numeric_limits<QuicPacketCount>::max();
  return (max_protected_packet_ - min_protected_packet_ + 1) - num_received_;
}

bool QuicFecGroup::CanRevive() const { return !StaleLayout() && NumMissingPackets() == 1; }

bool QuicFecGroup::IsFinished() const { return !StaleLayout() && NumMissingPackets() == 0; }

bool QuicFecGroup::IsWaitingForPacketBefore(QuicPacketNumber num) const {
  if (StaleLayout()) return false;
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
  if (StaleLayout()) return StringPiece();
  if (unkept_payload_) {
    detailed_error_ = "finished group of 256 payloads: its accumulator was not kept";
    return StringPiece();
  }
  if (EnsureParity() != QFEC_OK) return StringPiece();
  return StringPiece(reinterpret_cast<const char*>(parity_.p), payload_parity_len_);
}

size_t QuicFecGroup::ReviveInPlace(QuicPacketHeader* header, StringPiece* payload) {
  if (StaleLayout()) return 0;
  if (!CanRevive()) return 0;
  QuicPacketNumber missing = kInvalidPacketNumber;
  for (QuicPacketNumber i = min_protected_packet_; i <= max_protected_packet_; ++i) {
    if (!HasReceived(i)) {
      missing = i;
      break;
    }
  }
  if (missing == kInvalidPacketNumber) return 0;
  if (EnsureParity() != QFEC_OK) return 0;
  *payload = StringPiece(reinterpret_cast<const char*>(parity_.p), payload_parity_len_);
  header->packet_number = missing;
  header->entropy_flag = false;  // unknown entropy
  header->fec_flag = false;
  header->is_in_fec_group = IN_FEC_GROUP;
  header->fec_group = fec_group_number_;
  MarkReceived(missing);
  return payload_parity_len_;
}

size_t QuicFecGroup::Revive(QuicPacketHeader* header, char* decrypted_payload, size_t len) {
  if (StaleLayout()) return 0;
  if (!CanRevive()) return 0;
  if (EnsureParity() != QFEC_OK) return 0;
  if (payload_parity_len_ > len) {
    detailed_error_ = "revive buffer smaller than the redundancy";
    return 0;
  }
  StringPiece view;
  const size_t n = ReviveInPlace(header, &view);
  if (n) std::memcpy(decrypted_payload, view.data(), n);
  return n;
}

int QuicFecGroup::ComputeAll(qfec_ctx* ctx, const std::vector<QuicFecGroup*>& groups) {
  Pending p;
  Launch(ctx, groups, &p, /*async=*/false);
  return Finish(&p, /*wait=*/true);
}

QuicFecGroup::LaunchProfile& QuicFecGroup::launch_profile() {
  static thread_local LaunchProfile p;
  return p;
}

void QuicFecGroup::LaunchTables::Clear() {
  groups.clear();
  pkt_off.clear();
  pkt_len.clear();
  grp_ptr.assign(1, 0);
  parity_off.clear();
  in_base = out_base = UINTPTR_MAX;
  mapped = true;
  rc = QFEC_OK;
}

bool QuicFecGroup::LaunchTables::Append(QuicFecGroup* g) {
  if (StaleLayout(layout_tag) || (g && g->StaleLayout())) return false;
  if (!g || !g->dirty_) return true;
  if (g->lens_.empty()) {  // only empty payloads folded: parity is empty
    g->payload_parity_len_ = 0;
    g->dirty_ = false;
    return true;
  }
  if (!g->parity_.p) {
    g->parity_ = ArenaAlloc(kMaxPacketSize);
    if (!g->parity_.p) {
      g->detailed_error_ = "out of payload memory";
      rc = QFEC_ERR_INTERNAL;
      return false;
    }
  }
  mapped = mapped && g->payloads_mapped_ && static_cast<ArenaSlab*>(g->parity_.slab)->mapped;
  in_base = std::min(in_base, g->min_data_);
  const uintptr_t par = reinterpret_cast<uintptr_t>(g->parity_.p);
  out_base = std::min(out_base, par);
  pkt_off.insert(pkt_off.end(), g->addrs_.begin(), g->addrs_.end());
  pkt_len.insert(pkt_len.end(), g->lens_.begin(), g->lens_.end());
  grp_ptr.push_back(static_cast<uint32_t>(pkt_len.size()));
  parity_off.push_back(par);
  groups.push_back(g);
  return true;
}

int QuicFecGroup::Launch(qfec_ctx* ctx, const std::vector<QuicFecGroup*>& groups, Pending* pend,
                         bool async) {
  if (pend == nullptr || StaleLayout(pend->layout_tag)) return QFEC_ERR_INTERNAL;
  for (QuicFecGroup* g : groups)
    if (g && g->StaleLayout()) {  // refused whole: no group of it is launched
      pend->ctx = nullptr;
      pend->launched.clear();
      pend->plen.clear();
      pend->live = false;
      pend->ticket = 0;
      return pend->rc = QFEC_ERR_INTERNAL;
    }
  // the tables built here, in one pass over the groups (a thread-local table
  // set, cleared per launch with its capacity kept)
  static thread_local LaunchTables t;
  t.Clear();
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t i = 0; i < groups.size(); ++i) {
    // prefetch: the group object 8 ahead, its address / length arrays 4 ahead
    if (i + 8 < groups.size() && groups[i + 8]) __builtin_prefetch(groups[i + 8]);
    if (i + 4 < groups.size() && groups[i + 4]) {
      const QuicFecGroup* nx = groups[i + 4];
      const char* a4 = reinterpret_cast<const char*>(nx->addrs_.data());
      for (size_t b = 0; b < nx->addrs_.size() * sizeof(uint64_t); b += 64)
        __builtin_prefetch(a4 + b);
      __builtin_prefetch(nx->lens_.data());
    }
    if (!t.Append(groups[i])) break;
  }
  launch_profile().tables_us +=
      std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  return Launch(ctx, &t, pend, async);
}

int QuicFecGroup::Launch(qfec_ctx* ctx, LaunchTables* t, Pending* pend, bool async) {
  if (t == nullptr || pend == nullptr || StaleLayout(t->layout_tag) ||
      StaleLayout(pend->layout_tag))
    return QFEC_ERR_INTERNAL;
  const auto t0 = std::chrono::steady_clock::now();
  // reset, keeping the vectors' capacity (a batcher's Pending is reused every
  // loop turn: no large block freed and reallocated per launch)
  pend->ctx = nullptr;
  pend->launched.clear();
  pend->plen.clear();
  pend->rc = QFEC_OK;
  pend->live = false;
  pend->ticket = 0;
  if (!ctx) ctx = thread_default_ctx();
  pend->ctx = ctx;
  if (t->rc != QFEC_OK) {  // an accumulator could not be allocated
    pend->rc = t->rc;
    for (QuicFecGroup* g : t->groups) g->detailed_error_ = "out of payload memory";
    pend->launched.assign(t->groups.begin(), t->groups.end());
    t->Clear();
    return pend->rc;
  }
  if (t->groups.empty()) {
    t->Clear();
    return QFEC_OK;
  }
  pend->launched.assign(t->groups.begin(), t->groups.end());
  if (!ctx) {
    for (QuicFecGroup* g : pend->launched) g->detailed_error_ = qfec_last_error(nullptr);
    t->Clear();
    return pend->rc = QFEC_ERR_INTERNAL;
  }
  // Ragged CSR over every folded payload of every group, addressed IN PLACE:
  // the C-ABI takes one base pointer plus 64-bit offsets, so the base is the
  // lowest payload address and each packet's offset is its distance from it
  // (likewise for the accumulators).  When every payload and accumulator sits
  // in a mapped arena slab the kernel reads and writes them where they are
  // (QFEC_PTR_MAPPED); otherwise the host path gathers them into the
  // context's pinned staging (QFEC_PTR_HOST).
  for (uint64_t& o : t->pkt_off) o -= t->in_base;
  for (uint64_t& o : t->parity_off) o -= t->out_base;
  const size_t ng = pend->launched.size(), npk = t->pkt_len.size();
  pend->plen.assign(ng, 0);
  const uint32_t flags =
      t->mapped ? (QFEC_PTR_MAPPED | (async ? QFEC_ASYNC : 0u)) : QFEC_PTR_HOST;
  const auto t1 = std::chrono::steady_clock::now();
  pend->rc = qfec_encode_ragged(ctx, reinterpret_cast<const uint8_t*>(t->in_base),
                                t->pkt_off.data(), t->pkt_len.data(), t->grp_ptr.data(), ng,
                                reinterpret_cast<uint8_t*>(t->out_base), t->parity_off.data(),
                                pend->plen.data(), flags);
  LaunchProfile& prof = launch_profile();
  const auto t2 = std::chrono::steady_clock::now();
  prof.tables_us += std::chrono::duration<double, std::micro>(t1 - t0).count();
  prof.call_us += std::chrono::duration<double, std::micro>(t2 - t1).count();
  ++prof.launches;
  prof.groups += ng;
  prof.packets += npk;
  pend->ticket = pend->rc == QFEC_OK ? qfec_async_ticket(ctx) : 0;
  pend->live = pend->ticket != 0;  // else it completed synchronously
  t->Clear();
  return pend->rc;
}

int QuicFecGroup::Finish(Pending* pend, bool wait) {
  if (pend == nullptr || StaleLayout(pend->layout_tag)) return QFEC_ERR_INTERNAL;
  if (pend->live) {
    const int rc = qfec_complete_ticket(pend->ctx, pend->ticket, wait ? 1 : 0);
    if (rc == QFEC_PENDING) return QFEC_PENDING;
    pend->rc = rc;
    pend->live = false;
  }
  if (pend->rc != QFEC_OK) {
    const char* why = qfec_last_error(pend->ctx);
    for (QuicFecGroup* g : pend->launched) g->detailed_error_ = why;
  } else {
    for (size_t i = 0; i < pend->launched.size(); ++i) {
      QuicFecGroup* g = pend->launched[i];
      g->payload_parity_len_ = pend->plen[i];
      g->dirty_ = false;
    }
  }
  pend->launched.clear();
  return pend->rc;
}

}  // namespace net
