// test_layout_guard.cc — the QuicFecGroup layout guard.
//
// Built with -DQFEC_TEST_STALE_LAYOUT, which adds a member to QuicFecGroup in
// THIS translation unit only: the code here plays a caller compiled against
// an older quic_fec_group.h, linked with the library's host sources compiled
// without it (libquic_amd/build.py SAN_TESTS, under AddressSanitizer).  Round
// 4's stale tools/tune/host_cost build corrupted its heap in exactly this
// situation; every library entry point must now refuse (false / 0 /
// QFEC_ERR_INTERNAL) and write nothing -- ASan would report any write past
// the caller's objects.  A control group built with the matching layout
// cannot exist in this TU by construction; the regular sanitizer tests are
// that control.
#include <cstdio>
#include <memory>
#include <string>
#include <vector>

#include "quic_fec_group.h"

#ifndef QFEC_TEST_STALE_LAYOUT
#error "build with -DQFEC_TEST_STALE_LAYOUT"
#endif

using namespace net;

static int g_fail = 0, g_checks = 0;
#define EXPECT(cond)                                                         \
  do {                                                                       \
    ++g_checks;                                                              \
    if (!(cond)) {                                                           \
      ++g_fail;                                                              \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);   \
    }                                                                        \
  } while (0)

int main() {
  qfec_ctx* ctx = qfec_create(0);
  std::string payload(1000, 'x');
  QuicPacketHeader h;
  h.packet_number = 5;
  h.is_in_fec_group = IN_FEC_GROUP;
  h.fec_group = 5;
  {
    // heap objects: ASan sees a write past the caller's allocation
    std::unique_ptr<QuicFecGroup> g(new QuicFecGroup(5, ctx));
    EXPECT(!g->Update(ENCRYPTION_NONE, h, StringPiece(payload)));
    h.fec_flag = true;
    h.packet_number = 7;
    EXPECT(!g->UpdateFec(ENCRYPTION_NONE, h, StringPiece(payload)));
    EXPECT(!g->CanRevive());
    EXPECT(!g->IsFinished());
    EXPECT(!g->IsWaitingForPacketBefore(100));
    EXPECT(g->PayloadParity().size() == 0);
    char buf[kMaxPacketSize];
    EXPECT(g->Revive(&h, buf, sizeof(buf)) == 0);
    StringPiece sp;
    EXPECT(g->ReviveInPlace(&h, &sp) == 0);
    std::vector<QuicFecGroup*> v{g.get()};
    EXPECT(QuicFecGroup::ComputeAll(ctx, v) == QFEC_ERR_INTERNAL);
    std::unique_ptr<QuicFecGroup::Pending> p(new QuicFecGroup::Pending());
    EXPECT(QuicFecGroup::Launch(ctx, v, p.get(), true) == QFEC_ERR_INTERNAL);
    EXPECT(QuicFecGroup::Finish(p.get(), true) == QFEC_ERR_INTERNAL);
    std::unique_ptr<QuicFecGroup::LaunchTables> t(new QuicFecGroup::LaunchTables());
    EXPECT(!t->Append(g.get()));
    EXPECT(QuicFecGroup::Launch(ctx, t.get(), p.get(), true) == QFEC_ERR_INTERNAL);
    QuicFecGroup::PacketBuffer b = QuicFecGroup::AllocPacketBuffer(1350);
    EXPECT(b.empty());
    EXPECT(!g->UpdateInPlace(ENCRYPTION_NONE, h, &b, 0, 0));
  }  // destructor: releases nothing of the foreign layout
  qfec_destroy(ctx);
  std::printf("%d checks, %d failures\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
