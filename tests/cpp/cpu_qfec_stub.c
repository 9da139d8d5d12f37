/* cpu_qfec_stub.c — TEST INFRASTRUCTURE ONLY (the sanitizer build of the host
 * C++).  A CPU restatement of the few qfec C-ABI entry
 * points the host bookkeeping calls (quic_fec_group.cc, quic_fec_connection.cc),
 * so that QuicFecGroup / the payload arena / QuicFecReceiver / the batcher can
 * run under AddressSanitizer + UndefinedBehaviorSanitizer on a machine with no
 * GPU.  Never linked into libqfec.so or anything the product loads: the real
 * entry points are libquic_amd/csrc/qfec_capi.cpp over the gfx950 kernels.
 *
 * Semantics follow include/qfec.h: qfec_encode_ragged XORs every packet of a
 * group into parity_out (zero padded to the longest packet, parity_len_out =
 * max len — the historical QuicFecGroup::UpdateParity, quic_fec_group.cc);
 * QFEC_ASYNC work completes at once and qfec_complete reports it done.
 */
#define _POSIX_C_SOURCE 200112L
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "qfec.h"

struct qfec_ctx {
  int fail;
};

static char g_err[256] = "";

qfec_ctx* qfec_create(int device) {
  (void)device;
  return (qfec_ctx*)calloc(1, sizeof(qfec_ctx));
}

void qfec_destroy(qfec_ctx* ctx) { free(ctx); }

const char* qfec_last_error(const qfec_ctx* ctx) {
  (void)ctx;
  return g_err;
}

int qfec_debug_fail_launches(qfec_ctx* ctx, int on) {
  if (!ctx) return QFEC_ERR_INTERNAL;
  ctx->fail = on;
  return QFEC_OK;
}

void* qfec_host_alloc(size_t bytes) {
  void* p = NULL;
  if (posix_memalign(&p, 64, bytes ? bytes : 1) != 0) return NULL;
  return p;
}

void qfec_host_free(void* p) { free(p); }

int qfec_complete(qfec_ctx* ctx, int wait) {
  (void)ctx;
  (void)wait;
  return QFEC_OK;
}

/* No resident worker on the CPU: nothing to warm. */
int qfec_service_warm(qfec_ctx* ctx) {
  (void)ctx;
  return QFEC_OK;
}

/* Work completes inside the call: nothing is ever queued. */
uint64_t qfec_async_ticket(const qfec_ctx* ctx) {
  (void)ctx;
  return 0;
}

int qfec_complete_ticket(qfec_ctx* ctx, uint64_t ticket, int wait) {
  (void)ctx;
  (void)ticket;
  (void)wait;
  strcpy(g_err, "unknown or already completed ticket");
  return QFEC_ERR_INTERNAL;
}

int qfec_encode_ragged(qfec_ctx* ctx, const uint8_t* bytes, const uint64_t* pkt_off,
                       const uint16_t* pkt_len, const uint32_t* grp_ptr, uint64_t n_groups,
                       uint8_t* parity_out, const uint64_t* parity_off,
                       uint16_t* parity_len_out, uint32_t flags) {
  (void)flags;
  if (!ctx) {
    strcpy(g_err, "null context");
    return QFEC_ERR_INTERNAL;
  }
  if (ctx->fail) {
    strcpy(g_err, "launch failed (qfec_debug_fail_launches)");
    return QFEC_ERR_INTERNAL;
  }
  for (uint64_t g = 0; g < n_groups; ++g) {
    uint16_t mx = 0;
    for (uint32_t p = grp_ptr[g]; p < grp_ptr[g + 1]; ++p)
      if (pkt_len[p] > mx) mx = pkt_len[p];
    uint8_t* o = parity_out + parity_off[g];
    memset(o, 0, mx);
    for (uint32_t p = grp_ptr[g]; p < grp_ptr[g + 1]; ++p) {
      const uint8_t* in = bytes + pkt_off[p];
      for (uint16_t j = 0; j < pkt_len[p]; ++j) o[j] ^= in[j];
    }
    parity_len_out[g] = mx;
  }
  return QFEC_OK;
}
