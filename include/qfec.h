/*
 * qfec.h — C-ABI of the MI355X-native QUIC forward-error-correction path.
 *
 * The boundary replaces libquic's FEC group (XOR parity encode + single-packet
 * revive).  The reference's implementation is absent from the snapshot
 * (/root/reference/Makefile:5332-5384 still lists the removed
 * src/net/quic/quic_fec_group.cc and quic_fec_group_interface.cc;
 * src/net/quic/core/quic_protocol.h:373 "FEC related fields are removed from
 * wire format"), so each entry point cites the historical member it replaces
 * and the in-tree hook site that called it:
 *
 *   qfec_encode_batch / _strided / qfec_encode_ragged
 *       replaces QuicFecGroup::UpdateParity + QuicFecGroupInterface::XorBuffers
 *       over every data packet of a group, then QuicFecGroup::PayloadParity().
 *       Send-side hook: QuicPacketCreator::SerializePacket between
 *       QuicFramer::BuildDataPacket and EncryptInPlace
 *       (src/net/quic/core/quic_packet_creator.cc:517-563, :530, :549).
 *   qfec_recover_batch / _strided / qfec_recover_ragged
 *       replaces QuicFecGroup::UpdateFec + Update(received) + CanRevive() +
 *       Revive().  Receive-side hook: QuicConnection::ProcessValidatedPacket
 *       "Drop any FEC packet." (src/net/quic/core/quic_connection.cc:1388-1392).
 *   qfec_xor_into
 *       replaces QuicFecGroupInterface::XorBuffers(input, size, output).
 *
 * Semantics: parity[j] = XOR over packets with
 * j < len_i of p_i[j]; parity_len = max len_i (zero padding, PADDING_FRAME = 0,
 * quic_protocol.h:259; quic_data_writer.cc:136-143).  Revive output is
 * parity_len bytes; bytes past the lost packet's own length are 0 and parse as
 * one PADDING frame (quic_framer.cc:1224-1231).
 *
 * Errors mirror the framer's bool + RaiseError(code) + detailed string
 * (quic_framer.cc:1128-1135): every call returns 0 on success or a negative
 * QuicErrorCode (quic_protocol.h:530-550); qfec_last_error() returns the
 * detailed string.  Nothing aborts.
 *
 * Ownership mirrors the reference's caller-owned ALIGNAS(64) packet buffers
 * (quic_framer.cc:573, quic_packet_creator.cc:351,401) and non-owning
 * StringPiece views: every buffer is borrowed for the duration of the call
 * (device-pointer calls: until the work queued on the context stream has
 * completed — see qfec_sync).  The context owns its device scratch, pinned
 * staging and streams; the library never frees caller memory.
 *
 * Threading: the reference connection is single-threaded
 * (quic_connection.h:14 "this class is not thread-safe"); a qfec_ctx is
 * likewise thread-compatible — one context per host thread / device, no global
 * locks on the hot path.
 */
#ifndef QFEC_H_
#define QFEC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QFEC_ABI_VERSION 1

/* Limits (quic_protocol.h:56, :66; quic_framer.cc:1126-1136). */
#define QFEC_DEFAULT_MAX_PACKET_SIZE 1350u /* kDefaultMaxPacketSize */
#define QFEC_MAX_PACKET_SIZE 1452u         /* kMaxPacketSize */
#define QFEC_MAX_GROUP_PACKETS 255u        /* uint8 first_fec_protected_packet_offset */

/* Return codes: 0 or -QuicErrorCode (quic_protocol.h). */
#define QFEC_OK 0
#define QFEC_ERR_INTERNAL (-1)         /* -QUIC_INTERNAL_ERROR: HIP failure, bad ctx */
#define QFEC_ERR_INVALID_FEC_DATA (-5) /* -QUIC_INVALID_FEC_DATA */

/* flags */
#define QFEC_PTR_DEVICE 0u  /* all buffer arguments are device pointers (default) */
#define QFEC_PTR_HOST 1u    /* all buffer arguments are host pointers: the call
                               stages through the context (pinned, chunked,
                               overlapped H2D / kernel / D2H) and returns when the
                               results are back in host memory */
#define QFEC_CACHED 2u      /* fixed-shape device calls: use the default cache
                               policy instead of non-temporal (nt) loads and
                               stores — for small batches whose output is
                               consumed straight away from L2 / MALL */
#define QFEC_PTR_MAPPED 4u  /* FEC calls (fixed, ragged, xor_into): the payload
                               buffers (rows / bytes, parity, parity_out / out) are
                               pinned, device-mapped host memory (qfec_host_alloc,
                               qfec_host_register, or any hipHostMalloc'd memory) that the
                               kernels read and write IN PLACE over PCIe — no
                               staging copy, the packets cross the link once; the
                               index arrays (pkt_off, pkt_len, grp_ptr, parity_off,
                               parity_len, missing_idx, out_off, parity_len_out)
                               are ordinary host memory, staged by the call.
                               Returns when the results are in host memory. */
#define QFEC_ONE_PASS 8u    /* fixed-shape device calls: always the one-pass
                               kernel.  Without it a large nt batch (>= 6 phases,
                               about 184K groups at L = 1350 on 256 CUs) runs the
                               phased kernel: one workgroup per CU, reads and
                               parity writes in separate grid-wide phases, which
                               keeps its rate independent of where the buffers
                               sit in the DRAM.  Same results either way. */
#define QFEC_ASYNC 16u      /* with QFEC_PTR_MAPPED, ragged calls: return as soon
                               as the work is queued (index arrays staged, kernel
                               launched) instead of when it is done; the outputs
                               (payload bytes and parity_len_out) are valid once
                               qfec_complete() has returned QFEC_OK, and every
                               buffer stays borrowed until then.  A batch whose
                               index tables exceed one staging slot (64 MiB) runs
                               synchronously.  Up to 3 calls may be in flight on
                               a context; any other call that stages through the
                               context completes them first.  Ignored by other
                               calls.  (The event-loop form: launch the turn's
                               FEC work, serve sockets, complete it next turn.) */
#define QFEC_SCRATCH_OUTPUT 32u /* decrypt / open calls (NULL, ChaCha20-Poly1305,
                               AES-128-GCM-12; device pointers): the output of a
                               packet whose tag fails may hold its unverified
                               plaintext (ok[p] = 0 still), so the kernel reads
                               the ciphertext once (hash and copy together)
                               instead of twice.  QuicFramer::DecryptPayload
                               decrypts into a scratch buffer, retries the
                               alternative decrypter into the same buffer and
                               drops the packet on failure
                               (quic_framer.cc:1884-1930), so this is a drop-in
                               for that caller; without the flag the output is
                               untouched on failure, as NullDecrypter leaves it
                               (crypto/null_decrypter.cc:57-62). */
#define QFEC_SMALL_GROUPS 64u /* ragged device calls (round 6): a hint that the
                                * batch's groups carry few payload bytes each
                                * (under ~4 KiB on average: short packets or
                                * k <= 4), so a large batch runs two groups per
                                * wave instead of eight per block (+8-14% there,
                                * DESIGN.md §4 band table).  Host-pointer and
                                * mapped batches choose by themselves (the host
                                * holds their tables); results are identical. */

/* qfec_complete() with wait == 0: the QFEC_ASYNC work is still running. */
#define QFEC_PENDING 1

typedef struct qfec_ctx qfec_ctx;

/* ---- context ---------------------------------------------------------- */
/* Create a context bound to HIP device `device`.  NULL on failure (no device,
 * HIP error); the reason is then available from qfec_last_error(NULL). */
qfec_ctx* qfec_create(int device);
void qfec_destroy(qfec_ctx* ctx);
/* Use an existing hipStream_t (e.g. torch's current stream) for device-pointer
 * calls; NULL is HIP's null (default) stream, as in the HIP API.  A new
 * context uses a non-blocking stream of its own, returned by
 * qfec_own_stream() (pass it back to restore it). */
int qfec_set_stream(qfec_ctx* ctx, void* hip_stream);
void* qfec_get_stream(qfec_ctx* ctx);
void* qfec_own_stream(qfec_ctx* ctx);
/* Wait for all queued work; returns the first error latched by a kernel
 * (e.g. a missing index >= k or a ragged length > kMaxPacketSize found on the
 * device) since the previous qfec_sync, then clears it. */
int qfec_sync(qfec_ctx* ctx);
/* Finish the context's QFEC_ASYNC calls in issue order.  wait != 0 blocks
 * until all are done; wait == 0 returns QFEC_PENDING while one is still
 * running.  Returns the first error of the calls it finished (the same codes
 * the synchronous call would have returned), else QFEC_OK. */
int qfec_complete(qfec_ctx* ctx, int wait);
/* The ticket of the last ragged call on this context if it was queued
 * asynchronously (QFEC_ASYNC honoured), else 0. */
uint64_t qfec_async_ticket(const qfec_ctx* ctx);
/* Finish ONE queued op: wait blocks, otherwise QFEC_PENDING while it runs.
 * Returns that op's own code only (an op finished early by another call --
 * its staging slot reused, a synchronous call -- keeps its code for this);
 * QFEC_ERR_INTERNAL for an unknown or already claimed ticket.  The codes of
 * the last 4096 tickets stay claimable once each, also after qfec_complete
 * finished their ops (which reports an op's error once, to one of the two). */
int qfec_complete_ticket(qfec_ctx* ctx, uint64_t ticket, int wait);
/* Small-batch service hint (round 5; no counterpart in the reference): make
 * sure the context's resident worker runs.  An event loop that calls it when
 * a turn starts collecting groups finds the worker resident at the turn's
 * flush instead of relaunching it there (the worker leaves after 100 us
 * without work; a relaunch costs the calling thread 3-5 us and the flush
 * ~20 us).  One load when the worker runs; a no-op with the service off.
 * Returns a qfec_* code (a failed launch turns the service off for the
 * context, as a failed relaunch in a batch call does). */
int qfec_service_warm(qfec_ctx* ctx);
const char* qfec_strerror(int code);
/* Pinned, device-mapped host memory for QFEC_PTR_MAPPED payloads (the
 * registered receive / send buffers of a QUIC server: the GPU reads packets
 * where the socket wrote them).  NULL on failure (qfec_last_error(NULL)). */
void* qfec_host_alloc(size_t bytes);
void qfec_host_free(void* p);
/* Pin and device-map EXISTING host memory [p, p + bytes) for QFEC_PTR_MAPPED
 * calls (e.g. a server's recvmmsg ring allocated by the application), the
 * registration counterpart of qfec_host_alloc; the memory stays the caller's.
 * The GPU addresses it at the same virtual address as the host (the mapped
 * calls pass pointers through unchanged); a platform where that is not so is
 * refused (QFEC_ERR_INTERNAL).  Unregister before freeing the memory. */
int qfec_host_register(void* p, size_t bytes);
int qfec_host_unregister(void* p);
const char* qfec_last_error(const qfec_ctx* ctx);
int qfec_abi_version(void);

/* ---- fixed-shape batches ---------------------------------------------- */
/* rows:    n_groups x k x L bytes, group g row i at rows + g*k*L + i*L
 * parity:  n_groups x L bytes
 * Encode:  parity[g] = XOR_i rows[g][i]. */
int qfec_encode_batch(qfec_ctx* ctx, const uint8_t* rows, uint32_t k, uint32_t L,
                      uint64_t n_groups, uint8_t* parity_out, uint32_t flags);

/* Recover: out[g] = parity[g] XOR_{i != missing[g]} rows[g][i].
 * rows[g][missing[g]] is never read (the lost packet's slot).  missing[g] < k. */
int qfec_recover_batch(qfec_ctx* ctx, const uint8_t* rows, const uint8_t* parity,
                       const uint8_t* missing_idx, uint32_t k, uint32_t L, uint64_t n_groups,
                       uint8_t* out, uint32_t flags);

/* In-slot recover: the receiver has written the FEC packet's redundancy
 * (L bytes) into row missing_idx[g] of group g -- the slot of the lost packet,
 * where the framer would have put it -- so the lost packet is the XOR of the
 * group's k rows.  The kernels then read ONE contiguous stream of k rows per
 * group (qfec_recover_batch reads k-1 rows around the lost row's hole plus a
 * separate parity stream); the same 14,850 B per group at 10 x 1350 B.
 *   out != NULL: out[g] = XOR_i rows[g][i]; missing_idx is not read (may be
 *                NULL); the rows are not written.  Any pointer mode (flags).
 *   out == NULL: in place, rows[g][missing_idx[g]] receives the lost packet
 *                (missing_idx[g] < k, else -QUIC_INVALID_FEC_DATA as
 *                qfec_recover_batch); device pointers only.  Applying it twice
 *                restores the redundancy.
 * Replaces the same historical QuicFecGroup::UpdateFec + Revive as
 * qfec_recover_batch, at the receive hook QuicConnection::ProcessValidatedPacket
 * (src/net/quic/core/quic_connection.cc:1388-1392). */
int qfec_recover_inslot_batch(qfec_ctx* ctx, uint8_t* rows, const uint8_t* missing_idx, uint32_t k,
                              uint32_t L, uint64_t n_groups, uint8_t* out, uint32_t flags);

/* Strided forms (padding study: row_stride >= L, group_stride >= k*row_stride,
 * parity/out strides >= L; all in bytes). */
int qfec_encode_batch_strided(qfec_ctx* ctx, const uint8_t* rows, uint32_t k, uint32_t L,
                              uint64_t row_stride, uint64_t group_stride, uint64_t n_groups,
                              uint8_t* parity_out, uint64_t parity_stride, uint32_t flags);
int qfec_recover_batch_strided(qfec_ctx* ctx, const uint8_t* rows, const uint8_t* parity,
                               const uint8_t* missing_idx, uint32_t k, uint32_t L,
                               uint64_t row_stride, uint64_t group_stride,
                               uint64_t parity_stride, uint64_t n_groups, uint8_t* out,
                               uint64_t out_stride, uint32_t flags);
int qfec_recover_inslot_batch_strided(qfec_ctx* ctx, uint8_t* rows, const uint8_t* missing_idx,
                                      uint32_t k, uint32_t L, uint64_t row_stride,
                                      uint64_t group_stride, uint64_t n_groups, uint8_t* out,
                                      uint64_t out_stride, uint32_t flags);

/* ---- ragged batches (CSR) ---------------------------------------------- */
/* Group g holds packets p in [grp_ptr[g], grp_ptr[g+1]) (1..255 of them);
 * packet p is pkt_len[p] (1..1452) bytes at bytes + pkt_off[p].
 * Encode writes parity_len_out[g] = max len and that many parity bytes at
 * parity_out + parity_off[g]. */
int qfec_encode_ragged(qfec_ctx* ctx, const uint8_t* bytes, const uint64_t* pkt_off,
                       const uint16_t* pkt_len, const uint32_t* grp_ptr, uint64_t n_groups,
                       uint8_t* parity_out, const uint64_t* parity_off,
                       uint16_t* parity_len_out, uint32_t flags);
/* Recover writes parity_len[g] bytes at out + out_off[g]:
 * parity XOR every received packet of the group (zero padded).  The lost
 * packet's pkt_off / pkt_len entries (index grp_ptr[g] + missing_idx[g]) are
 * never read.  Every received packet must satisfy len <= parity_len[g]. */
int qfec_recover_ragged(qfec_ctx* ctx, const uint8_t* bytes, const uint64_t* pkt_off,
                        const uint16_t* pkt_len, const uint32_t* grp_ptr, uint64_t n_groups,
                        const uint8_t* parity, const uint64_t* parity_off,
                        const uint16_t* parity_len, const uint8_t* missing_idx, uint8_t* out,
                        const uint64_t* out_off, uint32_t flags);

/* ---- single buffer ------------------------------------------------------ */
/* out[j] ^= in[j] for j < n (QuicFecGroupInterface::XorBuffers). */
int qfec_xor_into(qfec_ctx* ctx, const uint8_t* in, uint64_t n, uint8_t* out, uint32_t flags);

/* ---- v<=31 FEC wire format (host memory; no device involved) ----------- */
/* What an FFI user (e.g. a cgo binding) needs around the parity bytes:
 *   private flags byte + 1-byte first_fec_protected_packet_offset, with the
 *   checks of QuicFramer::ProcessAuthenticatedHeader (quic_framer.cc:1102-1141:
 *   flags above the version's maximum are illegal — v > 31 allows only the
 *   entropy bit, quic_protocol.h:343-358 — and the offset must be below the
 *   packet number; the group is packet_number - offset);
 *   the ack frame's revived-packets list (count byte + N packet numbers of the
 *   largest-observed length, little-endian: quic_framer.cc:1477-1493 read,
 *   :2307-2317 write, kNumberOfRevivedPacketsSize quic_framer.h:64-65);
 *   an FEC packet body: private header (FEC | FEC_GROUP, offset) + redundancy.
 * Each returns the bytes written / consumed, or 0 on failure with the
 * framer's detailed error string in qfec_last_error(NULL). */
typedef struct qfec_fec_header {
  uint8_t entropy_flag;     /* PACKET_PRIVATE_FLAGS_ENTROPY */
  uint8_t fec_flag;         /* PACKET_PRIVATE_FLAGS_FEC: the payload is redundancy */
  uint8_t in_fec_group;     /* PACKET_PRIVATE_FLAGS_FEC_GROUP: offset byte follows */
  uint8_t fec_group_offset; /* packet_number - first protected packet number */
} qfec_fec_header;

size_t qfec_wire_write_private_header(const qfec_fec_header* h, uint8_t* buf, size_t cap);
size_t qfec_wire_parse_private_header(const uint8_t* buf, size_t len, int quic_version,
                                      uint64_t packet_number, qfec_fec_header* out);
size_t qfec_wire_write_revived(const uint64_t* revived, size_t n, size_t packet_number_length,
                               uint8_t* buf, size_t cap);
/* Parses into revived[0 .. *n_out) (at most 255 entries: size the array so). */
size_t qfec_wire_parse_revived(const uint8_t* buf, size_t len, size_t packet_number_length,
                               uint64_t* revived, size_t* n_out);
size_t qfec_wire_fec_packet_body(uint64_t packet_number, uint64_t fec_group, int entropy_flag,
                                 const uint8_t* redundancy, size_t redundancy_len, uint8_t* buf,
                                 size_t cap);

/* ---- packet protection around FEC (ENCRYPTION_NONE) -------------------- */
/* The NULL packet protection libquic applies before the handshake completes:
 * a 12-byte FNV-1a-128 tag of header || payload written in front of the
 * payload.  Batched over a CSR layout (one lane per packet on the device):
 * packet p's associated data (its packet header) is ad_len[p] bytes at
 * bytes + ad_off[p]; its payload in_len[p] bytes at bytes + in_off[p].
 *
 * qfec_null_encrypt_batch replaces NullEncrypter::EncryptPacket
 *   (src/net/quic/core/crypto/null_encrypter.cc:28-47), called per packet by
 *   QuicPacketCreator::SerializePacket -> EncryptInPlace
 *   (quic_packet_creator.cc:549): out + out_off[p] receives in_len[p] + 12
 *   bytes, tag first.  out + out_off[p] may equal bytes + in_off[p] (in place,
 *   as EncryptInPlace does) or must not overlap any input.
 * qfec_null_decrypt_batch replaces NullDecrypter::DecryptPacket
 *   (crypto/null_decrypter.cc:38-64), called by QuicFramer::DecryptPayload
 *   (quic_framer.cc:1884): ok[p] = 1 and in_len[p] - 12 payload bytes at
 *   out + out_off[p] when the tag verifies; ok[p] = 0 and the output untouched
 *   when it does not (or in_len[p] < 12; with QFEC_SCRATCH_OUTPUT a failed
 *   packet's output holds its unverified plaintext).  Output must not overlap
 *   the input.
 * flags: QFEC_PTR_DEVICE / QFEC_PTR_HOST as above, QFEC_SCRATCH_OUTPUT. */
int qfec_null_encrypt_batch(qfec_ctx* ctx, const uint8_t* bytes, const uint64_t* ad_off,
                            const uint16_t* ad_len, const uint64_t* in_off,
                            const uint16_t* in_len, uint64_t n_packets, uint8_t* out,
                            const uint64_t* out_off, uint32_t flags);
int qfec_null_decrypt_batch(qfec_ctx* ctx, const uint8_t* bytes, const uint64_t* ad_off,
                            const uint16_t* ad_len, const uint64_t* in_off,
                            const uint16_t* in_len, uint64_t n_packets, uint8_t* out,
                            const uint64_t* out_off, uint8_t* ok, uint32_t flags);

/* ChaCha20-Poly1305 packet protection (the AEAD libquic negotiates, 12-byte
 * tags), batched like the NULL forms above.  Packet p is protected under key
 * key_idx[p]: keys holds 32 bytes per key, prefixes the 4-byte nonce prefix
 * per key; the 12-byte nonce is prefix || LE64(path_id[p] << 56 |
 * packet_number[p]) (path_id may be NULL: all 0).
 * qfec_chacha20poly1305_seal_batch replaces ChaCha20Poly1305Encrypter::
 *   EncryptPacket (AeadBaseEncrypter::EncryptPacket,
 *   src/net/quic/core/crypto/aead_base_encrypter.cc:107-134 -> BoringSSL
 *   EVP_aead_chacha20_poly1305): out + out_off[p] receives in_len[p] + 12
 *   bytes, ciphertext then tag; it may equal bytes + in_off[p] (in place).
 * qfec_chacha20poly1305_open_batch replaces ChaCha20Poly1305Decrypter::
 *   DecryptPacket (aead_base_decrypter.cc): ok[p] = 1 and in_len[p] - 12
 *   plaintext bytes at out + out_off[p] when the tag verifies; ok[p] = 0 and
 *   the output untouched otherwise.  Output must not overlap the input. */
int qfec_chacha20poly1305_seal_batch(qfec_ctx* ctx, const uint8_t* keys, const uint8_t* prefixes,
                                     const uint32_t* key_idx, const uint64_t* packet_number,
                                     const uint8_t* path_id, const uint8_t* bytes,
                                     const uint64_t* ad_off, const uint16_t* ad_len,
                                     const uint64_t* in_off, const uint16_t* in_len,
                                     uint64_t n_packets, uint8_t* out, const uint64_t* out_off,
                                     uint32_t flags);
int qfec_chacha20poly1305_open_batch(qfec_ctx* ctx, const uint8_t* keys, const uint8_t* prefixes,
                                     const uint32_t* key_idx, const uint64_t* packet_number,
                                     const uint8_t* path_id, const uint8_t* bytes,
                                     const uint64_t* ad_off, const uint16_t* ad_len,
                                     const uint64_t* in_off, const uint16_t* in_len,
                                     uint64_t n_packets, uint8_t* out, const uint64_t* out_off,
                                     uint8_t* ok, uint32_t flags);

/* AES-128-GCM packet protection (12-byte tags), same batch form as the
 * ChaCha20-Poly1305 calls above with 16-byte keys (keys holds 16 bytes per
 * key).  Replaces Aes128Gcm12Encrypter::EncryptPacket / Aes128Gcm12Decrypter::
 * DecryptPacket (crypto/aes_128_gcm_12_encrypter.cc -> AeadBaseEncrypter,
 * BoringSSL EVP_aead_aes_128_gcm).  Throughput is best when runs of 64
 * consecutive packets share a key (one GHASH table per wave); mixed-key runs
 * are correct but take a bit-serial GHASH. */
int qfec_aes128gcm_seal_batch(qfec_ctx* ctx, const uint8_t* keys, const uint8_t* prefixes,
                              const uint32_t* key_idx, const uint64_t* packet_number,
                              const uint8_t* path_id, const uint8_t* bytes, const uint64_t* ad_off,
                              const uint16_t* ad_len, const uint64_t* in_off,
                              const uint16_t* in_len, uint64_t n_packets, uint8_t* out,
                              const uint64_t* out_off, uint32_t flags);
int qfec_aes128gcm_open_batch(qfec_ctx* ctx, const uint8_t* keys, const uint8_t* prefixes,
                              const uint32_t* key_idx, const uint64_t* packet_number,
                              const uint8_t* path_id, const uint8_t* bytes, const uint64_t* ad_off,
                              const uint16_t* ad_len, const uint64_t* in_off,
                              const uint16_t* in_len, uint64_t n_packets, uint8_t* out,
                              const uint64_t* out_off, uint8_t* ok, uint32_t flags);

/* ---- packet-entropy bookkeeping (QUIC <= v33) --------------------------- */
/* The 1-byte entropy hashes the sender records per packet and checks acks
 * against, batched over connections.  Connection c
 * holds the hashes of its packets first_pn[c] .. first_pn[c] + n_c - 1 at
 * entropy[conn_ptr[c] .. conn_ptr[c+1]) — QuicSentEntropyManager's deque after
 * ClearEntropyBefore(first_pn[c]) — and cum_base[c] is the cumulative entropy
 * through first_pn[c] - 1 (NULL: 0).  A packet's hash is
 * entropy_flag << (packet_number % 8) (QuicFramer::GetPacketEntropyHash,
 * quic_framer.cc:351-354).
 *
 * qfec_entropy_cumulative_batch: cum[i] = cum_base[c] ^ entropy[conn_ptr[c]]
 *   ^ ... ^ entropy[i] — QuicSentEntropyManager::GetCumulativeEntropy for every
 *   packet (quic_sent_entropy_manager.cc:33-41, :57-66); with 0 for packets not
 *   received it is the receiver's EntropyTracker::EntropyHash
 *   (quic_received_packet_manager.cc:40-56).  n_packets = conn_ptr[n_conns] -
 *   conn_ptr[0] is a launch-shape hint (lanes per connection from the mean
 *   window); 0 = unknown.  It never changes the result.
 * qfec_entropy_validate_batch: ack a of connection ack_conn[a] with
 *   largest_observed[a], missing packets as the disjoint intervals
 *   [range_lo[r], range_hi[r]), r in range_ptr[a] .. range_ptr[a+1] (the
 *   PacketNumberQueue), and the claimed hash: ok[a] = IsValidEntropy(...)
 *   (quic_sent_entropy_manager.cc:68-96, called by QuicConnection::
 *   ValidateAckFrame, quic_connection.cc:854), given `cum` from the first call.
 *   Where the reference's behaviour is undefined — a missing packet above the
 *   largest recorded one, largest_observed below the window, ack_conn out of
 *   range — ok[a] = 0.  An invalid ack is a result (ok = 0), not an error. */
int qfec_entropy_cumulative_batch(qfec_ctx* ctx, const uint8_t* entropy, const uint64_t* conn_ptr,
                                  const uint8_t* cum_base, uint64_t n_conns, uint64_t n_packets,
                                  uint8_t* cum, uint32_t flags);
int qfec_entropy_validate_batch(qfec_ctx* ctx, const uint8_t* cum, const uint64_t* conn_ptr,
                                const uint64_t* first_pn, const uint8_t* cum_base,
                                uint64_t n_conns, const uint32_t* ack_conn,
                                const uint64_t* largest_observed, const uint8_t* claimed,
                                const uint32_t* range_ptr, const uint64_t* range_lo,
                                const uint64_t* range_hi, uint64_t n_acks, uint8_t* ok,
                                uint32_t flags);

/* ---- measurement support (bench.py, device pointers) ------------------- */
/* Streaming bandwidth probe over n bytes of src (n rounded down to 16):
 * mode 0 = read only (nt loads, XOR-folded; dst receives at most 16 bytes),
 * mode 1 = copy src -> dst (nt loads + nt stores).  The measured ceilings the
 * FEC kernels' rates are compared with. */
int qfec_stream_probe(qfec_ctx* ctx, const uint8_t* src, uint64_t n, uint8_t* dst, int mode);
/* Number of phased fixed-shape launches on this context that gave up their
 * grid-wide meetings (a workgroup waited > 200 us: the GPU shared with other
 * work, so not every workgroup was resident) and ran to the end without them
 * — same results, one-pass-like speed.  Waits for the context's stream. */
int qfec_phase_abandons(qfec_ctx* ctx, uint32_t* count);
/* Large fixed-shape batches left to run with the one-pass kernel because a
 * phased launch of this context was abandoned (the GPU is contended: the
 * context then uses the one-pass kernel for the next 16 such batches and
 * tries the phased one again).  -1 for a null context. */
int qfec_phase_backoff(qfec_ctx* ctx);
/* Which kernel the context's last device-pointer fixed-shape call ran: 1 the
 * phased kernel, 0 the one-pass kernel, -1 none yet (or a null context).
 * The measurement names its roofline kernel from this, not from a copy of
 * the library's size rule. */
int qfec_last_fixed_phased(const qfec_ctx* ctx);
/* Test hook: the workgroup count of the last device fixed-shape launch if it
 * ran phased (one per CU, less the CUs other contexts' resident small-batch
 * workers hold), else 0. */
uint32_t qfec_debug_last_phase_grid(const qfec_ctx* ctx);
/* Test hook: launch `extra` workgroups beyond one per CU in phased launches
 * (0..64; they cannot all be resident, so the first meeting times out — the
 * abandon path; the backoff does not apply while extra > 0), and with
 * reset_backoff clear the contention backoff (forgetting abandoned launches
 * so far).  Waits for the stream. */
int qfec_debug_phase(qfec_ctx* ctx, uint32_t extra, int reset_backoff);
/* Test hook: fixed-shape batches of at least `min_phases` phases (a phase is
 * one workgroup per CU x 8 steps x the groups per workgroup step) run the
 * phased kernel; 0 restores the default (6 phases, about 184K headline
 * groups).  1 forces it for any batch, 0xFFFFFFFF never. */
int qfec_debug_phase_min(qfec_ctx* ctx, uint32_t min_phases);
/* Test hook: on == 0 runs phased launches without their register-held steps
 * (40 LDS steps per phase only, more phases); 1 restores the default.  For
 * the per-group-size A/B; results are identical. */
int qfec_debug_phase_regsteps(qfec_ctx* ctx, int on);
/* Test hook: the load batch of the runtime-k phased body (group sizes above
 * 16): 16 or 32 (0 restores the library's measured per-operation choice:
 * encode 16, recover 32 up to k = 32).  For the per-group-size A/B
 * (DESIGN.md §4); results are identical. */
int qfec_debug_phase_rtbatch(qfec_ctx* ctx, uint32_t batch);
/* Test hook: phased launches leave `cus` more CUs out of their grid (0..64),
 * as if other contexts' small-batch workers held them -- the A/B of the
 * round-6 CU arbitration; results are identical. */
int qfec_debug_phase_reserve(qfec_ctx* ctx, uint32_t cus);
/* Test hook: the CUs a phased launch on ctx would leave to other contexts'
 * small-batch workers now; *why (nullable) gets why they count (bit 0 a job
 * or warm in the last 2 ms, bit 1 a worker alive, bit 2 its stream busy). */
uint32_t qfec_debug_other_service_cus(qfec_ctx* ctx, uint32_t* why);
/* Test hook: fail != 0 makes every ragged call on this context fail with
 * QFEC_ERR_INTERNAL before touching the device (the GPU-failure path of the
 * connection integration: groups go without FEC). */
int qfec_debug_fail_launches(qfec_ctx* ctx, int on);

/* Small-batch service (round 4): QFEC_PTR_MAPPED ragged batches of at most 16
 * groups are taken by a resident worker kernel from a ring in host-mapped
 * memory instead of a kernel launch each; the worker leaves after 100 us
 * without work (or before a phased launch of its context) and is relaunched
 * by the next such batch.  on = 1 / 0
 * enables / disables it (0 also makes a running worker leave; -1 leaves the
 * setting; 2 enables it and writes the NEXT job's ring entry with a wrong job
 * number -- a malformed ring, whose job must fail with QFEC_ERR_INTERNAL and
 * turn the service off rather than report stale output); stats (may be NULL)
 * receives {worker launches, jobs finished, worker alive}; on = 3 leaves the
 * setting and fills stats[0..5] with those plus {worker stream busy, us since
 * the context's last service job or warm (the view the phased launches of
 * other contexts take of it), workers stopped for their 2-ms residency bound}.  Test / measurement hook; the service is on by
 * default.  Any failed service job turns the service off for the context
 * (small batches then launch). */
int qfec_debug_service(qfec_ctx* ctx, int on, uint64_t* stats);
/* Measurement hook of the service: on = 1 / 0 makes the worker record
 * 100-MHz wall-clock stamps of each job it finishes (-1 leaves the
 * setting); stamps (may be NULL, 6 entries) receives the last job's: work
 * seen, ring entry and tables in LDS, wave 0's first group done, every group
 * done, outputs made visible, token stored.  (Worker launched by a later
 * job picks the setting up at its start.) */
int qfec_debug_service_stamps(qfec_ctx* ctx, int on, uint64_t* stamps);
/* Measurement hook (round 6; stamps on through qfec_debug_service_stamps):
 * the last service job end to end, 44 words: [0..5] the leader's stamps as
 * above, [6] when the token was stored and [7] by which workgroup; [8 + 4w ..]
 * workgroup w's share: entry in LDS, groups done, outputs visible, counted
 * (100-MHz ticks); [40..43] the host's steady-clock ns of the last service
 * call: entry, job published, token seen, return. */
int qfec_debug_service_trace(qfec_ctx* ctx, uint64_t* out);
/* Measurement hook (round 6): on = 1 starts a native thread that owns ctx
 * (the caller must not use ctx until it is stopped) and flushes one-group
 * mapped batches of 10 x 1350 B in loop turns 20 us apart, warming the
 * small-batch worker at each turn's start; on = 0 stops it and returns its code, with stats
 * (nullable) = {batches flushed, batches whose parity was wrong}. */
int qfec_debug_service_feed(qfec_ctx* ctx, int on, uint64_t* stats);
/* Test hook: hold != 0 keeps the service's follower workgroups waiting at
 * their start (as if dispatched late behind another kernel) until it is
 * cleared; the leader runs on.  A split job's token then waits for them. */
int qfec_debug_service_hold(qfec_ctx* ctx, int hold);
/* Test hook (round 6): the small-batch worker's residency bound, ns (default
 * 2,000,000; 0 rotates the worker at every job published while it runs --
 * the successor queued behind it, no wait); returns the previous bound, or 0
 * for a null ctx. */
uint64_t qfec_debug_service_resident(qfec_ctx* ctx, uint64_t ns);
/* Test hook (round 6): the small-batch worker's idle time in us (default
 * 100), for workers launched from now on; returns the previous value, or 0
 * for a null ctx.  (A test that holds the followers back keeps the leader
 * resident with it: a leader that idles out meanwhile has its successor
 * queued behind the held kernel.) */
uint64_t qfec_debug_service_idle(qfec_ctx* ctx, uint64_t us);

/* ---- synthetic inputs (bench / parity-test support, device pointers) ---- */
/* Counter-based bytes: byte j of packet (g, i) is little-endian byte j%8 of
 * splitmix64(seed ^ ((g*256 + i) << 32) ^ (j/8)) — generated on the device so
 * that host and device agree without a 14 GB transfer.
 * Fills groups g0 .. g0+n_groups-1 into rows[(g-g0)*group_stride + i*row_stride]. */
int qfec_synth_fixed(qfec_ctx* ctx, uint8_t* rows, uint32_t k, uint32_t L, uint64_t row_stride,
                     uint64_t group_stride, uint64_t g0, uint64_t n_groups, uint64_t seed);
/* Fill the packets of a ragged CSR batch whose group g (global index g0+g)
 * packet i has pkt_len[grp_ptr[g]+i] bytes at pkt_off[...]. */
int qfec_synth_ragged(qfec_ctx* ctx, uint8_t* bytes, const uint64_t* pkt_off,
                      const uint16_t* pkt_len, const uint32_t* grp_ptr, uint64_t g0,
                      uint64_t n_groups, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif /* QFEC_H_ */
