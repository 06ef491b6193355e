/*
 * checked_batch.h -- batched CheckedMessage<Crc32Hasher> checksums over RPC
 * payloads held in pinned (device-accessible) host memory, part of
 * libphoton_checksum.so. SURVEY.md §8(f) row 1.
 *
 * Two pieces, both plain C-ABI:
 *
 * 1. A pinned-memory allocator with IOAlloc's callback signatures
 *    (common/io-alloc.h:31-85): photon_crc_pinned_allocate /
 *    photon_crc_pinned_deallocate can be bound as IOAlloc{Allocator,
 *    Deallocator} and handed to Skeleton::set_allocator (rpc/rpc.h:187,
 *    rpc.cpp:216-220), so socket readv lands in buffers the GPU can read in
 *    place (hipHostMalloc'd, mapped into every device's address space). Blocks
 *    come from size-class pools carved out of 64 MiB pinned slabs (pinning is
 *    slow; slabs are kept until photon_crc_pinned_release).
 *
 * 2. A message batch: instead of calling validate_checksum
 *    (rpc/serialize.h:266-275) on each received message, the receive path
 *    saves the message's m_checksum, zeroes it (exactly as validate_checksum
 *    does) and adds {payload iovector, struct body, saved checksum} to a
 *    batch; one submit checksums every message on the GPU (per-segment CRCs +
 *    crc32c_combine fold, the photon_crc32c_batch_msg_n kernels) and compares.
 *    The same batch serves the send side (add_checksum, serialize.h:258-261):
 *    add with expected = 0 and read the computed value.
 *    Result i == what the reference's validate_checksum(iov, body, len)
 *    returns for message i:
 *    - by default `body` is the message object itself, as
 *      DeserializerIOV::deserialize passes it (t->validate_checksum(iov, t,
 *      sizeof(*t)), serialize.h:462-463), whose first 4 bytes are m_checksum
 *      (the CheckedMessage<> base of every Photon message struct).
 *      Crc32Hasher accumulates the payload's CRC into m_checksum and then
 *      hashes the body holding it; a CRC whose init equals its first data
 *      word equals the CRC (init 0) of the data with that word zeroed, so the
 *      reference's checksum is crc32c(body with m_checksum = 0): the payload
 *      does NOT enter it (tests/golden/ioalloc_binding.json: the reference's
 *      own template over reference IOVectors). The batch reproduces that: it
 *      checksums the body with its first 4 bytes read as zero
 *      (validate_checksum's second line) and does not read the payload
 *      segments. It never writes the caller's message: m_checksum keeps the
 *      received claim (the reference leaves the recomputed value there,
 *      which equals the claim whenever the message is valid).
 *    - PHOTON_CRC_BATCH_DETACHED_BODY: `body` is a separate buffer (not the
 *      object holding m_checksum) or absent: Crc32Hasher::extend_hash over
 *      the payload segments, then the body, seed 0 (serialize.h:244-252;
 *      also the default's result when body is NULL, e.g. rpc.h:106).
 *
 * Memory rules: every segment and body must be device-accessible (pinned by
 * this allocator or any hipHostMalloc / hipHostRegister, or device memory);
 * photon_crc_msg_batch_add verifies that unless the batch was created with
 * PHOTON_CRC_BATCH_TRUSTED, and rejects other memory with -EFAULT (there is
 * no CPU fallback). Segments must stay valid and unmodified until the batch's
 * completion.
 *
 * Errors: negative errno codes; photon_crc_last_error() has the text.
 */
#ifndef PHOTON_CRC_CHECKED_BATCH_H
#define PHOTON_CRC_CHECKED_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include "crc32c_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------ pinned IOAlloc pool */

/* Same layout as IOAlloc::RangeSize {int min, max;} (io-alloc.h:33). */
typedef struct photon_crc_range {
    int min;
    int max;
} photon_crc_range;

/* IOAlloc::Allocator callback: allocate size.max bytes (size.min must be > 0
 * and size.max >= size.min, as default_allocator asserts, io-alloc.h:74-80)
 * of pinned host memory, 4 KiB aligned; returns the size allocated (> 0) or a
 * negative errno. `obj` is the Callback's bound object and is ignored. */
int photon_crc_pinned_allocate(void* obj, photon_crc_range size, void** ptr);

/* IOAlloc::Deallocator callback: return a block to its pool. 0, or -EINVAL
 * for a pointer this allocator did not hand out. */
int photon_crc_pinned_deallocate(void* obj, void* ptr);

/* Bytes pinned in slabs and bytes handed out. */
int photon_crc_pinned_stats(uint64_t* slab_bytes, uint64_t* in_use_bytes);

/* Unpin every slab with no block in use. Returns the number of bytes released. */
int64_t photon_crc_pinned_release(void);

/* ------------------------------------------------------------ message batch */

typedef struct photon_crc_msg_batch photon_crc_msg_batch;

#define PHOTON_CRC_BATCH_TRUSTED 1u /* skip the per-segment accessibility check */
#define PHOTON_CRC_BATCH_STAGED 2u  /* copy descriptors H2D and verdicts D2H instead of
                                       the kernels reading / writing the pinned staging */
#define PHOTON_CRC_BATCH_DETACHED_BODY 4u /* bodies are separate buffers: hash payload, then body */

/* A batch on the current device with room for max_messages messages and
 * max_segments segments in total: every iovec entry and every body counts
 * as one (a message-object body is hashed internally as two pieces, the zero
 * word standing for m_checksum and the rest of the object; the batch
 * reserves the extra piece itself). NULL on error. */
photon_crc_msg_batch* photon_crc_msg_batch_create(uint32_t max_messages, uint32_t max_segments, uint32_t flags);
void photon_crc_msg_batch_destroy(photon_crc_msg_batch* b);

/* Append one message: its payload iovector (iov[iovcnt], struct iovec layout)
 * followed by `body` (skipped when NULL or body_length == 0, as
 * validate_checksum does) and the checksum it must match. Unless the batch
 * is DETACHED_BODY, a body is the message object: it is checksummed with its
 * first 4 bytes (m_checksum) read as 0, as validate_checksum zeroes them,
 * at every submit, without writing the object (see 2. above). Returns the
 * message's index (>= 0) or -ENOSPC / -EFAULT / -EBUSY (submitted, not yet
 * reset) / -EINVAL. */
int64_t photon_crc_msg_batch_add(photon_crc_msg_batch* b, const photon_crc_iovec* iov, uint32_t iovcnt,
                                 const void* body, uint64_t body_length, uint32_t expected);

/* Launch the whole batch on `stream` (NULL = default stream): the kernels
 * read the descriptors from pinned staging and the segments in place, and
 * write the verdict CRCs to pinned memory (one launch; with
 * PHOTON_CRC_BATCH_STAGED the descriptors are copied H2D and the results
 * D2H around it). If `done` is non-NULL it is called once the results are on
 * the host, from a HIP runtime thread (it may call photon::semaphore::signal,
 * thread/thread.h:511-520, and photon_crc_msg_batch_result, which then needs
 * no HIP call); it must not call HIP, nor submit / reset / destroy this batch.
 * A completed batch may be submitted again (its payloads re-read, e.g. after
 * they were refilled); -EBUSY while a submit is still running or its `done`
 * callback has not returned yet (reset too; destroy waits for it). */
int photon_crc_msg_batch_submit(photon_crc_msg_batch* b, void* stream, void (*done)(void* arg), void* arg);

/* Wait for the submitted batch. Returns the number of messages whose checksum
 * did not match (>= 0), or a negative error. */
int64_t photon_crc_msg_batch_wait(photon_crc_msg_batch* b);

/* After completion: *crc = message i's computed checksum (if crc != NULL);
 * returns 1 if it equals the expected value, 0 if not, -EINVAL for a bad
 * index, -EBUSY before completion. */
int photon_crc_msg_batch_result(photon_crc_msg_batch* b, uint64_t i, uint32_t* crc);

/* Number of messages added so far. */
uint64_t photon_crc_msg_batch_count(const photon_crc_msg_batch* b);

/* Forget all messages (waits for an outstanding submit first). */
int photon_crc_msg_batch_reset(photon_crc_msg_batch* b);

#ifdef __cplusplus
}
#endif

#endif /* PHOTON_CRC_CHECKED_BATCH_H */
