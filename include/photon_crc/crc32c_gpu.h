/*
 * crc32c_gpu.h -- C-ABI of the MI355X CRC32C engine (libphoton_checksum.so).
 *
 * Plain pointers and sizes only; no HIP or torch types in the signatures
 * (`stream` is a hipStream_t passed as void*, NULL = the default stream).
 *
 * Semantics are PhotonLibOS's raw CRC-32C (common/checksum/crc32c.h:30-45):
 * reflected polynomial 0x82F63B78, init = caller's seed, no final xor.
 *   out[i] = crc32c_extend(buffer_i, nbytes_i, seed_i)
 * Every entry point below replaces a host loop over that reference call:
 *   photon_crc32c_batch_strided  <- loop of crc32c_extend (crc32c.h:30-33) over
 *                                   base + i*stride; with stride == nbytes and
 *                                   seeds == 0 it is crc32c_series
 *                                   (crc32c.h:52-57, crc.cpp:474-509)
 *   photon_crc32c_batch_iov      <- loop of crc32c_extend over struct iovec[]
 *                                   (common/iovector.h:56-230)
 *   photon_crc32c_batch_msg      <- Crc32Hasher::extend_hash over each
 *                                   message's iovector (rpc/serialize.h:239-252):
 *                                   per-segment CRC + crc32c_combine fold
 *                                   (crc.cpp:393-430)
 *   photon_crc32c_combine_batch  <- loop of crc32c_combine (crc32c.h:61-66)
 *
 * All batch calls are asynchronous on `stream`: inputs must stay valid and
 * outputs are ready only after the stream is synchronised. Buffers and
 * descriptor arrays must be device-accessible (hipMalloc'd or registered /
 * pinned host memory).
 *
 * Per device, the library keeps ≈1.3 MiB of constant table images for the
 * life of the process (the LDS tables every batch / long kernel copies
 * instead of building them, written on the device's first call) and, for
 * the small and mid kernels, ≈1.3 MiB more on the first call that needs them.
 *
 * Return value: 0 on success, a negative errno-style code otherwise
 * (-ENODEV no usable gfx950 device, -EINVAL bad arguments, -EIO HIP runtime
 * error; photon_crc_last_error() has the text). There is NO silent CPU
 * fallback: on error nothing is computed.
 */
#ifndef PHOTON_CRC32C_GPU_H
#define PHOTON_CRC32C_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same layout as struct iovec {void *iov_base; size_t iov_len;}
 * (common/iovector.h:56-230 uses struct iovec); a struct iovec array may be
 * passed directly. */
typedef struct photon_crc_iovec {
    const void* base;
    uint64_t len;
} photon_crc_iovec;

/* Same layout as CRC32C_Component {uint32_t crc; uint32_t size;}
 * (common/checksum/crc32c.h:76-79); a CRC32C_Component array may be passed. */
typedef struct photon_crc_component {
    uint32_t crc;
    uint32_t size;
} photon_crc_component;

/* Number of usable gfx950 devices (>0), or a negative error code. */
int photon_crc_device_count(void);

/* Text of the last error on this thread ("" if none). */
const char* photon_crc_last_error(void);

/* Device scratch the library keeps between calls (segment CRCs of two-kernel
 * message batches, long-buffer state): idle buffers over 64 MiB, and idle
 * scratch beyond 256 MiB per device, are freed automatically; this frees
 * every idle buffer whose last use has completed. Returns the bytes freed. */
int64_t photon_crc_scratch_release(void);

/* (i) Equal-length buffers: buffer i = d_base + i*stride, nbytes each.
 * seed_i = d_seeds ? d_seeds[i] : seed0. d_out[count] receives the CRCs. */
int photon_crc32c_batch_strided(const void* d_base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                uint32_t seed0, const uint32_t* d_seeds, uint32_t* d_out, void* stream);

/* (i-h) Host-memory batch, the path's real source (socket / file buffers in
 * host RAM feeding rpc/ and fs/): chunks of the batch are copied to the
 * device (stream-ordered, 2-D so any stride packs densely) while earlier
 * chunks are checksummed; the CRCs come back to h_out[count]. Synchronous.
 * h_base should be pinned (hipHostMalloc / hipHostRegister) for the copies to
 * overlap; h_seeds (optional) and h_out are host arrays. Buffers up to 256 MiB. */
int photon_crc32c_host_batch_strided(const void* h_base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                     uint32_t seed0, const uint32_t* h_seeds, uint32_t* h_out);

/* (i-h, many GPUs) The same host-memory batch sharded over the first `ndev`
 * gfx950 devices (0 = every device) of THIS process -- Photon runs one
 * process per host, not one per GPU: contiguous slices of the buffer indices,
 * one host thread per device driving that device's pipeline over its own
 * host link, results in h_out[count] exactly as the single-device call.
 * No collective. Synchronous. */
int photon_crc32c_host_batch_strided_multi(const void* h_base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                           uint32_t seed0, const uint32_t* h_seeds, uint32_t* h_out, int ndev);

/* (i-d, many GPUs) Device-resident shards, each on its own device: shard i is
 * photon_crc32c_batch_strided on `device` (pointers of that device, stream of
 * that device or NULL). Enqueues every shard and returns (async); the caller's
 * current device is restored. */
typedef struct photon_crc_shard {
    int device;
    const void* d_base;
    uint64_t stride;
    uint64_t nbytes;
    uint64_t count;
    uint32_t seed0;
    const uint32_t* d_seeds;
    uint32_t* d_out;
    void* stream;
} photon_crc_shard;
int photon_crc32c_batch_strided_shards(const photon_crc_shard* shards, int nshards);

/* (ii) Arbitrary buffers: d_iov[count] (device-resident descriptors); any
 * alignment, any length (0 returns the seed). */
int photon_crc32c_batch_iov(const photon_crc_iovec* d_iov, uint64_t count, uint32_t seed0,
                            const uint32_t* d_seeds, uint32_t* d_out, void* stream);

/* (iii) Scatter-gather messages: message m is segments
 * [d_msg_start[m], d_msg_start[m+1]) of d_iov (d_msg_start has nmsg+1
 * entries, d_msg_start[nmsg] = total segments). d_out[m] = the chained
 * crc32c_extend over the message's segments starting from seed_m.
 * d_seg_out (total segments entries), if non-NULL, receives each segment's
 * own CRC32C (seed 0); with NULL the segments are chained through the seed
 * (the faster form when there are many short messages). */
int photon_crc32c_batch_msg(const photon_crc_iovec* d_iov, const uint64_t* d_msg_start, uint64_t nmsg,
                            uint32_t seed0, const uint32_t* d_seeds, uint32_t* d_seg_out, uint32_t* d_out,
                            void* stream);
/* As photon_crc32c_batch_msg, with the total segment count nseg
 * (== d_msg_start[nmsg]) supplied by the caller: fully asynchronous
 * (photon_crc32c_batch_msg reads it back from the device and waits). */
int photon_crc32c_batch_msg_n(const photon_crc_iovec* d_iov, const uint64_t* d_msg_start, uint64_t nmsg,
                              uint64_t nseg, uint32_t seed0, const uint32_t* d_seeds, uint32_t* d_seg_out,
                              uint32_t* d_out, void* stream);

/* d_out[i] = crc32c_combine(d_crc1[i], d_crc2[i], d_len2[i]) with the
 * reference's shortcuts (crc1 == 0 -> crc2, len2 == 0 -> crc1). */
int photon_crc32c_combine_batch(const uint32_t* d_crc1, const uint32_t* d_crc2, const uint32_t* d_len2,
                                uint64_t count, uint32_t* d_out, void* stream);

/* Device forms of the contiguous-batch calls (crc32c.h:52-57, 71-74, 84-87),
 * same results as the drop-in host functions for the same inputs:
 *   series:          d_crc_parts[i] = crc32c(d_buffer + i*part_size, part_size)
 *                    with crc32c_series' semantics (the SSE4.2 engine that
 *                    crc32c_series_auto selects: part_size < 8 gives 0s);
 *   combine_series:  *d_result = crc32c_combine_series(d_crc, part_size,
 *                    n_parts), including n_parts == 0 -> 0 and the
 *                    part_size == 0 shortcut behaviour;
 *   trim_batch:      d_out[i] = crc32c_trim(d_all[i], d_prefix[i],
 *                    d_suffix[i]); an element whose sizes are inconsistent
 *                    gives 0 (the reference's EINVAL result) and, when d_nerr
 *                    is non-null, increments *d_nerr (zero it beforehand);
 *   extend_device:   *d_out = crc32c_extend(d_data, nbytes, seed) for ONE
 *                    long buffer in ONE launch over the whole device: chunks
 *                    on a grid anchored at a 4 KiB boundary, each lane group's
 *                    chunks folded in registers, the workgroups' values
 *                    XOR-combined by the last workgroup to finish; up to a
 *                    256 KiB block span, the latency path (up to 32 small
 *                    workgroups, no table prologue). Launches of more than
 *                    one workgroup share, per stream, the reduce's state (a
 *                    ticket counting every workgroup of the stream's
 *                    launches, a slot per workgroup): the calls are safe
 *                    from any number of streams and threads. Every call may
 *                    be captured into a HIP graph (even a process's first:
 *                    the per-device setup runs in relaxed capture mode); a
 *                    captured launch of more than one workgroup uses a
 *                    reduce state owned by the graph, reset by the launch
 *                    itself, so the graph replays any number of times, one
 *                    replay at a time: two executable graphs instantiated
 *                    from the same captured graph share those states and
 *                    must not run concurrently.
 * Asynchronous on `stream` like the batches. */
int photon_crc32c_series_device(const void* d_buffer, uint32_t part_size, uint32_t n_parts, uint32_t* d_crc_parts,
                                void* stream);
int photon_crc32c_combine_series_device(const uint32_t* d_crc, uint32_t part_size, uint32_t n_parts,
                                        uint32_t* d_result, void* stream);
int photon_crc32c_trim_batch(const photon_crc_component* d_all, const photon_crc_component* d_prefix,
                             const photon_crc_component* d_suffix, uint64_t count, uint32_t* d_out,
                             uint32_t* d_nerr, void* stream);
int photon_crc32c_extend_device(const void* d_data, uint64_t nbytes, uint32_t seed, uint32_t* d_out, void* stream);

/* (many GPUs) ONE logical buffer whose bytes lie on several devices of this
 * process: span i = [d_data, d_data + nbytes) on `device`, the spans in
 * buffer order. Every span runs photon_crc32c_extend_device (from seed 0) on
 * its own device, all devices at once; the host folds the span CRCs with
 * crc32c_combine's identity (crc.cpp:393-405): acc = seed, then acc =
 * acc * x^(8 len_i) ^ crc_i. 4 bytes per device cross the host link; no
 * collective. Synchronous: *h_result = crc32c_extend(buffer, total, seed).
 * The caller's current device is restored. */
typedef struct photon_crc_span {
    int device;
    const void* d_data;
    uint64_t nbytes;
} photon_crc_span;
int photon_crc32c_extend_spans(const photon_crc_span* spans, int nspans, uint32_t seed, uint32_t* h_result);

/* Route the drop-in entry points to the device when handed device memory:
 * with on != 0, crc32c_auto / crc32c_series_auto / crc32c_combine_series_auto
 * (crc.cpp:126-134) and crc64ecma_auto point to wrappers that ask HIP whether the data pointer
 * is device memory (hipMemoryTypeDevice) and, if so, run the calls above
 * synchronously on that pointer's device, else call the host engine. A
 * routed call runs on a non-blocking stream leased from a per-device pool
 * (never the legacy default stream, so it does not serialise against the
 * process's other streams; concurrent routed calls get streams of their
 * own) and its result is written by the kernel into pinned host memory. The
 * calling thread (a photon vCPU: its coroutines wait with it) does not spin
 * through a long kernel: a call whose bytes would take longer than the poll
 * window first sleeps through most of its expected time, then polls the
 * result words with a pause between reads for at most 40 us, then sleeps in
 * 10 us slices between reads (photon_crc_set_routed_wait, tuning.h). Off (the
 * default, also at load time) restores the host engines. The reference signatures have no error channel and the reference
 * always computes (crc.cpp:114-117), so a routed call whose device work
 * fails NEVER returns a made-up value: it is reported on stderr, counted,
 * errno is set to EIO, and the bytes are copied to the host and checksummed
 * by the host engine (same result as the reference); if even that copy fails
 * the process aborts with a message. Returns 0, or -EIO if a routed call
 * failed since the last switch (photon_crc_dispatch_fallbacks() counts them).
 * Ordering: like the reference's crc32c_extend (crc32c.h:30-33), a routed
 * call checksums the bytes that exist when it is called. It takes no stream
 * and orders against none of the caller's: the caller must have COMPLETED
 * every write to the buffer (kernel, copy, vDMA, peer write) before the call,
 * e.g. hipStreamSynchronize / hipEventSynchronize on the producer's stream.
 * A write still in flight may or may not be seen. For stream-ordered work use
 * photon_crc32c_extend_device / photon_crc64ecma_extend_device on the
 * producer's stream instead. */
int photon_crc_set_device_dispatch(int on);
/* Number of routed calls so far whose device work failed and that were
 * recomputed on the host (0 in a healthy process; tests assert it). */
uint64_t photon_crc_dispatch_fallbacks(void);

/* CRC-64/ECMA batches (reference crc64ecma.h:20-38: reflected polynomial
 * 0xC96C5795D7870F42, init and result inverted):
 *   out[i] = crc64ecma_extend(buffer_i, nbytes_i, seed_i)
 * Same shapes and rules as the CRC32C strided / iovec batches. */
int photon_crc64ecma_batch_strided(const void* d_base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                   uint64_t seed0, const uint64_t* d_seeds, uint64_t* d_out, void* stream);
int photon_crc64ecma_batch_iov(const photon_crc_iovec* d_iov, uint64_t count, uint64_t seed0,
                               const uint64_t* d_seeds, uint64_t* d_out, void* stream);

/* CRC-64/ECMA forms of the CRC32C calls above (crc64ecma.h:20-87):
 *   combine_batch: d_out[i] = crc64ecma_combine(d_crc1[i], d_crc2[i], d_len2[i])
 *                  (crc1 == 0 -> crc2, as the reference);
 *   batch_msg_n:   d_out[m] = crc64ecma_extend chained over message m's
 *                  segments from seed_m (e.g. an OSS object's iovector,
 *                  ecosystem/oss.h:217 expected_crc64); d_seg_out[s] = each
 *                  segment's crc64ecma(seg, 0); nseg == d_msg_start[nmsg];
 *   extend_device: *d_out = crc64ecma_extend(d_data, nbytes, seed) for ONE
 *                  long device buffer (one launch, as the CRC32C call). */
/* Same layout as CRC64ECMA_Component {uint64_t crc; uint64_t size;}
 * (common/checksum/crc64ecma.h:68-71). */
typedef struct photon_crc64_component {
    uint64_t crc;
    uint64_t size;
} photon_crc64_component;

/* d_out[i] = crc64ecma_trim(d_all[i], d_prefix[i], d_suffix[i])
 * (crc64ecma.h:73-87); inconsistent sizes give 0 and count in *d_nerr. */
int photon_crc64ecma_trim_batch(const photon_crc64_component* d_all, const photon_crc64_component* d_prefix,
                                const photon_crc64_component* d_suffix, uint64_t count, uint64_t* d_out,
                                uint32_t* d_nerr, void* stream);

/* photon_crc32c_host_batch_strided for CRC-64/ECMA: host (e.g. an OSS
 * upload's) buffers through the same chunked H2D + kernel + D2H pipeline. */
int photon_crc64ecma_host_batch_strided(const void* h_base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                        uint64_t seed0, const uint64_t* h_seeds, uint64_t* h_out);
int photon_crc64ecma_combine_batch(const uint64_t* d_crc1, const uint64_t* d_crc2, const uint32_t* d_len2,
                                   uint64_t count, uint64_t* d_out, void* stream);
/* photon_crc32c_batch_msg_n for CRC-64/ECMA: d_out[m] = crc64ecma_extend
 * chained over message m's segments from seed_m. d_seg_out (per-segment CRCs
 * from seed 0) is optional. */
int photon_crc64ecma_batch_msg_n(const photon_crc_iovec* d_iov, const uint64_t* d_msg_start, uint64_t nmsg,
                                 uint64_t nseg, uint64_t seed0, const uint64_t* d_seeds, uint64_t* d_seg_out,
                                 uint64_t* d_out, void* stream);
/* photon_crc32c_extend_device for CRC-64/ECMA (crc64ecma_extend, crc.cpp:
 * 119-122): the same latency path for spans up to 256 KiB (a small kernel of
 * up to 33 workgroups), one launch over the chip above, the same per-stream
 * state and capture rules. */
int photon_crc64ecma_extend_device(const void* d_data, uint64_t nbytes, uint64_t seed, uint64_t* d_out,
                                   void* stream);
/* photon_crc32c_extend_spans for CRC-64/ECMA (crc64ecma_combine's identity:
 * the inverted CRC folds the same way). */
int photon_crc64ecma_extend_spans(const photon_crc_span* spans, int nspans, uint64_t seed, uint64_t* h_result);

/* Synchronous convenience: photon_crc32c_batch_strided + stream sync. */
int photon_crc32c_batch_strided_sync(const void* d_base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                     uint32_t seed0, const uint32_t* d_seeds, uint32_t* d_out, void* stream);

/* Tuning knobs, the failure-injection hook and the bench data utilities are
 * declared in <photon_crc/tuning.h> (not for production callers). */

/* Producers outside device memory.
 * photon_crc_host_register: make an existing host range (e.g. the iovec
 * targets of IFile::preadv, fs/filesystem.h:54-70) readable by the kernels in
 * place (hipHostRegister, mapped); undo with photon_crc_host_unregister.
 * photon_crc32c_file_strided: h_out[i] = crc32c_extend(record i, nbytes,
 * seed0) for the records at file offset + i*stride of fd. A reader thread
 * pread()s 4 KiB-aligned chunks (so an O_DIRECT fd works: the device reads
 * what the disk DMA'd, the CPU touches no payload byte) into two pinned chunk
 * buffers while the GPU pipeline checksums the previous chunk. Synchronous;
 * -EIO if the file ends before the last record, -errno on a read error.
 * Concurrent callers each check out their own pinned chunk pair (pairs are
 * cached for reuse) and share one persistent pool of reader threads. */
int photon_crc_host_register(void* ptr, uint64_t len);
int photon_crc_host_unregister(void* ptr);
int photon_crc32c_file_strided(int fd, uint64_t offset, uint64_t stride, uint64_t nbytes, uint64_t count,
                               uint32_t seed0, uint32_t* h_out);

/* Runtime shim so that Photon code drives the batches without HIP headers
 * (host code stays Photon C++; HIP stays behind this library):
 *   stream_create / _destroy / _sync: a non-blocking stream of the current
 *       device (the `stream` argument of the calls above);
 *   stream_on_complete: run fn(arg) on a runtime thread once everything
 *       enqueued on `stream` so far has finished (fn may call
 *       photon::semaphore::signal, thread/thread.h:511-520; it must not call
 *       into this library or HIP);
 *   device_alloc / _free: device memory of the current device;
 *   memcpy_async: copy n bytes between any host/device pointers, ordered on
 *       `stream` (pinned host memory for true asynchrony).
 * 0 or a negative errno-style code, as everywhere. */
int photon_crc_stream_create(void** stream);
int photon_crc_stream_destroy(void* stream);
int photon_crc_stream_sync(void* stream);
int photon_crc_stream_on_complete(void* stream, void (*fn)(void* arg), void* arg);
int photon_crc_device_alloc(void** ptr, uint64_t nbytes);
int photon_crc_device_free(void* ptr);
int photon_crc_memcpy_async(void* dst, const void* src, uint64_t nbytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PHOTON_CRC32C_GPU_H */
