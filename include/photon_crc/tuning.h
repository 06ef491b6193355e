/*
 * tuning.h -- NOT for production callers of libphoton_checksum.so.
 *
 * Engine-shape knobs used by the tuning scripts and the parity tests (every
 * variant is parity-tested; the defaults are the measured-fastest shapes),
 * a failure-injection hook for the failure-contract test, and the bench's
 * synthetic-data utilities. Every knob is a process-wide atomic word that a
 * launch reads once, so changing one while other threads submit batches is
 * race-free (each launch runs entirely with the old or entirely with the new
 * shape); it is still a process-wide setting, which is why it is not part of
 * the production header <photon_crc/crc32c_gpu.h>.
 */
#ifndef PHOTON_CRC_TUNING_H
#define PHOTON_CRC_TUNING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Engine selection for photon_crc32c_batch_* (testing / tuning):
 * lanes per buffer G in {4,8,16,32,64}; 0 = automatic (default). */
int photon_crc_set_lanes_per_buffer(int g);

/* Workgroups of the CRC32C batch kernel's persistent grid (tuning: fewer
 * busy CUs at the same HBM rate); 0 = one per CU (default). */
int photon_crc_set_batch_grid(int workgroups);

/* Batch kernel variant (testing / tuning): -1 (default) = rows per step by
 * lane-group size (2 for 16-lane groups, else 4); 2, 4 or 8 = the generic
 * kernel with that many rows per step. (The fused and streaming kernels of
 * earlier rounds measured slower and were deleted in round 6.) */
int photon_crc_set_generic_rows(int rows_per_step);

/* Message batches (photon_crc32c_batch_msg[_n], the CheckedMessage batch),
 * testing / tuning: 0 = automatic (default: one kernel with a lane group per
 * message, chained through the seed, when no per-segment CRCs are requested
 * and there are >= 4096 wavefronts' worth of short messages; else parallel
 * segment CRCs + a fold kernel), 1 = always the one-kernel form, 2 = always
 * the two-kernel form. */
int photon_crc_set_msg_mode(int mode);

/* Rows per step of the one-kernel message form (tuning): 2 (default) or 4. */
int photon_crc_set_msg_rows(int rows_per_step);

/* Buffers over 256 KiB up to 16 MiB (block span <= 1,048,576 16-byte blocks)
 * of photon_crc32c_extend_device / photon_crc64ecma_extend_device
 * and of the routed calls: 1 (default) = the mid layout (the small kernel's
 * code over 512 workgroups: 1 MiB in 5.1 µs per call queued against 8.3 for
 * the long kernel), 0 = the long kernel (tests of its plan). DESIGN.md §4.0. */
int photon_crc_set_mid_kernel(int on);

/* One long buffer (photon_crc32c_extend_device / photon_crc64ecma_extend_device,
 * buffers over 16 MiB, or over 256 KiB with the mid kernel off): lanes per chunk (32 or 64) and chunks per lane
 * group of the full grid (rounds, 1..64); 0 = automatic, by buffer size and
 * CRC width (photonlibos_amd/csrc/long_plan.h long_plan_for, which lists the
 * measurements behind each step): CRC-32C 64 lanes x 2 rounds, 32 x 2 from
 * 512 MiB, 64 x 4 from 1.5 GiB, 64 x 2 from 3 GiB; CRC-64 64 lanes x 1
 * round, 64 x 2 from 512 MiB, 32 x 2 from 1 GiB, 64 x 4 from 1.5 GiB, 64 x 2
 * from 3 GiB. */
int photon_crc_set_long_shape(int lanes, int rounds);

/* CRC-64 batches of whole steps (aligned strided, one seed, nbytes a
 * multiple of 32 * lanes * rows_per_step): 0 = the generic batch kernel,
 * 1 = the full-row kernel (wave-uniform loop, two register sets), 2 = the
 * same with the next buffer's first rows issued before the finish, 3 = the
 * default: mode 2 for buffers that take lane groups of up to 16 lanes (up to
 * 32 KiB at 8 lanes), the generic kernel above, with 4 rows per step for
 * buffers of 8 KiB and more and 2 below (rows_per_step is then ignored);
 * modes 0-2 take rows_per_step 2 or 4. DESIGN.md §4.1 has the measurements. */
int photon_crc64_set_full_rows(int mode, int rows_per_step);

/* Routed drop-in calls (photon_crc_set_device_dispatch) collect their result
 * by polling tagged words in pinned memory for at most `spin_us` microseconds
 * (default 40, with a pause between reads), then sleep in 10 us slices,
 * reading the words after each; with sleep_ahead != 0 (the default) a call
 * whose bytes at a nominal 6.5 GB/ms would take longer than the window first
 * sleeps through 85 % of that time. spin_us = 0: no polling window. */
int photon_crc_set_routed_wait(int spin_us, int sleep_ahead);

/* Resident small-buffer service for routed crc32c_extend calls of up to 2 MiB
 * (block span <= 135,168 16-byte blocks; device pointers,
 * photon_crc_set_device_dispatch): idle_us > 0 keeps a
 * launch of 33 workgroups (256 threads, 14 KiB of LDS each) on the device
 * that polls a request doorbell (device memory the host writes through the
 * PCIe BAR; pinned memory without a large BAR), so a call costs no kernel
 * launch and no table load; the launch ends after idle_us without a request
 * (and after its life, photon_crc_set_small_service_life, 2 ms by default,
 * in any case; the next call starts a new one and is its first request). Default 200 (or the environment variable
 * PHOTON_CRC_SMALL_SERVICE at load); 0 = off, a launch per call; turning it
 * off ends running launches. crc64ecma_extend has a service of its own (34
 * KiB of LDS per workgroup). Every batch, message or long launch of this
 * library ends the running services of its device first, and no routed call
 * starts a service launch while one is queued or running (it takes the launch
 * path), so those kernels never run beside them. One call at a time uses it; concurrent calls take
 * the launch path. While it runs, hipDeviceSynchronize() and anything else
 * that waits for every stream of the device wait until it ends: at most
 * idle_us after the last call, and at most the launch's life (below) under
 * steady traffic; the library ends it before its own hipFree calls. An idle
 * launch naps between doorbell polls after 20 us without a request. DESIGN.md
 * §4.0 has the latency. */
int photon_crc_set_small_service(int idle_us);
/* Life of one service launch, 100..1000000 us (default 2000): under steady
 * routed traffic a launch ends after it and the next call starts another, so
 * it bounds how long a device-wide wait can stall behind the service. */
int photon_crc_set_small_service_life(int life_us);
/* The service's doorbell: 1 (default) = device memory the host writes through
 * the PCIe BAR, used only when the device reports a large BAR and the host
 * mapping was verified at creation (fault-free probe: the kernel copies the
 * words to and from a pipe, EFAULT if unmapped); 0 = the pinned host area
 * (also PHOTON_CRC_SVC_DOORBELL=host in the environment at load). Ends
 * running launches; the next launch uses the new doorbell. */
int photon_crc_set_service_doorbell(int bar);
/* The doorbell the current device's service of `kind` (0 CRC-32C, 1 CRC-64)
 * rings: 1 BAR, 0 pinned host memory, -ENOENT if it was never started. */
int photon_crc_small_service_doorbell(int kind);
/* Routed small calls served by the service, launches of it, and calls that
 * found it ending and took the launch path (tests). */
int photon_crc_small_service_stats(uint64_t* served, uint64_t* starts, uint64_t* missed);
/* Routed small calls that would have started a service launch while a batch,
 * message or long launch of this library was still queued or running on the
 * device, and took the launch path instead (the two never share the chip:
 * their workgroups do not fit on one CU together). */
uint64_t photon_crc_small_service_deferred(void);

/* Lanes per buffer the engine picks for buffers of typical length n (the
 * lane-group table of DESIGN.md §4, or the override when one is set). */
int photon_crc_lanes_for(uint64_t nbytes);

/* Failure injection (tests only): the next `n` device entry points called on
 * this thread return -EIO before enqueuing anything ("injected failure"). */
void photon_crc_test_fail_next(int n);

/* The constants this library GENERATES (gf2.h), for pinning against the
 * reference's compiled tables (crc_tables.cpp:104-107, 147-164): which =
 *   0 host x^(8*2^i)            (= crc32c_lshift_table_sw, 32)
 *   1 host x^-(8*2^i)           (= crc32c_rshift_table_sw, 32)
 *   2 host x^(8*2^i - 33)       ([4..31] = crc32c_lshift_table_hw[0..27])
 *   3 host x^-(8*2^i + 33)      (= crc32c_rshift_table_hw, 32)
 *   4 device x^(8*2^i)          (combine / fold kernels, 32)
 *   5 device x^-(8*2^i)         (trim kernel, 32)
 *   6 device row shifts x^(8*16*G), G = 4..64 (5)
 *   7 device lane-combine x^(128*2^k) (image of x^0, 6)
 *   8 host slicing table T[b] (crc.cpp:82-97, 256)
 *   9 device finish tables x^(32+128*d), d < 8 (image of x^0, 8)
 * Returns the number of words written to out[n], or a negative error. */
int photon_crc_test_tables(int which, uint32_t* out, int n);

/* The long-buffer plan and launch constants (photonlibos_amd/csrc/long_plan.h)
 * the library would use for a buffer at address `addr` (not dereferenced) of
 * n bytes on a device with `cus` compute units, shape as
 * photon_crc_set_long_shape (0, 0 = automatic), CRC-64 constants if crc64.
 * out[0..8] = head, chunk, nchunks, last, rounds, grid, stride, lead, lanes;
 * then CRC-32C: xsb[32], xb[32], zt[16], ft[grid]; CRC-64: xsb[64], x,
 * zt[16], ft[grid] (one word each). For CPU tests that replay the kernels'
 * staged combine with the oracle. Returns the words written, or -EINVAL. */
int photon_crc_test_long_plan(uint64_t addr, uint64_t n, int cus, int lanes, int rounds, int crc64, uint64_t* out,
                              int nout);

/* Test/bench utility (not on the checksum path): fill count buffers of
 * nbytes at d_base + i*stride with the splitmix64 byte stream of seed
 * (seed_base + i), i.e. word k = mix64(seed + (k+1)*0x9E3779B97F4A7C15),
 * little-endian; identical to photonlibos_amd.datagen. */
int photon_crc_util_fill_splitmix(void* d_base, uint64_t stride, uint64_t nbytes, uint64_t count,
                                  uint64_t seed_base, void* stream);

/* Bench utility (not on the checksum path): read nbytes (16-byte aligned
 * base) once with the CRC kernels' loads and access pattern (one persistent
 * 1024-thread workgroup per CU, waves sweeping 64 KiB pieces in 1 KiB rows,
 * 4 rows in flight) and fold them into d_sink (>= 1024 words; grid =
 * min(CUs, sink_words/1024)): the achievable HBM-read rate the roofline is
 * compared against. */
int photon_crc_util_read_stream(const void* d_base, uint64_t nbytes, uint32_t* d_sink, uint64_t sink_words,
                                void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PHOTON_CRC_TUNING_H */
