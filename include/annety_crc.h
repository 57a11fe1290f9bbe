/*
 * annety_crc.h — C-ABI of the MI355X batch checksum engine (libannety_crc.so).
 *
 * Drop-in boundary for annety's checksum path. The reference API is the header-only class
 * annety::Crc32c (include/Crc32c.h:22-83) over the tables in src/Crc32c.cc:20-92; it has no FFI.
 * This header is what a foreign-language binding (ctypes, cgo, JNI, N-API) binds: plain pointers
 * and sizes, `void*` for the hipStream_t, no C++ or torch types. The C++ drop-in header
 * include/annety/Crc32c.h is layered on top of it.
 *
 * Checksum = CRC-32/ISO-HDLC (reflected poly 0xEDB88320, init 0xFFFFFFFF, xorout 0xFFFFFFFF), the
 * exact function annety names "Crc32c" (SURVEY.md §0.1). Check value: crc("123456789") = 0xCBF43926.
 *
 * Error model (the reference functions are total): every entry point that can fail
 * returns an int status, 0 on success, a negative ANNETY_CRC_E* code otherwise, and never aborts.
 * Thread safety: all entry points are reentrant; device state is initialised once per device.
 * Devices: device entry points run on the CURRENT device (hipSetDevice), and `stream` must belong to it:
 * a stream of another device returns ANNETY_CRC_EINVAL (never another device's tables). NULL,
 * hipStreamPerThread and hipStreamLegacy name streams of the current device. A process driving several
 * GPUs from one thread sets the device to the stream's before each call (or uses the device groups below).
 * Streams: the variable, arena and split paths keep per-call device scratch per (device, stream), reused
 * in stream order with no per-call event and no host wait (hipStreamPerThread is keyed per calling
 * thread, since that handle names a different stream in every thread). Up to 64 streams per device
 * (ANNETY_CRC_STREAM_SLOTS) hold their own. While all 64 are taken, every call records an event on its own
 * stream right after its work, and a new stream takes the least recently used scratch over by waiting for
 * that event; a scratch whose last call predates the table filling up is taken over after one device-wide
 * synchronisation instead. The library never records on, or waits for, a stream other than the calling
 * one, so a stream destroyed without annety_crc_stream_release is harmless; releasing it (before
 * hipStreamDestroy) returns its scratch at once and avoids that synchronisation. A new stream whose handle
 * value equals a destroyed one's takes that scratch over in its own order (hipStreamDestroy has completed
 * the old stream's work by then).
 * Failures: annety_crc_last_hip_error names the HIP error and annety_crc_last_error_stage the step of the
 * host path that saw it (per thread). Work queued on a stream reports its failure at the next synchronising
 * call; with ANNETY_CRC_SYNC_STAGES=1 the host-memory paths synchronise after every step so that the stage
 * named is the one that failed (a diagnostic mode, slower).
 */
#ifndef ANNETY_CRC_H
#define ANNETY_CRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ANNETY_CRC_ABI_VERSION 6

enum {
  ANNETY_CRC_OK = 0,
  ANNETY_CRC_EINVAL = -1,  /* bad argument (null pointer with n > 0, misaligned, length out of range) */
  ANNETY_CRC_EHIP = -2,    /* HIP runtime error (see annety_crc_last_hip_error) */
  ANNETY_CRC_ENOMEM = -3,  /* device or pinned-host allocation failed */
  ANNETY_CRC_ENODEV = -4,  /* no usable gfx950 device */
  ANNETY_CRC_ERCCL = -5    /* collective failure (multi-GPU helpers) */
};

/* ---- library / device lifecycle ---- */
int annety_crc_abi_version(void);
/* Uploads the LDS table images to `device` (idempotent; called lazily by every device entry point
 * for the current device). */
int annety_crc_init(int device);
/* Frees device images and staging buffers of every initialised device. */
int annety_crc_shutdown(void);
const char* annety_crc_strerror(int status);
/* Last hipError_t seen by this thread (0 if none). */
int annety_crc_last_hip_error(void);
/* The host-path step ("upload (packed)", "arena verify", "final sync", ...) of this thread's last HIP
 * failure ("" if none). Static string. */
const char* annety_crc_last_error_stage(void);
/* The kernels this thread's latest device entry point enqueued, in launch order, joined by " + " (e.g.
 * "crc32_onekib_nt_kernel" for BASELINE config 1, "crc32_arena_lines_kernel + crc32_arena_stitch_kernel" for
 * an arena batch). Valid until the thread's next call; "" before any. */
const char* annety_crc_last_kernels(void);
/* Leave n CUs of every device free of the batch kernels (which otherwise take one workgroup per CU), so
 * that work on other streams - e.g. the RCCL kernels of a digest gather overlapped with the next chunk -
 * runs beside them instead of between them. 0 (default) uses every CU. Process-wide. */
int annety_crc_reserve_cus(int n);
/* Long-payload split policy, process-wide (initial values from ANNETY_CRC_SPLIT / ANNETY_CRC_SEG, read
 * once): mode -1 = auto (split when the batch is too small to fill the chip), 0 = never, 1 = whenever a
 * payload spans two segments; min_segment = smallest segment in bytes (power of two >= 4096), 0 = default
 * 64 KiB. Digests do not depend on it. */
int annety_crc_set_split(int mode, uint64_t min_segment);
/* Variable batches on the length-sorted path run each payload of more than 128 KiB as 16 KiB segments (1 MiB
 * segments past 256 MiB), digests and update registers alike. extra_segments bounds the segment descriptors one
 * call may add (default and maximum 262144 = 2^18, 4 MiB of per-stream scratch; 0 = never split); payloads that
 * find no room run whole. Process-wide; results do not depend on it. ANNETY_CRC_EINVAL above the maximum. */
int annety_crc_set_split_cap(uint32_t extra_segments);
/* Host frame walks (annety_lhc_parse, annety_*_verify_host*): a buffer of at least two segments of
 * `bytes` (0 = default 64 MiB, at least 4096) is walked in segments side by side, each later segment from
 * a speculative entry that the in-order join confirms or redoes (crc32_capi.cpp FrameWalks). Results do
 * not depend on it. Process-wide. */
int annety_crc_set_walk_segment(uint64_t bytes);
/* Drops `stream`'s per-stream scratch on the current device (stream-ordered free, no wait). Call before
 * destroying a stream that ran variable, arena or split batches. */
int annety_crc_stream_release(void* stream);
/* Scratch bookkeeping of `device` (test and tuning visibility): streams holding a slot, hand-overs of a
 * slot between streams so far, device-wide synchronisations so far (0 outside annety_crc_shutdown). */
int annety_crc_scratch_stats(int device, uint64_t* slots, uint64_t* handoffs, uint64_t* device_syncs);
/* The path annety_crc32_batch_var / annety_crc32_update_batch_var take, process-wide (initial value from
 * ANNETY_CRC_VAR_PATH = auto | sorted; ANNETY_CRC_VAR_AUTO=0 means sorted): 0 = automatic arena or
 * length-sorted choice from recorded extents (below), 1 = the length-sorted path. Any other mode returns
 * ANNETY_CRC_EINVAL. Digests do not depend on it. get returns the current mode. */
int annety_crc_set_var_path(int mode);
int annety_crc_get_var_path(void);
/* Calls of annety_crc32_batch_var / annety_crc32_update_batch_var on `device` (n >= 1024) whose path the host chose
 * from recorded extents - the arena path (and how many of those ran without recording their extent, between two
 * recording calls) or the sorted path - and calls whose path the device chose from the call's own extent (test and
 * tuning visibility). Any pointer may be NULL. */
int annety_crc_var_path_stats(int device, uint64_t* arena, uint64_t* sorted, uint64_t* arena_unrecorded,
                              uint64_t* device_chosen);

/* ---- host scalar API: exact replacements of the reference's inline methods ----
 * annety_crc32_long   replaces Crc32c::crc32_long(const char*, size_t)   include/Crc32c.h:58-69
 * annety_crc32_short  replaces Crc32c::crc32_short(const char*, size_t)  include/Crc32c.h:41-55
 * annety_crc32_update replaces Crc32c::crc32_update(uint32_t*, ...)      include/Crc32c.h:71-82
 * These run on the calling CPU thread: a single frame is far below the size at which a device
 * round trip pays; batches go through the device entry points below. */
uint32_t annety_crc32_long(const char* buff, size_t len);
uint32_t annety_crc32_short(const char* buff, size_t len);
void annety_crc32_update(uint32_t* crc, const char* buff, size_t len);
/* crc(A||B) from crc(A), crc(B) and |B| (GF(2) shift; not in the reference, used to join partials). */
uint32_t annety_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
/* The reference's table globals annety::internal::crc32_table16/256 (src/Crc32c.cc:20-92), read-only. */
const uint32_t* annety_crc32_table16(void);
const uint32_t* annety_crc32_table256(void);

/* ---- device-resident batches (pointers are device memory of the current device) ----
 * Fixed length: payload i occupies [d_base + i*stride, d_base + i*stride + len); d_out[i] receives
 * crc32_long(payload i). Fast path: d_base 16-byte aligned, stride % 16 == 0, len % 16 == 0; other
 * shapes are accepted and routed to the general kernel. `stream` is a hipStream_t (NULL = default).
 * Asynchronous with respect to the host: results are valid after the stream is synchronised. */
int annety_crc32_batch_fixed(const void* d_base, size_t n, size_t len, size_t stride, uint32_t* d_out,
                             void* stream);
/* Variable length: payload i = [d_base + d_off[i], + d_len[i]) (any alignment).
 * Path choice is automatic. A recording call runs the extent kernel (a few us), which publishes the batch's
 * extent; once two completed recording calls on the same stream with the same (d_base, d_off, d_len, n) have
 * shown a dense batch (payload bytes >= 2/3 of the span) that is either sorted (starts ascending, gaps < 4 KiB)
 * or lies inside one device allocation (any order, any gaps), calls take the arena path over that span; once a
 * completed record for those pointers rules the arena out (sparse, or unsorted across allocations), and for
 * n < 1024, the length-sorted path. Until then - and on every call of a caller that passes fresh offset / length
 * arrays each time - the device chooses within the call: after the extent kernel, both paths' launches are
 * enqueued and only the chosen one runs (the arena iff the batch is dense, sorted with gaps < 4 KiB, and its
 * scratch fits the stream's, which grows to the densest span recorded on the stream). On the arena path one
 * call in 8 records: it re-checks its own extent on the device and, if the layout changed under the same
 * pointers, folds every payload directly from its own bytes. The 7 calls in between skip the extent kernel
 * and the device check: the span is checked on the host to lie inside one device allocation (so the line
 * pass reads only mapped memory), and the stitch folds any payload outside the span from its own bytes. In
 * every call each digest depends only on its payload's bytes: a changed layout costs time, never a wrong
 * digest or a read of unmapped memory. ANNETY_CRC_VAR_AUTO=0: sorted path only.
 * n must be below 2^31 (ANNETY_CRC_EINVAL otherwise): the sorted list keeps bit 31 of an index for segments. */
int annety_crc32_batch_var(const void* d_base, const uint64_t* d_off, const uint32_t* d_len, size_t n,
                           uint32_t* d_out, void* stream);
/* Raw-register update (crc32_update semantics) for a fixed-length batch: d_state[i] is the register
 * before payload i on input and after it on output (no init, no final xor). Any alignment. */
int annety_crc32_update_batch_fixed(uint32_t* d_state, const void* d_base, size_t n, size_t len, size_t stride,
                                    void* stream);
/* Streaming update: one fragment per stream, fragment i = [d_base + d_off[i],
 * + d_len[i]) advances stream i's register d_state[i] in place (crc32_update, include/Crc32c.h:71-82).
 * A fragment of length 0 leaves its register unchanged. Seed with 0xFFFFFFFF and xor the final register
 * with 0xFFFFFFFF to get crc32_long of the whole stream. Path choice, the split of long fragments and the
 * bound on n as annety_crc32_batch_var. */
int annety_crc32_update_batch_var(uint32_t* d_state, const void* d_base, const uint64_t* d_off, const uint32_t* d_len,
                                  size_t n, void* stream);

/* Arena variants of the two entry points above, for payloads that lie in one buffer of arena_bytes
 * bytes at d_arena (a NetBuffer's readable bytes, a frame stream, a packed batch; offsets are relative
 * to d_arena). One pass streams every 128-byte line of the arena whatever the length mix, then one lane
 * per payload joins its lines, so the cost follows arena_bytes: use these when the
 * payloads cover most of the arena, and the two entry points above for sparse batches. A payload that
 * reaches outside [0, arena_bytes) is still computed correctly (its lines are folded directly).
 * Same results and argument rules as annety_crc32_batch_var / annety_crc32_update_batch_var. */
int annety_crc32_batch_var_arena(const void* d_arena, size_t arena_bytes, const uint64_t* d_off,
                                 const uint32_t* d_len, size_t n, uint32_t* d_out, void* stream);
int annety_crc32_update_batch_var_arena(uint32_t* d_state, const void* d_arena, size_t arena_bytes,
                                        const uint64_t* d_off, const uint32_t* d_len, size_t n, void* stream);

/* ---- host-memory batch (payloads off a NetBuffer/socket): staged through pinned buffers (packed by a
 * small host thread pool, ANNETY_CRC_PACK_THREADS), H2D -> kernel -> D2H, pipelined on two streams.
 * Synchronous. ---- */
int annety_crc32_batch_fixed_host(const void* h_base, size_t n, size_t len, size_t stride, uint32_t* h_out);
/* Pin (hipHostRegister) / unpin a long-lived host buffer, e.g. a NetBuffer arena: host batches whose
 * payloads lie inside one buffer pinned here are copied to the device in place, without the staging pack.
 * h_ptr must be page-aligned, and the buffer's pages must not overlap a buffer already pinned here
 * (ANNETY_CRC_EINVAL otherwise): the runtime pins whole pages, and registrations sharing a page leave its
 * lookup two answers. Only buffers pinned through this call are DMA'd in place; any other host memory
 * (including memory pinned by other means) goes through the pack. unregister takes the same h_ptr
 * (ANNETY_CRC_EINVAL for a pointer not pinned here). */
int annety_crc_host_register(void* h_ptr, size_t bytes);
int annety_crc_host_unregister(void* h_ptr);

/* ---- device groups: one process, several gfx950 devices ----
 * A group is an RCCL communicator over `devices` (ncclCommInitAll, single process) plus a compute and a
 * communication stream per device. Payloads are independent, so a batch shards into contiguous blocks
 * with no data-path collective; the only exchange is the digests' trip to the root device (devices[0]).
 * The C++ callers of annety (one process, N event loops: src/EventLoopPool.cc:55-66) use these to spread
 * a batch over the GPUs of a node without torch.distributed. */
typedef struct annety_crc_group annety_crc_group;
/* Contiguous block shards of n payloads over nshards: shard k = [first[k], first[k] + count[k]), sizes
 * within one of each other. Host only (no device needed). */
int annety_crc_shard_plan(size_t n, int nshards, size_t* first, size_t* count);
/* The transfer schedule annety_crc32_group_batch_fixed runs (host only): shard k is cut into `chunks`
 * near-equal pieces; for piece c of shard k, plan[(c*nd + k)*3 + 0] = its first payload within the shard,
 * [+1] = its payload count (0: nothing to do), [+2] = the index in d_root_out where its digests land
 * (sum(n_shard[0..k-1]) + first). plan holds chunks*nd*3 entries. */
int annety_crc_group_schedule(const size_t* n_shard, int nd, size_t chunks, size_t* plan);
/* ANNETY_CRC_ENODEV if a device is missing or not gfx950, ANNETY_CRC_EINVAL for a repeated device,
 * ANNETY_CRC_ERCCL if the communicator cannot be built. */
int annety_crc_group_create(const int* devices, int ndev, annety_crc_group** out);
int annety_crc_group_destroy(annety_crc_group* group);
int annety_crc_group_size(const annety_crc_group* group);
/* Device-resident shards: device k (the group's k-th) holds n_shard[k] payloads of len bytes at
 * d_shard[k] (stride apart, memory of device k). d_root_out (memory of devices[0]) receives all
 * sum(n_shard) digests in device order. Each shard is checksummed in `chunks` pieces and piece c's
 * digests travel to the root (RCCL send/recv over xGMI) while piece c+1 is computed. Synchronous;
 * ANNETY_CRC_ERCCL on a collective failure. */
int annety_crc32_group_batch_fixed(annety_crc_group* group, const void* const* d_shard, const size_t* n_shard,
                                   size_t len, size_t stride, uint32_t* d_root_out, size_t chunks);
/* Host-memory batch spread over the group: payload shard k (annety_crc_shard_plan) is staged over device
 * k's own PCIe link and checksummed there, all devices at once; h_out[i] = crc32_long(payload i). */
int annety_crc32_group_batch_fixed_host(annety_crc_group* group, const void* h_base, size_t n, size_t len,
                                        size_t stride, uint32_t* h_out);

/* ---- LengthHeaderCodec wire format, batched ----
 * frame = [length: T bytes big-endian, T = 1/2/4/8][payload: length-4 bytes][crc32(payload): 4 bytes BE]
 * (include/codec/LengthHeaderCodec.h:33-46; decode :71-137; encode :146-201; checksum enabled). */

/* Host walk of a receive stream, exactly LengthHeaderCodec::decode's framing without the CRC:
 * from h_stream[0], for each complete frame writes its payload offset/length (relative to h_stream),
 * stopping at the first incomplete frame, at max_frames, or at an invalid length (length < 4, or
 * length > max_payload when max_payload > 0, or a negative signed length as peek_int* would read it).
 * *n_frames = frames written, *consumed = bytes of those frames. Returns 0; 1 when it stopped on an
 * invalid length at offset *consumed (decode's -1); ANNETY_CRC_EINVAL for a bad argument or a complete
 * frame whose payload is 4 GiB or more (lengths here are 32-bit). */
int annety_lhc_parse(const void* h_stream, size_t size, int length_type, int64_t max_payload, uint64_t* payload_off,
                     uint32_t* payload_len, size_t max_frames, size_t* n_frames, size_t* consumed);
/* Device verify of n frames already located (offsets/lengths from annety_lhc_parse, copied to the
 * device): d_ok[i] = 1 if crc32_long(payload i) equals its big-endian trailer, else 0 (decode :123-132).
 * d_digest (optional, may be NULL) receives the computed CRCs. */
int annety_lhc_verify_batch(const void* d_stream, const uint64_t* d_payload_off, const uint32_t* d_payload_len,
                            size_t n, uint8_t* d_ok, uint32_t* d_digest, void* stream);
/* Same as annety_lhc_verify_batch over the arena path: d_stream holds stream_bytes bytes (the received
 * stream the frames were parsed from), so the payload CRCs take one pass over the stream. */
int annety_lhc_verify_stream(const void* d_stream, size_t stream_bytes, const uint64_t* d_payload_off,
                             const uint32_t* d_payload_len, size_t n, uint8_t* d_ok, uint32_t* d_digest,
                             void* stream);
/* Codec::recv over a host receive buffer (include/codec/Codec.h:52-76, the NetBuffer of
 * src/TcpConnection.cc:438-461): the header walk of annety_lhc_parse runs on the walk pool (in segments
 * side by side, annety_crc_set_walk_segment) while the stream is copied to the current device (in place
 * when h_stream is pinned), then every complete frame's CRC is verified on the device (arena path over the
 * stream). Outputs as annety_lhc_parse plus h_ok[i] = 1 if frame i's trailer matches. Returns 0, 1 (the
 * walk stopped on an invalid length: decode's -1) or a negative error. Synchronous. Reuse the output
 * arrays across calls: arrays of max_frames entries allocated per call cost more than the verify (a
 * 1 GiB stream through fresh 110 MB arrays: 28 against 49 GiB/s). */
int annety_lhc_verify_host(const void* h_stream, size_t size, int length_type, int64_t max_payload,
                           uint64_t* h_payload_off, uint32_t* h_payload_len, uint8_t* h_ok, size_t max_frames,
                           size_t* n_frames, size_t* consumed);
/* Codec::recv over K connections' receive buffers in one call (one input NetBuffer per TcpConnection,
 * src/TcpConnection.cc:438-461, each walked as include/codec/Codec.h:55-78 does): the buffers are gathered
 * into one device stream (pinned staging; pinned buffers are DMA'd in place), each is walked exactly as
 * annety_lhc_parse walks one, and every complete frame's CRC is verified on the device in one arena pass.
 * Frames of connection c occupy output entries [sum(conn_frames[0..c-1]), + conn_frames[c]); their
 * h_payload_off are relative to h_bufs[c]. conn_consumed[c] = bytes of c's complete frames; conn_rt[c] = 0
 * (walk stopped at an incomplete frame or the end), 1 (invalid length: decode's -1, the connection is
 * shut down) or ANNETY_CRC_EINVAL (a frame of 4 GiB or more). max_frames bounds the output arrays over all
 * connections; connections past the bound report 0 frames. Returns 0 or a negative error. Synchronous. */
int annety_lhc_verify_host_iov(const void* const* h_bufs, const size_t* sizes, size_t k, int length_type,
                               int64_t max_payload, uint64_t* h_payload_off, uint32_t* h_payload_len, uint8_t* h_ok,
                               size_t max_frames, size_t* conn_frames, size_t* conn_consumed, int* conn_rt);
/* How annety_*_verify_host(_iov) uploads receive buffers that are not pinned here: 1 (default; initial value
 * from ANNETY_CRC_FRAMES_PACK) packs them into the library's pinned ring with the pack threads, 0 hands them
 * to the runtime's pageable copy. Process-wide; results do not depend on it. */
int annety_crc_set_frames_pack(int pack);
/* Host plan for a batch of LengthHeaderCodec::encode calls (:169-176): h_rt[i] (optional) = 1, or 0 for
 * an empty payload, or -1 for len > max_payload (max_payload > 0); h_frame_off[i] = where frame i starts
 * when the frames of accepted payloads are packed back to back (rejected ones take no bytes);
 * *total = bytes of all frames. As in the reference, a length field too wide for T keeps its low T bytes. */
int annety_lhc_encode_plan(const uint32_t* h_len, size_t n, int length_type, int64_t max_payload,
                           uint64_t* h_frame_off, int8_t* h_rt, uint64_t* total);
/* Device encode: for each accepted payload i = [d_src + d_src_off[i], + d_len[i]) writes header,
 * payload copy and CRC trailer at d_dst + d_frame_off[i] (offsets from annety_lhc_encode_plan with the
 * same length_type and max_payload); rejected payloads write nothing. */
int annety_lhc_encode_batch(const void* d_src, const uint64_t* d_src_off, const uint32_t* d_len, size_t n,
                            int length_type, int64_t max_payload, void* d_dst, const uint64_t* d_frame_off,
                            void* stream);

/* ---- ProtobufCodec framing, batched (include/protobuf/ProtobufCodec.h, checksum on) ----
 * The same frame layout with T = 4 and the codec's fixed limits: decode accepts a length field
 * (payload + 4) in [10, 64 MiB] (min_payload() = nameLen 4 + 2 + checksum 4, :279-283; max_payload()
 * 64 MiB, unconditional, :273-277; decode :127-173), encode accepts payloads of 6 .. 64 MiB bytes
 * (:225-247). The CRC covers the whole payload (nameLen + typeName + protobuf bytes, :235-247), so the
 * message itself stays opaque here: parsing it needs libprotobuf and is the caller's.
 * Verify with annety_lhc_verify_batch / annety_lhc_verify_stream (format-independent once located). */
int annety_pbc_parse(const void* h_stream, size_t size, uint64_t* payload_off, uint32_t* payload_len,
                     size_t max_frames, size_t* n_frames, size_t* consumed);
int annety_pbc_verify_host(const void* h_stream, size_t size, uint64_t* h_payload_off, uint32_t* h_payload_len,
                           uint8_t* h_ok, size_t max_frames, size_t* n_frames, size_t* consumed);
int annety_pbc_verify_host_iov(const void* const* h_bufs, const size_t* sizes, size_t k, uint64_t* h_payload_off,
                               uint32_t* h_payload_len, uint8_t* h_ok, size_t max_frames, size_t* conn_frames,
                               size_t* conn_consumed, int* conn_rt);
int annety_pbc_encode_plan(const uint32_t* h_len, size_t n, uint64_t* h_frame_off, int8_t* h_rt, uint64_t* total);
int annety_pbc_encode_batch(const void* d_src, const uint64_t* d_src_off, const uint32_t* d_len, size_t n,
                            void* d_dst, const uint64_t* d_frame_off, void* stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* ANNETY_CRC_H */
