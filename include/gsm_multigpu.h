/*
 * gsm_multigpu.h -- screen-slab partition of one frame across GPUs.
 *
 * The reference renders on one Metal device; these entry points are the build's
 * multi-GPU extension of GlobalRenderer.render (GlobalRenderer.swift:201-238).
 * Protocol, one process and one renderer per GPU, slabs = contiguous tile rows:
 *   1. every rank projects its contiguous range of gaussian ids once
 *      (gsm_global_project_partition) and gets, per slab, the records of the
 *      gaussians whose ellipse meets a tile of that slab, in ascending id order;
 *   2. the records reach slab s's owner concatenated in source-rank order (so
 *      ascending id order overall);
 *   3. the owner, with gsm_global_set_tile_rows(slab), renders its rows from them
 *      (gsm_global_render_records).
 * The slab's pixels are bit-identical to a single-GPU gsm_global_render of the frame:
 * projection is per gaussian, and the ascending-id concatenation preserves the
 * stable-sort tie order (determinism contract).
 *
 * gsm_multigpu_* run the whole protocol inside the library with no host round trip and no
 * collective library in the frame: every rank owns one fine-grained "exchange" allocation
 * (control words, the count matrix, its receive buffer of records and, on rank 0, the gathered
 * colour and depth frames), the ranks open each other's exchange allocations once (IPC handles),
 * and per frame the counts, the records and the slab pixels are written straight into the owners'
 * memory by the producing kernels (xGMI stores between GPUs) with system-coherent write-through
 * stores; the producers drain them and then arrive at a device-side flag barrier themselves, and
 * every consumer load of exchange data is system-coherent.
 * gsm_global_project_partition / gsm_global_render_records remain for callers that move the
 * records themselves.
 */
#ifndef GSM_MULTIGPU_H
#define GSM_MULTIGPU_H

#include "gsm_renderer.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GSM_SPLAT_RECORD_BYTES 48 /* projected gaussian: render data, blend record, tile rect */
#define GSM_MAX_SLABS 16
#define GSM_MULTIGPU_HANDLE_BYTES 256 /* one rank's exchange handle (gsm_multigpu_handle) */

/* Project gaussians [first, first + count) of `input` (count <= config.max_gaussians) for a
 * width x height frame and pack, slab by slab, the records of those that meet slab s =
 * tile rows [slab_rows[s], slab_rows[s+1]) into `send` (device memory, capacity in
 * records; count * num_slabs always suffices).  send_counts (device, num_slabs uint32)
 * receives the records per slab; slab s starts at record sum(send_counts[0..s)).
 * slab_rows is a host array of num_slabs + 1 non-decreasing tile rows <= tiles_y.
 * Enqueue-only on `stream`. */
gsm_status gsm_global_project_partition(gsm_renderer *renderer, void *stream,
                                        const gsm_gaussian_input *input,
                                        const gsm_camera_params *camera, uint32_t width,
                                        uint32_t height, uint32_t first, uint32_t count,
                                        const uint32_t *slab_rows, uint32_t num_slabs, void *send,
                                        uint64_t send_capacity_records, uint32_t *send_counts);

/* Render the renderer's tile rows (gsm_global_set_tile_rows) of a width x height frame
 * from `count` received records (device memory, count <= config.max_gaussians) into the
 * full-frame-addressed color/depth targets (rows outside the slab are not written). */
gsm_status gsm_global_render_records(gsm_renderer *renderer, void *stream, const void *records,
                                     uint32_t count, uint32_t width, uint32_t height,
                                     void *color_rgba16f, size_t color_pitch_bytes,
                                     void *depth_r16f, size_t depth_pitch_bytes);

/* --- the frame across the ranks of a node ---------------------------------------------------
 * One renderer per rank (gsm_global_create on that rank's GPU; every rank with the same
 * max_width / max_height).  Set-up is collective and happens once, in two steps around an
 * exchange the caller performs with any transport (torch.distributed, MPI, sockets, ...):
 *   gsm_multigpu_prepare   allocates this rank's exchange memory (fine-grained device memory:
 *                          control words, 2 x W x W counts, 2 x max_gaussians x 48-B records
 *                          (frame parity),
 *                          and on rank 0 the gathered colour frame and r16f depth frame,
 *                          max_width x max_height pixels each) and the renderer's partition
 *                          buffers, and writes its GSM_MULTIGPU_HANDLE_BYTES handle into `handle`.
 *                          GSM_MG_MEM=cached (ordinary device memory; one GPU only: refused at
 *                          connect across processes) is the A/B of DESIGN.md 7;
 *                          GSM_MG_MEM=uncached returns GSM_ERR_UNSUPPORTED: uncached memory
 *                          renders wrong slabs on MI355X;
 *                          GSM_MG_PIPELINE=1 (every rank alike, checked at connect): phases 0-1 of a
 *                          frame run on a stream of the library's own and phases 2-3 on the caller's,
 *                          joined by events, so frame f + 1's projection and record push run beside
 *                          frame f's slab render (rank 0 then holds two gathered frames that alternate,
 *                          and a gather target must be the caller's own memory: the library frames
 *                          are refused with GSM_ERR_INVALID_ARGUMENT);
 *   (caller)               all-gathers the handles: all[r * GSM_MULTIGPU_HANDLE_BYTES] = rank r's;
 *   gsm_multigpu_connect   opens every peer's exchange memory (hipIpcOpenMemHandle; a handle
 *                          from the same process is used directly) and checks that the ranks
 *                          agree on the world, the frame limits and the options (row layout,
 *                          pipelining, transport): GSM_ERR_INVALID_ARGUMENT otherwise.  It then
 *                          checks every mapping it will store into or poll (own and peers'): one
 *                          word per 4 KiB page written with the frame's system-coherent store form
 *                          from workgroups spread over every XCD, read back with the barrier's poll
 *                          form from other workgroups and through the host, twice with different
 *                          values, and finally re-zeroes the control words with write-through stores
 *                          (never a cached memset) -- GSM_ERR_DEVICE_NOT_AVAILABLE when a word was
 *                          not seen (r06: a range last mapped uncached by any library of the process
 *                          and reused lost flag stores in r05).
 * The frame capacity is the smallest max_gaussians of all ranks (a slab receives every id at
 * most once): a frame with more gaussians returns GSM_ERR_INVALID_GAUSSIAN_COUNT on every rank
 * alike, before anything is enqueued.
 * gsm_multigpu_create does all three over an RCCL communicator (ncclComm_t as void*;
 * libgsm_amd loads RCCL at run time and uses the copy the process has already loaded, so a
 * communicator from torch.distributed works): GSM_ERR_UNSUPPORTED when no RCCL can be loaded,
 * GSM_ERR_INVALID_ARGUMENT when rank / world_size do not match the communicator or
 * world_size > GSM_MAX_SLABS. */
typedef struct gsm_multigpu gsm_multigpu;

/* Per-renderer choices of the partitioned frame (r06), every rank alike (checked at
 * connect; GSM_ERR_INVALID_ARGUMENT otherwise).  gsm_multigpu_default_options fills the defaults; the
 * entry points without options use them, with the environment variables GSM_MG_ROWS=interleaved and
 * GSM_MG_PIPELINE=1 applied on top as test overrides (explicit options ignore the environment). */
typedef enum {
    GSM_MG_ROWS_CONTIGUOUS = 0,  /* rank r owns tile rows [r ceil(tiles_y / W), +ceil(tiles_y / W)): each
                                    record travels to the fewest ranks (faster on centred content) */
    GSM_MG_ROWS_INTERLEAVED = 1  /* rank r owns rows r, r + W, ...: balanced on off-centre content
                                    (the heaviest contiguous rank can sort 2.8x the mean) */
} gsm_multigpu_rows;
typedef enum {
    GSM_MG_TRANSPORT_PEER_STORES = 0, /* the producing kernels store counts, records and pixels straight
                                         into the peers' fine-grained exchange memory (IPC mappings) and
                                         meet at device flag barriers: no collective, no host sync */
    GSM_MG_TRANSPORT_RCCL = 1         /* the same per-slab runs moved by RCCL over `nccl_comm`: the count
                                         rows all-gathered and copied to the host once per frame, the
                                         records by grouped ncclSend / ncclRecv into each owner's receive
                                         buffer at the count matrix's offsets (source-rank order), the
                                         slab rows of colour and depth by grouped send / recv to rank 0.
                                         No IPC and no device barrier: for nodes where peer mappings
                                         cannot be opened (SURVEY.md 8e's all-to-all) */
} gsm_multigpu_transport;
typedef struct {
    uint32_t struct_bytes; /* sizeof(gsm_multigpu_options): set by gsm_multigpu_default_options */
    int32_t rows;          /* gsm_multigpu_rows */
    int32_t pipelined;     /* 1: phases 0-1 on a stream of the library's own, overlapping the previous
                              frame's slab render (peer-stores transport only; GSM_ERR_UNSUPPORTED with
                              RCCL) -- rank 0 then holds two alternating gathered frames */
    int32_t transport;     /* gsm_multigpu_transport */
    uint32_t timeout_ms;   /* device barrier timeout (peer stores), 0 = 10000 */
    uint32_t reserved;
    void *nccl_comm;       /* transport RCCL: the ncclComm_t the frames run their collectives on
                              (gsm_multigpu_create_with_options: its own argument) */
} gsm_multigpu_options;
void gsm_multigpu_default_options(gsm_multigpu_options *options);
gsm_status gsm_multigpu_prepare(gsm_renderer *renderer, int rank, int world_size, gsm_multigpu **out,
                                void *handle);
gsm_status gsm_multigpu_prepare_with_options(gsm_renderer *renderer, int rank, int world_size,
                                             const gsm_multigpu_options *options, gsm_multigpu **out,
                                             void *handle);
gsm_status gsm_multigpu_create_with_options(gsm_renderer *renderer, void *nccl_comm, int rank, int world_size,
                                            const gsm_multigpu_options *options, gsm_multigpu **out);
gsm_status gsm_multigpu_connect(gsm_multigpu *multigpu, const void *all_handles);
gsm_status gsm_multigpu_create(gsm_renderer *renderer, void *nccl_comm, int rank, int world_size,
                               gsm_multigpu **out);
void gsm_multigpu_destroy(gsm_multigpu *multigpu);

/* One frame of gsm_global_render (GlobalRenderer.swift:201-238) across the ranks.  Collective:
 * every rank calls it once per frame with the same input (device pointers on its own GPU; it
 * reads only its id range [r * ceil(N / W), +ceil(N / W))), camera, size and gather choice.
 * Rank r owns tile rows [r * ceil(tiles_y / W), +ceil(tiles_y / W)), or -- when every rank's
 * process has GSM_MG_ROWS=interleaved in its environment at gsm_multigpu_prepare -- rows r, r + W,
 * r + 2W, ... (balances content off the frame's centre; a record then travels to every rank one of
 * its rect's rows maps to).  Per frame, on `stream`:
 *   1. projection of the rank's ids, per-slab record counts written into every rank's count
 *      matrix, flag barrier;
 *   2. every record written straight into its slab owner's receive buffer (offsets from the
 *      count matrix: rank order), flag barrier;
 *   3. the owner renders its rows from the received records (their count read on the device);
 *      when gathering, colour goes to rank 0's gathered frame and -- when depth_r16f is non-NULL
 *      -- depth to rank 0's gathered depth frame (GlobalRenderer.swift:350 writes depth with
 *      every frame); without gathering both go to the rank's own targets (full-frame addressed,
 *      rows outside the slab untouched; depth nullable);
 *   4. gathering: every rank's blend signals rank 0, whose stream waits for all slabs; a
 *      gather_color other than gsm_multigpu_frame's buffer (a depth_r16f other than
 *      gsm_multigpu_frame_depth's) then receives a copy of the frame.
 * Gathering: gather_color non-NULL on every rank (ranks other than 0 pass any non-NULL value;
 * their color may then be NULL); depth gathered when depth_r16f is non-NULL, the same choice on
 * every rank (ranks other than 0 pass any non-NULL value).  No host synchronisation anywhere in
 * the frame.
 * Errors: everything a rank could refuse is checked before it enqueues anything; a refused rank
 * returns the error but still performs every barrier step of the frame (zero counts, arrivals
 * marked failed), so the ranks stay in step and the next frame renders normally; its peers finish
 * the frame without its records or band and count a failed peer arrival (gsm_multigpu_errors).
 * A barrier that waits longer than the timeout (default 10 s; a peer that never calls) gives up,
 * counts the event (gsm_multigpu_status) and lets the frame finish with undefined pixels (the
 * frame's later waits are skipped; the next frame waits again): no wait on the device is
 * unbounded. */
gsm_status gsm_multigpu_render(gsm_multigpu *multigpu, void *stream, const gsm_gaussian_input *input,
                               const gsm_camera_params *camera, uint32_t width, uint32_t height,
                               void *color_rgba16f, size_t color_pitch_bytes, void *depth_r16f,
                               size_t depth_pitch_bytes, void *gather_color);

/* Rank 0's gathered frame (library memory, valid until destroy): *color = its device pointer,
 * *pitch_bytes = max_width x bytes per pixel of the configured colour format.  Passing it as
 * gather_color skips the copy.  Other ranks: *color = NULL.  Pipelined (GSM_MG_PIPELINE=1): the
 * frame of the last frame issued (two alternate); not a valid gather target. */
gsm_status gsm_multigpu_frame(gsm_multigpu *multigpu, void **color, size_t *pitch_bytes);
/* Rank 0's gathered r16f depth frame (library memory): *depth = its device pointer, *pitch_bytes its
 * row pitch.  Passing it as depth_r16f skips the copy.  Other ranks: *depth = NULL. */
gsm_status gsm_multigpu_frame_depth(gsm_multigpu *multigpu, void **depth, size_t *pitch_bytes);

/* Barrier timeouts since create (or the last clear), synchronous: 0 on a healthy run. */
gsm_status gsm_multigpu_status(gsm_multigpu *multigpu, uint32_t *timeouts, int clear);
/* Barrier timeouts and failed peer arrivals (a peer's frame was refused: its arrival carried the
 * failure mark) since create or the last clear, synchronous: 0 and 0 on a healthy run. */
gsm_status gsm_multigpu_errors(gsm_multigpu *multigpu, uint32_t *timeouts, uint32_t *failed_peer_arrivals,
                               int clear);
/* Barrier timeout in milliseconds (default 10000, at least 1). */
gsm_status gsm_multigpu_set_timeout_ms(gsm_multigpu *multigpu, uint32_t ms);

/* Rank 0: copy rows [0, height) x width pixels of the gathered frame into host memory (dst_pitch
 * bytes per row), synchronous (after the frame's stream work); GSM_ERR_INVALID_ARGUMENT elsewhere. */
gsm_status gsm_multigpu_debug_copy_frame(gsm_multigpu *multigpu, void *host_dst, size_t dst_pitch_bytes,
                                         uint32_t width, uint32_t height);

/* Rank 0: the same for the gathered r16f depth frame (dst_pitch >= 2 x width). */
gsm_status gsm_multigpu_debug_copy_depth(gsm_multigpu *multigpu, void *host_dst, size_t dst_pitch_bytes,
                                         uint32_t width, uint32_t height);

/* The first `bytes` of this rank's exchange allocation (control words from byte 0, the count matrix
 * from byte 1024, the received records of even frames from byte 4096, of odd frames after them at the
 * next 4096-byte boundary), synchronous. */
gsm_status gsm_multigpu_debug_copy_exchange(gsm_multigpu *multigpu, void *host_dst, size_t bytes);

/* The last frame's world x world record counts (row = source rank, column = slab), synchronous. */
gsm_status gsm_multigpu_debug_counts(gsm_multigpu *multigpu, uint32_t *host_counts);

/* Test surface (r05): the barrier epoch of the last frame becomes `epoch` (taken modulo 2^31, 0 -> 1) and
 * this rank's flag words are set as if every peer had reached it -- so a test reaches the epoch wrap
 * (2^31 - 1 -> 1) in a few frames.  Every rank alike, with no frame pending or in flight (synchronous);
 * GSM_ERR_PHASE_ORDER while a frame is pending. */
gsm_status gsm_multigpu_debug_set_epoch(gsm_multigpu *multigpu, uint32_t epoch);

/* gsm_multigpu_render in four phases (0: projection + counts + barrier; 1: records + barrier;
 * 2: slab render + the gather signal; 3: rank 0's gather wait + copy); render = phases 0..3, each
 * called even after an earlier phase of the frame returned an error.  A phase called out of order
 * returns GSM_ERR_PHASE_ORDER and enqueues nothing (r05; GSM_ERR_INVALID_ARGUMENT before): a caller
 * that stopped part way through a frame calls gsm_multigpu_finish_frame before the next phase 0.
 * For W ranks driven from ONE host thread (virtual ranks of a test or a timing tool, e.g. W
 * renderers on one GPU sharing one stream): issue phase p of every rank before phase p + 1 of
 * any, so that every barrier waits only for work enqueued before it. */
gsm_status gsm_multigpu_render_phase(gsm_multigpu *multigpu, int phase, void *stream,
                                     const gsm_gaussian_input *input, const gsm_camera_params *camera,
                                     uint32_t width, uint32_t height, void *color_rgba16f,
                                     size_t color_pitch_bytes, void *depth_r16f, size_t depth_pitch_bytes,
                                     void *gather_color);

/* The phases a caller left unfinished in the current frame (r05): phase 1's record push
 * still runs when phase 0 published this rank's counts (the owners expect the records); from phase 2
 * on the frame is abandoned on this rank -- barrier steps only, its arrival at the gather barrier
 * marked failed -- so every rank's epochs stay in step and the next frame renders normally.
 * Enqueued on `stream`; GSM_OK and nothing enqueued when no frame is pending. */
gsm_status gsm_multigpu_finish_frame(gsm_multigpu *multigpu, void *stream);

/* Inputs written on another stream (r05): the next frame's phase 0 makes the stream its
 * projection runs on wait for `event` (a hipEvent_t the caller recorded after writing that frame's
 * gaussians / harmonics).  Pipelined (GSM_MG_PIPELINE=1) phases 0-1 run on the library's own stream,
 * which is otherwise ordered only after the caller's stream finished frame f - 2: without this call
 * the caller must not change the input buffers of a frame it has issued until that frame's phase 1
 * completed.  One-shot (the next phase 0 consumes it); NULL clears it. */
gsm_status gsm_multigpu_wait_event(gsm_multigpu *multigpu, void *event);

#ifdef __cplusplus
}
#endif
#endif
