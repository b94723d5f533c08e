/*
 * gsm_multigpu.h -- screen-slab partition of one frame across GPUs.
 *
 * The reference renders on one Metal device; these entry points are the build's
 * multi-GPU extension of GlobalRenderer.render (GlobalRenderer.swift:201-238).
 * Protocol, one process and one renderer per GPU, slabs = contiguous tile rows:
 *   1. every rank projects its contiguous range of gaussian ids once
 *      (gsm_global_project_partition) and gets, per slab, the records of the
 *      gaussians whose ellipse meets a tile of that slab, in ascending id order;
 *   2. an all-to-all(v) over the fabric (RCCL) delivers slab s's records to its owner,
 *      concatenated in source-rank order (so ascending id order overall);
 *   3. the owner, with gsm_global_set_tile_rows(slab), renders its rows from them
 *      (gsm_global_render_records).
 * The slab's pixels are bit-identical to a single-GPU gsm_global_render of the frame:
 * projection is per gaussian, and the ascending-id concatenation preserves the
 * stable-sort tie order (determinism contract).
 *
 * gsm_multigpu_* run the whole protocol inside the library over the caller's RCCL
 * communicator (steps 1-3 plus the band gather), enqueue-only with no host round trip;
 * gsm_global_project_partition / gsm_global_render_records remain for callers that move
 * the records themselves.
 */
#ifndef GSM_MULTIGPU_H
#define GSM_MULTIGPU_H

#include "gsm_renderer.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GSM_SPLAT_RECORD_BYTES 48 /* projected gaussian: render data, blend record, tile rect */
#define GSM_MAX_SLABS 16

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

/* --- the frame across a communicator ------------------------------------------------------
 * One renderer per rank (gsm_global_create on that rank's GPU, config.max_gaussians >= the
 * frame's gaussian count) and the rank's RCCL communicator (ncclComm_t as void*; libgsm_amd
 * loads RCCL at run time and uses the copy the process has already loaded, so a communicator
 * from torch.distributed works).  Collective: every rank of the communicator calls create,
 * each frame and destroy.  create allocates the send / receive buffers (48 B x max_gaussians
 * each) and opens every peer's receive buffer once from its IPC handle; GSM_ERR_UNSUPPORTED
 * when no RCCL can be loaded, GSM_ERR_INVALID_ARGUMENT when rank / world_size do not match the
 * communicator or world_size > GSM_MAX_SLABS. */
typedef struct gsm_multigpu gsm_multigpu;
gsm_status gsm_multigpu_create(gsm_renderer *renderer, void *nccl_comm, int rank, int world_size,
                               gsm_multigpu **out);
void gsm_multigpu_destroy(gsm_multigpu *multigpu);

/* One frame of gsm_global_render (GlobalRenderer.swift:201-238) across the communicator.  Every
 * rank passes the same input (device pointers on its own GPU; it reads only its id range
 * [r * ceil(N / W), +ceil(N / W))), camera and size.  Rank r owns tile rows
 * [r * ceil(tiles_y / W), +ceil(tiles_y / W)) and writes them into its full-frame-addressed
 * color / depth targets; per frame, on `stream`: projection of its ids, all-gather of the
 * per-slab record counts, peer writes of every record into its owner's receive buffer over
 * xGMI, one ordering all-reduce, the slab render with the record count read on the device, and,
 * when gather_color is set on rank 0 (it must then equal color, with color_pitch = 8 * width)
 * and on every other rank (any non-NULL value), the bands sent to rank 0's frame.  No host
 * synchronisation anywhere in the frame. */
gsm_status gsm_multigpu_render(gsm_multigpu *multigpu, void *stream, const gsm_gaussian_input *input,
                               const gsm_camera_params *camera, uint32_t width, uint32_t height,
                               void *color_rgba16f, size_t color_pitch_bytes, void *depth_r16f,
                               size_t depth_pitch_bytes, void *gather_color);

/* The last frame's world x world record counts (row = source rank, column = slab), synchronous. */
gsm_status gsm_multigpu_debug_counts(gsm_multigpu *multigpu, uint32_t *host_counts);

#ifdef __cplusplus
}
#endif
#endif
