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

#ifdef __cplusplus
}
#endif
#endif
