/*
 * gsm_debug.h -- introspection, stage profiling, multi-GPU slab control and
 * stand-alone sort for libgsm_amd.so.
 *
 * The reference exposes its intermediate buffers to its own tests through
 * `@testable import Renderer` (Tests/RendererTests/GlobalUnitTests.swift:2) and
 * per-view resources (GlobalResources.swift:6-362); these entry points are the
 * C-ABI equivalent used by the parity tests and the benchmark.  All readbacks
 * are synchronous host copies: call them after the frame's stream work is done.
 */
#ifndef GSM_DEBUG_H
#define GSM_DEBUG_H

#include "gsm_renderer.h"

#ifdef __cplusplus
extern "C" {
#endif

/* TileAssignmentHeader (BridgingTypes.h:99-104) + derived frame counters. */
typedef struct {
    uint32_t total_assignments; /* after the clamp to max_capacity */
    uint32_t max_capacity;      /* 4 * max_gaussians */
    uint32_t padded_count;      /* roundup(total, 1024) (GlobalShaders.metal:711-712) */
    uint32_t overflow;          /* 1 when the clamp fired (GlobalShaders.metal:697-701) */
    uint32_t tiles_x, tiles_y, tile_count;
    uint32_t gaussian_count;    /* of the last frame */
} gsm_debug_counters;

/* Buffers that can be copied back (reference resource named in brackets). */
typedef enum {
    GSM_BUF_RENDER_DATA = 0,   /* GaussianRenderData[count], 16 B each [interleavedGaussians]; kept only
                                  by captured frames (profiling bit 1 or 4; else
                                  GSM_ERR_MISSING_REQUIRED_BUFFER): the blend reads its own records */
    GSM_BUF_BOUNDS = 1,        /* int32[count][4] minTX,maxTX,minTY,maxTY [boundsCache] */
    GSM_BUF_TILE_COUNTS = 2,   /* uint32[count] tiles per gaussian [coverageBuffer] */
    GSM_BUF_KEYS = 3,          /* uint32[total] unsorted sort keys [sortKeys before sort] */
    GSM_BUF_VALUES = 4,        /* int32[total] unsorted gaussian ids [tileIndices] */
    GSM_BUF_SORTED_KEYS = 5,   /* uint32[total] [sortKeys after sort]; captured frames only (as
                                  RENDER_DATA): the blend walks per-half-tile lists instead */
    GSM_BUF_SORTED_VALUES = 6, /* int32[total] [sortedIndices]; captured frames only */
    GSM_BUF_HEADERS = 7,       /* GaussianHeader[tile_count] {offset,count} [orderedHeaders] */
    GSM_BUF_EXP_TABLE = 8,     /* uint16[65536] blend exp table indexed by fp16 quad-form bits */
    GSM_BUF_BLEND_TRACE = 9    /* uint64[blend units][4] {start, end (100 MHz ticks), count<<32 | entries
                                  walked, XCC_ID<<32 | HW_ID} of the last profiled frame (bit 2) */
} gsm_buffer_id;

gsm_status gsm_global_debug_counters(gsm_renderer *renderer, gsm_debug_counters *out);

/* The blend kernel the last enqueued frame launched (host-side choice, no sync): k_blend_px with
 * 16x8 quadrant units (small frames and multi-GPU slabs), k_blend_px with 16x16 half-tile units, or
 * the pair walk k_blend_pw (>= 6 half-tile units per wave slot on one GPU).  The benchmark attributes
 * its blend roofline and PMC counters to this kernel. */
typedef enum {
    GSM_BLEND_KERNEL_NONE = 0,
    GSM_BLEND_KERNEL_QUADRANT = 1,
    GSM_BLEND_KERNEL_HALF_TILE = 2,
    GSM_BLEND_KERNEL_PAIR_WALK = 3
} gsm_blend_kernel;
gsm_status gsm_global_debug_blend_kernel(gsm_renderer *renderer, int *kind);
/* Copies up to `bytes` of buffer `which` into host memory; *needed receives the full size. */
gsm_status gsm_global_debug_copy(gsm_renderer *renderer, int which, void *host_dst, size_t bytes,
                                 size_t *needed);
/* `enable` is a bit set: bit 0 brackets every stage by HIP events on the frame's stream,
 * bit 1 keeps the unsorted keys (GSM_BUF_KEYS/VALUES) for readback and captures (bit 4),
 * bit 4 captures the reference's intermediates the product path does not write
 * (GSM_BUF_RENDER_DATA, GSM_BUF_SORTED_KEYS/VALUES; the frame costs their writes), bit 2 records a
 * per-unit blend trace (GSM_BUF_BLEND_TRACE), bit 3 (without bit 0) brackets only the blend
 * (two events per frame; the other stages then report 0); bits 8-15, with bit 3: a period P > 1
 * brackets the blend on every P-th frame only (the average is over the bracketed frames).
 * Every event costs frame time (~10 us per bracketed frame at config 2). */
gsm_status gsm_global_set_profiling(gsm_renderer *renderer, int enable);

enum {
    GSM_STAGE_PROJECT = 0, /* project + cull + SH + tile count */
    GSM_STAGE_SCAN = 1,    /* prefix scan of tile counts */
    GSM_STAGE_SCATTER = 2, /* duplicate-with-keys */
    GSM_STAGE_SORT = 3,    /* radix sort */
    GSM_STAGE_HEADERS = 4, /* tile headers */
    GSM_STAGE_BLEND = 5,   /* clear + front-to-back blend */
    GSM_STAGE_COUNT = 6
};
/* Milliseconds of each stage of the last profiled frame (after stream sync). */
gsm_status gsm_global_stage_times(gsm_renderer *renderer, float *ms, int n);

/* Multi-GPU screen-slab partition: restrict tile assignment,
 * sort, headers and blend to tile rows [row_begin, row_end).  Pixels outside the
 * slab are not written.  (0, 0) restores the full frame. */
gsm_status gsm_global_set_tile_rows(gsm_renderer *renderer, uint32_t row_begin, uint32_t row_end);

/* Stable LSD radix sort of n (uint32 key, uint32 value) pairs in device memory,
 * in place, `key_bits` low key bits significant (the RadixSortEncoder unit-test
 * surface, GlobalUnitTests.swift:23-178).  Allocates its scratch; synchronises
 * `stream` before returning. */
gsm_status gsm_sort_pairs_u32(void *keys, void *values, uint32_t n, uint32_t key_bits, void *stream);

/* The create-time device probe behind the sorts' stable ranks: *lane_ordered = 1 when the lanes
 * of one ds_add_rtn_u32 that hit the same LDS address on `hip_device` receive their old values in
 * lane order (the sorts then rank with one LDS atomic per key), 0 when they do not (ranks from
 * ballot matches).  GSM_SORT_RANK=ballot in the environment at create forces the ballot ranks.
 * Cached per device and process; no reference counterpart (a gfx950 design choice). */
gsm_status gsm_debug_sort_rank_probe(int hip_device, int *lane_ordered);

/* The sorts' workspace guard (host only, no device call): the digit-count workspace bytes every
 * renderer allocates for a sort of `capacity` keys, and whether the passes the LSD sort plans for
 * `key_bits` bits (wide 9..11-bit digits allowed or not) fit `hist_bytes` of it -- GSM_OK, or
 * GSM_ERR_INVALID_ASSIGNMENT_CAPACITY, the status a frame whose sort would overrun its workspace
 * returns before launching any of its passes (an undersized histogram workspace faulted an r05
 * A/B build). */
size_t gsm_debug_sort_workspace_bytes(uint32_t capacity);
gsm_status gsm_debug_sort_plan_fits(uint32_t capacity, uint32_t key_bits, int wide, size_t hist_bytes);

/* The device steps of gsm_multigpu_render (gsm_multigpu.h) without RCCL, so W virtual ranks can run
 * the native exchange in one process on one GPU (tests): the caller plays the collectives --
 * gathers every rank's per-slab counts into the W x W matrix (row r = rank r) on the device and
 * orders the pushes before the renders by stream order.
 *   partition_counts: project ids [first, first + count) and count the records per slab
 *     (slab_rows: num_slabs + 1 tile-row boundaries) into d_send_counts (device, num_slabs words);
 *   partition_push: write every record of the last partition_counts straight into its slab
 *     owner's receive buffer (recv_buffers: host array of `world` device pointers, each holding
 *     GSM_SPLAT_RECORD_BYTES x max_gaussians) at the offset the count matrix d_counts gives;
 *     d_recv_count (device) receives this rank's incoming record count;
 *   render_records_device_count: gsm_global_render_records with the record count read on the
 *     device (d_count) and `capacity` records the grids cover. */
gsm_status gsm_debug_partition_counts(gsm_renderer *renderer, void *stream, const gsm_gaussian_input *input,
                                      const gsm_camera_params *camera, uint32_t width, uint32_t height,
                                      uint32_t first, uint32_t count, const uint32_t *slab_rows,
                                      uint32_t num_slabs, uint32_t *d_send_counts);
gsm_status gsm_debug_partition_push(gsm_renderer *renderer, void *stream, uint32_t world, uint32_t rank,
                                    const uint32_t *d_counts, void *const *recv_buffers, uint32_t *d_recv_count);
gsm_status gsm_debug_render_records_device_count(gsm_renderer *renderer, void *stream, const void *records,
                                                 uint32_t capacity, const uint32_t *d_count, uint32_t width,
                                                 uint32_t height, void *color, size_t color_pitch, void *depth,
                                                 size_t depth_pitch);

#ifdef __cplusplus
}
#endif
#endif
