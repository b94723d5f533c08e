/*
 * gsm_depthfirst.h -- C ABI of the DepthFirst stereo side-by-side path (libgsm_amd.so).
 *
 * Drop-in for the reference's DepthFirstRenderer.renderStereo(target: .sideBySide)
 * (Sources/Renderer/DepthFirstRenderer/DepthFirstRenderer.swift:205-223, 469-512, 595-831;
 * SURVEY.md 8(f) rank 1).  Its semantics differ from running the Global path once per eye:
 *   - one projection pass projects every gaussian into both eyes; SH colour is evaluated once,
 *     from the midpoint of the two camera centres (DepthFirstShaders.metal:419-424);
 *   - screen positions use ndcToScreen without the half-pixel shift (:291);
 *   - a gaussian is binned into the union of its two eyes' 16x16-tile rects (:426-442),
 *     depth-sorted first by the centre depth as a 32-bit float key (:33-37, :496), then the
 *     per-tile instances are stably sorted by tile (DepthFirstRenderer.swift:683-768);
 *   - one 64-lane wave per 16x16 tile blends both eyes, 2x2 pixels per lane with a joint
 *     left/right saturation break and the r^2 <= 9 cutoff (DepthFirstShaders.metal:1825-1982);
 *   - the two eyes land side by side in the target through the copy pass
 *     (DepthFirstStereoCopyEncoder.swift:29-99), which flips rows (target row y of an eye is
 *     row height-1-y of its slice; DESIGN.md "DepthFirst stereo").
 * Same conventions as gsm_renderer.h: device pointers, the stream as void*, enqueue-only.
 */
#ifndef GSM_DEPTHFIRST_H
#define GSM_DEPTHFIRST_H

#include "gsm_renderer.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gsm_depthfirst gsm_depthfirst;

/* DepthFirstRenderer.init(device:config:depthSortKeyPrecision:tileIdPrecision:)
 * (DepthFirstRenderer.swift:45-101) with its defaults: 32-bit depth keys, 16-bit tile ids.
 * Errors as GlobalRenderer.init: max_gaussians > 30M -> GSM_ERR_INVALID_GAUSSIAN_COUNT
 * (:51-56); a 16x16 tile grid of max_width x max_height over 65535 tiles (16-bit tile ids,
 * 0xFFFF is the tile sort's sentinel) -> GSM_ERR_INVALID_TILE_COUNT.  Scratch is allocated
 * here: max_gaussians records and 4 * max_gaussians instances (DepthFirstResources.swift:399). */
gsm_status gsm_depthfirst_create(const gsm_renderer_config *config, int hip_device, gsm_depthfirst **out);
void gsm_depthfirst_destroy(gsm_depthfirst *renderer);

/* renderStereo(commandBuffer:target:.sideBySide(colorTexture:depthTexture:)input:camera:width:height:)
 * (DepthFirstRenderer.swift:205-223, 469-512).  width/height are per eye (<= config max_width /
 * max_height); the colour target is 2 * width columns of config.color_format by height rows of
 * color_pitch_bytes: left eye in columns [0, width), right eye in [width, 2 * width).  The
 * reference ignores the depth texture of this target (:472), so there is none here.
 * near/far planes come from the left camera (makeStereoCameraUniforms, :583-584).
 * scene_transform: NULL for the identity of the side-by-side path, or 16 floats column-major
 * (StereoConfiguration.sceneTransform, GaussianRendererProtocol.swift:100-116).
 * Returns an error where the reference silently skips the frame (:478, :607). */
gsm_status gsm_depthfirst_render_stereo_sbs(gsm_depthfirst *renderer, void *stream,
                                            const gsm_gaussian_input *input,
                                            const gsm_camera_params *left, const gsm_camera_params *right,
                                            const float *scene_transform, uint32_t width, uint32_t height,
                                            void *color, size_t color_pitch_bytes);

/* DepthFirstHeader (BridgingTypes.h:209-219) + frame counters of the last frame. */
typedef struct {
    uint32_t gaussian_count;
    uint32_t visible;         /* visibleCount after compaction */
    uint32_t total_instances; /* after the clamp to max_instances */
    uint32_t max_instances;   /* 4 * max_gaussians */
    uint32_t overflow;        /* 1 when the clamp fired (DepthFirstShaders.metal:2191-2194) */
    uint32_t tiles_x, tiles_y, tile_count;
} gsm_depthfirst_counters;

/* Buffers of the last frame that can be copied back (reference resource in brackets). */
typedef enum {
    GSM_DF_BUF_RENDER_DATA = 0,      /* StereoTiledRenderData[count], 32 B [renderData]; culled entries undefined */
    GSM_DF_BUF_BOUNDS = 1,           /* int32[count][4] union tile rect [bounds] */
    GSM_DF_BUF_TOUCHED = 2,          /* uint32[count] tiles of the union rect [nTouchedTiles] */
    GSM_DF_BUF_DEPTH_KEYS = 3,       /* uint32[count] float_to_sortable_uint(centre depth) [preDepthKeys] */
    GSM_DF_BUF_DEPTH_ORDER = 4,      /* int32[visible] ids after the depth sort [primitiveIndices] */
    GSM_DF_BUF_INSTANCE_TILES = 5,   /* uint32[total_instances] sorted tile ids [instanceTileIds] */
    GSM_DF_BUF_INSTANCE_GAUSSIANS = 6, /* int32[total_instances] [instanceGaussianIndices] */
    GSM_DF_BUF_HEADERS = 7,          /* GaussianHeader[tile_count] {offset, count} [tileHeaders] */
    GSM_DF_BUF_BLEND_STATS = 8       /* uint64[4] (profiling bit 1): list entries the blend walked, of
                                        which had the eye's mean, of which blended; list entries */
} gsm_depthfirst_buffer;

gsm_status gsm_depthfirst_debug_counters(gsm_depthfirst *renderer, gsm_depthfirst_counters *out);
/* Copies min(bytes, size) bytes; *needed (nullable) receives the full size. */
gsm_status gsm_depthfirst_debug_copy(gsm_depthfirst *renderer, int which, void *host_dst, size_t bytes,
                                     size_t *needed);
/* bit 0: bracket every stage with HIP events (GSM_DF_STAGE_*); bit 1: count the blend's walk
 * (GSM_DF_BUF_BLEND_STATS); bit 3: only the blend (two events per frame, for timing the blend
 * inside a timed loop); bits 8-15 with bit 3: a period P > 1 brackets every P-th frame only. */
gsm_status gsm_depthfirst_set_profiling(gsm_depthfirst *renderer, int enable);
typedef enum {
    GSM_DF_STAGE_PROJECT = 0, /* project both eyes + visibility compaction */
    GSM_DF_STAGE_DEPTH_SORT = 1,
    GSM_DF_STAGE_INSTANCES = 2, /* ordered counts, scan, instance expansion */
    GSM_DF_STAGE_TILE_SORT = 3, /* stable tile sort + tile ranges */
    GSM_DF_STAGE_BLEND = 4,     /* both eyes, written side by side into the target */
    GSM_DF_STAGE_COUNT = 5
} gsm_depthfirst_stage;
/* Average milliseconds per stage over the profiled frames (after stream sync). */
gsm_status gsm_depthfirst_stage_times(gsm_depthfirst *renderer, float *ms, int n);
/* DepthFirstRenderer.lastGPUTime (DepthFirstRenderer.swift:43): seconds of the last profiled frame. */
gsm_status gsm_depthfirst_last_gpu_time(gsm_depthfirst *renderer, double *seconds);

#ifdef __cplusplus
}
#endif
#endif
