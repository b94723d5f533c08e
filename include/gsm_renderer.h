/*
 * gsm_renderer.h -- C ABI of the MI355X-native GlobalRenderer (libgsm_amd.so).
 *
 * Drop-in boundary for the reference's GlobalRenderer operator surface
 * (LuckyIYI/gsm-renderer, Swift + Metal).  Each declaration cites the reference
 * interface it replaces (paths relative to the reference repository root).
 * Plain pointers and sizes only: device buffers are HIP device pointers, the
 * stream is a hipStream_t passed as void*.  No torch / HIP types appear here.
 *
 * Threading: one in-flight frame per handle (the reference's GlobalRenderer owns
 * a single scratch set, GlobalRenderer.swift:72,94); handles are independent and
 * each is bound to one HIP device.
 */
#ifndef GSM_RENDERER_H
#define GSM_RENDERER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSM_ABI_VERSION 1

/* RendererError (Sources/Renderer/Shared/GaussianRendererProtocol.swift:274-292). */
typedef enum {
    GSM_OK = 0,
    GSM_ERR_DEVICE_NOT_AVAILABLE = 1,        /* .deviceNotAvailable */
    GSM_ERR_FAILED_TO_CREATE_LIBRARY = 2,    /* .failedToCreateLibrary */
    GSM_ERR_FAILED_TO_CREATE_PIPELINE = 3,   /* .failedToCreatePipeline */
    GSM_ERR_FAILED_TO_ALLOCATE_BUFFER = 4,   /* .failedToAllocateBuffer */
    GSM_ERR_FAILED_TO_ALLOCATE_TEXTURE = 5,  /* .failedToAllocateTexture */
    GSM_ERR_INVALID_GAUSSIAN_COUNT = 6,      /* .invalidGaussianCount */
    GSM_ERR_INVALID_DIMENSIONS = 7,          /* .invalidDimensions */
    GSM_ERR_INVALID_BUFFER_SIZE = 8,         /* .invalidBufferSize */
    GSM_ERR_INVALID_TILE_COUNT = 9,          /* .invalidTileCount */
    GSM_ERR_INVALID_ASSIGNMENT_CAPACITY = 10,/* .invalidAssignmentCapacity */
    GSM_ERR_RENDER_FAILED = 11,              /* .renderFailed */
    GSM_ERR_ENCODER_CREATION_FAILED = 12,    /* .encoderCreationFailed */
    GSM_ERR_MISSING_REQUIRED_BUFFER = 13,    /* .missingRequiredBuffer */
    GSM_ERR_INVALID_ARGUMENT = 14,           /* null handle / pointer (no Swift analogue) */
    GSM_ERR_UNSUPPORTED = 15,                /* renderStereo on Global: fatalError in the reference */
    GSM_ERR_PHASE_ORDER = 16                 /* gsm_multigpu_render_phase out of order (gsm_multigpu.h) */
} gsm_status;

/* RenderPrecision (GaussianRendererProtocol.swift:4-7). */
typedef enum { GSM_PRECISION_FLOAT32 = 0, GSM_PRECISION_FLOAT16 = 1 } gsm_precision;
/* RendererConfig.GaussianColorSpace (GaussianRendererProtocol.swift:196-201). */
typedef enum { GSM_COLOR_SPACE_LINEAR = 0, GSM_COLOR_SPACE_SRGB = 1 } gsm_color_space;

/* Pixel format of the colour target (RendererConfig.colorFormat, GaussianRendererProtocol.swift:207;
 * the reference's Global path writes half4 into whatever texture it is given and Metal converts
 * on the write, GlobalShaders.metal:1155-1186).  With raw device pointers the format of the
 * target is declared here.  Conversion of the blended fp16 value c (alpha = 1 - T):
 *   RGBA16F: as is (8 B/px);  RGBA32F: exact widening (16 B/px);
 *   *8_UNORM: u8 = RTNE(clamp(c, 0, 1) * 255), clamp by IEEE maxNum/minNum (NaN -> 0) (4 B/px);
 *   *8_UNORM_SRGB: the same after the linear->sRGB encode of R, G, B:
 *     c <= 0.0031308 ? 12.92 c : 1.055 powr(c, 1 / 2.4) - 0.055 (fp32, powr of the numeric contract).
 * BGRA formats store B, G, R, A.  The Metal rounding of unorm / sRGB writes is not specified
 * to the bit: parity for the 8-bit formats is against this definition. */
typedef enum {
    GSM_COLOR_FORMAT_RGBA16F = 0,
    GSM_COLOR_FORMAT_RGBA32F = 1,
    GSM_COLOR_FORMAT_RGBA8_UNORM = 2,
    GSM_COLOR_FORMAT_RGBA8_UNORM_SRGB = 3,
    GSM_COLOR_FORMAT_BGRA8_UNORM = 4,
    GSM_COLOR_FORMAT_BGRA8_UNORM_SRGB = 5 /* the reference's RendererConfig default (.bgra8Unorm_srgb) */
} gsm_color_format;

/* RendererConfig (GaussianRendererProtocol.swift:195-228).  back_to_front is accepted and
 * ignored, as in the reference Global path. */
typedef struct {
    uint32_t max_gaussians;        /* default 6_000_000, <= 30_000_000 (GlobalRenderer.swift:73) */
    uint32_t max_width;            /* default 1920 */
    uint32_t max_height;           /* default 1080 */
    uint32_t precision;            /* gsm_precision, default FLOAT16 */
    uint32_t color_format;         /* gsm_color_format of the colour target, default RGBA16F */
    uint32_t gaussian_color_space; /* gsm_color_space, default SRGB */
    uint32_t back_to_front;        /* ignored */
} gsm_renderer_config;

/* GaussianInput (GaussianRendererProtocol.swift:9-26).  Device pointers owned by
 * the caller; they must stay valid until the stream work of the frame is done.
 * gaussians: PackedWorldGaussian (48 B) when precision == FLOAT32, else
 * PackedWorldGaussianHalf (32 B) (BridgingTypes.h:57-73).  harmonics: planar
 * per-gaussian SH [R0..Rk-1, G0.., B0..], float (FLOAT32) or half (FLOAT16). */
typedef struct {
    const void *gaussians;
    const void *harmonics;
    uint32_t gaussian_count;
    uint32_t sh_components;
} gsm_gaussian_input;

/* CameraParams (GaussianRendererProtocol.swift:28-54).  Matrices are column-major
 * (simd_float4x4 memory layout).  focal_x/focal_y are ignored by the Global path
 * (focal comes from the projection matrix, GaussianShared.h:353-355). */
typedef struct {
    float view[16];
    float proj[16];
    float position[3];
    float focal_x;
    float focal_y;
    float near_plane; /* default 0.1 */
    float far_plane;  /* default 10.0 */
} gsm_camera_params;

typedef struct gsm_renderer gsm_renderer;

/* RendererConfig() defaults (GaussianRendererProtocol.swift:211-219). */
void gsm_renderer_config_default(gsm_renderer_config *config);
/* CameraParams.init defaults near = 0.1, far = 10 (GaussianRendererProtocol.swift:37-45). */
void gsm_camera_params_init(gsm_camera_params *camera, const float view[16], const float proj[16],
                            const float position[3], float focal_x, float focal_y);

/* GlobalRenderer.init(device:config:) (GlobalRenderer.swift:110-193).  Allocates
 * every scratch buffer up front (4 * max_gaussians assignment capacity,
 * GlobalResources.swift:79).  hip_device < 0 selects the current device. */
gsm_status gsm_global_create(const gsm_renderer_config *config, int hip_device, gsm_renderer **out);
void gsm_global_destroy(gsm_renderer *renderer);

/* GlobalRenderer.render(commandBuffer:colorTexture:depthTexture:input:camera:width:height:)
 * (GlobalRenderer.swift:201-238; protocol GaussianRendererProtocol.swift:248-256).
 * Enqueue-only on `stream` (the analogue of encoding into the caller's command
 * buffer; the caller synchronises).  color: config.color_format (rgba16Float by default),
 * height rows of color_pitch bytes; depth: r16Float or NULL (the reference then renders into
 * its own internal depth texture, GlobalRenderer.swift:350).  Returns an error
 * where the reference silently skips the frame (GlobalRenderer.swift:295-299). */
gsm_status gsm_global_render(gsm_renderer *renderer, void *stream, const gsm_gaussian_input *input,
                             const gsm_camera_params *camera, uint32_t width, uint32_t height,
                             void *color_rgba16f, size_t color_pitch_bytes, void *depth_r16f,
                             size_t depth_pitch_bytes);

/* GlobalRenderer.renderStereo (GlobalRenderer.swift:240-255) calls fatalError for
 * every target; this entry returns GSM_ERR_UNSUPPORTED instead. */
gsm_status gsm_global_render_stereo(gsm_renderer *renderer, void *stream,
                                    const gsm_gaussian_input *input,
                                    const gsm_camera_params *left, const gsm_camera_params *right,
                                    uint32_t width_per_eye, uint32_t height, void *color_rgba16f,
                                    size_t color_pitch_bytes, void *depth_r16f,
                                    size_t depth_pitch_bytes);

/* Config 5: both eyes of a stereo pair through the Global
 * path into one side-by-side target -- left eye in columns [0, width_per_eye), right eye in
 * [width_per_eye, 2 * width_per_eye) of rows of color_pitch bytes.  Each half equals
 * gsm_global_render of that eye (the two views are independent Global frames; the
 * DepthFirst renderer's shared-colour stereo semantics are not reproduced).  width_per_eye
 * is bounded by config.max_width. */
gsm_status gsm_global_render_stereo_sbs(gsm_renderer *renderer, void *stream,
                                        const gsm_gaussian_input *input,
                                        const gsm_camera_params *left, const gsm_camera_params *right,
                                        uint32_t width_per_eye, uint32_t height, void *color_rgba16f,
                                        size_t color_pitch_bytes, void *depth_r16f,
                                        size_t depth_pitch_bytes);

/* GlobalRenderer.debugReadTotalAssignments() (GlobalRenderer.swift:196-199): reads
 * the GPU counter; call after the frame's stream work has completed. */
uint32_t gsm_global_debug_read_total_assignments(gsm_renderer *renderer);

/* GaussianRenderer.lastGPUTime (GaussianRendererProtocol.swift:245, declared but
 * never assigned in the reference).  Seconds of the last frame measured with HIP
 * events when profiling is enabled (gsm_debug.h); returns GSM_ERR_RENDER_FAILED
 * when no measurement is available. */
gsm_status gsm_global_last_gpu_time(gsm_renderer *renderer, double *seconds);

const char *gsm_status_string(gsm_status status);
int gsm_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
