/*
 * gsm_oracle.h -- CPU restatement of the reference GlobalRenderer hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * implementation in gsm-renderer_amd/.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product never links it.
 *
 * Reference (LuckyIYI/gsm-renderer, read-only at /root/reference):
 *   Sources/Renderer/GlobalRenderer/GlobalShaders.metal   (kernels)
 *   Sources/Renderer/Shared/GaussianShared.h              (projection math)
 *   Sources/Renderer/GlobalRenderer/GlobalRenderer.swift  (frame orchestration)
 *   Sources/RendererTypes/include/BridgingTypes.h         (wire formats)
 *
 * Parity status: the reference is Swift+Metal and cannot be compiled or run in
 * this environment.  The radix-sort key format and sort
 * are pinned by the reference's own known-answer tests
 * (Tests/RendererTests/GlobalUnitTests.swift:23-178, regenerated bit-exactly
 * from glibc drand48, see tests/test_oracle_kat.py).  Projection and blend
 * arithmetic follow the Metal source line by line with the declared numeric
 * choices of DESIGN.md ("Numeric contract"); against real Metal output they
 * are "parity unpinned" (Metal's -ffast-math transcendentals are unknowable).
 */
#ifndef GSM_ORACLE_H
#define GSM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* BridgingTypes.h:57-64 PackedWorldGaussian (48 B, align 16). */
typedef struct {
    float px, py, pz;
    float opacity;
    float sx, sy, sz;
    float pad0;
    float rot[4]; /* quaternion x,y,z,w */
} og_world32;

/* BridgingTypes.h:66-73 PackedWorldGaussianHalf (32 B). fp16 fields as raw bits. */
typedef struct {
    float px, py, pz;
    uint16_t opacity;
    uint16_t sx, sy, sz;
    uint16_t rx, ry, rz, rw;
    uint16_t pad0, pad1;
} og_world16;

/* BridgingTypes.h:75-84 GaussianRenderData (16 B). */
typedef struct {
    uint16_t meanX, meanY; /* fp16 */
    uint16_t theta;        /* [0,pi) * 65535/pi */
    uint16_t sigma1, sigma2, depth; /* fp16 */
    uint8_t colorR, colorG, colorB, opacity;
} og_render_data;

/* GaussianRendererProtocol.swift:28-54 CameraParams (matrices column-major, simd layout). */
typedef struct {
    float view[16];
    float proj[16];
    float position[3];
    float focal_x, focal_y; /* accepted, ignored by the Global path */
    float near_plane, far_plane;
} og_camera;

/* GaussianRendererProtocol.swift:195-228 RendererConfig (subset the Global path reads). */
typedef struct {
    uint32_t max_gaussians;
    uint32_t max_width, max_height;
    uint32_t precision;   /* 0 = float32 (PackedWorldGaussian + f32 SH), 1 = float16 */
    uint32_t color_space; /* 0 = linear, 1 = srgb (decode to linear in projection) */
} og_config;

/* Everything one frame produces; owned by the oracle, freed by og_frame_free. */
typedef struct {
    uint32_t count, width, height;
    uint32_t tiles_x, tiles_y, tile_count;
    uint32_t max_assignments;
    uint32_t total_assignments; /* after the 4*maxGaussians clamp */
    uint32_t overflow;
    uint32_t visible;
    uint32_t active_tiles;
    og_render_data *render_data; /* [count]; culled entries zero-filled */
    int32_t *bounds;             /* [count*4] minTX,maxTX,minTY,maxTY ((0,-1,0,-1) = culled) */
    uint8_t *mask;               /* [count] */
    uint32_t *tile_counts;       /* [count] tiles each gaussian is assigned to */
    uint32_t *keys;              /* [total] (tile<<16)|(fp16(depth)^0x8000), assignment order */
    int32_t *values;             /* [total] gaussian index, assignment order */
    uint32_t *sorted_keys;       /* [total] */
    int32_t *sorted_values;      /* [total] */
    uint32_t *headers;           /* [tile_count*2] {offset,count} */
    uint16_t *color;             /* [height*width*4] rgba16f bits */
    uint16_t *depth;             /* [height*width]   r16f bits */
    uint32_t *group_iters;       /* [tile_count*64] entries each 4x2 thread group processed before its break */
    double t_project, t_assign, t_sort, t_headers, t_blend; /* seconds */
} og_frame;

enum {
    OG_OK = 0,
    OG_ERR_INVALID_GAUSSIAN_COUNT = 5,
    OG_ERR_INVALID_DIMENSIONS = 6,
    OG_ERR_INVALID_ARGUMENT = 10,
    OG_ERR_OUT_OF_MEMORY = 11
};

/* GlobalRenderer.render (GlobalRenderer.swift:201-238) for one frame.
 * gaussians: og_world32[count] (precision 0) or og_world16[count] (precision 1)
 * harmonics: planar SH per gaussian, float or fp16 bits.
 * nthreads <= 0 uses all online CPUs. */
int og_render(const og_config *cfg, const void *gaussians, const void *harmonics,
              uint32_t count, uint32_t sh_components, const og_camera *cam,
              uint32_t width, uint32_t height, int nthreads, og_frame **out);
void og_frame_free(og_frame *f);

/* Stage entry points for unit tests (same code the frame uses). */
uint32_t og_sort_key(uint32_t tile, uint16_t depth_h);
/* Stable LSD radix sort of (key,value) pairs, 8-bit digits (RadixSortEncoder.swift:41-101). */
void og_radix_sort_pairs(uint32_t *keys, int32_t *values, uint32_t n);

/* The colour target's pixel format (include/gsm_renderer.h gsm_color_format): converts n
 * rgba16f pixels (the frame's colour) into dst -- 0 rgba16f copy, 1 rgba32f, 2 rgba8 unorm,
 * 3 rgba8 unorm sRGB, 4 bgra8 unorm, 5 bgra8 unorm sRGB.  Returns bytes per pixel or 0. */
int og_convert_color(const uint16_t *rgba16f, size_t n, int format, void *dst);

/* fp16 helpers (round-to-nearest-even, IEEE binary16). */
uint16_t og_f2h(float f);
float og_h2f(uint16_t h);
uint16_t og_d2h(double d);
/* Correctly rounded fp16 e^x for every fp16 x (DESIGN.md numeric contract). */
uint16_t og_exp_h(uint16_t x_bits);
/* fp16 a*b + c with one rounding to nearest even (the blend's fused `C += c * w`) */
uint16_t og_hfma(uint16_t a, uint16_t b, uint16_t c);
/* Deterministic fp32 math (fixed polynomials, see tools/fit_polys.py). */
float og_atan2f(float y, float x);
float og_log2f(float x);
float og_exp2f(float x);

/* Reference test-fixture generators (Tests/RendererTests/TestUtils.swift). drand48-seeded. */
void og_srand48(long seed);
double og_drand48(void);
/* generateVisibleGaussians (TestUtils.swift:189-231) packed as makePackedBuffers
 * (TestUtils.swift:236-276): PackedWorldGaussian + 3 float harmonics (SH0). */
void og_gen_visible_gaussians(uint32_t count, long seed, og_world32 *world, float *harmonics);
/* generateGridGaussians (TestUtils.swift:144-185). */
void og_gen_grid_gaussians(uint32_t count, long seed, og_world32 *world, float *harmonics);
/* makeCameraParams (TestUtils.swift:74-94), OpenCV convention, identity view. */
void og_make_camera(uint32_t width, uint32_t height, og_camera *cam);

/* ---- DepthFirst stereo side-by-side ---------------------------- */
/* BridgingTypes.h:250-276 StereoTiledRenderData (32 B).  fp16 fields as raw bits; an eye the
 * gaussian is not visible in has mean = fp16(-1e10) = -inf and zero conic/depth. */
typedef struct {
    uint16_t leftMeanX, leftMeanY, leftCxx, leftCyy, leftCxy2, leftDepth;
    uint16_t rightMeanX, rightMeanY, rightCxx, rightCyy, rightCxy2, rightDepth;
    uint8_t colorR, colorG, colorB, opacity;
    uint16_t centerDepth, pad0;
} og_stereo_render_data;

typedef struct {
    uint32_t count, width, height; /* width, height: per eye */
    uint32_t tiles_x, tiles_y, tile_count, max_instances;
    uint32_t visible, total_instances, overflow, active_tiles;
    og_stereo_render_data *render_data; /* [count]; culled entries zero-filled */
    int32_t *bounds;      /* [count*4] union tile rect, (0,-1,0,-1) when culled */
    uint32_t *touched;    /* [count] tiles of the union rect, 0 when culled */
    uint32_t *depth_keys; /* [count] float_to_sortable_uint(centre depth), 0xFFFFFFFF when culled */
    int32_t *depth_order; /* [visible] gaussian ids after the stable 32-bit depth sort */
    uint32_t *inst_tiles; /* [total_instances] tile ids after the stable tile sort */
    int32_t *inst_gids;   /* [total_instances] */
    uint32_t *headers;    /* [tile_count*2] {offset, count} */
    uint16_t *eye_color;  /* [2][height][width][4] the intermediate rgba16f slices (0 = left) */
    uint16_t *color;      /* [height][2*width][4] the side-by-side target after the copy */
    double t_project, t_sort, t_blend;
} og_df_frame;

/* DepthFirstRenderer.renderStereo(target: .sideBySide) (DepthFirstRenderer.swift:205-223,
 * 469-512, 595-831).  scene_transform: 16 floats column-major (StereoConfiguration.sceneTransform,
 * GaussianRendererProtocol.swift:106) or NULL for the identity the side-by-side path uses. */
int og_df_render_stereo(const og_config *cfg, const void *gaussians, const void *harmonics,
                        uint32_t count, uint32_t sh_components, const og_camera *left,
                        const og_camera *right, const float *scene_transform, uint32_t width,
                        uint32_t height, int nthreads, og_df_frame **out);
void og_df_frame_free(og_df_frame *f);
/* sin/cos of an fp32 angle (numeric contract) and float_to_sortable_uint. */
void og_sincos_theta(float th, float *s, float *c);
uint32_t og_float_to_sortable(float v);

#ifdef __cplusplus
}
#endif
#endif
