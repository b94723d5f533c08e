// gsm_types.h -- wire formats shared by the host orchestration and the gfx950 kernels.
//
// Layouts are byte-identical to the reference's C bridging header
// (Sources/RendererTypes/include/BridgingTypes.h); sizes are pinned by static_asserts
// (measured with clang in SURVEY.md section 2).  fp16 fields are carried as raw
// uint16 bits so host and device agree without relying on a host half type.
#pragma once
#include <cstddef>
#include <cstdint>

namespace gsm {

// BridgingTypes.h:57-64 -- 48 B, align 16.
struct alignas(16) PackedWorldGaussian {
    float px, py, pz;
    float opacity;
    float sx, sy, sz;
    float pad0;
    float rot[4];  // x, y, z, w
};
static_assert(sizeof(PackedWorldGaussian) == 48, "PackedWorldGaussian must be 48 B");

// BridgingTypes.h:66-73 -- 32 B (the Swift doc comment's "24 bytes" is wrong).
struct PackedWorldGaussianHalf {
    float px, py, pz;
    uint16_t opacity;
    uint16_t sx, sy, sz;
    uint16_t rx, ry, rz, rw;
    uint16_t pad0, pad1;
};
static_assert(sizeof(PackedWorldGaussianHalf) == 32, "PackedWorldGaussianHalf must be 32 B");
static_assert(offsetof(PackedWorldGaussianHalf, opacity) == 12, "layout");
static_assert(offsetof(PackedWorldGaussianHalf, rx) == 20, "layout");

// BridgingTypes.h:75-84 -- 16 B projected splat.
struct GaussianRenderData {
    uint16_t meanX, meanY;  // fp16 pixel-centred screen position
    uint16_t theta;         // [0, pi) * 65535 / pi
    uint16_t sigma1, sigma2;
    uint16_t depth;         // fp16 clip.w
    uint8_t colorR, colorG, colorB, opacity;
};
static_assert(sizeof(GaussianRenderData) == 16, "GaussianRenderData must be 16 B");

// BridgingTypes.h:22-39 -- 208 B camera constants (simd_float3 occupies 16 B).
struct alignas(16) CameraUniforms {
    float view[16];
    float proj[16];
    float cameraCenter[3];
    float cameraCenterPad;
    float pixelFactor;
    float focalX, focalY;
    float width, height;
    float nearPlane, farPlane;
    uint32_t shComponents;
    uint32_t gaussianCount;
    float inputIsSRGB;
    float pad1, pad2, pad3;
};
static_assert(sizeof(CameraUniforms) == 208, "CameraUniforms must be 208 B");
static_assert(offsetof(CameraUniforms, pixelFactor) == 144, "layout");
static_assert(offsetof(CameraUniforms, width) == 156, "layout");
static_assert(offsetof(CameraUniforms, shComponents) == 172, "layout");
static_assert(offsetof(CameraUniforms, inputIsSRGB) == 180, "layout");

// BridgingTypes.h:86-97 -- 40 B projection/binning constants.
struct TileBinningParams {
    uint32_t gaussianCount;
    uint32_t tilesX, tilesY;
    uint32_t tileWidth, tileHeight;
    uint32_t surfaceWidth, surfaceHeight;
    uint32_t maxCapacity;
    float alphaThreshold;
    float totalInkThreshold;
};
static_assert(sizeof(TileBinningParams) == 40, "TileBinningParams must be 40 B");

// BridgingTypes.h:99-104 -- GPU-side assignment counters.
struct TileAssignmentHeader {
    uint32_t totalAssignments;
    uint32_t maxCapacity;
    uint32_t paddedCount;
    uint32_t overflow;
};
static_assert(sizeof(TileAssignmentHeader) == 16, "TileAssignmentHeader must be 16 B");

// BridgingTypes.h:52-55.
struct GaussianHeader {
    uint32_t offset;
    uint32_t count;
};
static_assert(sizeof(GaussianHeader) == 8, "GaussianHeader must be 8 B");

// BridgingTypes.h:41-50.
struct RenderParams {
    uint32_t width, height, tileWidth, tileHeight, tilesX, tilesY, activeTileCount, gaussianCount;
};
static_assert(sizeof(RenderParams) == 32, "RenderParams must be 32 B");

// Build-internal per-gaussian blend record (not a reference type): the values
// globalRender recomputes per (tile, thread, entry) (GlobalShaders.metal:1094-1105)
// computed once per gaussian by the projection kernel.  All fields fp16 bits.
//   a.x = meanX | meanY<<16, a.y = cxx | cyy<<16, a.z = cxy2 | opacity<<16,
//   a.w = colR | colG<<16, b = colB | depth<<16
struct BlendRecordA {
    uint32_t x, y, z, w;
};
// The blend reads a record as one 16-B and one 4-B load of the same 32-B slot: one 64-B memory
// segment per gathered entry instead of one per array (tools/exp/fetch_calib.hip: a gather costs a
// 64-B segment whatever its width).
struct BlendRecord {
    BlendRecordA a;
    uint32_t b;
    float bandX, bandHalfWidth;  // the half-tile skip band (k_project / k_records_in -> k_scatter)
    uint32_t pad;
};
static_assert(sizeof(BlendRecord) == 32, "BlendRecord is one 32-B slot");

// BridgingTypes.h:250-276 -- 32 B projected splat of the DepthFirst stereo path: per eye fp16
// mean, conic (cxx, cyy, 2*cxy) and depth; shared u8 colour/opacity and fp16 centre depth.
struct StereoTiledRenderData {
    uint16_t leftMeanX, leftMeanY, leftCxx, leftCyy, leftCxy2, leftDepth;
    uint16_t rightMeanX, rightMeanY, rightCxx, rightCyy, rightCxy2, rightDepth;
    uint8_t colorR, colorG, colorB, opacity;
    uint16_t centerDepth, pad0;
};
static_assert(sizeof(StereoTiledRenderData) == 32, "StereoTiledRenderData must be 32 B");
static_assert(offsetof(StereoTiledRenderData, rightMeanX) == 12, "layout");
static_assert(offsetof(StereoTiledRenderData, colorR) == 24, "layout");

// Tile-slab bookkeeping for one frame.
struct FrameGeometry {
    uint32_t tilesX, tilesY, tileCount;
    uint32_t rowBegin, rowEnd;  // tile rows owned by this renderer: rowBegin, + rowStride, ... < rowEnd
    uint32_t rowStride, rowCount;
    uint32_t width, height;     // frame (camera) size
    uint32_t maxAssignments;
};

constexpr uint32_t kTileWidth = 32;   // GlobalRenderer.swift:74
constexpr uint32_t kTileHeight = 16;  // GlobalRenderer.swift:75
constexpr uint32_t kMaxSupportedGaussians = 30000000u;  // GlobalRenderer.swift:73

}  // namespace gsm
