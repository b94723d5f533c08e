// gsm_df_internal.h -- device buffers, kernel arguments and launchers of the DepthFirst stereo
// side-by-side path (gsm_df_kernels.hip; host orchestration in gsm_depthfirst.hip).
// Reference: Sources/Renderer/DepthFirstRenderer/ (DepthFirstRenderer.swift:469-831,
// DepthFirstShaders.metal) -- SURVEY.md 8(f) rank 1.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gsm_internal.h"
#include "gsm_types.h"

namespace gsm {

constexpr uint32_t kDfTile = 16;  // DepthFirstRenderer.swift:8-9 (16x16 tiles)

// Per-eye uniforms of projectToEye (DepthFirstShaders.metal:249-339): the eye's matrices and
// the projectCovariance2D terms evaluated once on the host.
struct DfEyeConst {
    float view[16], proj[16];
    float limX, limY, focalX, focalY;
};

// StereoCameraUniforms + TileBinningParams of one frame (BridgingTypes.h:222-248, 86-97).
struct DfArgs {
    DfEyeConst eye[2];
    float scene[16];    // sceneTransform, column-major
    float sceneScale;   // length(sceneTransform[0].xyz)
    float width, height, nearPlane, farPlane;  // per eye; near/far of the left camera
    float maxEig, adjFar, adjDen;
    float mid[3];       // midpoint of the two camera centres (SH direction)
    float inputIsSRGB;
    uint32_t shComponents, count, tilesX, tilesY, tileCount, maxInstances;
    uint32_t schedUnits;  // > 0: the projection launch also orders this many blend units (block 0)
};

// The DepthFirstResources analogue (DepthFirstResources.swift:380-470), sized at create time.
struct DfArena {
    StereoTiledRenderData* renderData = nullptr;  // [maxG]
    short4* bounds = nullptr;                     // [maxG] union tile rect
    uint32_t* touched = nullptr;                  // [maxG] nTouchedTiles
    uint32_t* depthKeys = nullptr;                // [maxG] preDepthKeys
    uint32_t* blockSums = nullptr;                // [ceil(maxG/256) + 1] visible counts per block
    uint32_t* instSums = nullptr;                 // [ceil(maxG/256) + 1] instance counts per block
    TileAssignmentHeader* visHdr = nullptr;       // totalAssignments = visibleCount
    TileAssignmentHeader* instHdr = nullptr;      // totalAssignments = totalInstances (clamped)
    uint32_t* dkeys[2] = {nullptr, nullptr};      // [maxG] depth sort ping-pong
    uint32_t* dvals[2] = {nullptr, nullptr};
    uint32_t* ikeys[2] = {nullptr, nullptr};      // [maxInstances] tile ids
    uint32_t* ivals[2] = {nullptr, nullptr};      // [maxInstances] gaussian ids
    uint32_t* radixHist = nullptr;
    size_t radixHistBytes = 0;
    uint32_t* radixBinTotals = nullptr;
    uint32_t* starts = nullptr;                   // [tileCount + 1] first instance of each tile
    uint32_t* queue = nullptr;                    // blend work counter
    uint16_t* expTable = nullptr;                 // [65536] stereo alpha table (r^2 cutoff folded)
    uint16_t* unitCost = nullptr;                 // [2 * maxTiles] entries each (tile, eye) unit walked
    uint32_t* unitOrder = nullptr;                // [2 * maxTiles] units, longest last-frame walk first
    uint32_t* costMax = nullptr;                  // [kCostMaxSlots] longest walk of the last blend
    unsigned long long* blendStats = nullptr;     // [4] profiling bit 1: entries walked / with a real
                                                  // mean / blended, list entries (null: not counted)
};
inline SortSpace sort_space(const DfArena& A) { return SortSpace{A.radixHist, A.radixHistBytes, A.radixBinTotals, kSortTotalsWords}; }

constexpr int kDfBlock = 256;
// instance values: gaussian id in bits 0-29 (max_gaussians <= 30M < 2^30); bit 30 + e set when eye e
// provably adds nothing to the instance's tile (k_df_expand, df_eye_misses_tile)
constexpr uint32_t kDfSkipShift = 30;
constexpr uint32_t kDfGidMask = (1u << kDfSkipShift) - 1u;


// depthFirstStereoProjectCullKernel (DepthFirstShaders.metal:341-499) + per-block visible counts
void df_launch_project(bool halfInput, uint32_t shDegree, const void* world, const void* harmonics,
                       const DfArgs& a, const DfArena& A, hipStream_t stream);
// visibilityScatterCompactKernel (:589-621): (depth key, id) of the visible gaussians, ascending id
void df_launch_compact(const DfArgs& a, const DfArena& A, hipStream_t stream);
// applyDepthOrderingKernel + instance prefix sum + createInstancesStereoKernel (:623-640, :790-826)
void df_launch_instance_counts(const uint32_t* order, const DfArgs& a, const DfArena& A, hipStream_t stream);
void df_launch_instances(const uint32_t* order, const DfArgs& a, const DfArena& A, hipStream_t stream);
// extractTileRangesKernel (:1258-1313)
// clearStereoRenderTextureKernel + depthFirstStereoRender + DepthFirstStereoCopyEncoder
// (:1813-1982; DepthFirstStereoCopyEncoder.swift:29-99) in one persistent kernel
// costOrder: hand the units out longest-last-frame-walk first (A.unitOrder, filled by block 0 of
// the projection launch from A.unitCost); the blend records this frame's walks into A.unitCost
// and each wave's longest into A.costMax
void df_launch_blend(const uint32_t* sortedGids, const DfArgs& a, const DfArena& A, void* color, size_t pitch,
                     int colorFormat, int numCUs, bool costOrder, hipStream_t stream);

}  // namespace gsm
