/*
 * gsm_ply.h -- PLY ingestion for the GlobalRenderer input.
 *
 * Restates the reference's PLYLoader.load (Sources/Renderer/Utils/PLYLoader.swift:254-742:
 * standard 3DGS PLY with logit / log-space detection, placeholder skip, planar SH re-layout
 * and recentering; PlayCanvas "splat-transform" compressed PLY with 256-vertex chunks),
 * GaussianSceneBuilder.bounds and sortByMortonCode (Sources/Renderer/Utils/Scene.swift:54-187),
 * and the packing into the renderer's GaussianInput buffers (PackedWorldGaussian /
 * PackedWorldGaussianHalf init, Sources/Renderer/Shared/KernelTypes.swift:12-53, as
 * Tests/RendererTests/PLYBenchmarkTests.swift:137-147 does it).  Host memory only: the caller
 * copies the packed buffers to the device and passes them to gsm_global_render.
 */
#ifndef GSM_PLY_H
#define GSM_PLY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* PLYLoaderError (PLYLoader.swift:220-247) and PLYHeader.DecodeError (:91-113). */
typedef enum {
    GSM_PLY_OK = 0,
    GSM_PLY_ERR_IO = 1,                          /* file cannot be opened / read (Data(contentsOf:) throws) */
    GSM_PLY_ERR_INVALID_HEADER = 2,              /* .invalidHeader: no end_header line */
    GSM_PLY_ERR_UNSUPPORTED_FORMAT = 3,          /* .unsupportedFormat: ascii / big endian */
    GSM_PLY_ERR_MISSING_VERTEX_ELEMENT = 4,      /* .missingVertexElement */
    GSM_PLY_ERR_MISSING_REQUIRED_PROPERTIES = 5, /* .missingRequiredProperties(["x","y","z"]) */
    GSM_PLY_ERR_LIST_PROPERTIES_NOT_SUPPORTED = 6, /* .listPropertiesNotSupported */
    GSM_PLY_ERR_INSUFFICIENT_DATA = 7,           /* .insufficientData */
    GSM_PLY_ERR_MISSING_CHUNK_ELEMENT = 8,       /* .missingChunkElement */
    GSM_PLY_ERR_HEADER_FORMAT_MISSING = 9,       /* DecodeError.headerFormatMissing */
    GSM_PLY_ERR_HEADER_INVALID_CHARACTERS = 10,  /* DecodeError.headerInvalidCharacters */
    GSM_PLY_ERR_HEADER_UNKNOWN_KEYWORD = 11,     /* DecodeError.headerUnknownKeyword */
    GSM_PLY_ERR_HEADER_UNEXPECTED_KEYWORD = 12,  /* DecodeError.headerUnexpectedKeyword */
    GSM_PLY_ERR_HEADER_INVALID_LINE = 13,        /* DecodeError.headerInvalidLine */
    GSM_PLY_ERR_HEADER_INVALID_FORMAT_TYPE = 14, /* DecodeError.headerInvalidFileFormatType */
    GSM_PLY_ERR_HEADER_UNKNOWN_PROPERTY_TYPE = 15, /* DecodeError.headerUnknownPropertyType */
    GSM_PLY_ERR_INVALID_ARGUMENT = 16            /* null pointer / short output buffer */
} gsm_ply_status;

/* GaussianDataset (Scene.swift:141-158): records + planar harmonics; opaque. */
typedef struct gsm_ply_scene gsm_ply_scene;

/* PLYLoader.load(url:) (PLYLoader.swift:254-287).  `path` is a file path; `bytes`/`size`
 * load from memory instead (path == NULL).  On error *out is NULL and the message of the
 * failure is available from gsm_ply_last_error(). */
gsm_ply_status gsm_ply_load(const char *path, gsm_ply_scene **out);
gsm_ply_status gsm_ply_load_memory(const void *bytes, size_t size, gsm_ply_scene **out);
const char *gsm_ply_last_error(void);
const char *gsm_ply_status_string(gsm_ply_status s);
void gsm_ply_free(gsm_ply_scene *scene);

/* dataset.records.count, dataset.shComponents; compressed: 1 when the file was compressed */
uint32_t gsm_ply_count(const gsm_ply_scene *scene);
uint32_t gsm_ply_sh_components(const gsm_ply_scene *scene);
int gsm_ply_is_compressed(const gsm_ply_scene *scene);

/* The records as arrays (any pointer may be NULL): positions [n][3], scales [n][3] (linear),
 * rotations [n][4] as (x, y, z, w) = (imag, real) of the simd_quatf, opacities [n] (linear),
 * harmonics [n * 3 * sh_components] planar per gaussian [R0..Rk-1, G.., B..]. */
gsm_ply_status gsm_ply_records(const gsm_ply_scene *scene, float *positions, float *scales, float *rotations,
                               float *opacities, float *harmonics);

/* GaussianSceneBuilder.bounds(of:) (Scene.swift:172-196): center[3], radius. */
gsm_ply_status gsm_ply_bounds(const gsm_ply_scene *scene, float center[3], float *radius);

/* GaussianSceneBuilder.sortByMortonCode (Scene.swift:74-138), in place; ties keep file order. */
gsm_ply_status gsm_ply_sort_morton(gsm_ply_scene *scene);

/* GaussianInput buffers on the host: precision 0 -> PackedWorldGaussian (48 B) + float SH,
 * 1 -> PackedWorldGaussianHalf (32 B) + half SH (KernelTypes.swift:12-53; Float16(x) rounds
 * to nearest even).  Sizes: gsm_ply_packed_sizes. */
gsm_ply_status gsm_ply_packed_sizes(const gsm_ply_scene *scene, int precision, size_t *gaussian_bytes,
                                    size_t *harmonic_bytes);
gsm_ply_status gsm_ply_pack(const gsm_ply_scene *scene, int precision, void *gaussians, size_t gaussian_bytes,
                            void *harmonics, size_t harmonic_bytes);

#ifdef __cplusplus
}
#endif
#endif /* GSM_PLY_H */
