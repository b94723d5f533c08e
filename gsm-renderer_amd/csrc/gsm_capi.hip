// gsm_capi.hip -- extern "C" entry points declared in include/gsm_renderer.h and
// include/gsm_debug.h.  Thin, exception-free shims over gsm::GlobalRenderer.
#include <hip/hip_runtime.h>

#include <cstring>
#include <new>

#include "../../include/gsm_debug.h"
#include "../../include/gsm_multigpu.h"
#include "../../include/gsm_renderer.h"
#include "gsm_internal.h"
#include "gsm_renderer_impl.h"

extern "C" {

int gsm_abi_version(void) { return GSM_ABI_VERSION; }

const char* gsm_status_string(gsm_status s) {
    // RendererError.description (GaussianRendererProtocol.swift:294-323)
    switch (s) {
        case GSM_OK: return "ok";
        case GSM_ERR_DEVICE_NOT_AVAILABLE: return "HIP device not available";
        case GSM_ERR_FAILED_TO_CREATE_LIBRARY: return "Failed to create kernel library";
        case GSM_ERR_FAILED_TO_CREATE_PIPELINE: return "Failed to create pipeline";
        case GSM_ERR_FAILED_TO_ALLOCATE_BUFFER: return "Failed to allocate buffer";
        case GSM_ERR_FAILED_TO_ALLOCATE_TEXTURE: return "Failed to allocate texture";
        case GSM_ERR_INVALID_GAUSSIAN_COUNT: return "Gaussian count exceeds maximum";
        case GSM_ERR_INVALID_DIMENSIONS: return "Dimensions exceed maximum";
        case GSM_ERR_INVALID_BUFFER_SIZE: return "Buffer has invalid size";
        case GSM_ERR_INVALID_TILE_COUNT: return "Tile count exceeds maximum";
        case GSM_ERR_INVALID_ASSIGNMENT_CAPACITY: return "Required tile assignment capacity exceeds available";
        case GSM_ERR_RENDER_FAILED: return "Render failed";
        case GSM_ERR_ENCODER_CREATION_FAILED: return "Failed to create stage";
        case GSM_ERR_MISSING_REQUIRED_BUFFER: return "Missing required buffer";
        case GSM_ERR_INVALID_ARGUMENT: return "Invalid argument";
        case GSM_ERR_UNSUPPORTED: return "GlobalRenderer does not support stereo rendering";
        case GSM_ERR_PHASE_ORDER: return "Multi-GPU frame phase called out of order (gsm_multigpu_finish_frame)";
    }
    return "unknown status";
}

void gsm_renderer_config_default(gsm_renderer_config* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->max_gaussians = 6000000u;
    c->max_width = 1920u;
    c->max_height = 1080u;
    c->precision = GSM_PRECISION_FLOAT16;
    c->color_format = 0u;
    c->gaussian_color_space = GSM_COLOR_SPACE_SRGB;
    c->back_to_front = 0u;
}

void gsm_camera_params_init(gsm_camera_params* cam, const float view[16], const float proj[16],
                            const float position[3], float focal_x, float focal_y) {
    if (!cam) return;
    std::memset(cam, 0, sizeof(*cam));
    if (view) std::memcpy(cam->view, view, sizeof(cam->view));
    if (proj) std::memcpy(cam->proj, proj, sizeof(cam->proj));
    if (position) std::memcpy(cam->position, position, sizeof(cam->position));
    cam->focal_x = focal_x;
    cam->focal_y = focal_y;
    cam->near_plane = 0.1f;
    cam->far_plane = 10.0f;
}

gsm_status gsm_global_create(const gsm_renderer_config* config, int hip_device, gsm_renderer** out) {
    if (!out) return GSM_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    gsm_renderer_config cfg;
    if (config) cfg = *config;
    else gsm_renderer_config_default(&cfg);
    gsm::GlobalRenderer* impl = nullptr;
    gsm_status st = gsm::GlobalRenderer::create(cfg, hip_device, &impl);
    if (st != GSM_OK) return st;
    gsm_renderer* h = new (std::nothrow) gsm_renderer;
    if (!h) {
        delete impl;
        return GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    h->impl = impl;
    *out = h;
    return GSM_OK;
}

void gsm_global_destroy(gsm_renderer* r) {
    if (!r) return;
    delete r->impl;
    delete r;
}

gsm_status gsm_global_render(gsm_renderer* r, void* stream, const gsm_gaussian_input* input,
                             const gsm_camera_params* camera, uint32_t width, uint32_t height,
                             void* color, size_t color_pitch, void* depth, size_t depth_pitch) {
    if (!r || !r->impl || !input || !camera) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->render((hipStream_t)stream, *input, *camera, width, height, color, color_pitch,
                           depth, depth_pitch);
}

gsm_status gsm_global_project_partition(gsm_renderer* r, void* stream, const gsm_gaussian_input* input,
                                        const gsm_camera_params* camera, uint32_t width, uint32_t height,
                                        uint32_t first, uint32_t count, const uint32_t* slab_rows,
                                        uint32_t num_slabs, void* send, uint64_t send_capacity,
                                        uint32_t* send_counts) {
    if (!r || !r->impl || !input || !camera) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->projectPartition((hipStream_t)stream, *input, *camera, width, height, first, count,
                                     slab_rows, num_slabs, send, send_capacity, send_counts);
}

gsm_status gsm_global_render_records(gsm_renderer* r, void* stream, const void* records, uint32_t count,
                                     uint32_t width, uint32_t height, void* color, size_t color_pitch,
                                     void* depth, size_t depth_pitch) {
    if (!r || !r->impl) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->renderRecords((hipStream_t)stream, records, count, width, height, color, color_pitch,
                                  depth, depth_pitch);
}

gsm_status gsm_global_render_stereo_sbs(gsm_renderer* r, void* stream, const gsm_gaussian_input* input,
                                        const gsm_camera_params* left, const gsm_camera_params* right,
                                        uint32_t width_per_eye, uint32_t height, void* color, size_t color_pitch,
                                        void* depth, size_t depth_pitch) {
    if (!r || !r->impl || !input || !left || !right) return GSM_ERR_INVALID_ARGUMENT;
    if (!color) return GSM_ERR_MISSING_REQUIRED_BUFFER;
    gsm_status st = r->impl->render((hipStream_t)stream, *input, *left, width_per_eye, height, color,
                                    color_pitch, depth, depth_pitch);
    if (st != GSM_OK) return st;
    char* rc = (char*)color + (size_t)width_per_eye * 8;
    char* rd = depth ? (char*)depth + (size_t)width_per_eye * 2 : nullptr;
    return r->impl->render((hipStream_t)stream, *input, *right, width_per_eye, height, rc, color_pitch, rd,
                           depth_pitch);
}

gsm_status gsm_global_render_stereo(gsm_renderer* r, void*, const gsm_gaussian_input*,
                                    const gsm_camera_params*, const gsm_camera_params*, uint32_t,
                                    uint32_t, void*, size_t, void*, size_t) {
    if (!r) return GSM_ERR_INVALID_ARGUMENT;
    return GSM_ERR_UNSUPPORTED;  // GlobalRenderer.swift:248-254 fatalError
}

uint32_t gsm_global_debug_read_total_assignments(gsm_renderer* r) {
    if (!r || !r->impl) return 0;
    gsm_debug_counters c;
    if (r->impl->counters(&c) != GSM_OK) return 0;
    return c.total_assignments;
}

gsm_status gsm_global_last_gpu_time(gsm_renderer* r, double* seconds) {
    if (!r || !r->impl || !seconds) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->lastGpuTime(seconds);
}

gsm_status gsm_global_debug_counters(gsm_renderer* r, gsm_debug_counters* out) {
    if (!r || !r->impl || !out) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->counters(out);
}

gsm_status gsm_global_debug_blend_kernel(gsm_renderer* r, int* kind) {
    if (!r || !r->impl || !kind) return GSM_ERR_INVALID_ARGUMENT;
    *kind = r->impl->lastBlendKernel();
    return GSM_OK;
}

gsm_status gsm_global_debug_copy(gsm_renderer* r, int which, void* dst, size_t bytes, size_t* needed) {
    if (!r || !r->impl) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->debugCopy(which, dst, bytes, needed);
}

gsm_status gsm_global_set_profiling(gsm_renderer* r, int enable) {
    if (!r || !r->impl) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->setProfiling(enable);
}

gsm_status gsm_global_stage_times(gsm_renderer* r, float* ms, int n) {
    if (!r || !r->impl || !ms) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->stageTimes(ms, n);
}

gsm_status gsm_global_set_tile_rows(gsm_renderer* r, uint32_t b, uint32_t e) {
    if (!r || !r->impl) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->setTileRows(b, e);
}

size_t gsm_debug_sort_workspace_bytes(uint32_t capacity) { return gsm::radix_workspace_bytes(capacity); }

gsm_status gsm_debug_sort_plan_fits(uint32_t capacity, uint32_t key_bits, int wide, size_t hist_bytes) {
    if (key_bits == 0 || key_bits > 32) return GSM_ERR_INVALID_ARGUMENT;
    // (placeholder pointers: the plan only compares footprints, nothing is dereferenced or launched)
    const gsm::SortSpace ws{(uint32_t*)(uintptr_t)16, hist_bytes, (uint32_t*)(uintptr_t)16, gsm::kSortTotalsWords};
    return gsm::sort_bits_plan_fits(capacity, key_bits, wide != 0, ws) ? GSM_OK : GSM_ERR_INVALID_ASSIGNMENT_CAPACITY;
}

gsm_status gsm_sort_pairs_u32(void* keys, void* values, uint32_t n, uint32_t key_bits, void* stream) {
    if ((!keys || !values) && n > 0) return GSM_ERR_INVALID_ARGUMENT;
    if (n == 0) return GSM_OK;
    if (key_bits == 0 || key_bits > 32) key_bits = 32;
    hipStream_t s = (hipStream_t)stream;
    uint32_t *k2 = nullptr, *v2 = nullptr, *hist = nullptr, *bins = nullptr, *np = nullptr;
    gsm_status st = GSM_OK;
    if (hipMalloc(&k2, (size_t)n * 4) != hipSuccess || hipMalloc(&v2, (size_t)n * 4) != hipSuccess ||
        hipMalloc(&hist, gsm::radix_workspace_bytes(n)) != hipSuccess || hipMalloc(&bins, 256 * 4) != hipSuccess ||
        hipMalloc(&np, 4) != hipSuccess) {
        st = GSM_ERR_FAILED_TO_ALLOCATE_BUFFER;
    }
    if (st == GSM_OK) {
        hipMemcpyAsync(np, &n, 4, hipMemcpyHostToDevice, s);
        hipMemsetAsync(hist, 0, gsm::radix_workspace_bytes(n), s);
        uint32_t* kb[2] = {(uint32_t*)keys, k2};
        uint32_t* vb[2] = {(uint32_t*)values, v2};
        const int digits = (int)((key_bits + 7) / 8);
        int dev = 0;
        hipGetDevice(&dev);
        const gsm::Tuning tn = gsm::tuning_from_env(dev);  // read per call: no renderer here
        const gsm::SortSpace ws{hist, gsm::radix_workspace_bytes(n), bins, 256};
        int res = gsm::radix_sort_pairs(kb, vb, np, n, 0, digits, ws, s, tn.ballotRank, tn.sortScanless);
        if (res == gsm::kSortNoSpace) st = GSM_ERR_INVALID_ASSIGNMENT_CAPACITY;
        if (res == 1) {
            hipMemcpyAsync(keys, k2, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
            hipMemcpyAsync(values, v2, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
        }
        if (hipStreamSynchronize(s) != hipSuccess) st = GSM_ERR_RENDER_FAILED;
    }
    hipFree(k2);
    hipFree(v2);
    hipFree(hist);
    hipFree(bins);
    hipFree(np);
    return st;
}

gsm_status gsm_debug_sort_rank_probe(int hip_device, int* lane_ordered) {
    if (!lane_ordered) return GSM_ERR_INVALID_ARGUMENT;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || hip_device < 0 || hip_device >= ndev) {
        (void)hipGetLastError();
        return GSM_ERR_DEVICE_NOT_AVAILABLE;
    }
    *lane_ordered = gsm::sort_lane_ordered_atomics(hip_device) ? 1 : 0;
    return GSM_OK;
}

gsm_status gsm_debug_partition_counts(gsm_renderer* r, void* stream, const gsm_gaussian_input* input,
                                      const gsm_camera_params* camera, uint32_t width, uint32_t height,
                                      uint32_t first, uint32_t count, const uint32_t* slab_rows,
                                      uint32_t num_slabs, uint32_t* d_send_counts) {
    if (!r || !r->impl || !input || !camera || !slab_rows || !d_send_counts) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->partitionCounts((hipStream_t)stream, *input, *camera, width, height, first, count, slab_rows,
                                    num_slabs, d_send_counts);
}

gsm_status gsm_debug_partition_push(gsm_renderer* r, void* stream, uint32_t world, uint32_t rank,
                                    const uint32_t* d_counts, void* const* recv_buffers, uint32_t* d_recv_count) {
    if (!r || !r->impl || !d_counts || !recv_buffers || !d_recv_count || world < 1 || world > gsm::kMaxSlabs ||
        rank >= world)
        return GSM_ERR_INVALID_ARGUMENT;
    gsm::SlabPeers peers{};
    for (uint32_t p = 0; p < world; ++p) {
        if (!recv_buffers[p]) return GSM_ERR_INVALID_ARGUMENT;
        peers.recv[p] = (gsm::SplatRecord*)recv_buffers[p];
        peers.cap[p] = r->impl->maxGaussians();  // (gsm_debug.h: each holds max_gaussians records)
    }
    return r->impl->partitionPush((hipStream_t)stream, world, rank, d_counts, peers, d_recv_count, gsm::MgArrive{});
}

gsm_status gsm_debug_render_records_device_count(gsm_renderer* r, void* stream, const void* records,
                                                 uint32_t capacity, const uint32_t* d_count, uint32_t width,
                                                 uint32_t height, void* color, size_t color_pitch, void* depth,
                                                 size_t depth_pitch) {
    if (!r || !r->impl || !d_count) return GSM_ERR_INVALID_ARGUMENT;
    return r->impl->renderRecords((hipStream_t)stream, records, capacity, width, height, color, color_pitch, depth,
                                  depth_pitch, d_count);
}

}  // extern "C"
