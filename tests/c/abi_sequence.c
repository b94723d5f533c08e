/* The call sequence of the Swift wrapper (swift/Sources/GsmRendererHIP) through the C ABI, in C:
 * RendererConfig defaults -> gsm_global_create -> device buffers -> CameraParams init -> render on a
 * stream -> synchronise -> debugReadTotalAssignments / lastGPUTime -> the error paths the wrapper maps
 * (invalid dimensions, stereo unsupported) -> read back -> destroy.  Test infrastructure: run by
 * tests/test_c_abi.py, which writes the scene and compares the frame with the oracle.
 *
 * usage: abi_sequence world.bin harm.bin count sh width height cam.bin out_color.bin */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>

#include "gsm_debug.h"
#include "gsm_renderer.h"

static void* slurp(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    *n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    void* p = malloc(*n ? *n : 1);
    if (fread(p, 1, *n, f) != *n) {
        fclose(f);
        free(p);
        return NULL;
    }
    fclose(f);
    return p;
}

#define CHECK(cond, msg)                       \
    do {                                       \
        if (!(cond)) {                         \
            fprintf(stderr, "FAIL: %s\n", msg); \
            return 1;                          \
        }                                      \
    } while (0)

int main(int argc, char** argv) {
    if (argc != 9) {
        fprintf(stderr, "usage: %s world harm count sh width height cam out\n", argv[0]);
        return 2;
    }
    size_t wn = 0, hn = 0, cn = 0;
    void* world = slurp(argv[1], &wn);
    void* harm = slurp(argv[2], &hn);
    float* camf = (float*)slurp(argv[7], &cn); /* view[16] proj[16] pos[3] fx fy near far */
    const uint32_t count = (uint32_t)atoi(argv[3]), sh = (uint32_t)atoi(argv[4]);
    const uint32_t W = (uint32_t)atoi(argv[5]), H = (uint32_t)atoi(argv[6]);
    CHECK(world && harm && camf && cn == 39 * sizeof(float), "inputs");

    gsm_renderer_config cfg;
    gsm_renderer_config_default(&cfg);
    CHECK(cfg.max_gaussians == 6000000 && cfg.max_width == 1920 && cfg.precision == GSM_PRECISION_FLOAT16,
          "RendererConfig defaults");
    cfg.max_gaussians = count;
    cfg.max_width = W;
    cfg.max_height = H;
    cfg.color_format = GSM_COLOR_FORMAT_RGBA16F;
    cfg.gaussian_color_space = GSM_COLOR_SPACE_LINEAR;
    gsm_renderer* r = NULL;
    CHECK(gsm_global_create(&cfg, 0, &r) == GSM_OK && r, "gsm_global_create");

    void *dw = NULL, *dh = NULL, *dc = NULL, *dd = NULL;
    CHECK(hipMalloc(&dw, wn) == hipSuccess && hipMalloc(&dh, hn) == hipSuccess &&
              hipMalloc(&dc, (size_t)W * H * 8) == hipSuccess && hipMalloc(&dd, (size_t)W * H * 2) == hipSuccess,
          "hipMalloc");
    CHECK(hipMemcpy(dw, world, wn, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(dh, harm, hn, hipMemcpyHostToDevice) == hipSuccess,
          "upload");
    gsm_camera_params cam;
    gsm_camera_params_init(&cam, camf, camf + 16, camf + 32, camf[35], camf[36]);
    CHECK(cam.near_plane == 0.1f && cam.far_plane == 10.0f, "CameraParams defaults");
    cam.near_plane = camf[37];
    cam.far_plane = camf[38];
    gsm_gaussian_input in = {dw, dh, count, sh};
    hipStream_t stream = NULL;
    CHECK(hipStreamCreate(&stream) == hipSuccess, "stream");

    CHECK(gsm_global_render(r, stream, &in, &cam, W, H, dc, (size_t)W * 8, dd, (size_t)W * 2) == GSM_OK, "render");
    CHECK(hipStreamSynchronize(stream) == hipSuccess, "sync");
    const uint32_t total = gsm_global_debug_read_total_assignments(r);
    double secs = 0.0;
    CHECK(gsm_global_last_gpu_time(r, &secs) == GSM_ERR_RENDER_FAILED, "lastGPUTime is nil without profiling");
    /* the wrapper's error mapping: validateLimits and the Global stereo fatalError */
    CHECK(gsm_global_render(r, stream, &in, &cam, W + 1, H, dc, (size_t)W * 8, dd, (size_t)W * 2) ==
              GSM_ERR_INVALID_DIMENSIONS, "invalid dimensions");
    CHECK(gsm_global_render_stereo(r, stream, &in, &cam, &cam, W, H, dc, (size_t)W * 8, NULL, 0) ==
              GSM_ERR_UNSUPPORTED, "stereo unsupported");
    /* a profiled frame gives lastGPUTime */
    CHECK(gsm_global_set_profiling(r, 1) == GSM_OK, "profiling");
    CHECK(gsm_global_render(r, stream, &in, &cam, W, H, dc, (size_t)W * 8, dd, (size_t)W * 2) == GSM_OK, "render 2");
    CHECK(hipStreamSynchronize(stream) == hipSuccess, "sync 2");
    CHECK(gsm_global_last_gpu_time(r, &secs) == GSM_OK && secs > 0.0, "lastGPUTime");

    void* host = malloc((size_t)W * H * 8);
    CHECK(hipMemcpy(host, dc, (size_t)W * H * 8, hipMemcpyDeviceToHost) == hipSuccess, "download");
    FILE* f = fopen(argv[8], "wb");
    CHECK(f && fwrite(host, 1, (size_t)W * H * 8, f) == (size_t)W * H * 8, "write");
    fclose(f);
    hipStreamDestroy(stream);
    hipFree(dw);
    hipFree(dh);
    hipFree(dc);
    hipFree(dd);
    gsm_global_destroy(r);
    printf("total_assignments %u gpu_time_s %.6f abi %d\n", total, secs, gsm_abi_version());
    return 0;
}
