// shim_smallpt.cpp -- drop-in replacement for the device half of smallptgpu-v1.6/smallptGPU.cpp.
//
// Link this translation unit (plus shim_smallpt_main.cpp where the app uses
// mainGPU, and librt_hip.so) into the reference app in place of
// smallptGPU.cpp.  It defines the globals smallptGPU.cpp defined
// (useGPU, useOpenCL, camera, currentSample, spheres, sphereCount:
// smallptGPU.cpp:51-52,71-74) and the entry points the rest of the app
// calls -- UpdateRenderingGPU (:642-782), ReInitSceneGPU (:784-803),
// ReInitGPU (:805-830) -- and reads displayfunc.cpp's width / height /
// pixels / captionBuffer (displayfunc.cpp:61-64) as the reference did.
//
// Where rendering_kernel.cl computed a different image (seed slot = gid,
// OpenCL sign(0) = 0, clang argument order: SURVEY.md §8(a) S10), the HIP
// path computes the CPU path's (UpdateRenderingCPU, smallptCPU.cpp:77-132).
// Buffers stay device-resident across passes; only the RGBA8 frame is read
// back per UpdateRenderingGPU call, as clEnqueueReadBuffer did (:760).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime.h>
#include "../../include/rt_hip.h"

int useGPU = 1;                        // smallptGPU.cpp:51-52
int useOpenCL = 1;
rt_camera camera;                      // Camera camera;        (:72, camera.h:29-34 layout)
int currentSample = 0;                 // (:73)
rt_sphere *spheres;                    // Sphere *spheres;      (:74, geom.h:43-47 layout)
unsigned int sphereCount;
int smallptHipMode = SPT_PATH_TRACING; // rendering_kernel.cl vs rendering_kernel_dl.cl

extern int width;                      // displayfunc.cpp:61-64
extern int height;
extern unsigned int *pixels;
extern char captionBuffer[256];
extern void UpdateCamera();            // displayfunc.cpp:182-195
extern double WallClockTime();         // displayfunc.cpp:69-80

namespace {
spt_scene *scene = nullptr;
float *d_colors = nullptr;
uint32_t *d_seeds = nullptr, *d_pixels = nullptr;
uint32_t *h_seeds = nullptr;
hipStream_t stream = nullptr;

void die(const char *what, int rc)
{
    fprintf(stderr, "%s: %s (%d)\n", what, rt_last_error(), rc);
    exit(-1);
}

void die_hip(const char *what, hipError_t e)
{
    fprintf(stderr, "%s: %s (%d)\n", what, hipGetErrorString(e), (int)e);
    exit(-1);
}

void upload_scene()
{
    if (scene) spt_scene_destroy(scene);
    scene = nullptr;
    int rc = spt_scene_create(spheres, sphereCount, &scene);
    if (rc) die("Failed to write the HIP scene buffer", rc);
}

// FreeBuffers (smallptGPU.cpp:76-98)
void FreeBuffers()
{
    if (d_colors) (void)hipFree(d_colors);
    if (d_seeds) (void)hipFree(d_seeds);
    if (d_pixels) (void)hipFree(d_pixels);
    d_colors = nullptr;
    d_seeds = d_pixels = nullptr;
    free(h_seeds);
    free(pixels);
    h_seeds = nullptr;
    pixels = nullptr;
}

// AllocateBuffers (smallptGPU.cpp:100-167): seeds from rand() (>= 2),
// pixels preset to their index ("Test colors", :111-113), device buffers.
void AllocateBuffers()
{
    const int pixelCount = width * height;
    h_seeds = (uint32_t *)malloc(sizeof(uint32_t) * pixelCount * 2);
    for (int i = 0; i < pixelCount * 2; i++) {
        h_seeds[i] = (uint32_t)rand();
        if (h_seeds[i] < 2) h_seeds[i] = 2;
    }
    pixels = (unsigned int *)malloc(sizeof(unsigned int) * pixelCount);
    for (int i = 0; i < pixelCount; ++i) pixels[i] = i;
    hipError_t e = hipMalloc(&d_colors, sizeof(float) * 3 * pixelCount);
    if (e != hipSuccess) die_hip("Failed to create HIP output buffer", e);
    e = hipMalloc(&d_pixels, sizeof(uint32_t) * pixelCount);
    if (e != hipSuccess) die_hip("Failed to create HIP pixel buffer", e);
    e = hipMalloc(&d_seeds, sizeof(uint32_t) * pixelCount * 2);
    if (e != hipSuccess) die_hip("Failed to create HIP seed buffer", e);
    e = hipMemcpy(d_seeds, h_seeds, sizeof(uint32_t) * pixelCount * 2, hipMemcpyHostToDevice);
    if (e != hipSuccess) die_hip("Failed to write the HIP seeds buffer", e);
}

// ExecuteKernel (smallptGPU.cpp:617-640): one pass = one sample per pixel.
void ExecuteKernel()
{
    int rc = spt_scene_render_async(scene, &camera, d_colors, d_seeds, d_seeds, d_pixels, width, height, 0,
                                    height, currentSample, 1, smallptHipMode, nullptr, stream);
    if (rc) die("Failed to enqueue HIP work", rc);
}
}  // namespace

// SetUpOpenCL (smallptGPU.cpp:209-615): device, stream, scene and buffers.
void SetUpHIP()
{
    if (rt_device_count() < 1) {
        fprintf(stderr, "Failed to find a HIP device: %s\n", rt_last_error());
        exit(-1);
    }
    int rc = rt_set_device(0);
    if (rc) die("Failed to select HIP device 0", rc);
    hipError_t e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
    if (e != hipSuccess) die_hip("Failed to create HIP stream", e);
    upload_scene();
    AllocateBuffers();
}

// UpdateRenderingGPU (smallptGPU.cpp:642-782): a single pass for the first
// 20 samples, then passes until 0.5 * min(currentSample - 20, 100) / 100 s
// have elapsed; then the blocking read of the RGBA8 frame and the caption.
void UpdateRenderingGPU()
{
    double startTime = WallClockTime();
    int startSampleCount = currentSample;
    if (currentSample < 20) {
        ExecuteKernel();
        currentSample++;
    } else {
        const int c = currentSample - 20;
        const float k = (c < 100 ? c : 100) / 100.f;
        const float tresholdTime = 0.5f * k;
        for (;;) {
            ExecuteKernel();
            hipError_t e = hipStreamSynchronize(stream);
            if (e != hipSuccess) die_hip("Failed to finish HIP work", e);
            currentSample++;
            const float elapsedTime = WallClockTime() - startTime;
            if (elapsedTime > tresholdTime) break;
        }
    }
    hipError_t e = hipMemcpyAsync(pixels, d_pixels, sizeof(unsigned int) * width * height,
                                  hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) die_hip("Failed to read the HIP pixel buffer", e);
    const double elapsedTime = WallClockTime() - startTime;
    const int samples = currentSample - startSampleCount;
    const double sampleSec = samples * height * width / elapsedTime;
    sprintf(captionBuffer, "Rendering time %.3f sec (pass %d)  Sample/sec  %.1fK\n", elapsedTime,
            currentSample, sampleSec / 1000.f);
}

// ReInitSceneGPU (smallptGPU.cpp:784-803)
void ReInitSceneGPU()
{
    currentSample = 0;
    upload_scene();
}

// ReInitGPU (smallptGPU.cpp:805-830).  The camera travels by value with every
// launch, so there is no camera buffer to rewrite.
void ReInitGPU(const int reallocBuffers)
{
    if (reallocBuffers) {
        FreeBuffers();
        UpdateCamera();
        AllocateBuffers();
    } else {
        UpdateCamera();
    }
    currentSample = 0;
}

// Test / tooling hook: the device HDR accumulator (Vec per flipped slot).
void SmallptHipReadColors(float *out)
{
    hipError_t e = hipMemcpy(out, d_colors, sizeof(float) * 3 * width * height, hipMemcpyDeviceToHost);
    if (e != hipSuccess) die_hip("Failed to read the HIP colour buffer", e);
}

// Test / tooling hook: the seeds AllocateBuffers drew (host copy, 2*W*H).
const unsigned int *SmallptHipInitialSeeds() { return h_seeds; }
