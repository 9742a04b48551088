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
// Frames are tiled in row bands over every visible gfx950 GPU (spt_multi:
// each pixel's accumulator and RNG words live on its band's device, so a pass
// needs no exchange); buffers stay device-resident across passes and only
// the RGBA8 frame is read back per UpdateRenderingGPU call, band by band, as
// clEnqueueReadBuffer did (:760).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

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
// The frame, tiled in row bands over every GPU the shim drives (one band on
// a one-GPU node); accumulators and RNG words stay on their band's device.
spt_multi *frame = nullptr;
std::vector<int> devices;
uint32_t *h_seeds = nullptr;

void die(const char *what, int rc)
{
    fprintf(stderr, "%s: %s (%d)\n", what, rt_last_error(), rc);
    exit(-1);
}

// The devices to tile frames over: RT_SPT_DEVICES="0,1,..." (a device may
// repeat: several bands on one GPU), else every visible gfx950 GPU, at most
// RT_SPT_GPUS of them.  (The reference picks one OpenCL device,
// smallptGPU.cpp:225-300.)
void pick_devices()
{
    devices.clear();
    if (const char *e = getenv("RT_SPT_DEVICES")) {
        for (const char *p = e; *p;) {
            char *end;
            const long d = strtol(p, &end, 10);
            if (end == p) break;
            devices.push_back((int)d);
            p = *end == ',' ? end + 1 : end;
        }
    } else {
        const int n = rt_device_count();
        int cap = n;
        if (const char *g = getenv("RT_SPT_GPUS")) cap = atoi(g) > 0 ? atoi(g) : n;
        for (int d = 0; d < n && (int)devices.size() < cap; d++) {
            hipDeviceProp_t prop;
            if (hipGetDeviceProperties(&prop, d) == hipSuccess && !strncmp(prop.gcnArchName, "gfx950", 6))
                devices.push_back(d);
        }
    }
    if (devices.empty()) {
        fprintf(stderr, "Failed to find a gfx950 HIP device: %s\n", rt_last_error());
        exit(-1);
    }
}

// FreeBuffers (smallptGPU.cpp:76-98)
void FreeBuffers()
{
    if (frame) spt_multi_destroy(frame);
    frame = nullptr;
    free(h_seeds);
    (void)rt_host_free(pixels);
    h_seeds = nullptr;
    pixels = nullptr;
}

// AllocateBuffers (smallptGPU.cpp:100-167): seeds from rand() (>= 2),
// pixels preset to their index ("Test colors", :111-113), device buffers
// (scene, accumulator, seeds, pixels) on every band's device.
void AllocateBuffers()
{
    const int pixelCount = width * height;
    h_seeds = (uint32_t *)malloc(sizeof(uint32_t) * pixelCount * 2);
    for (int i = 0; i < pixelCount * 2; i++) {
        h_seeds[i] = (uint32_t)rand();
        if (h_seeds[i] < 2) h_seeds[i] = 2;
    }
    // page-locked: the blocking read after every pass (ReadKernelBuffer)
    // then runs at DMA speed
    void *px = nullptr;
    int rc0 = rt_host_alloc(sizeof(unsigned int) * pixelCount, &px);
    if (rc0) die("Failed to allocate the pixel buffer", rc0);
    pixels = (unsigned int *)px;
    for (int i = 0; i < pixelCount; ++i) pixels[i] = i;
    int rc = spt_multi_create(spheres, sphereCount, width, height, devices.data(), (int)devices.size(), &frame);
    if (rc) die("Failed to create HIP buffers", rc);
    rc = spt_multi_upload(frame, nullptr, h_seeds);
    if (rc) die("Failed to write the HIP seeds buffer", rc);
}

// ExecuteKernel (smallptGPU.cpp:617-640): one pass = one sample per pixel,
// every band on its own device; passes > 1 runs that many consecutive passes
// in one launch (samples currentSample .. currentSample + passes - 1, the
// same results as one launch per pass: the kernel keeps each pixel's
// sample order).
void ExecuteKernel(int passes = 1)
{
    int rc = spt_multi_render_async(frame, &camera, currentSample, passes, smallptHipMode, 0);
    if (rc) die("Failed to enqueue HIP work", rc);
}

void Finish()                          // clFinish (smallptGPU.cpp:748)
{
    int rc = spt_multi_sync(frame);
    if (rc) die("Failed to finish HIP work", rc);
}
}  // namespace

// SetUpOpenCL (smallptGPU.cpp:209-615): devices, scene and buffers.
void SetUpHIP()
{
    if (rt_device_count() < 1) {
        fprintf(stderr, "Failed to find a HIP device: %s\n", rt_last_error());
        exit(-1);
    }
    pick_devices();
    AllocateBuffers();
}

// UpdateRenderingGPU (smallptGPU.cpp:642-782): a single pass for the first
// 20 samples, then passes until 0.5 * min(currentSample - 20, 100) / 100 s
// have elapsed; then the blocking read of the RGBA8 frame and the caption.
// The reference launches and waits for (clFinish) every pass of the time
// box; here a launch runs a batch of passes sized from the measured pass
// time to about an eighth of the time left (at least one pass), so the
// kernel keeps a pixel's samples in-lane and the host waits once per batch
// -- the same sample sequence per pixel, the box overshot by at most a
// batch.  RT_SPT_SHIM_BATCH=1: one pass per launch, as the reference.
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
        const char *be = getenv("RT_SPT_SHIM_BATCH");
        const int max_batch = be && atoi(be) > 0 ? atoi(be) : 256;
        int batch = 1;
        for (;;) {
            const double t0 = WallClockTime();
            ExecuteKernel(batch);
            Finish();
            currentSample += batch;
            const double now = WallClockTime();
            const float elapsedTime = now - startTime;
            if (elapsedTime > tresholdTime) break;
            const double per_pass = (now - t0) / batch;
            const double left = tresholdTime - elapsedTime;
            int next = per_pass > 0 ? (int)(left / per_pass / 8.0) : 1;
            batch = next < 1 ? 1 : (next > max_batch ? max_batch : next);
        }
    }
    int rc = spt_multi_download(frame, nullptr, nullptr, pixels);   // every band's rows
    if (rc) die("Failed to read the HIP pixel buffer", rc);
    const double elapsedTime = WallClockTime() - startTime;
    const int samples = currentSample - startSampleCount;
    // (in double: the reference's int product overflows past ~1,000 samples
    // per call at 1080p, which its OpenCL device never reached in one call)
    const double sampleSec = (double)samples * height * width / elapsedTime;
    sprintf(captionBuffer, "Rendering time %.3f sec (pass %d)  Sample/sec  %.1fK\n", elapsedTime,
            currentSample, sampleSec / 1000.f);
}

// ReInitSceneGPU (smallptGPU.cpp:784-803)
void ReInitSceneGPU()
{
    currentSample = 0;
    int rc = spt_multi_set_scene(frame, spheres, sphereCount);
    if (rc) die("Failed to write the HIP scene buffer", rc);
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
    int rc = spt_multi_download(frame, out, nullptr, nullptr);
    if (rc) die("Failed to read the HIP colour buffer", rc);
}

// Test / tooling hook: the seeds AllocateBuffers drew (host copy, 2*W*H).
const unsigned int *SmallptHipInitialSeeds() { return h_seeds; }

// Test / tooling hook: the number of row bands (GPUs) frames are tiled over.
int SmallptHipBands() { return (int)devices.size(); }
