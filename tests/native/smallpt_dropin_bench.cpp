// tests/native/smallpt_dropin_bench.cpp -- bench harness (bench.py "dropin"):
// the reference's own host path over the HIP drop-in (csrc/shim_smallpt.cpp
// in place of smallptgpu-v1.6/smallptGPU.cpp): displayfunc.cpp's idle loop
// calling UpdateRenderingGPU on the Cornell scene at W x H -- 20 single
// passes, then time-boxed calls (smallptGPU.cpp:739-755) for about argv[3]
// seconds -- printing one JSON line with the samples/s the reference's
// caption reports (smallptGPU.cpp:777-781: samples * H * W / elapsed).
#include <stdio.h>
#include <stdlib.h>
#include <sys/time.h>
#include "../../include/rt_hip.h"
#include "../../oracle/oracle.h"

int width = 1920, height = 1080;                  // displayfunc.cpp:61-64
unsigned int *pixels;
char captionBuffer[256];
int amiSmallptCPU;

extern rt_camera camera;
extern int currentSample;
extern rt_sphere *spheres;
extern unsigned int sphereCount;
void SetUpHIP();
void UpdateRenderingGPU();

void UpdateCamera() { ors_update_camera((or_camera *)&camera, width, height); }
double WallClockTime()
{
    struct timeval t;
    gettimeofday(&t, NULL);
    return t.tv_sec + t.tv_usec / 1000000.0;
}

int main(int argc, char **argv)
{
    if (argc > 1) width = atoi(argv[1]);
    if (argc > 2) height = atoi(argv[2]);
    const double seconds = argc > 3 ? atof(argv[3]) : 3.0;
    static rt_sphere cs[9];
    ors_cornell((or_sphere *)cs, 9);
    spheres = cs;
    sphereCount = 9;
    camera.orig = {50.f, 45.f, 205.6f};
    camera.target = {50.f, 45 - 0.042612f, (float)204.6};
    UpdateCamera();
    if (rt_device_count() < 1) { fprintf(stderr, "no HIP device\n"); return 1; }
    srand(1);
    SetUpHIP();
    UpdateRenderingGPU();                          // warm-up pass (first launch, allocations)
    const double px = (double)width * height;
    double t0 = WallClockTime();
    while (currentSample < 20) UpdateRenderingGPU();
    const double t_single = WallClockTime() - t0;
    const int single = 19;
    int calls = 0;
    const int s0 = currentSample;
    t0 = WallClockTime();
    while (WallClockTime() - t0 < seconds) {
        UpdateRenderingGPU();
        calls++;
    }
    const double t_box = WallClockTime() - t0;
    const int boxed = currentSample - s0;
    char cap[256];
    snprintf(cap, sizeof(cap), "%s", captionBuffer);
    for (char *c = cap; *c; c++)
        if (*c == '\n' || *c == '"') *c = ' ';
    printf("{\"frame\": [%d, %d], \"single_passes\": {\"passes\": %d, \"ms_per_pass\": %.4f, "
           "\"Msamples_per_s\": %.2f}, \"timeboxed\": {\"calls\": %d, \"samples\": %d, \"seconds\": %.3f, "
           "\"Msamples_per_s\": %.2f}, \"last_caption\": \"%s\"}\n",
           width, height, single, t_single * 1e3 / single, single * px / t_single / 1e6, calls, boxed, t_box,
           boxed * px / t_box / 1e6, cap);
    return 0;
}
