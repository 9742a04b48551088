// tests/native/smallpt_app.cpp -- test harness: displayfunc.cpp's globals and
// the idle loop (displayfunc.cpp:197-204 -> UpdateRenderingGPU) over the HIP
// drop-in shim (csrc/shim_smallpt.cpp).  UpdateCamera is the oracle's
// restatement (test infrastructure).  Runs argv[3] UpdateRenderingGPU calls
// -- or, with argv[5], a script of comma-separated steps: "pN" N
// UpdateRenderingGPU calls, "R" ReInitGPU(1) (FreeBuffers + AllocateBuffers:
// fresh rand() seeds), "r" ReInitGPU(0), "S" move sphere 6 by +1 in x and
// ReInitSceneGPU (the keyboard handler's edit, displayfunc.cpp:300-420) --
// and writes pixels (W*H u32), the device HDR colours (3*W*H f32), the seeds
// the last AllocateBuffers drew, currentSample, the number of row bands and
// currentSample after each step to argv[4].
#include <stdio.h>
#include <stdlib.h>
#include <sys/time.h>
#include <vector>
#include "../../include/rt_hip.h"
#include "../../oracle/oracle.h"

int width = 640, height = 480;                    // displayfunc.cpp:61-64
unsigned int *pixels;
char captionBuffer[256];
int amiSmallptCPU;

extern rt_camera camera;
extern int currentSample;
extern rt_sphere *spheres;
extern unsigned int sphereCount;
void SetUpHIP();
void UpdateRenderingGPU();
void ReInitGPU(const int);
void ReInitSceneGPU();
int SmallptHipBands();
void SmallptHipReadColors(float *out);
const unsigned int *SmallptHipInitialSeeds();

void UpdateCamera() { ors_update_camera((or_camera *)&camera, width, height); }
double WallClockTime()
{
    struct timeval t;
    gettimeofday(&t, NULL);
    return t.tv_sec + t.tv_usec / 1000000.0;
}

int main(int argc, char **argv)
{
    if (argc < 5) { fprintf(stderr, "usage: smallpt_app W H passes out.bin\n"); return 2; }
    width = atoi(argv[1]); height = atoi(argv[2]);
    const int passes = atoi(argv[3]);
    static rt_sphere cs[9];
    ors_cornell((or_sphere *)cs, 9);                                   // mainGPU (smallptGPU.cpp:847-851)
    spheres = cs; sphereCount = 9;
    camera.orig = {50.f, 45.f, 205.6f};
    camera.target = {50.f, 45 - 0.042612f, (float)204.6};
    UpdateCamera();
    // The HIP runtime may draw from rand() while it initialises; bring it up
    // first so AllocateBuffers' seeds are the srand(1) stream the oracle uses.
    if (rt_device_count() < 1) { fprintf(stderr, "no HIP device\n"); return 1; }
    srand(1);
    SetUpHIP();
    std::vector<int> after;
    if (argc > 5) {
        for (const char *p = argv[5]; *p;) {
            if (*p == 'p') {
                char *end;
                const long n = strtol(p + 1, &end, 10);
                for (long i = 0; i < n; i++) UpdateRenderingGPU();
                p = end;
            } else if (*p == 'R' || *p == 'r') {
                ReInitGPU(*p == 'R');
                p++;
            } else if (*p == 'S') {
                cs[6].p.x += 1.f;
                ReInitSceneGPU();
                p++;
            } else {
                fprintf(stderr, "bad script step '%c'\n", *p);
                return 2;
            }
            after.push_back(currentSample);
            if (*p == ',') p++;
        }
    } else {
        for (int i = 0; i < passes; i++) UpdateRenderingGPU();
    }
    float *col = (float *)malloc(sizeof(float) * 3 * width * height);
    SmallptHipReadColors(col);
    FILE *f = fopen(argv[4], "wb");
    fwrite(pixels, 4, (size_t)width * height, f);
    fwrite(col, 4, (size_t)3 * width * height, f);
    fwrite(SmallptHipInitialSeeds(), 4, (size_t)2 * width * height, f);
    fwrite(&currentSample, 4, 1, f);
    const int bands = SmallptHipBands();
    fwrite(&bands, 4, 1, f);
    if (!after.empty()) fwrite(after.data(), 4, after.size(), f);
    fclose(f);
    fprintf(stderr, "%s", captionBuffer);
    return 0;
}
