// tests/native/smallpt_main_app.cpp -- test harness for the drop-in's own
// main/mainGPU (csrc/shim_smallpt_main.cpp, smallptGPU.cpp:832-884): the app
// is linked exactly as the reference links smallptGPU (main -> mainGPU ->
// UpdateCamera, SetUpHIP, InitGlut, glutMainLoop), with displayfunc.cpp's
// globals (:61-64) and a GLUT stand-in whose main loop runs the idle
// callback (displayfunc.cpp:197-204 -> UpdateRenderingGPU) RT_TEST_PASSES
// times, writes pixels (W*H u32), currentSample and the seeds AllocateBuffers
// drew to RT_TEST_OUT, and exits.  UpdateCamera is the oracle's restatement
// (test infrastructure).  The stand-in exists only because this image has no
// GLUT; it is not part of the product.
#include <stdio.h>
#include <stdlib.h>
#include <sys/time.h>
#include "../../include/rt_hip.h"
#include "../../oracle/oracle.h"

int width = 640, height = 480;                    // displayfunc.cpp:61-64
unsigned int *pixels;
char captionBuffer[256];
int amiSmallptCPU;

extern rt_camera camera;
extern int currentSample;
void UpdateRenderingGPU();
const unsigned int *SmallptHipInitialSeeds();

void UpdateCamera() { ors_update_camera((or_camera *)&camera, width, height); }
double WallClockTime()
{
    struct timeval t;
    gettimeofday(&t, NULL);
    return t.tv_sec + t.tv_usec / 1000000.0;
}

static char *g_title;
void InitGlut(int, char *[], char *windowTittle) { g_title = windowTittle; }   // displayfunc.cpp:422-439

extern "C" void glutMainLoop(void)
{
    const int passes = getenv("RT_TEST_PASSES") ? atoi(getenv("RT_TEST_PASSES")) : 1;
    for (int i = 0; i < passes; i++) UpdateRenderingGPU();   // idleFunc (displayfunc.cpp:197-204)
    FILE *f = fopen(getenv("RT_TEST_OUT"), "wb");
    if (!f) exit(3);
    fwrite(pixels, 4, (size_t)width * height, f);
    fwrite(&currentSample, 4, 1, f);
    fwrite(SmallptHipInitialSeeds(), 4, (size_t)2 * width * height, f);
    fclose(f);
    fprintf(stderr, "%s: %s", g_title, captionBuffer);
    exit(0);
}

int mainCPU(int, char **) { return 1; }   // smallptCPU.cpp:169 (not this app)
