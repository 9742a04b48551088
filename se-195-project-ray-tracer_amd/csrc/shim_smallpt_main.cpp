// shim_smallpt_main.cpp -- mainGPU of smallptgpu-v1.6/smallptGPU.cpp:832-870 on the
// HIP shim.  Separate from shim_smallpt.cpp because it needs the app's GLUT
// front end (InitGlut, displayfunc.cpp:422-439, and glutMainLoop).
#include "../../include/rt_hip.h"

extern rt_camera camera;
extern rt_sphere *spheres;
extern unsigned int sphereCount;
extern int amiSmallptCPU;
extern void UpdateCamera();
extern void InitGlut(int argc, char *argv[], char *windowTittle);
extern "C" void glutMainLoop(void);
void SetUpHIP();

// CornellSpheres, scene.h:29-40
static rt_sphere CornellSpheres[] = {
    {1e4f, {1e4f + 1.f, 40.8f, 81.6f}, {0.f, 0.f, 0.f}, {.75f, .25f, .25f}, 0},
    {1e4f, {-1e4f + 99.f, 40.8f, 81.6f}, {0.f, 0.f, 0.f}, {.25f, .25f, .75f}, 0},
    {1e4f, {50.f, 40.8f, 1e4f}, {0.f, 0.f, 0.f}, {.75f, .75f, .75f}, 0},
    {1e4f, {50.f, 40.8f, -1e4f + 270.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, 0},
    {1e4f, {50.f, 1e4f, 81.6f}, {0.f, 0.f, 0.f}, {.75f, .75f, .75f}, 0},
    {1e4f, {50.f, -1e4f + 81.6f, 81.6f}, {0.f, 0.f, 0.f}, {.75f, .75f, .75f}, 0},
    {16.5f, {27.f, 16.5f, 47.f}, {0.f, 0.f, 0.f}, {.9f, .9f, .9f}, 1},
    {16.5f, {73.f, 16.5f, 78.f}, {0.f, 0.f, 0.f}, {.9f, .9f, .9f}, 2},
    {7.f, {50.f, 81.6f - 15.f, 81.6f}, {12.f, 12.f, 12.f}, {0.f, 0.f, 0.f}, 0},
};

int mainGPU(int argc, char **argv)
{
    amiSmallptCPU = 0;
    spheres = CornellSpheres;
    sphereCount = sizeof(CornellSpheres) / sizeof(rt_sphere);
    camera.orig = {50.f, 45.f, 205.6f};
    camera.target = {50.f, 45 - 0.042612f, (float)204.6};
    UpdateCamera();
    SetUpHIP();
    InitGlut(argc, argv, (char *)"SmallPT GPU V1.6 (HIP / MI355X)");
    glutMainLoop();
    return 0;
}

int mainCPU(int argc, char **argv);     // smallptCPU.cpp:169
extern int useGPU, useOpenCL;

// main, smallptGPU.cpp:874-884 (lives in the file this shim replaces).
int main(int argc, char **argv)
{
    useOpenCL = 1;
    useGPU = 1;
    if (useOpenCL) return mainGPU(argc, argv);
    return mainCPU(argc, argv);
}
