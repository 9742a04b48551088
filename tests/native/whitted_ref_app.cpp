// tests/native/whitted_ref_app.cpp -- test harness: the reference app's
// OpenCL launch sequence (testapp.cpp:57-136, useOpenCL = 1) over the HIP
// drop-in shim (csrc/shim_whitted.cpp), linked with the reference's OWN
// scene.cpp and surface.cpp (compiled unmodified where they lie under
// /root/reference by tests/native/Makefile; never copied).  Only
// raytracer.cpp's Engine_Constructor / Engine_SetTarget / Engine_InitRender
// (raytracer.cpp:12-24, 278-294) are restated here, because raytracer.cpp
// includes <windows.h>, which this image lacks.
//
// Writes the Surface after ReadKernelBuffer (W*H uint32) to argv[3].  The
// app's text overlay (Surface_InitCharset / Surface_Print, testapp.cpp:62,
// 71-91) is not drawn: it is out of scope, and surface.cpp's
// Surface_SetChar copies 6 bytes into each char[5] font row
// (surface.cpp:52-58, surface.h:15), which this image's fortified glibc
// aborts on.
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include "common.h"
#include "raytracer.h"
#include "scene.h"
#include "surface.h"

int useOpenCL = 1;                                               // testapp.cpp:25-28
int useGPU = 1;

char *openCLcode();                                              // testapp.cpp:32-46
void AllocateBuffers();
void SetKernelArguments();
void ExecuteKernel();
void ReadKernelBuffer();
extern std::string outputLine2, outputLine3, outputLine4, outputLine5, outputLine6, outputLine7, outputLine8,
    outputLine9;

// raytracer.cpp:12-24
void Engine_Constructor() { m_Scene = (Scene *)malloc(sizeof(Scene)); }
void Engine_SetTarget(Pixel *a_Dest, int a_Width, int a_Height)
{
    m_Dest = a_Dest;
    m_Width = a_Width;
    m_Height = a_Height;
}
// raytracer.cpp:278-294 (the float view scalars are the device path's own;
// the shim reads m_CurrLine)
void Engine_InitRender()
{
    m_CurrLine = 20;
    m_PPos = 20 * m_Width;
    m_WX1 = -3, m_WX2 = 3, m_WY1 = m_SY = 2.25f, m_WY2 = -2.25f;
    m_DX = (m_WX2 - m_WX1) / m_Width;
    m_DY = (m_WY2 - m_WY1) / m_Height;
    m_SY += 20 * m_DY;
}

int main(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: whitted_ref_app W H out.bin\n"); return 2; }
    const int W = atoi(argv[1]), H = atoi(argv[2]);
    Surface *surface = Surface_Create(W, H);                      // testapp.cpp:59-61
    Pixel *buffer = Surface_GetBuffer(surface);
    Surface_Clear(surface, 0);
    Engine_Constructor();                                         // :65-68
    TracedRays_init();
    Scene_InitScene();
    Engine_SetTarget(Surface_GetBuffer(surface), W, H);
    char *ret = openCLcode();                                     // :71-92 (text overlay not drawn)
    AllocateBuffers();                                            // :106-111
    SetKernelArguments();
    Engine_InitRender();                                          // :123
    AllocateBuffers();                                            // :128-136
    SetKernelArguments();
    ExecuteKernel();
    ReadKernelBuffer();

    FILE *f = fopen(argv[3], "wb");
    fwrite(buffer, 4, (size_t)W * H, f);
    fclose(f);
    fprintf(stderr, "%s | %s\n", ret, outputLine5.c_str());
    return 0;
}
