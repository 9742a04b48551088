// tests/native/whitted_app.cpp -- test harness: the reference app's launch
// sequence (testapp.cpp:57-178, useOpenCL = 1 branch) over the HIP drop-in
// shim (csrc/shim_whitted.cpp).  Stands in for the app side only: the
// scene.cpp globals are defined here and the scene is built by the oracle's
// Scene_InitScene restatement (test infrastructure).  Writes the Surface
// buffer (W*H uint32) to argv[3].
#include <stdio.h>
#include <stdlib.h>
#include <string>
#include "../../include/rt_hip.h"
#include "../../oracle/oracle.h"

struct Scene { int m_Primitives; or_primitive *m_Primitive; };   // raytracer.h:34-37
Scene *m_Scene;                                                   // scene.cpp:13-17
unsigned int *m_Dest = NULL;
int m_Width, m_Height, m_CurrLine, m_PPos;
int useGPU = 1;                                                   // testapp.cpp:30

char *openCLcode();
void AllocateBuffers();
void SetKernelArguments();
void ExecuteKernel();
void ReadKernelBuffer();
extern std::string outputLine1, outputLine2;

int main(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: whitted_app W H out.bin\n"); return 2; }
    const int W = atoi(argv[1]), H = atoi(argv[2]);
    unsigned int *buffer = (unsigned int *)calloc((size_t)W * H, 4);    // Surface_Create + Clear(0)
    m_Scene = (Scene *)malloc(sizeof(Scene));                            // Scene_InitScene
    m_Scene->m_Primitive = (or_primitive *)calloc(50, sizeof(or_primitive));
    m_Scene->m_Primitives = orw_scene_init(m_Scene->m_Primitive, 50);
    m_Dest = buffer; m_Width = W; m_Height = H;                          // Engine_SetTarget
    char *desc = openCLcode();
    fprintf(stderr, "%s | %s\n", desc, outputLine2.c_str());
    AllocateBuffers();
    SetKernelArguments();
    m_CurrLine = 20; m_PPos = 20 * W;                                    // Engine_InitRender
    AllocateBuffers();
    SetKernelArguments();
    ExecuteKernel();
    ReadKernelBuffer();
    FILE *f = fopen(argv[3], "wb");
    fwrite(buffer, 4, (size_t)W * H, f);
    fclose(f);
    return 0;
}
