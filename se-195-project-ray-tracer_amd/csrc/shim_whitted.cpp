// shim_whitted.cpp -- drop-in replacement for raytracer3.0.06.no_rec.samp/openCLcode.cpp.
//
// Link this translation unit (and librt_hip.so) into the reference app in
// place of openCLcode.cpp: testapp.cpp's declarations (testapp.cpp:32-46)
// resolve to the functions and strings below unchanged, and the app's own
// globals from scene.cpp (m_Scene, m_Dest, m_Width, m_Height, m_CurrLine;
// raytracer.h:50-54) are read exactly as openCLcode.cpp read them.  Where the
// OpenCL kernel computed a different image (openCLcode.cl: 2x2 sub-samples,
// x64 scale, rows [20,530)), the HIP path computes the
// CPU path's image (Engine_Render, raytracer.cpp:301-530) bit for bit over
// the rows Engine_Render covers: [m_CurrLine, m_Height - 70).
//
// With RT_WHITTED_SEMANTICS=opencl in the environment the shim computes what
// the reference's own OpenCL kernel computes instead (rtw_render_ocl_async:
// rows [20, min(530, h)), 2x2 sub-samples, light colour, x64).
//
// Error behaviour follows the reference host: print to stderr and exit(-1).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>

#include <hip/hip_runtime.h>
#include "../../include/rt_hip.h"

// raytracer.h:34-37 (layout of the app's Scene; Primitive is rt_primitive's twin)
struct Scene;
struct rt_scene_view { int m_Primitives; rt_primitive *m_Primitive; };

extern Scene *m_Scene;                 // scene.cpp:14
extern unsigned int *m_Dest;           // scene.cpp:15 (Pixel = unsigned int, common.h:12)
extern int m_Width, m_Height, m_CurrLine;  // scene.cpp:17
extern int useGPU;                     // testapp.cpp:30 (openCLcode.cpp:19)

std::string outputLine1 = "1:";        // openCLcode.cpp:22-30
std::string outputLine2 = "2:";
std::string outputLine3 = "3:";
std::string outputLine4 = "4:";
std::string outputLine5 = "5:";
std::string outputLine6 = "6:";
std::string outputLine7 = "7:";
std::string outputLine8 = "8:";
std::string outputLine9 = "9:";

namespace {
rt_primitive *d_prims = nullptr;       // device copy of m_Scene->m_Primitive
uint32_t *d_dest = nullptr;            // device frame (m_Width * m_Height)
int dev_w = 0, dev_h = 0, dev_nprims = 0, prim_cap = 0;
int arg_w = 0, arg_h = 0, arg_nprims = 0, arg_row0 = 20;
hipStream_t stream = nullptr;

bool opencl_semantics()
{
    const char *e = getenv("RT_WHITTED_SEMANTICS");
    return e && strcmp(e, "opencl") == 0;
}

// Rows the device writes: Engine_Render's [m_CurrLine, m_Height - 70), or
// raytrace_kernel's [20, min(530, height)).
void window(int *r0, int *r1)
{
    if (opencl_semantics()) {
        *r0 = 20;
        *r1 = arg_h < 530 ? arg_h : 530;
    } else {
        *r0 = arg_row0;
        *r1 = arg_h - 70;
    }
}

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
}  // namespace

// openCLcode() (openCLcode.cpp:162-535): device selection + "program build".
// Returns a malloc'd description string as the reference's _strdup'd
// platform string (printed into the framebuffer by testapp.cpp:73-76).
char *openCLcode()
{
    int n = rt_device_count();
    if (n < 1) {
        fprintf(stderr, "Failed to find a HIP device: %s\n", rt_last_error());
        exit(-1);
    }
    int rc = rt_set_device(0);
    if (rc) die("Failed to select HIP device 0", rc);
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, 0);
    if (e != hipSuccess) die_hip("Failed to query HIP device", e);
    e = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
    if (e != hipSuccess) die_hip("Failed to create HIP stream", e);
    outputLine1 = std::string("1: HIP device 0: ") + prop.name + " (" + prop.gcnArchName + ")";
    outputLine2 = "2: compute units: " + std::to_string(prop.multiProcessorCount);
    outputLine3 = "3: global memory: " + std::to_string(prop.totalGlobalMem >> 20) + " MB";
    outputLine4 = "4: LDS per block: " + std::to_string(prop.sharedMemPerBlock) + " B";
    outputLine5 = "5: kernels: rt::whitted::root/level/tir/backacc/final_kernel (gfx950)";
    outputLine6 = "6: useGPU = " + std::to_string(useGPU);
    return strdup(outputLine1.c_str());
}

// AllocateBuffers (openCLcode.cpp:64-120): device frame sized to the
// Surface, primitives uploaded.  Unlike the reference (which leaks a cl_mem
// pair per frame, testapp.cpp:109,130), buffers are reused across calls.
void AllocateBuffers()
{
    const rt_scene_view *sc = reinterpret_cast<const rt_scene_view *>(m_Scene);
    const int np = sc->m_Primitives;
    hipError_t e;
    if (!d_dest || dev_w != m_Width || dev_h != m_Height) {
        if (d_dest) (void)hipFree(d_dest);
        e = hipMalloc(&d_dest, sizeof(uint32_t) * (size_t)m_Width * m_Height);
        if (e != hipSuccess) die_hip("Failed to create HIP output buffer", e);
        dev_w = m_Width;
        dev_h = m_Height;
    }
    if (!d_prims || prim_cap < np) {
        if (d_prims) (void)hipFree(d_prims);
        e = hipMalloc(&d_prims, sizeof(rt_primitive) * (np > 0 ? np : 1));
        if (e != hipSuccess) die_hip("Failed to create HIP scene buffer", e);
        prim_cap = np;
    }
    e = hipMemcpyAsync(d_prims, sc->m_Primitive, sizeof(rt_primitive) * np, hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) die_hip("Failed to write the HIP scene buffer", e);
    dev_nprims = np;
}

// SetKernelArguments (openCLcode.cpp:562-624): height, width, pixels,
// primitives, count -- captured here for the next ExecuteKernel.
void SetKernelArguments()
{
    arg_h = m_Height;
    arg_w = m_Width;
    arg_nprims = dev_nprims;
    arg_row0 = m_CurrLine;
}

// ExecuteKernel (openCLcode.cpp:537-560): one launch over the render window.
void ExecuteKernel()
{
    int row0, row1;
    window(&row0, &row1);
    if (row1 <= row0) return;           // the reference loop would not run either
    const int rc = opencl_semantics()
                       ? rtw_render_ocl_async(d_prims, arg_nprims, d_dest, arg_w, arg_h, nullptr, stream)
                       : rtw_render_async(d_prims, arg_nprims, d_dest, arg_w, arg_h, row0, row1, nullptr, stream);
    if (rc) die("Failed to enqueue HIP work", rc);
}

// ReadKernelBuffer (openCLcode.cpp:626-643): blocking read into m_Dest.  Only
// the window rows are copied: rows outside [m_CurrLine, m_Height-70) keep the
// host's contents (the CPU path never writes them).
void ReadKernelBuffer()
{
    int row0, row1;
    window(&row0, &row1);
    hipError_t e;
    if (row1 > row0) {
        const size_t off = (size_t)row0 * arg_w, len = (size_t)(row1 - row0) * arg_w;
        e = hipMemcpyAsync(m_Dest + off, d_dest + off, sizeof(uint32_t) * len, hipMemcpyDeviceToHost, stream);
        if (e != hipSuccess) die_hip("Failed to read the HIP pixel buffer", e);
    }
    e = hipStreamSynchronize(stream);
    if (e != hipSuccess) die_hip("Failed to read the HIP pixel buffer", e);
}

// FreeBuffers (openCLcode.cpp:50-62; never called by the reference app).
void FreeBuffers()
{
    if (d_dest) (void)hipFree(d_dest);
    if (d_prims) (void)hipFree(d_prims);
    d_dest = nullptr;
    d_prims = nullptr;
    dev_w = dev_h = prim_cap = 0;
}
