// shim_queue.cpp -- drop-in replacement for Raytracer3.2.03's
// raytracer_non_OpenCL.c (the CPU queue tracer raytracer.c:756 calls).
//
// Link this translation unit (and librt_hip.so) into the reference app in
// place of raytracer_non_OpenCL.c: raytracer.c's declaration
//   extern void raytracer_non_kernel(uchar_4 *pixels, int width, int height,
//                                    Primitive_2 *primitives, int n_primitives);
// (raytracer.c:11-16, C++ linkage -- the project compiles its .c files as
// C++) resolves to the function below, which renders the same frame bit for
// bit on the GPU (rtq_render).  The two structs are declared here with the
// reference's names and layouts (raytracer_non_OpenCL.c:42-81, common.h:11-63)
// so the mangled symbol is the one raytracer.c references.
//
// Error behaviour: raytracer_non_kernel returns void and cannot fail in the
// reference; a device failure here prints rt_last_error() and exits(-1), as
// the reference's OpenCL host does on every failed call (raytracer.c:84-640).
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include "../../include/rt_hip.h"

typedef struct { float x, y, z, w; } float_4;                  // raytracer_non_OpenCL.c:42-44
typedef struct { unsigned char x, y, z, w; } uchar_4;          // :46-48
typedef enum { PLANE = 0, SPHERE = 1 } prim_type;              // :62-65
typedef struct {                                               // :67-81
    float_4 m_color;
    float m_refl, m_diff, m_refr, m_refr_index, m_spec, dummy_3;
    prim_type type;
    bool is_light;
    float_4 normal, center;
    float depth, radius, sq_radius, r_radius;
} Primitive_2;

static_assert(sizeof(Primitive_2) == sizeof(rtq_primitive), "Primitive_2 is rtq_primitive's twin");
static_assert(sizeof(uchar_4) == sizeof(uint32_t), "uchar_4 is one 32-bit pixel");

void raytracer_non_kernel(uchar_4 *pixels, int width, int height, Primitive_2 *primitives, int n_primitives)
{
    const int rc = rtq_render((const rtq_primitive *)primitives, n_primitives, (uint32_t *)pixels, width, height,
                              nullptr);
    if (rc != RT_OK) {
        fprintf(stderr, "Error: raytracer_non_kernel on the GPU failed: %s\n", rt_last_error());
        exit(-1);
    }
}
