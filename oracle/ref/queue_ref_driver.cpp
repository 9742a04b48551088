/*
 * oracle/ref/queue_ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * Links the reference's own Raytracer3.2.03 CPU path into
 * oracle/_ref/libref_queue.so: raytracer_non_OpenCL.c (the queue tracer
 * raytracer_non_kernel, :285-449), scene.c (create_scene, :48-128) and
 * bitmap.c (write_bmp_file, :8-74), all compiled unmodified where they lie
 * under /root/reference, as C++ like the reference's project does
 * (OpenCL Raytracer.vcxproj:85-121 <CompileAs>CompileAsCpp</CompileAs>),
 * against the system's Khronos <CL/cl.h> (common.h:9) -- no stand-in
 * headers.  raytracer.c itself includes <Windows.h> (:4), absent here, so its
 * main() sequence is restated below: create_scene, the Primitive ->
 * Primitive_2 copy (raytracer.c:720-746), raytracer_non_kernel (:756), the
 * Pixel copy and write_bmp_file (:777-787).
 */
#include <stdlib.h>
#include <string.h>
#include "common.h"
#include "scene.h"
#include "bitmap.h"

extern void raytracer_non_kernel(uchar_4 *pixels, int width, int height, Primitive_2 *primitives,
                                 int n_primitives);

// create_scene + the copy of raytracer.c:721-746 (field for field).
extern "C" int ref_q_scene(Primitive_2 *out, int cap)
{
    cl_uint n = 0;
    Primitive *pl = create_scene(n);
    if (!pl || (int)n > cap) { free(pl); return -1; }
    memset(out, 0, sizeof(Primitive_2) * n);
    for (int i = 0; i < (int)n; i++) {
        out[i].center.x = pl[i].center.s[0];
        out[i].center.y = pl[i].center.s[1];
        out[i].center.z = pl[i].center.s[2];
        out[i].center.w = pl[i].center.s[3];
        out[i].depth = pl[i].depth;
        out[i].dummy_3 = pl[i].material.dummy_3;
        out[i].is_light = pl[i].is_light;
        out[i].m_color.x = pl[i].material.color.s[0];
        out[i].m_color.y = pl[i].material.color.s[1];
        out[i].m_color.z = pl[i].material.color.s[2];
        out[i].m_color.w = pl[i].material.color.s[3];
        out[i].m_diff = pl[i].material.diff;
        out[i].m_refl = pl[i].material.refl;
        out[i].m_refr = pl[i].material.refr;
        out[i].m_refr_index = pl[i].material.refr_index;
        out[i].m_spec = pl[i].material.spec;
        out[i].normal.x = pl[i].normal.s[0];
        out[i].normal.y = pl[i].normal.s[1];
        out[i].normal.z = pl[i].normal.s[2];
        out[i].normal.w = pl[i].normal.s[3];
        out[i].radius = pl[i].radius;
        out[i].r_radius = pl[i].r_radius;
        out[i].sq_radius = pl[i].sq_radius;
        out[i].type = pl[i].type;
    }
    free(pl);
    return (int)n;
}

// raytracer_non_kernel over the whole frame (the reference has no row window).
extern "C" void ref_q_render(uchar_4 *pixels, int width, int height, Primitive_2 *prims, int n)
{
    raytracer_non_kernel(pixels, width, height, prims, n);
}

// raytracer.c:777-787: uchar_4 -> Pixel (cl_uchar4), then write_bmp_file.
extern "C" int ref_q_write_bmp(const uchar_4 *px, int width, int height, char *path)
{
    Pixel *out = (Pixel *)malloc(sizeof(Pixel) * (size_t)width * height);
    if (!out) return 0;
    for (size_t i = 0; i < (size_t)width * height; i++) {
        out[i].s[0] = px[i].x;
        out[i].s[1] = px[i].y;
        out[i].s[2] = px[i].z;
        out[i].s[3] = px[i].w;
    }
    int ok = write_bmp_file(out, width, height, path);
    free(out);
    return ok;
}

extern "C" int ref_q_sizeof_primitive(void) { return (int)sizeof(Primitive_2); }
