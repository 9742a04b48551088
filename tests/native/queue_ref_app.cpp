// tests/native/queue_ref_app.cpp -- test harness: Raytracer3.2.03's main()
// (raytracer.c:705-797) over the HIP drop-in (csrc/shim_queue.cpp), linked
// with the reference's OWN scene.c and bitmap.c (compiled unmodified, as C++,
// where they lie under /root/reference by tests/native/Makefile; never
// copied).  raytracer.c itself includes <Windows.h>, which this image lacks,
// so its main() sequence is restated: create_scene (initialize_host
// :17-42), the Primitive -> Primitive_2 copy (:716-746),
// raytracer_non_kernel (:756), the Pixel copy (:777-783) and
// write_bmp_file (:787).  OpenCL initialisation and the timing printout are
// left out (the kernel run they set up is commented out in the reference,
// :753-754).  Writes the BMP to argv[3] (the reference: test.bmp).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "common.h"
#include "scene.h"
#include "bitmap.h"

extern void raytracer_non_kernel(uchar_4 *pixels, int width, int height, Primitive_2 *primitives,
                                 int n_primitives);

int main(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: queue_ref_app W H out.bmp\n"); return 2; }
    const cl_uint width = (cl_uint)atoi(argv[1]), height = (cl_uint)atoi(argv[2]);
    cl_uint n_primitives = 0;
    Primitive *primitive_list = create_scene(n_primitives);                  // :20
    Pixel *out_pixels = (Pixel *)malloc(sizeof(Pixel) * width * height);     // :29-42
    memset(out_pixels, 0, sizeof(Pixel) * width * height);
    int int_width = (int)width, int_height = (int)height, int_n_primitives = (int)n_primitives;
    uchar_4 *out_pixels_2 = (uchar_4 *)malloc(sizeof(uchar_4) * width * height);
    Primitive_2 *primitive_list_2 = (Primitive_2 *)malloc(sizeof(Primitive_2) * 50);
    for (int i = 0; i < int_n_primitives; i++) {
        primitive_list_2[i].center.x = primitive_list[i].center.s[0];
        primitive_list_2[i].center.y = primitive_list[i].center.s[1];
        primitive_list_2[i].center.z = primitive_list[i].center.s[2];
        primitive_list_2[i].center.w = primitive_list[i].center.s[3];
        primitive_list_2[i].depth = primitive_list[i].depth;
        primitive_list_2[i].dummy_3 = primitive_list[i].material.dummy_3;
        primitive_list_2[i].is_light = primitive_list[i].is_light;
        primitive_list_2[i].m_color.x = primitive_list[i].material.color.s[0];
        primitive_list_2[i].m_color.y = primitive_list[i].material.color.s[1];
        primitive_list_2[i].m_color.z = primitive_list[i].material.color.s[2];
        primitive_list_2[i].m_color.w = primitive_list[i].material.color.s[3];
        primitive_list_2[i].m_diff = primitive_list[i].material.diff;
        primitive_list_2[i].m_refl = primitive_list[i].material.refl;
        primitive_list_2[i].m_refr = primitive_list[i].material.refr;
        primitive_list_2[i].m_refr_index = primitive_list[i].material.refr_index;
        primitive_list_2[i].m_spec = primitive_list[i].material.spec;
        primitive_list_2[i].normal.x = primitive_list[i].normal.s[0];
        primitive_list_2[i].normal.y = primitive_list[i].normal.s[1];
        primitive_list_2[i].normal.z = primitive_list[i].normal.s[2];
        primitive_list_2[i].normal.w = primitive_list[i].normal.s[3];
        primitive_list_2[i].radius = primitive_list[i].radius;
        primitive_list_2[i].r_radius = primitive_list[i].r_radius;
        primitive_list_2[i].sq_radius = primitive_list[i].sq_radius;
        primitive_list_2[i].type = primitive_list[i].type;
    }
    raytracer_non_kernel(out_pixels_2, int_width, int_height, primitive_list_2, int_n_primitives);
    const cl_uint cnt = width * height;
    for (cl_uint i = 0; i < cnt; i++) {
        out_pixels[i].s[0] = out_pixels_2[i].x;
        out_pixels[i].s[1] = out_pixels_2[i].y;
        out_pixels[i].s[2] = out_pixels_2[i].z;
        out_pixels[i].s[3] = out_pixels_2[i].w;
    }
    write_bmp_file(out_pixels, (int)width, (int)height, argv[3]);
    free(primitive_list);
    free(out_pixels);
    free(out_pixels_2);
    free(primitive_list_2);
    return 0;
}
