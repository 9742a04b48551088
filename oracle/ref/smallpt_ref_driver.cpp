/*
 * oracle/ref/smallpt_ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * Builds the reference's own smallpt radiance core (geomfunc.h, simplernd.h,
 * vec.h, scene.h from /root/reference/smallptgpu-v1.6, included in place,
 * unmodified, no stand-in headers) into oracle/_ref/libref_smallpt.so so the
 * C restatement in oracle/smallpt_oracle.c can be checked against it.
 * Compiled with g++ like the reference (argument-evaluation order of
 * geomfunc.h:138 matters).  The pixel loop below restates
 * UpdateRenderingCPU (smallptCPU.cpp:84-123), whose file also pulls in GLUT.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>     /* smallptCPU.cpp:36 includes math.h before the scene headers */

#include "camera.h"
#include "scene.h"

extern "C" int ref_cornell(Sphere *out, int cap)
{
    int n = (int)(sizeof(CornellSpheres) / sizeof(Sphere));
    if (cap < n) return -1;
    memcpy(out, CornellSpheres, sizeof(CornellSpheres));
    return n;
}

extern "C" float ref_get_random(unsigned int *s0, unsigned int *s1) { return GetRandom(s0, s1); }

extern "C" void ref_smallpt_render(const Sphere *spheres, unsigned sphereCount, const Camera *cam,
                                   Vec *colors, unsigned int *seeds, unsigned int *pixels,
                                   int width, int height, int row_begin, int row_end,
                                   int first_sample, int nsamples, int direct_lighting)
{
    const float invWidth = 1.f / width;
    const float invHeight = 1.f / height;
    for (int y = row_begin; y < row_end; y++) {
        for (int x = 0; x < width; x++) {
            const int i = (height - y - 1) * width + x;
            const int i2 = 2 * i;
            for (int k = 0; k < nsamples; k++) {
                const int currentSample = first_sample + k;
                const float r1 = GetRandom(&seeds[i2], &seeds[i2 + 1]) - .5f;
                const float r2 = GetRandom(&seeds[i2], &seeds[i2 + 1]) - .5f;
                const float kcx = (x + r1) * invWidth - .5f;
                const float kcy = (y + r2) * invHeight - .5f;
                Vec rdir;
                vinit(rdir,
                      cam->x.x * kcx + cam->y.x * kcy + cam->dir.x,
                      cam->x.y * kcx + cam->y.y * kcy + cam->dir.y,
                      cam->x.z * kcx + cam->y.z * kcy + cam->dir.z);
                Vec rorig;
                vsmul(rorig, 0.1f, rdir);
                vadd(rorig, rorig, cam->orig)
                vnorm(rdir);
                const Ray ray = {rorig, rdir};
                Vec r;
                if (direct_lighting)
                    RadianceDirectLighting(spheres, sphereCount, &ray, &seeds[i2], &seeds[i2 + 1], &r);
                else
                    RadiancePathTracing(spheres, sphereCount, &ray, &seeds[i2], &seeds[i2 + 1], &r);
                if (currentSample == 0)
                    colors[i] = r;
                else {
                    const float k1 = currentSample;
                    const float k2 = 1.f / (k1 + 1.f);
                    colors[i].x = (colors[i].x * k1 + r.x) * k2;
                    colors[i].y = (colors[i].y * k1 + r.y) * k2;
                    colors[i].z = (colors[i].z * k1 + r.z) * k2;
                }
            }
            if (nsamples > 0)
                pixels[y * width + x] = toInt(colors[i].x) | (toInt(colors[i].y) << 8) |
                                        (toInt(colors[i].z) << 16);
        }
    }
}
