/*
 * oracle/ref/whitted_ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * Links the reference's own raytracer3.0.06.no_rec.samp/scene.cpp (compiled
 * unmodified from /root/reference) into oracle/_ref/libref_whitted_scene.so,
 * exposing Scene_InitScene / Primitive_Intersect / Primitive_GetNormal so the
 * C restatement in oracle/whitted_oracle.c can be checked against them.
 * raytracer.cpp (Engine_Raytrace / Engine_Render) includes <windows.h>, which
 * this image lacks: it is not built (no stand-in headers); the full-frame pin
 * for the Whitted path is the reference-produced known-answer hashes of
 * SURVEY.md §8(c) (tests/golden/known_answers.json).
 */
#include <string.h>
#include "common.h"
#include "raytracer.h"
#include "scene.h"

extern "C" int ref_whitted_scene(Primitive *out, int cap)
{
    Scene_InitScene();
    int n = m_Scene->m_Primitives;
    if (cap < n) return -1;
    memcpy(out, m_Scene->m_Primitive, sizeof(Primitive) * n);
    return n;
}

extern "C" int ref_primitive_intersect(Primitive *p, const float ray[6], float *dist)
{
    Ray r;
    r.m_Origin.x = ray[0]; r.m_Origin.y = ray[1]; r.m_Origin.z = ray[2];
    r.m_Direction.x = ray[3]; r.m_Direction.y = ray[4]; r.m_Direction.z = ray[5];
    return Primitive_Intersect(p, &r, dist);
}

extern "C" void ref_primitive_normal(const Primitive *p, const float pos[3], float out[3])
{
    vector3 q, n;
    q.x = pos[0]; q.y = pos[1]; q.z = pos[2];
    Primitive_GetNormal(&n, *p, q);
    out[0] = n.x; out[1] = n.y; out[2] = n.z;
}

extern "C" int ref_sizeof_primitive(void) { return (int)sizeof(Primitive); }
