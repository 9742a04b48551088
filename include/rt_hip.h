/*
 * rt_hip.h -- C-ABI of the MI355X (gfx950) per-pixel ray-trace hot path.
 *
 * Drop-in device path for the two reference renderers of
 * markrosoft/se-195-project-ray-tracer:
 *
 *   Whitted (raytracer3.0.06.no_rec.samp): rtw_* replace the OpenCL device
 *     path of openCLcode.cpp -- AllocateBuffers (:64-120), SetKernelArguments
 *     (:562-624), ExecuteKernel / clEnqueueNDRangeKernel (:537-560) and
 *     ReadKernelBuffer (:626-643) -- and compute what the CPU path
 *     Engine_Render (raytracer.cpp:301-530) computes, bit for bit.
 *   smallpt (smallptgpu-v1.6): spt_* replace ExecuteKernel (smallptGPU.cpp:617-640)
 *     and the buffer traffic of UpdateRenderingGPU (:642-782) / ReInit*GPU
 *     (:784-830), computing UpdateRenderingCPU's per-pixel result
 *     (smallptCPU.cpp:84-123: flipped colour/seed slot, running average, toInt).
 *   Queue tracer (Raytracer3.2.03): rtq_* replace raytracer_non_kernel
 *     (raytracer_non_OpenCL.c:285-449), the CPU twin its raytracer.c:756
 *     calls in place of run_openCL_kernel (:417-640), computing its uchar4
 *     frame bit for bit.
 *
 * Plain pointers and sizes only.  Every entry point returns RT_OK (0) or a
 * negative RT_ERR_* code; rt_last_error() describes the last failure of the
 * calling thread.  Struct layouts are byte-identical to the reference's.
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK 0
#define RT_ERR_INVALID -1   /* bad argument (null pointer, size, row range) */
#define RT_ERR_HIP -2       /* HIP runtime failure (rt_last_error has the text) */
#define RT_ERR_NODEVICE -3  /* no gfx950 device visible */

typedef struct { float x, y, z; } rt_vec3;

/* raytracer.h:23-32 (Material :18-21, plane common.h:49-53) -- 96 bytes */
typedef struct {
    int32_t type;                 /* SPHERE = 1, PLANE = 2, BOX = 3 */
    int32_t m_Light;
    rt_vec3 m_Centre;
    float m_SqRadius, m_Radius, m_RRadius;
    rt_vec3 plane_N;
    float plane_D;
    float plane_cell[4];
    rt_vec3 m_Color;
    float m_Refl, m_Refr, m_Diff, m_Spec, m_RIndex;
} rt_primitive;

/* smallptgpu-v1.6/geom.h:43-47 -- 44 bytes */
typedef struct {
    float rad;
    rt_vec3 p, e, c;
    int32_t refl;                 /* DIFF = 0, SPEC = 1, REFR = 2 */
} rt_sphere;

/* smallptgpu-v1.6/camera.h:29-34 -- 60 bytes */
typedef struct {
    rt_vec3 orig, target;
    rt_vec3 dir, x, y;
} rt_camera;

/* Raytracer3.2.03 raytracer_non_OpenCL.c:42-44 float_4 */
typedef struct { float x, y, z, w; } rtq_float4;

/* Raytracer3.2.03 raytracer_non_OpenCL.c:67-81 Primitive_2 -- 96 bytes
 * (the C++ bool is_light is one byte). */
typedef struct {
    rtq_float4 m_color;
    float m_refl, m_diff, m_refr, m_refr_index, m_spec, dummy_3;
    int32_t type;                 /* PLANE = 0, SPHERE = 1 */
    uint8_t is_light;
    uint8_t pad_[3];
    rtq_float4 normal, center;
    float depth, radius, sq_radius, r_radius;
} rtq_primitive;

/* ------------------------------------------------------------ runtime */
const char *rt_last_error(void);
int rt_device_count(void);
/* Select the HIP device used by the calling thread's subsequent calls. */
int rt_set_device(int device);
/* Release the per-device buffers the blocking entry points cache. */
int rt_release(void);
/* Bytes of device memory the blocking entry points currently cache. */
size_t rt_cached_bytes(void);
/* Page-locked host memory (hipHostMalloc) for frames the host reads back
 * every pass -- the smallpt drop-in's `pixels` (smallptGPU.cpp:111, a plain
 * malloc there, read by ReadKernelBuffer :626 after every pass): its
 * device-to-host copy then runs at DMA speed instead of through a staging
 * buffer.  rt_host_free(NULL) is a no-op. */
int rt_host_alloc(size_t bytes, void **out);
int rt_host_free(void *p);

/* ------------------------------------------------------------ Whitted */
/* Blocking, host buffers.  Renders rows [row_begin,row_end) of the w x h
 * frame into xrgb (uint32 0x00RRGGBB, row-major), leaving other rows
 * untouched; the reference window is [20, h-70) (raytracer.cpp:281,307).
 * Requires 20 <= row_begin < row_end <= h (m_SY's recurrence starts at row 20).
 * counters (nullable, host, 4 x u64): traced rays, shadow rays,
 * Primitive_Intersect calls, total-internal-reflection events -- the same
 * quantities oracle/orw_render counts. */
int rtw_render(const rt_primitive *prims, int nprims, uint32_t *xrgb, int w, int h,
               int row_begin, int row_end, uint64_t *counters);

/* Asynchronous, device-resident.  d_prims: device copy of the primitive
 * array; d_xrgb: device frame (w*h); d_counters: device u64[4] accumulated
 * into (nullable); stream: hipStream_t (NULL = default stream).  Work is
 * ordered on `stream`: a large frame also runs on a library-owned second
 * stream, forked from `stream` and joined back to it by events before the
 * call's last operation. */
int rtw_render_async(const rt_primitive *d_prims, int nprims, uint32_t *d_xrgb, int w, int h,
                     int row_begin, int row_end, uint64_t *d_counters, void *stream);

/* The reference's own device kernel instead of its CPU path: raytrace_kernel
 * of raytracer3.0.06.no_rec.samp/openCLcode.cl:5-247 with openCLcode.h's
 * Engine_Raytrace (ExecuteKernel, openCLcode.cpp:537-560) -- rows
 * [20, min(530, h)) (openCLcode.cl:66-67), SX = WX1 + x*DX per pixel (:22-23),
 * 2x2 sub-samples (:66), a light hit adds the light's colour
 * (openCLcode.h:176-182), reflection child folded before the refraction child
 * (:199-233), x(256/4) scale (:238-240).  The OpenCL built-ins (sqrt, '/',
 * exp, pow) are computed as the CPU path's correctly rounded / glibc
 * functions.  Same counters as rtw_render.  Rows outside the window are not
 * written. */
int rtw_render_ocl(const rt_primitive *prims, int nprims, uint32_t *xrgb, int w, int h,
                   uint64_t *counters);
int rtw_render_ocl_async(const rt_primitive *d_prims, int nprims, uint32_t *d_xrgb, int w, int h,
                         uint64_t *d_counters, void *stream);

/* ------------------------------------------------------------ smallpt */
#define SPT_PATH_TRACING 0       /* RadiancePathTracing    geomfunc.h:167-338 */
#define SPT_DIRECT_LIGHTING 1    /* RadianceDirectLighting geomfunc.h:340-483 */
/* Flag OR-ed into `mode` of the device-resident entry points: with
 * d_counters, count only counters[0] (Intersect calls), [1] (IntersectP
 * calls) and [3] (samples) -- SURVEY §8(d)'s rays -- and leave counters[2]
 * (sphere tests) untouched.  The sphere-test count needs IntersectP's
 * early-exit position (geomfunc.h:94-110: the highest-index occluder), which
 * costs hierarchy scenes a longer shadow walk; the call counts do not. */
#define SPT_COUNT_RAYS 0x100
/* Flag OR-ed into `mode` of spt_scene_render_list_async with d_group_cost:
 * each listed group's entry receives the LONGEST of its tiles' wave times
 * (atomic max) instead of their sum -- the length of the group's slowest
 * pixel chain, the order key for the heavy-tile treatment (list such groups
 * first), where the sum is the load to balance. */
#define SPT_COST_MAX 0x200
/* Flag OR-ed into `mode` of spt_scene_render_list_async only: the caller
 * guarantees that d_groups is already a set (no repeats, every entry in
 * range -- rtamd.dist.ListGather checks its lists on the host), so the
 * per-call dedup pass (a stream-ordered scratch allocation, a fill, one
 * small kernel, the free) is skipped.  A list that breaks the promise may
 * render a group twice in one launch: results are then undefined. */
#define SPT_LIST_SET 0x800

/* Blocking, host buffers, whole frame.  Runs samples first_sample ..
 * first_sample+nsamples-1 of every pixel, exactly as nsamples successive
 * UpdateRenderingCPU passes with currentSample = first_sample, ...:
 *   colors  float[3*w*h]  Vec per pixel, slot (h-y-1)*w+x      (in/out)
 *   seeds   uint32[2*w*h] two MWC words per slot (h-y-1)*w+x    (in/out)
 *   pixels  uint32[w*h]   toInt(r) | toInt(g)<<8 | toInt(b)<<16 at y*w+x (out)
 * mode: SPT_PATH_TRACING or SPT_DIRECT_LIGHTING.  counters (nullable,
 * host, 4 x u64): Intersect calls, IntersectP calls, sphere tests, samples. */
int spt_render(const rt_sphere *spheres, unsigned nspheres, const rt_camera *camera,
               float *colors, uint32_t *seeds, uint32_t *pixels, int w, int h,
               int first_sample, int nsamples, int mode, uint64_t *counters);

/* Device-resident buffers, rows [row_begin,row_end) of the frame.  Buffers
 * are full-frame device arrays laid out as above; seeds are read from
 * d_seeds_in and the advanced state written to d_seeds_out (may alias).
 * camera is read on the host at call time (passed by value to the kernel).
 * Reads the sphere array back (synchronising `stream` once) to find or
 * prepare the device's cached scene -- prepared again only when the array's
 * contents change -- then launches asynchronously; use spt_scene_* to stay
 * fully asynchronous.  spt_render uses the same cache. */
int spt_render_async(const rt_sphere *d_spheres, unsigned nspheres, const rt_camera *camera,
                     float *d_colors, const uint32_t *d_seeds_in, uint32_t *d_seeds_out,
                     uint32_t *d_pixels, int w, int h, int row_begin, int row_end,
                     int first_sample, int nsamples, int mode, uint64_t *d_counters,
                     void *stream);

/* Prepared scene: uploads the sphere array once (device SoA of geometry,
 * materials and per-light records; for >= 256 spheres also the exact-culling
 * sphere hierarchy).  Reuse it across frames. */
typedef struct spt_scene spt_scene;
int spt_scene_create(const rt_sphere *spheres, unsigned nspheres, spt_scene **out);
int spt_scene_destroy(spt_scene *scene);
/* spt_render_async on a prepared scene: asynchronous on `stream`
 * (graph-capturable).  Hierarchy scenes (>= 256 spheres) learn a dispatch
 * order: the first launch of a (window, camera, nsamples, mode) key records
 * each tile group's wave time and queues a 32-KB-class read-back of it; once
 * that has landed, launches of the key dispatch the heaviest groups first
 * (one small upload).  Scheduling only -- results are identical; during
 * stream capture the learnt order is used but not updated.  A scene's order
 * is updated by the calling thread: render one scene from one host thread
 * at a time.  Hierarchy scenes give every launch one of 64 work-counter
 * entries; a launch captured into a graph keeps its entry for the graph's
 * life (the graph may be replayed at any time), so at most 64 captured
 * launches of one scene can exist -- the next capture fails RT_ERR_INVALID
 * until spt_scene_release_captures. */
int spt_scene_render_async(const spt_scene *scene, const rt_camera *camera, float *d_colors,
                           const uint32_t *d_seeds_in, uint32_t *d_seeds_out, uint32_t *d_pixels,
                           int w, int h, int row_begin, int row_end, int first_sample, int nsamples,
                           int mode, uint64_t *d_counters, void *stream);

/* Hands the work-counter entries held by captured launches of `scene` out
 * again.  Call it only once every graph captured from this scene's launches
 * has been destroyed (a replay after it could share an entry with a new
 * launch). */
int spt_scene_release_captures(const spt_scene *scene);

/* spt_scene_render_async over an interleaved window: every pixel row y with
 * (y / 8) % ngroups == group, i.e. 8-row groups group, group + ngroups, ...
 * (0 <= group < ngroups).  The ngroups windows of a frame partition it; a
 * multi-GPU frame split this way gives each GPU the same mix of the image
 * (contiguous bands differ in cost with their content).  Same results per
 * pixel as any other window. */
int spt_scene_render_groups_async(const spt_scene *scene, const rt_camera *camera, float *d_colors,
                                  const uint32_t *d_seeds_in, uint32_t *d_seeds_out, uint32_t *d_pixels,
                                  int w, int h, int group, int ngroups, int first_sample, int nsamples,
                                  int mode, uint64_t *d_counters, void *stream);

/* Tile groups: group g is the 8x8-pixel tiles 4g .. 4g+3 of the frame in
 * row-major tile order (ceil(w/8) tiles per row) -- a 32x8 strip when
 * ceil(w/8) is a multiple of 4.  spt_group_count(w, h) = ceil(ceil(w/8) *
 * ceil(h/8) / 4) (or a negative RT_ERR_*). */
int spt_group_count(int w, int h);

/* spt_scene_render_async over an explicit set of tile groups: d_groups
 * (device, ngroups entries in [0, spt_group_count(w, h)); entries outside
 * are skipped; the list is taken as a set -- a repeated group renders once,
 * at the dispatch slot of one of its copies) in dispatch order -- the first
 * ones start first, so list the costliest first.  A multi-GPU frame split by per-rank lists
 * balanced on measured costs (rtamd.dist.balanced_partition).  d_group_cost
 * (nullable, device, spt_group_count(w, h) words; hierarchy scenes only,
 * left unchanged otherwise): each listed group's wave time in 100 MHz ticks
 * is ADDED to its entry (zero it first).  With full counters (d_counters
 * set, no SPT_COUNT_RAYS) a lane that finishes its pixel takes the next one
 * (pixel refill), so there the unit is a pixel: the entry receives the sum
 * of its pixels' durations, or with SPT_COST_MAX the longest one -- a lane
 * time, not a wave time.  No order is learnt on this path.
 * Same results per pixel as any other window. */
int spt_scene_render_list_async(const spt_scene *scene, const rt_camera *camera, float *d_colors,
                                const uint32_t *d_seeds_in, uint32_t *d_seeds_out, uint32_t *d_pixels,
                                int w, int h, const int *d_groups, int ngroups, int first_sample,
                                int nsamples, int mode, uint64_t *d_counters, unsigned *d_group_cost,
                                void *stream);

/* The accumulator of listed tile groups to / from a packed buffer of 768
 * floats per group (its four tiles in turn, 64 pixels each in row-major
 * order, r g b; pixels outside the frame pack as 0 and are not unpacked):
 * the exchange of a frame split by group lists (one all-gather of the packed
 * shares).  Exact copies, asynchronous on `stream`. */
int spt_groups_pack_async(const float *d_colors, int w, int h, const int *d_groups, int ngroups,
                          float *d_out, void *stream);
int spt_groups_unpack_async(float *d_colors, int w, int h, const int *d_groups, int ngroups,
                            const float *d_in, void *stream);

/* The toInt pack of UpdateRenderingCPU (smallptCPU.cpp:120-122, vec.h:62)
 * alone: d_pixels[y*w+x] for rows [row_begin,row_end) from the accumulator
 * slots (h-y-1)*w+x of d_colors -- the pixels a render call writes, rebuilt
 * from colours that arrived from other ranks (a row-band frame assembled by
 * one colour all-gather).  Asynchronous on `stream`. */
int spt_pack_pixels_async(const float *d_colors, uint32_t *d_pixels, int w, int h, int row_begin,
                          int row_end, void *stream);

/* ------------------------------------------------------------ smallpt, several GPUs */
/* One frame tiled over the GPUs of a node in row bands:
 * band k owns the k-th contiguous chunk of the flipped colour / seed slots,
 * i.e. pixel rows [h - e_k, h - s_k) with B = ceil(h/ngpus), s_k = min(h, k*B),
 * e_k = min(h, (k+1)*B) -- equal bands (the last one shorter, or empty), so
 * one in-place all-gather of B rows per band assembles the frame.
 * Every pixel keeps its RNG words and accumulator on its band's device, so
 * rendering needs no exchange; samples of a pixel are never split.  One host
 * thread drives all devices (one stream each), as the reference's single
 * host thread drove its one OpenCL queue (smallptGPU.cpp:617-640,739-760).
 *
 * devices: ngpus device ordinals (NULL: 0..ngpus-1).  A device may repeat
 * (several bands on one GPU -- the same band/assemble code on one device).
 * Each band holds a full-frame colour / seed / pixel array on its device;
 * only its own rows are authoritative until spt_multi_gather_async. */
typedef struct spt_multi spt_multi;
int spt_multi_create(const rt_sphere *spheres, unsigned nspheres, int w, int h, const int *devices,
                     int ngpus, spt_multi **out);
int spt_multi_destroy(spt_multi *m);
/* Re-uploads the scene to every band's device (ReInitSceneGPU). */
int spt_multi_set_scene(spt_multi *m, const rt_sphere *spheres, unsigned nspheres);
/* Pixel-row bounds: rows[k] .. rows[k+1] hold band k's rows in FLIPPED
 * order, i.e. band k renders pixel rows [h - rows[k+1], h - rows[k]).
 * rows: ngpus + 1 ints. */
int spt_multi_bands(const spt_multi *m, int *rows);
/* Host -> bands: each band's rows of seeds (2*w*h words, flipped slots) and,
 * when colors is not NULL, of the accumulator (3*w*h floats).  Blocking. */
int spt_multi_upload(spt_multi *m, const float *colors, const uint32_t *seeds);
/* Samples first_sample .. first_sample+nsamples-1 of every pixel, each band
 * on its own device, asynchronous.  counters: accumulate the four
 * spt_render counters (read with spt_multi_counters). */
int spt_multi_render_async(spt_multi *m, const rt_camera *camera, int first_sample, int nsamples,
                           int mode, int counters);
/* Assembles the whole HDR accumulator on every band's device and repacks
 * each device's RGBA8 frame from it (spt_pack_pixels_async).  Distinct
 * devices: one in-place ncclAllGather of the equal (padded) bands over xGMI
 * (the padding rows past h are never read); repeated devices or
 * RT_SPT_GATHER=peer: stream-ordered peer copies (RT_SPT_GATHER=rccl runs the
 * RCCL all-gather even for a single band).  Asynchronous. */
int spt_multi_gather_async(spt_multi *m);
/* Waits for every band's device work. */
int spt_multi_sync(spt_multi *m);
/* Bands -> host, blocking: each band's rows of colors / seeds / pixels
 * (each nullable) -- the assembled frame, no collective needed. */
int spt_multi_download(spt_multi *m, float *colors, uint32_t *seeds, uint32_t *pixels);
/* Band k's whole device frame -> host, blocking (after a gather: the
 * assembled frame as band k's device holds it).  Either pointer nullable. */
int spt_multi_read_frame(spt_multi *m, int k, float *colors, uint32_t *pixels);
/* Sums the per-band counters into out[4] (blocking) and zeroes them. */
int spt_multi_counters(spt_multi *m, uint64_t *out);
/* Band k's device frame and stream (after a gather: the whole frame). */
int spt_multi_band_buffers(const spt_multi *m, int k, int *device, float **d_colors, uint32_t **d_seeds,
                           uint32_t **d_pixels, void **stream);

/* spt_render over several GPUs (SURVEY.md §8(b) "spt_render(..., ngpus)"):
 * the same contract and results as spt_render, the frame tiled in row bands
 * over devices[0..ngpus-1] (NULL: 0..ngpus-1), host buffers assembled band
 * by band.  Blocking.  The band context (per band: scene, buffers, stream)
 * is kept across calls: the same devices and frame size reuse it, a changed
 * sphere array re-prepares only the scenes; rt_release frees it. */
int spt_render_multi(const rt_sphere *spheres, unsigned nspheres, const rt_camera *camera,
                     float *colors, uint32_t *seeds, uint32_t *pixels, int w, int h,
                     int first_sample, int nsamples, int mode, uint64_t *counters,
                     const int *devices, int ngpus);
/* Diagnostics of spt_render_multi's cached context: out[0] = band contexts
 * built, out[1] = scene preparations (both since the process started). */
int spt_multi_cache_info(uint64_t *out);

/* ------------------------------------------------------------ queue tracer (3.2.03) */
/* Blocking, host buffers, whole frame: raytracer_non_kernel(pixels, w, h,
 * prims, nprims) (raytracer_non_OpenCL.c:285-449).  pixels: w*h uchar_4
 * (r, g, b, 0) row-major -- as uint32, r | g<<8 | b<<16.  counters (nullable,
 * host, 4 x u64): rays traced (raytrace calls), shadow rays, intersect calls,
 * undefined-behaviour events.  The last counts what the reference leaves
 * undefined and this library defines as "no child rays": a ray at depth < 5
 * that hits nothing (the reference then reads primitives[-1], :373) or hits a
 * light with m_refl or m_refr > 0 (point_intersect is uninitialised, :197).
 * Neither occurs in the reference scene (scene.c:53-97). */
int rtq_render(const rtq_primitive *prims, int nprims, uint32_t *pixels, int w, int h,
               uint64_t *counters);
/* Asynchronous, device-resident: rows [row_begin,row_end) of the w x h frame
 * (0 <= row_begin < row_end <= h; other rows untouched) into d_pixels (w*h);
 * d_counters: device u64[4] accumulated into (nullable).  Ordered on
 * `stream` as rtw_render_async (a frame of several slabs also uses the
 * library's second stream, forked and joined by events). */
int rtq_render_async(const rtq_primitive *d_prims, int nprims, uint32_t *d_pixels, int w, int h,
                     int row_begin, int row_end, uint64_t *d_counters, void *stream);

/* Host helper: AllocateBuffers' seed fill (smallptGPU.cpp:105-110) --
 * srand(seed); seeds[i] = max(rand(), 2) for i < n, with the host libc's
 * rand() (glibc on the reference's Linux build). */
void spt_seed_fill(uint32_t *seeds, size_t n, unsigned seed);

#ifdef __cplusplus
}
#endif
#endif
