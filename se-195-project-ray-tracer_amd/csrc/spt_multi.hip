// spt_multi.hip -- smallpt frames tiled over the GPUs of one node
// (include/rt_hip.h "smallpt, several GPUs"; SURVEY.md §8(b) spt_render(...,
// ngpus) and §8(e)).
//
// The reference drives one OpenCL device from one host thread
// (smallptGPU.cpp:617-640 ExecuteKernel, :739-760 the progressive loop).
// Here one host thread drives N devices, each on its own non-blocking
// stream: band k owns the k-th contiguous chunk of the flipped colour / seed
// slots ((h-y-1)*w+x, smallptCPU.cpp:86), so its accumulator and RNG words
// never leave its device and a render call needs no exchange at all.  The
// host-buffer paths (spt_render_multi, spt_multi_download) assemble the frame
// in the caller's memory band by band.  Only a device-resident frame on every
// GPU needs a collective: the bands are equal (B = ceil(h/N) rows; the last
// is shorter, its padding rows past h never read), so one in-place
// ncclAllGather over xGMI assembles the accumulator on every device, which
// then repacks its RGBA8 frame with the kernel's own toInt
// (spt_pack_pixels_async).  RCCL is loaded on first use (dlopen), so the
// single-GPU library needs nothing but the HIP runtime.
#include <algorithm>
#include <dlfcn.h>
#include <mutex>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include "rt_runtime.h"
#include "spt_band.h"
#include <rccl/rccl.h>

namespace {

struct Band {
    int device = -1;
    int s0 = 0, s1 = 0;                // flipped slot rows [s0, s1) = pixel rows [h-s1, h-s0)
    hipStream_t stream = nullptr;
    hipEvent_t rendered = nullptr;     // after this band's render (peer gather source)
    hipEvent_t gathered = nullptr;     // after this band's peer gather copies
    spt_scene *scene = nullptr;
    float *d_col = nullptr;
    uint32_t *d_seed = nullptr, *d_px = nullptr;
    unsigned long long *d_cnt = nullptr;
};

// RCCL entry points (dlopen'ed once per process).
struct Rccl {
    bool tried = false, ok = false;
    char why[200] = "";
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
};
Rccl g_rccl;
std::mutex g_rccl_mu;

const Rccl *rccl()
{
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_rccl.tried) return &g_rccl;
    g_rccl.tried = true;
    // An RCCL the process already holds (e.g. PyTorch's) first, so one
    // RCCL and one HIP runtime serve the process; else the system's.
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        snprintf(g_rccl.why, sizeof(g_rccl.why), "dlopen librccl: %s", dlerror());
        return &g_rccl;
    }
    g_rccl.init_all = (decltype(g_rccl.init_all))dlsym(h, "ncclCommInitAll");
    g_rccl.destroy = (decltype(g_rccl.destroy))dlsym(h, "ncclCommDestroy");
    g_rccl.group_start = (decltype(g_rccl.group_start))dlsym(h, "ncclGroupStart");
    g_rccl.group_end = (decltype(g_rccl.group_end))dlsym(h, "ncclGroupEnd");
    g_rccl.all_gather = (decltype(g_rccl.all_gather))dlsym(h, "ncclAllGather");
    g_rccl.err = (decltype(g_rccl.err))dlsym(h, "ncclGetErrorString");
    g_rccl.ok = g_rccl.init_all && g_rccl.destroy && g_rccl.group_start && g_rccl.group_end &&
                g_rccl.all_gather && g_rccl.err;
    if (!g_rccl.ok) snprintf(g_rccl.why, sizeof(g_rccl.why), "librccl lacks an nccl* entry point");
    return &g_rccl;
}

int fail_nccl(const Rccl *r, ncclResult_t e, const char *what)
{
    char m[256];
    snprintf(m, sizeof(m), "%s: %s (%d)", what, r->err ? r->err(e) : "rccl error", (int)e);
    return rtrt::fail(RT_ERR_HIP, m);
}

}  // namespace

struct spt_multi {
    int w = 0, h = 0;
    int brows = 0;                     // rows per band (the last band may hold fewer, or none)
    std::vector<Band> bands;
    bool distinct = true;              // no device repeats: RCCL gather possible
    std::vector<ncclComm_t> comms;     // one per band (created on first RCCL gather)
};

namespace {

int release_band(Band &b)
{
    if (b.device < 0) return RT_OK;
    (void)hipSetDevice(b.device);
    if (b.stream) (void)hipStreamSynchronize(b.stream);
    if (b.scene) spt_scene_destroy(b.scene);
    (void)hipSetDevice(b.device);
    if (b.d_col) (void)hipFree(b.d_col);
    if (b.d_seed) (void)hipFree(b.d_seed);
    if (b.d_px) (void)hipFree(b.d_px);
    if (b.d_cnt) (void)hipFree(b.d_cnt);
    if (b.rendered) (void)hipEventDestroy(b.rendered);
    if (b.gathered) (void)hipEventDestroy(b.gathered);
    if (b.stream) (void)hipStreamDestroy(b.stream);
    b = Band();
    return RT_OK;
}

void destroy_multi(spt_multi *m)
{
    if (!m) return;
    rtrt::DeviceScope scope;
    if (!m->comms.empty()) {
        const Rccl *r = rccl();
        for (ncclComm_t c : m->comms)
            if (c && r->ok) (void)r->destroy(c);
    }
    for (Band &b : m->bands) release_band(b);
    delete m;
}

// First pixel / slot index of row s.
inline size_t px_off(const spt_multi &m, int s) { return (size_t)s * m.w; }

// Stream-ordered peer copies instead of RCCL: a device repeats (several
// bands on one GPU), or RT_SPT_GATHER=peer.
bool peer_gather(const spt_multi &m)
{
    const char *g = getenv("RT_SPT_GATHER");
    return !m.distinct || (g && !strcmp(g, "peer"));
}

int scene_on_band(Band &b, rtrt::DeviceScope &scope, const rt_sphere *spheres, unsigned n)
{
    int rc = scope.select(b.device);
    if (rc) return rc;
    if (b.scene) {
        (void)hipStreamSynchronize(b.stream);
        spt_scene_destroy(b.scene);
        b.scene = nullptr;
        if ((rc = scope.select(b.device))) return rc;
    }
    return spt_scene_create(spheres, n, &b.scene);
}

int sync_all(spt_multi &m, rtrt::DeviceScope &scope)
{
    for (Band &b : m.bands) {
        int rc = scope.select(b.device);
        if (rc) return rc;
        hipError_t e = hipStreamSynchronize(b.stream);
        if (e != hipSuccess) return rtrt::fail_hip(e, "spt_multi sync");
    }
    return RT_OK;
}

}  // namespace

extern "C" int spt_multi_create(const rt_sphere *spheres, unsigned nspheres, int w, int h, const int *devices,
                                int ngpus, spt_multi **out)
{
    if (!spheres || !out || nspheres < 1 || w < 1 || h < 1 || ngpus < 1 || ngpus > 64 || ngpus > h)
        return rtrt::fail(RT_ERR_INVALID, "spt_multi_create: bad arguments");
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess) return rtrt::fail_hip(e, "hipGetDeviceCount");
    rtrt::DeviceScope scope;
    spt_multi *m = new spt_multi();
    m->w = w;
    m->h = h;
    m->bands.resize(ngpus);
    m->brows = sptband::rows_per_band(h, ngpus);
    const size_t npx = (size_t)w * h;
    const size_t npad = sptband::padded_floats(w, h, ngpus) / 3;   // pixels incl. the all-gather's padding
    int rc = RT_OK;
    for (int k = 0; k < ngpus && rc == RT_OK; k++) {
        Band &b = m->bands[k];
        const int dev = devices ? devices[k] : k;
        if (dev < 0 || dev >= ndev) { rc = rtrt::fail(RT_ERR_NODEVICE, "spt_multi_create: no such device"); break; }
        for (int j = 0; j < k; j++)
            if (m->bands[j].device == dev) m->distinct = false;
        b.device = dev;
        sptband::span(h, ngpus, k, &b.s0, &b.s1);
        if ((rc = scope.select(dev))) break;
        if ((rc = spt_scene_create(spheres, nspheres, &b.scene))) break;   // checks gfx950 too
        if ((rc = scope.select(dev))) break;
        e = hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&b.rendered, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&b.gathered, hipEventDisableTiming);
        if (e == hipSuccess) e = hipMalloc(&b.d_col, 3 * sizeof(float) * npad);
        if (e == hipSuccess) e = hipMalloc(&b.d_seed, 2 * sizeof(uint32_t) * npx);
        if (e == hipSuccess) e = hipMalloc(&b.d_px, sizeof(uint32_t) * npx);
        if (e == hipSuccess) e = hipMalloc(&b.d_cnt, 4 * sizeof(unsigned long long));
        if (e == hipSuccess) e = hipMemsetAsync(b.d_col, 0, 3 * sizeof(float) * npad, b.stream);
        if (e == hipSuccess) e = hipMemsetAsync(b.d_px, 0, sizeof(uint32_t) * npx, b.stream);
        if (e == hipSuccess) e = hipMemsetAsync(b.d_cnt, 0, 4 * sizeof(unsigned long long), b.stream);
        if (e == hipSuccess) e = hipEventRecord(b.gathered, b.stream);
        if (e != hipSuccess) rc = rtrt::fail_hip(e, "spt_multi_create");
    }
    if (rc == RT_OK) rc = sync_all(*m, scope);
    if (rc) { destroy_multi(m); return rc; }
    *out = m;
    return RT_OK;
}

extern "C" int spt_multi_destroy(spt_multi *m)
{
    destroy_multi(m);
    return RT_OK;
}

extern "C" int spt_multi_set_scene(spt_multi *m, const rt_sphere *spheres, unsigned nspheres)
{
    if (!m || !spheres || nspheres < 1) return rtrt::fail(RT_ERR_INVALID, "spt_multi_set_scene: bad arguments");
    rtrt::DeviceScope scope;
    for (Band &b : m->bands) {
        int rc = scene_on_band(b, scope, spheres, nspheres);
        if (rc) return rc;
    }
    return RT_OK;
}

extern "C" int spt_multi_bands(const spt_multi *m, int *rows)
{
    if (!m || !rows) return rtrt::fail(RT_ERR_INVALID, "spt_multi_bands: null pointer");
    for (size_t k = 0; k < m->bands.size(); k++) rows[k] = m->bands[k].s0;
    rows[m->bands.size()] = m->h;
    return RT_OK;
}

extern "C" int spt_multi_upload(spt_multi *m, const float *colors, const uint32_t *seeds)
{
    if (!m || !seeds) return rtrt::fail(RT_ERR_INVALID, "spt_multi_upload: null pointer");
    rtrt::DeviceScope scope;
    for (Band &b : m->bands) {
        int rc = scope.select(b.device);
        if (rc) return rc;
        const size_t o = px_off(*m, b.s0), n = px_off(*m, b.s1) - o;
        hipError_t e = hipMemcpyAsync(b.d_seed + 2 * o, seeds + 2 * o, 2 * sizeof(uint32_t) * n,
                                      hipMemcpyHostToDevice, b.stream);
        if (e == hipSuccess && colors)
            e = hipMemcpyAsync(b.d_col + 3 * o, colors + 3 * o, 3 * sizeof(float) * n, hipMemcpyHostToDevice,
                               b.stream);
        if (e != hipSuccess) return rtrt::fail_hip(e, "spt_multi_upload");
    }
    return sync_all(*m, scope);
}

extern "C" int spt_multi_render_async(spt_multi *m, const rt_camera *camera, int first_sample, int nsamples,
                                      int mode, int counters)
{
    if (!m || !camera) return rtrt::fail(RT_ERR_INVALID, "spt_multi_render_async: null pointer");
    rtrt::DeviceScope scope;
    for (Band &b : m->bands) {
        int rc = scope.select(b.device);
        if (rc) return rc;
        // The previous peer gather still reads this band's rows on other
        // streams: order the overwrite after every band's copies.
        if (peer_gather(*m))
            for (Band &o : m->bands) {
                if (&o == &b) continue;
                hipError_t e = hipStreamWaitEvent(b.stream, o.gathered, 0);
                if (e != hipSuccess) return rtrt::fail_hip(e, "spt_multi_render_async wait");
            }
        const int r0 = m->h - b.s1, r1 = m->h - b.s0;
        rc = spt_scene_render_async(b.scene, camera, b.d_col, b.d_seed, b.d_seed, b.d_px, m->w, m->h, r0, r1,
                                    first_sample, nsamples, mode,
                                    counters ? (uint64_t *)b.d_cnt : nullptr, b.stream);
        if (rc) return rc;
        hipError_t e = hipEventRecord(b.rendered, b.stream);
        if (e != hipSuccess) return rtrt::fail_hip(e, "spt_multi_render_async record");
    }
    return RT_OK;
}

extern "C" int spt_multi_gather_async(spt_multi *m)
{
    if (!m) return rtrt::fail(RT_ERR_INVALID, "spt_multi_gather_async: null pointer");
    const int n = (int)m->bands.size();
    const char *g = getenv("RT_SPT_GATHER");
    const bool force_rccl = g && !strcmp(g, "rccl");
    if (n == 1 && !force_rccl) return RT_OK;
    rtrt::DeviceScope scope;
    const bool peer = peer_gather(*m);
    int rc;
    if (!peer) {
        const Rccl *r = rccl();
        if (!r->ok) return rtrt::fail(RT_ERR_HIP, r->why);
        if (m->comms.empty()) {
            std::vector<int> devs(n);
            for (int k = 0; k < n; k++) devs[k] = m->bands[k].device;
            m->comms.assign(n, nullptr);
            ncclResult_t ne = r->init_all(m->comms.data(), n, devs.data());
            if (ne != ncclSuccess) { m->comms.clear(); return fail_nccl(r, ne, "ncclCommInitAll"); }
        }
        // One in-place all-gather: rank k sends its band (slot rows
        // [k B, (k+1) B), padded) from where the full buffer holds it.
        const size_t cnt = sptband::gather_count(m->w, m->h, n);
        ncclResult_t ne = r->group_start();
        if (ne != ncclSuccess) return fail_nccl(r, ne, "ncclGroupStart");
        for (int k = 0; k < n && ne == ncclSuccess; k++) {
            Band &b = m->bands[k];
            if ((rc = scope.select(b.device))) { (void)r->group_end(); return rc; }
            ne = r->all_gather(b.d_col + sptband::send_offset(m->w, m->h, n, k), b.d_col, cnt, ncclFloat32,
                               m->comms[k], b.stream);
        }
        ncclResult_t ge = r->group_end();
        if (ne != ncclSuccess) return fail_nccl(r, ne, "ncclAllGather");
        if (ge != ncclSuccess) return fail_nccl(r, ge, "ncclGroupEnd");
    } else {
        for (Band &b : m->bands) {
            if ((rc = scope.select(b.device))) return rc;
            for (Band &src : m->bands) {
                if (&src == &b) continue;
                const size_t o = 3 * px_off(*m, src.s0), cnt = 3 * px_off(*m, src.s1) - o;
                hipError_t e = hipStreamWaitEvent(b.stream, src.rendered, 0);
                if (e == hipSuccess)
                    e = hipMemcpyPeerAsync(b.d_col + o, b.device, src.d_col + o, src.device, sizeof(float) * cnt,
                                           b.stream);
                if (e != hipSuccess) return rtrt::fail_hip(e, "spt_multi_gather_async peer copy");
            }
            hipError_t e = hipEventRecord(b.gathered, b.stream);
            if (e != hipSuccess) return rtrt::fail_hip(e, "spt_multi_gather_async record");
        }
    }
    // Every device repacks the rows it did not render (its own rows already
    // hold the render call's pack of the same colours).
    for (Band &b : m->bands) {
        if ((rc = scope.select(b.device))) return rc;
        int win[2][2];
        sptband::repack_windows(m->h, b.s0, b.s1, win);
        for (const auto &wn : win)
            if (wn[1] > wn[0] && (rc = spt_pack_pixels_async(b.d_col, b.d_px, m->w, m->h, wn[0], wn[1], b.stream)))
                return rc;
    }
    return RT_OK;
}

extern "C" int spt_multi_sync(spt_multi *m)
{
    if (!m) return rtrt::fail(RT_ERR_INVALID, "spt_multi_sync: null pointer");
    rtrt::DeviceScope scope;
    return sync_all(*m, scope);
}

extern "C" int spt_multi_download(spt_multi *m, float *colors, uint32_t *seeds, uint32_t *pixels)
{
    if (!m) return rtrt::fail(RT_ERR_INVALID, "spt_multi_download: null pointer");
    rtrt::DeviceScope scope;
    for (Band &b : m->bands) {
        int rc = scope.select(b.device);
        if (rc) return rc;
        const size_t o = px_off(*m, b.s0), n = px_off(*m, b.s1) - o;
        const size_t po = px_off(*m, m->h - b.s1);     // pixel rows [h-s1, h-s0)
        hipError_t e = hipSuccess;
        if (seeds)
            e = hipMemcpyAsync(seeds + 2 * o, b.d_seed + 2 * o, 2 * sizeof(uint32_t) * n, hipMemcpyDeviceToHost,
                               b.stream);
        if (e == hipSuccess && colors)
            e = hipMemcpyAsync(colors + 3 * o, b.d_col + 3 * o, 3 * sizeof(float) * n, hipMemcpyDeviceToHost,
                               b.stream);
        if (e == hipSuccess && pixels)
            e = hipMemcpyAsync(pixels + po, b.d_px + po, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, b.stream);
        if (e != hipSuccess) return rtrt::fail_hip(e, "spt_multi_download");
    }
    return sync_all(*m, scope);
}

extern "C" int spt_multi_read_frame(spt_multi *m, int k, float *colors, uint32_t *pixels)
{
    if (!m || k < 0 || k >= (int)m->bands.size()) return rtrt::fail(RT_ERR_INVALID, "spt_multi_read_frame: bad band");
    rtrt::DeviceScope scope;
    Band &b = m->bands[k];
    int rc = scope.select(b.device);
    if (rc) return rc;
    const size_t npx = px_off(*m, m->h);
    hipError_t e = hipSuccess;
    if (colors) e = hipMemcpyAsync(colors, b.d_col, 3 * sizeof(float) * npx, hipMemcpyDeviceToHost, b.stream);
    if (e == hipSuccess && pixels)
        e = hipMemcpyAsync(pixels, b.d_px, sizeof(uint32_t) * npx, hipMemcpyDeviceToHost, b.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(b.stream);
    return e == hipSuccess ? RT_OK : rtrt::fail_hip(e, "spt_multi_read_frame");
}

extern "C" int spt_multi_counters(spt_multi *m, uint64_t *out)
{
    if (!m || !out) return rtrt::fail(RT_ERR_INVALID, "spt_multi_counters: null pointer");
    rtrt::DeviceScope scope;
    for (int i = 0; i < 4; i++) out[i] = 0;
    for (Band &b : m->bands) {
        int rc = scope.select(b.device);
        if (rc) return rc;
        unsigned long long c[4];
        hipError_t e = hipMemcpyAsync(c, b.d_cnt, sizeof(c), hipMemcpyDeviceToHost, b.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(b.stream);
        if (e == hipSuccess) e = hipMemsetAsync(b.d_cnt, 0, sizeof(c), b.stream);
        if (e != hipSuccess) return rtrt::fail_hip(e, "spt_multi_counters");
        for (int i = 0; i < 4; i++) out[i] += c[i];
    }
    return sync_all(*m, scope);
}

extern "C" int spt_multi_band_buffers(const spt_multi *m, int k, int *device, float **d_colors, uint32_t **d_seeds,
                                      uint32_t **d_pixels, void **stream)
{
    if (!m || k < 0 || k >= (int)m->bands.size())
        return rtrt::fail(RT_ERR_INVALID, "spt_multi_band_buffers: bad band");
    const Band &b = m->bands[k];
    if (device) *device = b.device;
    if (d_colors) *d_colors = b.d_col;
    if (d_seeds) *d_seeds = b.d_seed;
    if (d_pixels) *d_pixels = b.d_px;
    if (stream) *stream = b.stream;
    return RT_OK;
}

namespace {
// spt_render_multi's band context, kept across calls as spt_render keeps its
// scene (smallptGPU.cpp:100-167,209-615 create the buffers once and reuse
// them every pass): the same devices and frame size reuse every band's
// buffers, stream and scene; a changed sphere array (compared byte for byte)
// re-prepares only the scenes; anything else builds a new context.
struct MultiCache {
    std::vector<int> devices;
    int w = 0, h = 0;
    std::vector<rt_sphere> host;
    std::string hooks;                 // the scenes' preparation hooks (spt_scene_create's getenv)
    spt_multi *m = nullptr;
    unsigned long long contexts = 0, preps = 0;
};
MultiCache g_multi_cache;
std::mutex g_multi_mu;

}  // namespace

namespace rtrt {
void release_cached_multi()
{
    std::lock_guard<std::mutex> lk(g_multi_mu);
    destroy_multi(g_multi_cache.m);
    g_multi_cache.m = nullptr;
    g_multi_cache.host.clear();
    g_multi_cache.devices.clear();
}
}  // namespace rtrt

extern "C" int spt_multi_cache_info(uint64_t *out)
{
    if (!out) return rtrt::fail(RT_ERR_INVALID, "spt_multi_cache_info: null pointer");
    std::lock_guard<std::mutex> lk(g_multi_mu);
    out[0] = g_multi_cache.contexts;
    out[1] = g_multi_cache.preps;
    return RT_OK;
}

extern "C" int spt_render_multi(const rt_sphere *spheres, unsigned nspheres, const rt_camera *camera,
                                float *colors, uint32_t *seeds, uint32_t *pixels, int w, int h, int first_sample,
                                int nsamples, int mode, uint64_t *counters, const int *devices, int ngpus)
{
    if (!spheres || !camera || !colors || !seeds || !pixels || w < 1 || h < 1 || nspheres < 1 ||
        first_sample < 0 || nsamples < 0 || ngpus < 1 || ngpus > 64)
        return rtrt::fail(RT_ERR_INVALID, "spt_render_multi: bad arguments");
    std::lock_guard<std::mutex> lk(g_multi_mu);
    MultiCache &c = g_multi_cache;
    std::vector<int> devs(ngpus);
    for (int k = 0; k < ngpus; k++) devs[k] = devices ? devices[k] : k;
    const std::string hooks = rtrt::scene_prep_hooks();
    int rc = RT_OK;
    if (!(c.m && c.devices == devs && c.w == w && c.h == h)) {
        destroy_multi(c.m);
        c.m = nullptr;
        c.host.clear();
        if ((rc = spt_multi_create(spheres, nspheres, w, h, devs.data(), ngpus, &c.m))) {
            c.m = nullptr;
            return rc;
        }
        c.devices = devs;
        c.w = w;
        c.h = h;
        c.host.assign(spheres, spheres + nspheres);
        c.hooks = hooks;
        c.contexts++;
        c.preps++;
    } else if (!(c.host.size() == nspheres && c.hooks == hooks &&
                 memcmp(c.host.data(), spheres, sizeof(rt_sphere) * nspheres) == 0)) {
        c.host.clear();
        if ((rc = spt_multi_set_scene(c.m, spheres, nspheres))) return rc;
        c.host.assign(spheres, spheres + nspheres);
        c.hooks = hooks;
        c.preps++;
    }
    spt_multi *m = c.m;
    if (counters) {                                    // start from zero (a failed call may have left counts)
        uint64_t z[4];
        if ((rc = spt_multi_counters(m, z))) return rc;
    }
    rc = spt_multi_upload(m, first_sample > 0 ? colors : nullptr, seeds);
    if (rc == RT_OK) rc = spt_multi_render_async(m, camera, first_sample, nsamples, mode, counters != nullptr);
    if (rc == RT_OK) rc = spt_multi_download(m, nsamples > 0 ? colors : nullptr, seeds, nsamples > 0 ? pixels : nullptr);
    if (rc == RT_OK && counters) rc = spt_multi_counters(m, counters);
    return rc;
}
