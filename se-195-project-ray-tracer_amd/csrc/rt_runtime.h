// rt_runtime.h -- host-side runtime of the C-ABI: per-thread error text,
// per-device state (stream, cached device buffers of the blocking entry
// points), HIP error mapping.  Defined in rt_api.hip.
#ifndef RT_RUNTIME_H
#define RT_RUNTIME_H

#include <hip/hip_runtime.h>
#include <mutex>
#include <stddef.h>
#include <string>
#include "../../include/rt_hip.h"

namespace rtrt {

constexpr int NSCRATCH = 11;
constexpr int SLOT_VIEW = 7;

struct DeviceState {
    int device = -1;
    int cus = 0;                       // compute units (launch shaping)
    hipStream_t stream = nullptr;      // stream of the blocking entry points
    void *buf[NSCRATCH] = {};          // grow-only device buffers
    size_t cap[NSCRATCH] = {};
    size_t cached_bytes = 0;
    // Held by an entry point while it uses this state's buffers / stream
    // (recursive: the blocking entry points call the asynchronous ones).
    std::recursive_mutex mu;
    // Whitted view tables (m_SX / m_SY, or openCLcode.cl's) for frame size
    // (vt_w, vt_h) and semantics vt_ocl in scratch slot SLOT_VIEW, and the
    // level-pass arena: both are reused by every frame on this device, on
    // whatever stream it is issued.  wf_done is recorded after each frame's
    // kernels; the next frame's stream waits on it (frames on different
    // streams are serialised, never interleaved), and a buffer is regrown
    // only after it has completed (whitted.hip).
    int vt_w = 0, vt_h = 0, vt_ocl = -1;
    hipEvent_t wf_done = nullptr;
    bool wf_pending = false;
    // Record pools of the level passes (POOL_WHITTED, POOL_QUEUE) as a
    // fraction of a slab's trees, learnt per (pass, slab size).  A frame whose
    // nodes did not all fit (the trees left over are re-evaluated exactly by
    // the fixup kernels, one lane per tree: correct but slow) raises its
    // entry's flag in host-mapped memory (pool_ovf, written by the fixup
    // kernel); the next frame of that size then sizes its pool 1.25x larger
    // (pool_fraction).
    struct PoolFit { int which = -1; long long trees = 0; double frac = 0.0; };
    PoolFit pool_fit[16];
    int pool_fit_next = 0;
    int *pool_ovf = nullptr;           // host-mapped [16]
    int *pool_ovf_dev = nullptr;       // its device address
    // A second stream for the level pass's concurrent slabs (aux_stream):
    // forked from and joined back to the caller's stream by events.
    hipStream_t aux = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
};

constexpr int POOL_WHITTED = 0, POOL_QUEUE = 1, POOL_FITS = 16;
constexpr double POOL_FRAC_MAX = 8.0;

// Records msg (plus the HIP error string) for rt_last_error(); returns code.
int fail(int code, const char *msg);
int fail_hip(hipError_t e, const char *what);
// hipGetLastError() after a launch, mapped to RT_ERR_HIP.
int check_launch(const char *what);
// State of the calling thread's current device (created on first use).
int state(DeviceState **out);
// Device buffer slot `slot` of at least `bytes` (grow-only, reused).
int scratch(DeviceState &st, int slot, size_t bytes, void **out);
// Pool fraction of level pass `which` for the next frame of `trees` trees
// per slab (starts at `initial`; grown after an overflowed frame of that
// size) and, in *flag_dev, the device address of that entry's overflow flag.
double pool_fraction(DeviceState &st, int which, long long trees, double initial, int **flag_dev);
// The state's second stream and its fork / join events (created on first use).
int aux_stream(DeviceState &st);
// An error after a frame forked work onto aux: joins aux back into s (and
// records wf_done, so the next frame and any buffer regrowth wait for it);
// returns rc.
int join_aux_on_error(DeviceState &st, hipStream_t s, int rc);
// Frees the per-device scenes cached by spt_render / spt_render_async
// (smallpt.hip; rt_release).
void release_cached_scenes();
// Frees spt_render_multi's cached band context (spt_multi.hip; rt_release).
void release_cached_multi();
// The environment test hooks spt_scene_create reads (RT_SPT_NO_BVH,
// RT_SPT_GEO, RT_SPT_WIDE) as one key: the scene caches
// of spt_render and spt_render_multi rebuild when it changes (smallpt.hip).
std::string scene_prep_hooks();
// The calling thread's rt_set_device choice (-1: none, HIP's current device).
int thread_device();
// Saves the calling thread's device selection (rt_set_device and HIP's
// current device) and restores both on scope exit: the multi-device entry
// points drive several devices from one host thread.
struct DeviceScope {
    int saved_rt, saved_hip = 0;
    DeviceScope();
    ~DeviceScope();
    int select(int device);   // rt_set_device for the scope's duration
};

}  // namespace rtrt

#endif
