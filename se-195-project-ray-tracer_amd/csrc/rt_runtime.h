// rt_runtime.h -- host-side runtime of the C-ABI: per-thread error text,
// per-device state (stream, cached device buffers of the blocking entry
// points), HIP error mapping.  Defined in rt_api.hip.
#ifndef RT_RUNTIME_H
#define RT_RUNTIME_H

#include <hip/hip_runtime.h>
#include <mutex>
#include <stddef.h>
#include "../../include/rt_hip.h"

namespace rtrt {

constexpr int NSCRATCH = 9;
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
};

// Records msg (plus the HIP error string) for rt_last_error(); returns code.
int fail(int code, const char *msg);
int fail_hip(hipError_t e, const char *what);
// hipGetLastError() after a launch, mapped to RT_ERR_HIP.
int check_launch(const char *what);
// State of the calling thread's current device (created on first use).
int state(DeviceState **out);
// Device buffer slot `slot` of at least `bytes` (grow-only, reused).
int scratch(DeviceState &st, int slot, size_t bytes, void **out);
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
