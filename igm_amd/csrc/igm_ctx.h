// Internal context / workspace / error plumbing shared by the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/igm_hip.h"

struct igm_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    // named device workspaces, grown on demand (never shrunk until destroy)
    std::map<std::string, std::pair<void*, size_t>> ws;
    // per kernel family: (start, stop) events of its last launch on `stream`
    std::map<std::string, std::pair<hipEvent_t, hipEvent_t>> kev;
    // volumetric maps staged by igm_mstep_set_volumes (device copies live in ws slots
    // "vol_maps", "vol_vox", "vol_smap")
    int vol_nmap = 0, vol_nsmap = 0;
    int num_cus = 256;
    // last HBM-size anneal: {K, slots, builds, re-cuts, largest resident set, largest
    // owned set, abort (0: the domain-decomposed engine ran; -1 / > 0: the population
    // engine ran, by choice / after an abort)}
    size_t lds_per_block = 65536;
    // auxiliary streams (+ one event each) for independent work inside one call,
    // created on first use: the population engine runs its structure groups on them
    std::vector<hipStream_t> aux;
    std::vector<hipEvent_t> aux_ev;
    hipEvent_t fork_ev = nullptr;
    // events ordering work between the auxiliary streams inside one call (pop_event)
    std::vector<hipEvent_t> step_ev;
};

namespace igm {

inline int fail(igm_ctx* c, int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

#define IGM_HIP_CHECK(ctx, expr)                                                           \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return ::igm::fail((ctx), IGM_E_HIP, "%s:%d %s -> %s", __FILE__, __LINE__,    \
                               #expr, hipGetErrorString(_e));                              \
    } while (0)

#define IGM_TRY(expr)               \
    do {                            \
        int _r = (expr);            \
        if (_r != IGM_OK) return _r; \
    } while (0)

// Device workspace slot `name` of at least `bytes` (contents undefined).
inline int workspace(igm_ctx* c, const char* name, size_t bytes, void** out) {
    auto& slot = c->ws[name];
    if (slot.second < bytes) {
        if (slot.first) {
            (void)hipStreamSynchronize(c->stream);
            (void)hipFree(slot.first);
            slot.first = nullptr;
            slot.second = 0;
        }
        size_t sz = bytes < 256 ? 256 : bytes;
        if (hipMalloc(&slot.first, sz) != hipSuccess) {
            (void)hipGetLastError();
            return fail(c, IGM_E_NOMEM, "hipMalloc(%zu) failed for workspace '%s'", sz, name);
        }
        slot.second = sz;
    }
    *out = slot.first;
    return IGM_OK;
}

// Get a device view of a caller array: either the pointer itself (device mode)
// or a staged copy in workspace `name`.
template <typename T>
inline int to_device(igm_ctx* c, uint32_t flags, const char* name, const T* p, size_t n, const T** out) {
    if (flags & IGM_DEVICE_PTRS || p == nullptr || n == 0) {
        *out = p;
        return IGM_OK;
    }
    void* d;
    IGM_TRY(workspace(c, name, n * sizeof(T), &d));
    IGM_HIP_CHECK(c, hipMemcpyAsync(d, p, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
    *out = static_cast<const T*>(d);
    return IGM_OK;
}

template <typename T>
inline int out_device(igm_ctx* c, uint32_t flags, const char* name, T* p, size_t n, T** out) {
    if (flags & IGM_DEVICE_PTRS || p == nullptr || n == 0) {
        *out = p;
        return IGM_OK;
    }
    void* d;
    IGM_TRY(workspace(c, name, n * sizeof(T), &d));
    *out = static_cast<T*>(d);
    return IGM_OK;
}

template <typename T>
inline int to_host(igm_ctx* c, uint32_t flags, T* host, const T* dev, size_t n) {
    if (flags & IGM_DEVICE_PTRS || host == nullptr || n == 0 || host == dev) return IGM_OK;
    IGM_HIP_CHECK(c, hipMemcpyAsync(host, dev, n * sizeof(T), hipMemcpyDeviceToHost, c->stream));
    return IGM_OK;
}

inline int finish(igm_ctx* c, uint32_t flags) {
    if (!(flags & IGM_ASYNC) || !(flags & IGM_DEVICE_PTRS)) IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    IGM_HIP_CHECK(c, hipGetLastError());
    return IGM_OK;
}

// Event-bracketed region on the context stream (elapsed time is read lazily by
// igm_last_kernel_ms, so timing never adds a host synchronisation).
struct Timed {
    igm_ctx* c;
    std::pair<hipEvent_t, hipEvent_t>* ev;
    Timed(igm_ctx* c_, const char* name) : c(c_) {
        auto& e = c->kev[name];
        if (!e.first) {
            (void)hipEventCreate(&e.first);
            (void)hipEventCreate(&e.second);
        }
        ev = &e;
        (void)hipEventRecord(e.first, c->stream);
    }
    ~Timed() { (void)hipEventRecord(ev->second, c->stream); }
};

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// at least n auxiliary streams; the work on them is forked from and joined into c->stream
inline int aux_streams(igm_ctx* c, int n) {
    if (!c->fork_ev) IGM_HIP_CHECK(c, hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming));
    while ((int)c->aux.size() < n) {
        hipStream_t st;
        hipEvent_t ev;
        IGM_HIP_CHECK(c, hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        IGM_HIP_CHECK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        c->aux.push_back(st);
        c->aux_ev.push_back(ev);
    }
    return IGM_OK;
}

// event k of the context's cross-stream events (created on first use, timing disabled)
inline int pop_event(igm_ctx* c, int k, hipEvent_t* out) {
    while ((int)c->step_ev.size() <= k) {
        hipEvent_t ev;
        IGM_HIP_CHECK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        c->step_ev.push_back(ev);
    }
    *out = c->step_ev[k];
    return IGM_OK;
}

// the first n auxiliary streams wait for the work queued so far on c->stream
inline int aux_fork(igm_ctx* c, int n) {
    IGM_HIP_CHECK(c, hipEventRecord(c->fork_ev, c->stream));
    for (int g = 0; g < n; ++g) IGM_HIP_CHECK(c, hipStreamWaitEvent(c->aux[g], c->fork_ev, 0));
    return IGM_OK;
}

// c->stream waits for the work queued on the first n auxiliary streams
inline int aux_join(igm_ctx* c, int n) {
    for (int g = 0; g < n; ++g) {
        IGM_HIP_CHECK(c, hipEventRecord(c->aux_ev[g], c->aux[g]));
        IGM_HIP_CHECK(c, hipStreamWaitEvent(c->stream, c->aux_ev[g], 0));
    }
    return IGM_OK;
}

}  // namespace igm
