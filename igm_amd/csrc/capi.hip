// Context management of libigmhip.so (include/igm_hip.h).
#include "igm_ctx.h"

extern "C" {

const char* igm_version(void) { return "igm_amd 0.1 gfx950"; }

int igm_ctx_create(int device, igm_ctx** out) {
    if (!out) return IGM_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return IGM_E_HIP;
    if (device < 0 || device >= ndev) return IGM_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return IGM_E_HIP;
    igm_ctx* c = new igm_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return IGM_E_HIP;
    }
    c->stream = c->own_stream;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
        c->num_cus = prop.multiProcessorCount;
        c->lds_per_block = prop.sharedMemPerBlock;
    }
    *out = c;
    return IGM_OK;
}

void igm_ctx_destroy(igm_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto& kv : c->ws)
        if (kv.second.first) (void)hipFree(kv.second.first);
    for (auto& kv : c->kev) {
        if (kv.second.first) (void)hipEventDestroy(kv.second.first);
        if (kv.second.second) (void)hipEventDestroy(kv.second.second);
    }
    for (size_t g = 0; g < c->aux.size(); ++g) {
        (void)hipStreamSynchronize(c->aux[g]);
        (void)hipStreamDestroy(c->aux[g]);
        (void)hipEventDestroy(c->aux_ev[g]);
    }
    if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
    for (hipEvent_t ev : c->step_ev) (void)hipEventDestroy(ev);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

const char* igm_last_error(const igm_ctx* c) { return c ? c->err.c_str() : "null context"; }

int igm_ctx_set_stream(igm_ctx* c, void* s) {
    if (!c) return IGM_E_INVALID;
    c->stream = s ? static_cast<hipStream_t>(s) : c->own_stream;
    return IGM_OK;
}

int igm_ctx_synchronize(igm_ctx* c) {
    if (!c) return IGM_E_INVALID;
    IGM_HIP_CHECK(c, hipStreamSynchronize(c->stream));
    return IGM_OK;
}

double igm_last_kernel_ms(const igm_ctx* c, const char* name) {
    if (!c || !name) return -1.0;
    auto it = c->kev.find(name);
    if (it == c->kev.end()) return -1.0;
    if (hipEventSynchronize(it->second.second) != hipSuccess) return -1.0;
    float ms = -1.f;
    if (hipEventElapsedTime(&ms, it->second.first, it->second.second) != hipSuccess) return -1.0;
    return ms;
}

}  // extern "C"
