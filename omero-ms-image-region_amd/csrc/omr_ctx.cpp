// omr_ctx.cpp — per-worker-thread context: device, stream, workspace, pinned staging.
// One context per Vert.x worker thread replaces the per-request Renderer construction
// (ImageRegionRequestHandler.java:436-440) as the unit of state; the reference's only
// parallelism (worker-verticle instances, ImageRegionMicroserviceVerticle.java:149-165)
// maps to one context per thread, or one per GPU for batched launches.
#include "omr_internal.h"

#include <cstdio>
#include <cstdlib>

namespace omr {

omr_status fail(Ctx* c, omr_status s, const std::string& msg) {
    if (c) c->last_error = msg;
    return s;
}

omr_status hip_fail(Ctx* c, hipError_t e, const char* what) {
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    return fail(c, e == hipErrorOutOfMemory ? OMR_OOM : OMR_DEVICE, m);
}

int bytes_per_pixel(int32_t t) {
    switch (t) {
    case OMR_PIXELS_INT8: case OMR_PIXELS_UINT8: return 1;
    case OMR_PIXELS_INT16: case OMR_PIXELS_UINT16: return 2;
    case OMR_PIXELS_INT32: case OMR_PIXELS_UINT32: case OMR_PIXELS_FLOAT: return 4;
    case OMR_PIXELS_DOUBLE: return 8;
    default: return 0;
    }
}

omr_status ensure_workspace(Ctx* c, size_t bytes) {
    if (bytes <= c->ws_cap) return OMR_OK;
    size_t cap = align_up(bytes + bytes / 4, 1 << 20);
    if (c->ws) {
        OMR_HIP(c, hipStreamSynchronize(c->stream));
        OMR_HIP(c, hipFree(c->ws));
        c->ws = nullptr;
        c->ws_cap = 0;
    }
    OMR_HIP(c, hipMalloc(&c->ws, cap));
    c->ws_cap = cap;
    return OMR_OK;
}

omr_status ensure_host_out(Ctx* c, size_t bytes) {
    if (bytes <= c->h_out_cap) return OMR_OK;
    if (c->h_out) {
        OMR_HIP(c, hipStreamSynchronize(c->stream));
        OMR_HIP(c, hipHostFree(c->h_out));
        c->h_out = nullptr;
        c->h_out_cap = 0;
    }
    OMR_HIP(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_out), bytes, hipHostMallocCoherent | hipHostMallocMapped));
    c->h_out_cap = bytes;
    return OMR_OK;
}

omr_status ensure_aux(Ctx* c, size_t bytes) {
    if (bytes <= c->aux_cap) return OMR_OK;
    if (c->aux) {
        OMR_HIP(c, hipStreamSynchronize(c->stream));
        OMR_HIP(c, hipFree(c->aux));
        c->aux = nullptr;
        c->aux_cap = 0;
    }
    OMR_HIP(c, hipMalloc(&c->aux, bytes));
    c->aux_cap = bytes;
    return OMR_OK;
}

omr_status stage_h2d2(Ctx* c, void* dst1, const void* src1, size_t n1, void* dst2, const void* src2, size_t n2) {
    const size_t off2 = align_up(n1, 16), bytes = off2 + n2;
    if (bytes == 0) return OMR_OK;
    if (bytes > c->pin_cap) {
        for (int i = 0; i < Ctx::kPinSlots; ++i) {
            if (c->pin[i]) {
                OMR_HIP(c, hipEventSynchronize(c->pin_ev[i]));
                OMR_HIP(c, hipHostFree(c->pin[i]));
                c->pin[i] = nullptr;
            }
        }
        size_t cap = align_up(bytes, 1 << 16);
        for (int i = 0; i < Ctx::kPinSlots; ++i)   // fine-grained: the copy kernel must never see a stale GPU-cached line
            OMR_HIP(c, hipHostMalloc(&c->pin[i], cap, hipHostMallocCoherent | hipHostMallocMapped));
        c->pin_cap = cap;
    }
    const int s = c->pin_slot;
    c->pin_slot = (s + 1) % Ctx::kPinSlots;
    OMR_HIP(c, hipEventSynchronize(c->pin_ev[s]));  // previous copy out of this slot is done
    uint8_t* slot = static_cast<uint8_t*>(c->pin[s]);
    if (n1) std::memcpy(slot, src1, n1);
    if (n2) std::memcpy(slot + off2, src2, n2);
    // A small kernel reads the parameter blocks straight from the pinned slot (device-mapped host
    // memory): unlike hipMemcpyAsync, which hands the copy to a DMA engine and makes the next
    // kernel wait on a cross-engine signal, it orders with the request's kernels like any launch.
    // Two blocks (e.g. plan + plane-pointer table) share one launch.
    OMR_HIP(c, launch_h2d_small(c->stream, dst1, slot, n1, dst2, slot + off2, n2));
    OMR_HIP(c, hipEventRecord(c->pin_ev[s], c->stream));
    return OMR_OK;
}

omr_status stage_h2d(Ctx* c, void* dst, const void* src, size_t bytes) {
    return stage_h2d2(c, dst, src, bytes, nullptr, nullptr, 0);
}

static hipEvent_t pooled_event(Ctx* c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    // Timing events skip the system-scope release fence (a write-back of L2 to memory visible to
    // the host) that a default event performs when it completes: the fence sits between a timed
    // kernel's end and the stop timestamp and inflated ~18 us kernels by ~4 us against rocprofv3's
    // kernel trace.  OMR_TIMING_FENCE=1 restores default events for comparison.
    static const bool fence = [] {
        const char* e = std::getenv("OMR_TIMING_FENCE");
        return e && *e && *e != '0';
    }();
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, fence ? hipEventDefault : hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return e;
}

thread_local KernelTimer* tl_ext_timer = nullptr;

KernelTimer::KernelTimer(Ctx* ctx, int k, bool ext_launch) : c(ctx), kind(k) {
    if (!c->timing) return;
    start = pooled_event(c);
    stop = pooled_event(c);
    if (!start || !stop) { stop = nullptr; return; }
    (void)hipEventRecord(start, c->stream);     // re-stamped by an ext launch
    c->timed.push_back({start, stop, kind});
    if (ext_launch) {
        ext = true;
        prev = tl_ext_timer;
        tl_ext_timer = this;
    }
}

KernelTimer::~KernelTimer() {
    if (ext) tl_ext_timer = prev;
    if (stop && !used) (void)hipEventRecord(stop, c->stream);
}

}  // namespace omr

using namespace omr;

extern "C" {

int32_t omr_abi_version(void) { return OMR_ABI_VERSION; }

omr_status omr_ctx_create(int32_t device_ordinal, omr_ctx** out) {
    if (!out) return OMR_INVALID_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return OMR_DEVICE;
    if (device_ordinal < 0 || device_ordinal >= n) return OMR_INVALID_ARGUMENT;
    omr_ctx* c = new omr_ctx();
    c->device = device_ordinal;
    hipError_t e = hipSetDevice(device_ordinal);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&c->d_flag, 256);
    if (e == hipSuccess) e = hipMemset(c->d_flag, 0, 256);
    if (e == hipSuccess)
        e = hipHostMalloc(reinterpret_cast<void**>(&c->h_flag), 64, hipHostMallocCoherent | hipHostMallocMapped);
    for (int i = 0; i < Ctx::kPinSlots && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->pin_ev[i], hipEventDisableTiming);
    if (e == hipSuccess) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device_ordinal) == hipSuccess) c->cu_count = prop.multiProcessorCount;
    }
    if (e != hipSuccess) {
        omr_ctx_destroy(c);
        return e == hipErrorOutOfMemory ? OMR_OOM : OMR_DEVICE;
    }
    c->stream = c->own_stream;
    if (const char* v = std::getenv("OMR_K2_NT_STORE")) c->k2_nt_store = std::atoi(v) != 0;
    if (const char* v = std::getenv("OMR_K3R")) c->k3r = std::atoi(v) != 0;
    if (const char* v = std::getenv("OMR_PNG_DEVICE_D3")) c->png_device_d3 = std::atoi(v) != 0;
    if (const char* v = std::getenv("OMR_PNG_SINGLE_BATCHED")) c->png_single_batched = std::atoi(v) != 0;
    if (const char* v = std::getenv("OMR_F1_F32")) c->f1_f32 = std::atoi(v) != 0;
    // B4a / B6 grids for 0.4 B per pixel (C2 q 0.9 streams are 0.37; longer ones loop): same-box A/B
    // 210.2k (1.0 B/px, the round-3 sizing) -> 213.5k C2 tiles/s fused (profiles/r04/ab_jpeg_est_groups.txt)
    c->jpeg_est_centibpp = 40;
    if (const char* v = std::getenv("OMR_JPEG_EST_CENTIBPP")) c->jpeg_est_centibpp = std::max(5, std::atoi(v));
    if (const char* v = std::getenv("OMR_K2_EVAL_CPT")) {   // 2 / 4 plain grid stride, -1 / -2 pipelined
        const int k = std::atoi(v);
        c->k2_eval_cpt = (k == 4 || k == 2 || k == -1 || k == -3) ? k : -2;
    }
    *out = c;
    return OMR_OK;
}

omr_status omr_ctx_enable_kernel_timing(omr_ctx* c, int32_t enable) {
    if (!c) return OMR_INVALID_ARGUMENT;
    c->timing = enable != 0;
    return OMR_OK;
}

int32_t omr_ctx_kernel_timings(omr_ctx* c, float* ms_out, int32_t* kind_out, int32_t cap) {
    if (!c) return -1;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return -1;
    int32_t n = 0;
    for (auto& t : c->timed) {
        float ms = 0.f;
        (void)hipEventSynchronize(t.stop);
        if (hipEventElapsedTime(&ms, t.start, t.stop) != hipSuccess) ms = -1.f;
        if (n < cap && ms_out) {
            ms_out[n] = ms;
            if (kind_out) kind_out[n] = t.kind;
        }
        ++n;
        c->event_pool.push_back(t.start);
        c->event_pool.push_back(t.stop);
    }
    c->timed.clear();
    return n < cap ? n : cap;
}

void omr_ctx_destroy(omr_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->pixbuf_state && c->pixbuf_state_free) c->pixbuf_state_free(c->pixbuf_state);
    for (auto& t : c->timed) { c->event_pool.push_back(t.start); c->event_pool.push_back(t.stop); }
    for (auto e : c->event_pool) (void)hipEventDestroy(e);
    for (int i = 0; i < Ctx::kPinSlots; ++i) {
        if (c->pin_ev[i]) (void)hipEventDestroy(c->pin_ev[i]);
        if (c->pin[i]) (void)hipHostFree(c->pin[i]);
    }
    if (c->ws) (void)hipFree(c->ws);
    if (c->aux) (void)hipFree(c->aux);
    if (c->d_crc_pow) (void)hipFree(c->d_crc_pow);
    for (auto& l : c->dev_luts) (void)hipFree(l.d);
    if (c->d_flag) (void)hipFree(c->d_flag);
    if (c->h_flag) (void)hipHostFree(c->h_flag);
    if (c->h_out) (void)hipHostFree(c->h_out);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

const char* omr_last_error(const omr_ctx* c) { return c ? c->last_error.c_str() : "null context"; }

omr_status omr_ctx_synchronize(omr_ctx* c) {
    if (!c) return OMR_INVALID_ARGUMENT;
    // the status word rides behind the queued work (and is cleared there): one sync, no
    // separate D2H copy and second wait
    OMR_HIP(c, launch_flag_out(c->stream, c->d_flag, c->h_flag));
    OMR_HIP(c, hipStreamSynchronize(c->stream));
    const int32_t flag = *static_cast<volatile int32_t*>(c->h_flag);
    if (flag) return fail(c, OMR_QUANTIZATION, "pixel value outside the quantization LUT domain");
    return OMR_OK;
}

omr_status omr_ctx_set_stream(omr_ctx* c, void* s) {
    if (!c) return OMR_INVALID_ARGUMENT;
    c->stream = s ? static_cast<hipStream_t>(s) : c->own_stream;
    return OMR_OK;
}

omr_status omr_ctx_set_semantics(omr_ctx* c, uint32_t flags) {
    if (!c) return OMR_INVALID_ARGUMENT;
    if (flags & ~(uint32_t)OMR_SEM_ALL) return fail(c, OMR_INVALID_ARGUMENT, "unknown semantics flag");
    c->sem = flags;
    return OMR_OK;
}

uint32_t omr_ctx_get_semantics(const omr_ctx* c) { return c ? c->sem : 0u; }

void* omr_ctx_get_stream(omr_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

void* omr_pinned_alloc(omr_ctx* c, size_t bytes) {
    void* p = nullptr;
    if (!c || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void omr_pinned_free(omr_ctx* c, void* p) {
    if (p) (void)hipHostFree(p);
}

}  // extern "C"
