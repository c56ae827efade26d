// omr_batcher.cpp — coalescing concurrent tile requests into GPU batches.
//
// The reference serves every render_image_region request on its own Vert.x worker thread
// (ImageRegionMicroserviceVerticle.java:149-165 deploys the worker verticles; each request
// builds its own Renderer, ImageRegionRequestHandler.java:436-440) and caches finished regions
// in Redis under ImageRegionCtx.cacheKey (ImageRegionCtx.java:165-177).  Here worker threads
// submit tile jobs to a batcher that owns one GPU context: a dispatcher thread takes whatever is
// pending (up to max_batch jobs, or whatever arrived within max_wait_us of the oldest job),
// groups jobs with the same image and rendering settings, renders each group with one pipelined
// pixel-buffer call (omr_render_pixel_buffer_tiles, device output) and one batched JPEG encode,
// and hands every job its own file.  Identical requests in flight together (the same cache key)
// are rendered once.
//
// Dispatch lanes (round 6): a batcher runs `lanes` dispatcher threads (default 2, env
// OMR_BATCH_LANES), each with its own context (stream, pixel-buffer staging, device buffers).  A
// round is synchronous on its lane -- tile upload, render, encode, readback -- so with one lane the
// PCIe link idled while a round rendered, encoded and read back, and clients with one request in
// flight split into two alternating halves that waited for each other.  With two lanes the next
// round's upload runs beside the current round's render and encode.  Only lane 0 takes projection
// jobs (it owns the HBM stack cache).  When no lane is busy the device is idle and a gather closes
// after a short grace (kIdleGapUs) instead of the full arrival pause.
#include "omr_internal.h"

#include <atomic>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>

namespace omr {

enum JobKind : int { kJobTile = 0, kJobProjection = 1, kJobMask = 2 };

// Device bytes one projection sub-batch may take for its full planes (ARGB + encoder output).
static constexpr size_t kProjectionBatchBytes = (size_t)2 << 30;

struct Job {
    uint64_t ticket = 0;
    int kind = kJobTile;
    const omr_pixel_buffer* pb = nullptr;
    omr_quantum_def qdef{};
    std::vector<omr_channel_binding> ch;
    std::vector<std::vector<uint8_t>> luts;     // owned copies of the .lut tables
    omr_tile_job spec{};
    omr_mask_job mask{};                         // kJobMask: bits point into mask_bits
    std::vector<uint8_t> mask_bits;
    uint32_t sem = 0;                            // OMR_SEM_* of the batcher when the job was submitted
    std::string group_key;                       // kind + image + settings + semantics + size + flip + format
    std::chrono::steady_clock::time_point t_submit;
};

struct Result {
    omr_status st = OMR_OK;
    std::string err;
    std::vector<uint8_t> bytes;
};

}  // namespace omr

namespace omr {
// One dispatcher thread with its own context and device buffers.
struct Lane {
    int index = 0;
    omr_ctx* ctx = nullptr;
    std::thread th;
    int last_round = 0;                      // jobs this lane's previous round took
    std::chrono::steady_clock::time_point t_round_end{};
    bool busy = false;                       // a round is in progress (under omr_batcher::m)
    // device buffers of the lane (grown on demand)
    uint32_t* d_argb = nullptr;
    size_t argb_cap = 0;
    uint8_t* d_jpeg = nullptr;                   // encoded files of a group (JPEG / PNG batch output)
    size_t jpeg_cap = 0;
    uint8_t* d_stack = nullptr;                  // projection jobs: scratch for stacks the cache cannot hold
    size_t stack_cap = 0;
    uint64_t* d_offs = nullptr;
    uint32_t* d_lens = nullptr;
    int32_t* d_stat = nullptr;
    int32_t* d_rstat = nullptr;    // per-tile render status (QuantizationException per tile)
    int meta_cap = 0;
};
constexpr int kIdleGapUs = 30;   // gather grace when no lane is busy (simultaneous submits still meet)
}  // namespace omr

struct omr_batcher {
    int device = 0;
    int max_batch = 64;
    int max_wait_us = 500;
    int gap_us = 200;                        // arrival pause that closes a gather (<= max_wait_us)
    // the same for lanes > 0 (env OMR_BATCH_LANE_GAP_US): an overlap lane gathers what arrived while
    // the lane below was busy, so a short pause closes it (30 us: the interactive serving leg's
    // best of 30 / 200 us, tools/serving_ab.py)
    int lane_gap_us = 30;
    std::chrono::steady_clock::time_point t_last_submit{};
    omr_ctx* ctx = nullptr;                  // lane 0's context (set_semantics and errors of the batcher)
    std::vector<std::unique_ptr<omr::Lane>> lanes;
    int busy_lanes = 0;                      // under m
    std::mutex m;
    std::condition_variable cv_in, cv_out;
    std::vector<std::unique_ptr<omr::Job>> pending;
    std::unordered_map<uint64_t, omr::Result> done;
    // cross-lane dedup: the cache key of every job a lane is rendering -> the tickets of identical
    // jobs another lane took meanwhile (answered with the same bytes when the render completes)
    std::unordered_map<std::string, std::vector<uint64_t>> inflight;
    uint64_t next_ticket = 1;
    bool stop = false;
    uint64_t n_jobs = 0, n_batches = 0, n_rendered = 0, n_dedup = 0;
    uint32_t sem = 0;                        // OMR_SEM_* copied into every job at submit (under m)
    std::atomic<int64_t> outstanding{0};     // jobs submitted and not yet completed (pool dispatch)
    // HBM stack cache (lane 0 only) (projection jobs): (pixel buffer, c, t) Z-stacks kept resident, LRU, up to
    // stack_cache_max bytes, so repeated p= requests on one image (other settings, ranges, flips)
    // skip the PCIe upload the reference repeats per request (ImageRegionRequestHandler.java:516-533)
    struct StackEntry { uint64_t serial; int32_t c, t; size_t bytes; uint8_t* d; uint64_t used; };
    std::vector<StackEntry> stacks;
    std::atomic<int64_t> stack_cache_max{(int64_t)4 << 30};
    std::atomic<uint64_t> stack_hits{0}, stack_misses{0}, stack_resident{0};
    uint64_t stack_tick = 0;
};

namespace omr {

static void append(std::string& k, const void* p, size_t n) { k.append(static_cast<const char*>(p), n); }

static std::string settings_key(const Job& j) {
    std::string k;
    if (j.kind == kJobMask) {                    // every mask of a round shares one batch call
        append(k, &j.kind, sizeof(j.kind));
        append(k, &j.sem, sizeof(j.sem));
        return k;
    }
    append(k, &j.pb, sizeof(j.pb));
    append(k, &j.qdef, sizeof(j.qdef));
    for (size_t c = 0; c < j.ch.size(); ++c) {
        const omr_channel_binding& b = j.ch[c];
        append(k, &b.active, sizeof(b.active));
        append(k, &b.family, sizeof(b.family));
        append(k, &b.coefficient, sizeof(b.coefficient));
        append(k, &b.noise_reduction, sizeof(b.noise_reduction));
        append(k, &b.reverse, sizeof(b.reverse));
        append(k, &b.input_start, sizeof(b.input_start));
        append(k, &b.input_end, sizeof(b.input_end));
        append(k, &b.global_min, sizeof(b.global_min));
        append(k, &b.global_max, sizeof(b.global_max));
        append(k, b.rgba, 4);
        const uint8_t has = b.lut ? 1 : 0;
        append(k, &has, 1);
        if (b.lut) append(k, b.lut, 768);
    }
    const omr_tile_job& s = j.spec;
    const int32_t geo[5] = {s.width, s.height, s.flip_h, s.flip_v, s.format};
    append(k, &j.kind, sizeof(j.kind));
    if (j.kind == kJobProjection) {             // the full plane: only the projection matters
        const int32_t pr[5] = {s.flip_h, s.flip_v, s.format, s.projection, s.projection_start};
        append(k, pr, sizeof(pr));
        append(k, &s.projection_end, sizeof(s.projection_end));
    } else {
        append(k, geo, sizeof(geo));
    }
    append(k, &j.sem, sizeof(j.sem));
    append(k, &s.quality, sizeof(s.quality));
    return k;
}

// Every pointer is cleared (and its capacity zeroed) as soon as it is freed, so a failed
// hipMalloc leaves nothing for omr_batcher_destroy to free twice.
template <typename T>
static omr_status regrow(omr_ctx* c, T*& p, size_t bytes) {
    if (p) {
        const hipError_t e = hipFree(p);
        p = nullptr;
        OMR_HIP(c, e);
    }
    OMR_HIP(c, hipMalloc(reinterpret_cast<void**>(&p), bytes));
    return OMR_OK;
}

static omr_status grow_dev(Lane* B, size_t argb, size_t jpeg, int n) {
    omr_ctx* c = B->ctx;
    omr_status st;
    if (argb > B->argb_cap) {
        B->argb_cap = 0;
        if ((st = regrow(c, B->d_argb, argb))) return st;
        B->argb_cap = argb;
    }
    if (jpeg > B->jpeg_cap) {
        B->jpeg_cap = 0;
        if ((st = regrow(c, B->d_jpeg, jpeg))) return st;
        B->jpeg_cap = jpeg;
    }
    if (n > B->meta_cap) {
        B->meta_cap = 0;
        if ((st = regrow(c, B->d_rstat, sizeof(int32_t) * n))) return st;
        if ((st = regrow(c, B->d_offs, sizeof(uint64_t) * n))) return st;
        if ((st = regrow(c, B->d_lens, sizeof(uint32_t) * n))) return st;
        if ((st = regrow(c, B->d_stat, sizeof(int32_t) * n))) return st;
        B->meta_cap = n;
    }
    return OMR_OK;
}
// Encode n device ARGB images of W x H (B->d_argb, tile i at i*W*H) in `format` into out[i] (skipping
// entries that already carry an error): JPEG and PNG in one batched launch each (sides up to
// 4096; larger planes, e.g. a projected full plane, one at a time), TIFF by the host writer, ARGB
// as the packed int[] itself.
// d_rstat (optional): the render's per-tile status on the device, read back with the encoder's
// lengths (one stream sync per round) and applied to out first.
static omr_status encode_group(Lane* B, int n, int W, int H, int format, float quality,
                               std::vector<Result>& out, const int32_t* d_rstat = nullptr) {
    omr_ctx* c = B->ctx;
    const size_t px = (size_t)W * H;
    const bool batched = W <= 4096 && H <= 4096;
    std::vector<int32_t> rstat(d_rstat ? n : 0);
    auto apply_rstat = [&]() {
        for (int i = 0; i < (int)rstat.size(); ++i)
            if (rstat[i] && !out[i].st) {
                out[i].st = rstat[i];
                out[i].err = "pixel value outside the quantization LUT domain";
            }
    };
    if ((format == OMR_FORMAT_JPEG || format == OMR_FORMAT_PNG) && batched) {
        const size_t cap = format == OMR_FORMAT_JPEG ? (size_t)n * (px * 4 + 65536)
                                                     : omr_png_batch_max_bytes(W, H, 3, n);
        omr_status st = grow_dev(B, 0, cap, n);
        if (st) return st;
        st = format == OMR_FORMAT_JPEG
                 ? omr_encode_jpeg_batch_device(c, B->d_argb, 0, n, W, H, quality, B->d_jpeg, cap, B->d_offs,
                                                B->d_lens, B->d_stat)
                 : omr_encode_png_batch_device(c, B->d_argb, 0, n, W, H, B->d_jpeg, cap, B->d_offs, B->d_lens,
                                               B->d_stat);
        if (st) return st;
        std::vector<uint64_t> offs(n);
        std::vector<uint32_t> lens(n);
        OMR_HIP(c, hipMemcpyAsync(offs.data(), B->d_offs, 8 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
        OMR_HIP(c, hipMemcpyAsync(lens.data(), B->d_lens, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
        if (d_rstat) OMR_HIP(c, hipMemcpyAsync(rstat.data(), d_rstat, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
        OMR_HIP(c, hipStreamSynchronize(c->stream));
        apply_rstat();
        uint64_t used = 0;
        for (int i = 0; i < n; ++i) {
            if (!lens[i]) return fail(c, OMR_INTERNAL, "encode batch buffer too small");
            used = std::max<uint64_t>(used, offs[i] + lens[i]);
        }
        std::vector<uint8_t> all(used);
        OMR_HIP(c, hipMemcpyAsync(all.data(), B->d_jpeg, used, hipMemcpyDeviceToHost, c->stream));
        OMR_HIP(c, hipStreamSynchronize(c->stream));
        for (int i = 0; i < n; ++i)
            if (!out[i].st) out[i].bytes.assign(all.begin() + offs[i], all.begin() + offs[i] + lens[i]);
    } else if (format == OMR_FORMAT_JPEG || format == OMR_FORMAT_PNG || format == OMR_FORMAT_TIFF) {
        if (d_rstat) {
            OMR_HIP(c, hipMemcpyAsync(rstat.data(), d_rstat, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
            OMR_HIP(c, hipStreamSynchronize(c->stream));
            apply_rstat();
        }
        const size_t cap = format == OMR_FORMAT_JPEG ? omr_jpeg_max_bytes(W, H)
                         : format == OMR_FORMAT_PNG  ? omr_png_max_bytes(W, H, 3)
                                                     : omr_tiff_max_bytes(W, H);   // TIFFImageWriter (:583-596)
        std::vector<uint8_t> buf(cap);
        for (int i = 0; i < n; ++i) {
            if (out[i].st) continue;
            size_t len = 0;
            const uint32_t* a = B->d_argb + px * i;
            const omr_status st = format == OMR_FORMAT_JPEG ? omr_encode_jpeg_device(c, a, W, H, quality, buf.data(), cap, &len)
                                : format == OMR_FORMAT_PNG  ? omr_encode_png_device(c, a, W, H, buf.data(), cap, &len)
                                                            : omr_encode_tiff_device(c, a, W, H, buf.data(), cap, &len);
            if (st) return st;
            out[i].bytes.assign(buf.begin(), buf.begin() + len);
        }
    } else {                                               // OMR_FORMAT_ARGB: the packed int[] itself
        if (d_rstat) OMR_HIP(c, hipMemcpyAsync(rstat.data(), d_rstat, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
        std::vector<uint8_t> all(px * 4 * n);
        OMR_HIP(c, hipMemcpyAsync(all.data(), B->d_argb, all.size(), hipMemcpyDeviceToHost, c->stream));
        OMR_HIP(c, hipStreamSynchronize(c->stream));
        apply_rstat();
        for (int i = 0; i < n; ++i)
            if (!out[i].st) out[i].bytes.assign(all.begin() + px * 4 * i, all.begin() + px * 4 * (i + 1));
    }
    return OMR_OK;
}

// Render + encode one group (same image, settings, size, flip, format).  jobs[u] are the
// distinct tiles; out[u] receives each one's bytes, or OMR_QUANTIZATION for a tile with a pixel
// outside the LUT domain — only that tile fails, as only that request's Renderer would throw
// in the reference (one Renderer per request, ImageRegionRequestHandler.java:436-440, :479-480).
static omr_status run_group(Lane* B, const std::vector<Job*>& jobs, std::vector<Result>& out) {
    omr_ctx* c = B->ctx;
    const Job& j0 = *jobs[0];
    c->sem = j0.sem;      // the group's semantics (every job of a group has the same), dispatcher thread only
    const int W = j0.spec.width, H = j0.spec.height;
    const size_t px = (size_t)W * H;
    // A tile outside the image (the reference's DimensionsOutOfBoundsException from the pixel
    // buffer) fails alone; the group renders the rest.
    int32_t dims[6];
    pixel_buffer_dims(j0.pb, dims);
    out.assign(jobs.size(), Result{});
    std::vector<int> live;
    std::vector<omr_tile_request> reqs;
    for (size_t i = 0; i < jobs.size(); ++i) {
        const omr_tile_job& s = jobs[i]->spec;
        if (s.z < 0 || s.z >= dims[2] || s.t < 0 || s.t >= dims[4] || s.x < 0 || s.y < 0 ||
            (int64_t)s.x + W > dims[0] || (int64_t)s.y + H > dims[1]) {
            out[i].st = OMR_INVALID_ARGUMENT;
            out[i].err = "tile outside the image";
            continue;
        }
        live.push_back((int)i);
        reqs.push_back({s.z, s.t, s.x, s.y});
    }
    const int n = (int)live.size();
    if (!n) return OMR_OK;
    omr_status st = grow_dev(B, px * 4 * n, 0, n);
    if (st) return st;
    st = render_pixel_buffer_tiles(c, j0.pb, &j0.qdef, j0.ch.data(), (int32_t)j0.ch.size(), reqs.data(), n, W, H,
                                   j0.spec.flip_h, j0.spec.flip_v, B->d_argb, 1, B->d_rstat);
    if (st) return st;
    std::vector<Result> sub(n);
    st = encode_group(B, n, W, H, j0.spec.format, j0.spec.quality, sub, B->d_rstat);
    if (st) return st;
    for (int i = 0; i < n; ++i) out[live[i]] = std::move(sub[i]);
    return OMR_OK;
}

// The cache slot of stack (serial, c, t): *resident = true when it is already in HBM; otherwise a
// buffer of `bytes` to upload into (least recently used stacks evicted, their memory reused when the
// size matches), or nullptr when the stack does not fit the cache beside the request's other stacks.
static uint8_t* stack_slot(omr_batcher* B, uint64_t serial, int32_t c, int32_t t, size_t bytes, uint64_t tick,
                           bool* resident, omr_status* st) {
    *resident = false;
    for (auto& e : B->stacks)
        if (e.serial == serial && e.c == c && e.t == t && e.bytes == bytes) {
            e.used = tick;
            *resident = true;
            B->stack_hits++;
            return e.d;
        }
    B->stack_misses++;
    const int64_t cap = B->stack_cache_max.load();
    uint8_t* reuse = nullptr;
    size_t resident_bytes = B->stack_resident.load();
    while (resident_bytes + bytes > (size_t)std::max<int64_t>(cap, 0)) {
        int lru = -1;
        for (int k = 0; k < (int)B->stacks.size(); ++k)
            if (B->stacks[k].used != tick && (lru < 0 || B->stacks[k].used < B->stacks[lru].used)) lru = k;
        if (lru < 0) break;                              // everything resident serves this request
        const omr_batcher::StackEntry e = B->stacks[lru];
        B->stacks.erase(B->stacks.begin() + lru);
        resident_bytes -= e.bytes;
        if (!reuse && e.bytes == bytes) {
            reuse = e.d;
        } else {
            const hipError_t he = hipFree(e.d);
            if (he != hipSuccess) { *st = hip_fail(B->ctx, he, "hipFree(stack cache)"); return nullptr; }
        }
    }
    B->stack_resident = resident_bytes;
    if (resident_bytes + bytes > (size_t)std::max<int64_t>(cap, 0)) {
        if (reuse) (void)hipFree(reuse);
        return nullptr;
    }
    if (!reuse) {
        const hipError_t he = hipMalloc(reinterpret_cast<void**>(&reuse), bytes);
        if (he != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;                              // HBM full: upload into the scratch instead
        }
    }
    B->stacks.push_back({serial, c, t, bytes, reuse, tick});
    B->stack_resident = resident_bytes + bytes;
    return reuse;
}

// A stack whose upload failed leaves the cache: its slot never held the (serial, c, t) planes, so a
// later request for them must upload (and fail or succeed) again rather than read stale HBM.
static void stack_drop(omr_batcher* B, const uint8_t* d) {
    for (size_t k = 0; k < B->stacks.size(); ++k)
        if (B->stacks[k].d == d) {
            B->stack_resident = B->stack_resident.load() - B->stacks[k].bytes;
            (void)hipFree(B->stacks[k].d);
            B->stacks.erase(B->stacks.begin() + (long)k);
            return;
        }
}

// Projection jobs of one group (same image, settings, projection, flips, format): for each
// distinct t the active channels' Z-stacks go to HBM (DMA from the registered ROMIO mapping),
// omr_render_projected_device projects and renders the full plane (the glue,
// ImageRegionRequestHandler.java:506-559), and the group's planes are encoded in one batch.
// A request whose render fails (OMR_QUANTIZATION, the quirk-3 OMR_INTERNAL, a bad z range) fails
// alone.
static omr_status run_projection_group(omr_batcher* B, Lane* L, const std::vector<Job*>& jobs,
                                       std::vector<Result>& out) {
    omr_ctx* c = L->ctx;
    const Job& j0 = *jobs[0];
    c->sem = j0.sem;
    int32_t dims[6];
    pixel_buffer_dims(j0.pb, dims);
    const int W = dims[0], H = dims[1], Z = dims[2], SC = dims[3], PT = dims[5];
    const int n = (int)jobs.size();
    const size_t px = (size_t)W * H;
    if ((int)j0.ch.size() != SC) return fail(c, OMR_INVALID_ARGUMENT, "channel bindings do not match sizeC");
    std::vector<int> act;
    for (int ch = 0; ch < SC; ++ch)
        if (j0.ch[ch].active) act.push_back(ch);
    const size_t stack_bytes = align_up(px * (size_t)bytes_per_pixel(PT) * Z, 256);
    const uint64_t serial = pixel_buffer_serial(j0.pb);
    omr_status st = grow_dev(L, px * 4 * n, 0, n);
    if (st) return st;
    const size_t scratch_bytes = stack_bytes * std::max<size_t>(1, act.size());
    auto scratch = [&](size_t a, uint8_t** d) -> omr_status {   // the uncached fallback, grown on first use
        if (scratch_bytes > L->stack_cap) {
            L->stack_cap = 0;
            const omr_status s2 = regrow(c, L->d_stack, scratch_bytes);
            if (s2) return s2;
            L->stack_cap = scratch_bytes;
        }
        *d = L->d_stack + stack_bytes * a;
        return OMR_OK;
    };
    out.assign(n, Result{});
    const int start = j0.spec.projection_start >= 0 ? j0.spec.projection_start : 0;   // :510-515
    const int end = j0.spec.projection_end >= 0 ? j0.spec.projection_end : Z - 1;
    std::vector<const void*> stacks(SC, nullptr);
    for (int i = 0; i < n; ++i) {
        const int t = jobs[i]->spec.t;
        if (t < 0 || t >= dims[4]) {                           // checked before any cache slot is taken
            out[i].st = OMR_INVALID_ARGUMENT;
            out[i].err = "projection t outside the image";
            continue;
        }
        const uint64_t tick = ++B->stack_tick;
        for (size_t a = 0; a < act.size() && !st; ++a) {
            bool resident = false;
            uint8_t* d = stack_slot(B, serial, act[a], t, stack_bytes, tick, &resident, &st);
            if (st) break;
            const bool cached = d != nullptr;
            if (!d && (st = scratch(a, &d))) break;              // larger than the cache: scratch
            stacks[act[a]] = d;
            if (!resident) {
                st = pixel_buffer_upload_stack(c, j0.pb, act[a], t, d);
                if (st && cached) stack_drop(B, d);
            }
        }
        if (!st)
            st = omr_render_projected_device(c, &j0.qdef, j0.ch.data(), SC, stacks.data(), PT, 1, W, H, Z,
                                             j0.spec.projection, start, end, 1, j0.spec.flip_h, j0.spec.flip_v,
                                             L->d_argb + px * i);
        if (!st) st = omr_ctx_synchronize(c);              // this request's QuantizationException, if any
        if (st) {
            if (st == OMR_DEVICE || st == OMR_OOM) return st;
            out[i].st = st;
            out[i].err = c->last_error;
            st = OMR_OK;
        }
    }
    return encode_group(L, n, W, H, j0.spec.format, j0.spec.quality, out);
}

// Every mask job of a dispatch round with the same semantics: one omr_render_shape_mask_png_batch.
static omr_status run_mask_group(Lane* B, const std::vector<Job*>& jobs, std::vector<Result>& out) {
    omr_ctx* c = B->ctx;
    c->sem = jobs[0]->sem;
    const int n = (int)jobs.size();
    std::vector<omr_mask_job> mj(n);
    size_t cap = 0;
    for (int i = 0; i < n; ++i) {
        mj[i] = jobs[i]->mask;
        // room only for masks the batch will encode: the ones it answers 404 (the single call's
        // checks) take none, so declared dimensions alone cannot size the buffer
        const int64_t npx = (int64_t)mj[i].width * mj[i].height;
        if (mj[i].width > 0 && mj[i].height > 0 && npx <= INT32_MAX && mj[i].bits &&
            (int64_t)mj[i].n_bytes * 8 >= npx)
            cap += omr_png_batch_max_bytes(mj[i].width, mj[i].height, 1, 1);
    }
    std::vector<uint8_t> buf(std::max<size_t>(cap, 16));
    std::vector<uint64_t> offs(n);
    std::vector<uint32_t> lens(n);
    std::vector<int32_t> stat(n);
    const omr_status st = omr_render_shape_mask_png_batch(c, mj.data(), n, buf.data(), buf.size(), offs.data(),
                                                          lens.data(), stat.data());
    if (st) return st;
    out.assign(n, Result{});
    for (int i = 0; i < n; ++i) {
        out[i].st = stat[i];
        if (stat[i]) out[i].err = "Cannot render Mask";      // ShapeMaskVerticle.java:119-128 -> 404
        else out[i].bytes.assign(buf.begin() + offs[i], buf.begin() + offs[i] + lens[i]);
    }
    return OMR_OK;
}

// The region / shape-mask cache key of a job within its group (ImageRegionCtx.java:165-177).
static std::string tile_key(const Job& jb) {
    const omr_tile_job& s = jb.spec;
    std::string key;
    if (jb.kind == kJobTile) {
        const int32_t k4[4] = {s.z, s.t, s.x, s.y};
        append(key, k4, sizeof(k4));
    } else if (jb.kind == kJobProjection) {
        append(key, &s.t, sizeof(s.t));
    } else {
        // the caller's byte count and null-ness too: an empty mask (padded to one zero byte) must
        // not share the result of a real 1-byte zero mask
        const int64_t nb = jb.mask.bits ? (int64_t)jb.mask.n_bytes : -1;
        const int32_t m4[4] = {jb.mask.width, jb.mask.height, jb.mask.flip_h, jb.mask.flip_v};
        append(key, m4, sizeof(m4));
        append(key, &nb, sizeof(nb));
        append(key, jb.mask.rgba, 4);
        append(key, jb.mask_bits.data(), jb.mask_bits.size());
    }
    return key;
}

static void dispatch_loop(omr_batcher* B, Lane* L) {
    (void)hipSetDevice(B->device);
    // lane 0 takes every kind; a higher lane takes tiles and masks, and gathers only while a lower
    // lane is busy: a second lane exists to overlap a round's upload with another round's render
    // and encode, not to split one burst into two smaller (and less deduplicated) rounds
    auto eligible = [&](const Job& j) { return L->index == 0 || j.kind != kJobProjection; };
    auto lower_busy = [&]() {
        for (int i = 0; i < L->index; ++i)
            if (B->lanes[i]->busy) return true;
        return false;
    };
    auto n_eligible = [&]() {
        int k = 0;
        for (auto& j : B->pending) k += eligible(*j);
        return k;
    };
    std::unique_lock<std::mutex> lk(B->m);
    for (;;) {
        B->cv_in.wait(lk, [&] { return B->stop || (n_eligible() > 0 && (L->index == 0 || lower_busy())); });
        if (B->stop && n_eligible() == 0) return;
        if (!B->stop && L->index > 0 && !lower_busy()) continue;
        // gather: up to max_batch jobs, what arrives within max_wait_us of the oldest one, or --
        // whichever comes first -- until the arrivals pause for gap_us.  A burst (a viewer's
        // screenful, the clients answered by the last round) is taken as soon as it has landed
        // instead of after the whole max_wait_us.  Right after a round, as many jobs as it took also
        // close the gather: clients that wait for their answer before asking again come back
        // together, and their round goes as soon as they are all in.  After an idle spell (longer
        // than max_wait_us) only the pause counts, so a fresh burst is still gathered whole (and its
        // duplicates rendered once).  With no lane busy the device is idle: the pause shrinks to
        // kIdleGapUs, enough for submits made together to meet.
        const Job* first = nullptr;
        for (auto& j : B->pending)
            if (eligible(*j)) { first = j.get(); break; }
        const bool follow = L->last_round > 0 &&
                            first->t_submit - L->t_round_end < std::chrono::microseconds(B->max_wait_us);
        for (;;) {
            const int ne = n_eligible();
            if (B->stop || ne >= B->max_batch || ne == 0) break;
            if (follow && ne >= L->last_round) break;
            const auto now = std::chrono::steady_clock::now();
            const int gap = B->busy_lanes == 0 ? std::min(B->gap_us, kIdleGapUs)
                          : L->index > 0          ? B->lane_gap_us
                                                  : B->gap_us;
            const auto deadline = std::min(first->t_submit + std::chrono::microseconds(B->max_wait_us),
                                           B->t_last_submit + std::chrono::microseconds(gap));
            if (now >= deadline) break;
            B->cv_in.wait_until(lk, deadline);
            first = nullptr;                             // another lane may have taken the oldest job
            for (auto& j : B->pending)
                if (eligible(*j)) { first = j.get(); break; }
            if (!first) break;
        }
        std::vector<std::unique_ptr<Job>> take;
        for (size_t i = 0; i < B->pending.size() && (int)take.size() < B->max_batch;) {
            if (eligible(*B->pending[i])) {
                take.push_back(std::move(B->pending[i]));
                B->pending.erase(B->pending.begin() + (long)i);
            } else {
                ++i;
            }
        }
        if (take.empty()) continue;
        // cross-lane dedup: a job identical to one another lane is rendering waits for that render
        std::vector<std::string> my_keys;
        uint64_t followed = 0;
        for (size_t i = 0; i < take.size();) {
            std::string key = take[i]->group_key + '\x01' + tile_key(*take[i]);
            auto it = B->inflight.find(key);
            if (it != B->inflight.end() &&
                std::find(my_keys.begin(), my_keys.end(), key) == my_keys.end()) {
                it->second.push_back(take[i]->ticket);
                take.erase(take.begin() + (long)i);
                ++followed;
                continue;
            }
            if (it == B->inflight.end()) {
                B->inflight.emplace(key, std::vector<uint64_t>());
                my_keys.push_back(std::move(key));
            }
            ++i;
        }
        B->n_dedup += followed;
        if (take.empty()) continue;
        L->last_round = (int)take.size();
        L->busy = true;
        B->busy_lanes++;
        lk.unlock();
        if (L->index + 1 < (int)B->lanes.size()) B->cv_in.notify_all();   // the next lane may gather now
        // group by settings; dedupe identical tiles (the region cache key) inside each group
        std::map<std::string, std::vector<Job*>> groups;
        for (auto& j : take) groups[j->group_key].push_back(j.get());
        std::vector<std::pair<uint64_t, Result>> results;
        std::vector<std::pair<std::string, size_t>> keyed;   // cache key of each rendered job -> its result
        uint64_t rendered = 0, dedup = 0;
        for (auto& g : groups) {
            std::vector<Job*> uniq;
            std::vector<int> slot(g.second.size());
            std::map<std::string, int> seen;
            const int kind = g.second[0]->kind;
            for (size_t i = 0; i < g.second.size(); ++i) {
                const std::string key = tile_key(*g.second[i]);
                auto it = seen.find(key);
                if (it == seen.end()) {
                    seen[key] = (int)uniq.size();
                    slot[i] = (int)uniq.size();
                    uniq.push_back(g.second[i]);
                } else {
                    slot[i] = it->second;
                    ++dedup;
                }
            }
            std::vector<Result> out;
            omr_status st = OMR_OK;
            size_t chunk = (size_t)B->max_batch;
            if (kind == kJobProjection) {
                // full planes: ARGB (px*4) + the batched JPEG's reservation (px*4 + 64 KiB) per plane,
                // kept under a fixed budget so a large image splits into sub-batches instead of
                // failing the whole group with OMR_OOM
                int32_t dims[6];
                pixel_buffer_dims(uniq[0]->pb, dims);
                const size_t per = (size_t)dims[0] * dims[1] * 8 + 65536;
                chunk = std::max<size_t>(1, std::min(chunk, kProjectionBatchBytes / per));
            }
            // each sub-batch answers its own jobs: a failure in a later sub-batch (OOM, a device
            // error) fails that sub-batch's jobs only, and the planes earlier ones rendered stand
            std::vector<omr_status> part_st(uniq.size(), OMR_OK);
            std::vector<std::string> part_err(uniq.size());
            for (size_t b0 = 0; b0 < uniq.size(); b0 += chunk) {
                const size_t b1 = std::min(uniq.size(), b0 + chunk);
                std::vector<Job*> part(uniq.begin() + b0, uniq.begin() + b1);
                std::vector<Result> po;
                try {
                    st = kind == kJobTile ? run_group(L, part, po)
                       : kind == kJobProjection ? run_projection_group(B, L, part, po)
                                                : run_mask_group(L, part, po);
                } catch (const std::bad_alloc&) {     // host memory: this sub-batch fails, the server lives
                    st = fail(L->ctx, OMR_OOM, "host allocation failed in the batcher");
                } catch (const std::exception& e) {
                    st = fail(L->ctx, OMR_INTERNAL, std::string("batcher: ") + e.what());
                }
                po.resize(part.size());
                for (size_t k = 0; k < part.size(); ++k) {
                    if (st) {
                        part_st[b0 + k] = st;
                        part_err[b0 + k] = L->ctx->last_error;
                    }
                    out.push_back(std::move(po[k]));
                }
                if (st == OMR_DEVICE) {               // a device error poisons the context: stop here
                    for (size_t k = b1; k < uniq.size(); ++k) {
                        part_st[k] = st;
                        part_err[k] = L->ctx->last_error;
                        out.emplace_back();
                    }
                    break;
                }
            }
            rendered += uniq.size();
            for (size_t i = 0; i < g.second.size(); ++i) {
                Result r;
                const int u = slot[i];
                if (part_st[u]) { r.st = part_st[u]; r.err = part_err[u]; }
                else if (out[u].st) { r.st = out[u].st; r.err = out[u].err; }
                else r.bytes = out[u].bytes;
                results.emplace_back(g.second[i]->ticket, std::move(r));
                if (std::find(uniq.begin(), uniq.end(), g.second[i]) != uniq.end())
                    keyed.emplace_back(g.second[i]->group_key + '\x01' + tile_key(*g.second[i]), results.size() - 1);
            }
        }
        lk.lock();
        size_t answered = results.size();
        for (auto& kr : keyed) {                  // the other lanes' identical jobs, same answer
            auto it = B->inflight.find(kr.first);
            if (it == B->inflight.end()) continue;
            for (uint64_t t : it->second) {
                B->done[t] = results[kr.second].second;
                ++answered;
            }
            B->inflight.erase(it);
        }
        for (const auto& k : my_keys) B->inflight.erase(k);   // (keys of jobs that failed before grouping)
        for (auto& r : results) B->done[r.first] = std::move(r.second);
        B->outstanding -= (int64_t)answered;
        B->n_batches += 1;
        L->t_round_end = std::chrono::steady_clock::now();
        L->busy = false;
        B->busy_lanes--;
        B->n_rendered += rendered;
        B->n_dedup += dedup;
        B->cv_out.notify_all();
    }
}

}  // namespace omr

using namespace omr;

extern "C" {

omr_status omr_batcher_create(int32_t device, int32_t max_batch, int32_t max_wait_us, omr_batcher** out) {
    if (!out || max_batch <= 0 || max_wait_us < 0) return OMR_INVALID_ARGUMENT;
    *out = nullptr;
    auto* B = new omr_batcher;
    B->device = device;
    B->max_batch = max_batch;
    B->max_wait_us = max_wait_us;
    int lanes = 2;
    if (const char* v = std::getenv("OMR_BATCH_LANES")) lanes = std::max(1, std::min(8, std::atoi(v)));
    for (int i = 0; i < lanes; ++i) {
        auto L = std::make_unique<Lane>();
        L->index = i;
        const omr_status st = omr_ctx_create(device, &L->ctx);
        if (st) {
            for (auto& x : B->lanes) omr_ctx_destroy(x->ctx);
            delete B;
            return st;
        }
        B->lanes.push_back(std::move(L));
    }
    B->ctx = B->lanes[0]->ctx;
    if (const char* v = std::getenv("OMR_STACK_CACHE_MB")) B->stack_cache_max = (int64_t)std::atoll(v) << 20;
    B->gap_us = std::min(max_wait_us, 200);
    if (const char* v = std::getenv("OMR_BATCH_GAP_US")) B->gap_us = std::max(0, std::min(max_wait_us, std::atoi(v)));
    B->lane_gap_us = std::min(B->gap_us, 30);
    if (const char* v = std::getenv("OMR_BATCH_LANE_GAP_US")) B->lane_gap_us = std::max(0, std::min(max_wait_us, std::atoi(v)));
    for (auto& L : B->lanes) L->th = std::thread(dispatch_loop, B, L.get());
    *out = B;
    return OMR_OK;
}

void omr_batcher_destroy(omr_batcher* B) {
    if (!B) return;
    {
        std::lock_guard<std::mutex> g(B->m);
        B->stop = true;
    }
    B->cv_in.notify_all();
    for (auto& L : B->lanes)
        if (L->th.joinable()) L->th.join();
    (void)hipSetDevice(B->device);
    for (auto& e : B->stacks) (void)hipFree(e.d);
    for (auto& L : B->lanes) {
        for (void* p : {(void*)L->d_argb, (void*)L->d_jpeg, (void*)L->d_offs, (void*)L->d_lens, (void*)L->d_stat,
                        (void*)L->d_rstat, (void*)L->d_stack})
            if (p) (void)hipFree(p);
        omr_ctx_destroy(L->ctx);
    }
    delete B;
}

static void enqueue(omr_batcher* B, std::unique_ptr<Job> j, uint64_t* ticket) {
    j->t_submit = std::chrono::steady_clock::now();
    {
        std::lock_guard<std::mutex> g(B->m);
        j->sem = B->sem;                  // semantics fixed at submit: a later set_semantics cannot
        j->group_key = settings_key(*j);  // reach a job already queued or a group in flight
        j->ticket = B->next_ticket++;
        *ticket = j->ticket;
        B->t_last_submit = j->t_submit;
        B->pending.push_back(std::move(j));
        B->n_jobs++;
        B->outstanding++;
    }
    B->cv_in.notify_all();     // every idle lane (lane 0 alone takes projection jobs)
}

omr_status omr_batcher_submit(omr_batcher* B, const omr_tile_job* job, uint64_t* ticket) {
    if (!B || !job || !ticket || !job->pb || !job->qdef || !job->channels || job->size_c <= 0)
        return OMR_INVALID_ARGUMENT;
    const bool proj = job->has_projection != 0;
    if (!proj && (job->width <= 0 || job->height <= 0)) return OMR_INVALID_ARGUMENT;
    if (proj && (job->projection < OMR_PROJECTION_MAX || job->projection > OMR_PROJECTION_SUM))
        return OMR_INVALID_ARGUMENT;
    if (job->format != OMR_FORMAT_JPEG && job->format != OMR_FORMAT_PNG && job->format != OMR_FORMAT_ARGB &&
        job->format != OMR_FORMAT_TIFF)
        return OMR_NOT_FOUND;                              // unknown format -> null -> 404 (:602-603)
    auto j = std::make_unique<Job>();
    j->kind = proj ? kJobProjection : kJobTile;
    j->pb = job->pb;
    j->qdef = *job->qdef;
    j->ch.assign(job->channels, job->channels + job->size_c);
    j->luts.resize(job->size_c);
    for (int c = 0; c < job->size_c; ++c)
        if (j->ch[c].lut) {
            j->luts[c].assign(j->ch[c].lut, j->ch[c].lut + 768);
            j->ch[c].lut = j->luts[c].data();
        }
    j->spec = *job;
    j->spec.qdef = nullptr;
    j->spec.channels = nullptr;
    enqueue(B, std::move(j), ticket);
    return OMR_OK;
}

omr_status omr_batcher_submit_mask(omr_batcher* B, const omr_mask_job* job, uint64_t* ticket) {
    if (!B || !job || !ticket) return OMR_INVALID_ARGUMENT;
    auto j = std::make_unique<Job>();
    j->kind = kJobMask;
    j->mask = *job;
    if (job->bits && job->n_bytes) j->mask_bits.assign(job->bits, job->bits + job->n_bytes);
    // a null mask stays null (the reference's NPE -> 404 at wait); an empty one points at the copy
    j->mask.bits = job->bits ? j->mask_bits.data() : nullptr;
    if (job->bits && !job->n_bytes) { j->mask_bits.assign(1, 0); j->mask.bits = j->mask_bits.data(); }
    enqueue(B, std::move(j), ticket);
    return OMR_OK;
}

omr_status omr_batcher_wait(omr_batcher* B, uint64_t ticket, uint8_t* out, size_t cap, size_t* len) {
    if (!B || !len) return OMR_INVALID_ARGUMENT;
    std::unique_lock<std::mutex> lk(B->m);
    B->cv_out.wait(lk, [&] { return B->done.count(ticket) > 0; });
    Result& r = B->done[ticket];
    if (r.st) {
        const omr_status st = r.st;
        B->done.erase(ticket);
        return st;
    }
    *len = r.bytes.size();
    if (!out || cap < r.bytes.size()) return OMR_BUFFER_TOO_SMALL;   // result kept: retry with room
    std::memcpy(out, r.bytes.data(), r.bytes.size());
    B->done.erase(ticket);
    return OMR_OK;
}

omr_status omr_batcher_set_semantics(omr_batcher* B, uint32_t flags) {
    if (!B) return OMR_INVALID_ARGUMENT;
    if (flags & ~(uint32_t)OMR_SEM_ALL) return OMR_INVALID_ARGUMENT;
    // jobs carry the flags from submit; the dispatcher applies a group's flags to its own context
    // (run_group), so this never touches the context another thread is rendering with
    std::lock_guard<std::mutex> g(B->m);
    B->sem = flags;
    return OMR_OK;
}

omr_status omr_batcher_set_stack_cache(omr_batcher* B, int64_t max_bytes) {
    if (!B || max_bytes < 0) return OMR_INVALID_ARGUMENT;
    B->stack_cache_max = max_bytes;      // the dispatcher evicts down to it on its next projection job
    return OMR_OK;
}

omr_status omr_batcher_stack_cache_stats(omr_batcher* B, uint64_t stats_out[3]) {
    if (!B || !stats_out) return OMR_INVALID_ARGUMENT;
    stats_out[0] = B->stack_hits.load();
    stats_out[1] = B->stack_misses.load();
    stats_out[2] = B->stack_resident.load();
    return OMR_OK;
}

omr_status omr_batcher_stats(omr_batcher* B, uint64_t stats_out[4]) {
    if (!B || !stats_out) return OMR_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(B->m);
    stats_out[0] = B->n_jobs;
    stats_out[1] = B->n_batches;
    stats_out[2] = B->n_rendered;
    stats_out[3] = B->n_dedup;
    return OMR_OK;
}

// ---- node-level pool: one batcher per GPU ------------------------------------
// The reference scales a node with N worker-verticle instances over one worker pool
// (ImageRegionMicroserviceVerticle.java:84-85, :149-165).  The pool spreads the workers' tile
// jobs over the node's GPUs: every device has its own batcher (context, stream, dispatcher thread,
// and its own plan / LUT replicas in its HBM), a job goes to the batcher with the fewest jobs
// queued or in flight (ties rotate), and the ticket remembers which batcher holds it.  Tiles are
// independent: there is no collective and no peer traffic.
struct omr_pool {
    std::vector<omr_batcher*> b;
    std::vector<int32_t> devices;
    std::atomic<uint32_t> rr{0};
};

static constexpr int kPoolIndexBits = 8;   // up to 256 batchers; ticket = batcher ticket << 8 | index

omr_status omr_pool_create(const int32_t* devices, int32_t n_devices, int32_t max_batch, int32_t max_wait_us,
                           omr_pool** out) {
    if (!out) return OMR_INVALID_ARGUMENT;
    *out = nullptr;
    if (!devices || n_devices <= 0 || n_devices > (1 << kPoolIndexBits) || max_batch <= 0 || max_wait_us < 0)
        return OMR_INVALID_ARGUMENT;
    auto* P = new omr_pool;
    for (int i = 0; i < n_devices; ++i) {
        omr_batcher* b = nullptr;
        const omr_status st = omr_batcher_create(devices[i], max_batch, max_wait_us, &b);
        if (st) {
            for (omr_batcher* x : P->b) omr_batcher_destroy(x);
            delete P;
            return st;
        }
        P->b.push_back(b);
        P->devices.push_back(devices[i]);
    }
    *out = P;
    return OMR_OK;
}

void omr_pool_destroy(omr_pool* P) {
    if (!P) return;
    for (omr_batcher* b : P->b) omr_batcher_destroy(b);
    delete P;
}

int32_t omr_pool_size(const omr_pool* P) { return P ? (int32_t)P->b.size() : 0; }

// The batcher with the fewest jobs queued or in flight, ties rotating from a moving start.
static int pool_pick(omr_pool* P) {
    const int n = (int)P->b.size();
    const uint32_t start = P->rr.fetch_add(1, std::memory_order_relaxed) % (uint32_t)n;
    int best = (int)start;
    int64_t best_q = P->b[best]->outstanding.load(std::memory_order_relaxed);
    for (int k = 1; k < n; ++k) {
        const int i = (int)((start + k) % (uint32_t)n);
        const int64_t q = P->b[i]->outstanding.load(std::memory_order_relaxed);
        if (q < best_q) { best = i; best_q = q; }
    }
    return best;
}

// Route by the request's cache identity (ImageRegionCtx.java:165-177: image, plane, region; the
// settings travel with it): identical requests in flight together land on the same batcher, so the
// pool deduplicates them as one batcher does, instead of each batcher rendering its own copy.  A
// home batcher more than `slack` jobs behind the least-queued one is bypassed (load balance wins
// over dedup for a hot key).
static uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001B3ull;
    return h;
}
static int pool_pick_keyed(omr_pool* P, uint64_t h, int64_t slack) {
    const int n = (int)P->b.size();
    const int home = (int)((h >> 17) % (uint64_t)n);
    const int least = pool_pick(P);
    const int64_t qh = P->b[home]->outstanding.load(std::memory_order_relaxed);
    const int64_t ql = P->b[least]->outstanding.load(std::memory_order_relaxed);
    return qh <= ql + slack ? home : least;
}

omr_status omr_pool_submit(omr_pool* P, const omr_tile_job* job, uint64_t* ticket) {
    if (!P || !ticket || !job) return OMR_INVALID_ARGUMENT;
    uint64_t h = 0xCBF29CE484222325ull;
    h = fnv1a(h, &job->pb, sizeof(job->pb));
    const int32_t id[7] = {job->z, job->t, job->x, job->y, job->width, job->height, job->has_projection};
    h = fnv1a(h, id, sizeof(id));
    const int best = pool_pick_keyed(P, h, P->b[0]->max_batch / 2);
    uint64_t t = 0;
    const omr_status st = omr_batcher_submit(P->b[best], job, &t);
    if (st) return st;
    *ticket = (t << kPoolIndexBits) | (uint64_t)best;
    return OMR_OK;
}

omr_status omr_pool_submit_mask(omr_pool* P, const omr_mask_job* job, uint64_t* ticket) {
    if (!P || !ticket || !job) return OMR_INVALID_ARGUMENT;
    uint64_t h = 0xCBF29CE484222325ull;
    const int32_t id[4] = {job->width, job->height, job->flip_h, job->flip_v};
    h = fnv1a(h, id, sizeof(id));
    h = fnv1a(h, job->rgba, 4);
    if (job->bits) h = fnv1a(h, job->bits, std::min<size_t>(job->n_bytes, 256));
    const int best = pool_pick_keyed(P, h, P->b[0]->max_batch / 2);
    uint64_t t = 0;
    const omr_status st = omr_batcher_submit_mask(P->b[best], job, &t);
    if (st) return st;
    *ticket = (t << kPoolIndexBits) | (uint64_t)best;
    return OMR_OK;
}

int32_t omr_pool_device_index(const omr_pool* P, uint64_t ticket) {
    if (!P) return -1;
    const uint64_t i = ticket & ((1u << kPoolIndexBits) - 1);
    return i < P->b.size() ? (int32_t)i : -1;
}

omr_status omr_pool_wait(omr_pool* P, uint64_t ticket, uint8_t* out, size_t cap, size_t* len) {
    const int32_t i = omr_pool_device_index(P, ticket);
    if (i < 0) return OMR_INVALID_ARGUMENT;
    return omr_batcher_wait(P->b[i], ticket >> kPoolIndexBits, out, cap, len);
}

omr_status omr_pool_set_semantics(omr_pool* P, uint32_t flags) {
    if (!P) return OMR_INVALID_ARGUMENT;
    if (flags & ~(uint32_t)OMR_SEM_ALL) return OMR_INVALID_ARGUMENT;
    for (omr_batcher* b : P->b) {
        const omr_status st = omr_batcher_set_semantics(b, flags);
        if (st) return st;
    }
    return OMR_OK;
}

omr_status omr_pool_set_stack_cache(omr_pool* P, int64_t max_bytes_per_device) {
    if (!P) return OMR_INVALID_ARGUMENT;
    for (omr_batcher* b : P->b) {
        const omr_status st = omr_batcher_set_stack_cache(b, max_bytes_per_device);
        if (st) return st;
    }
    return OMR_OK;
}

omr_status omr_pool_stats(omr_pool* P, uint64_t* stats_out, int32_t n_entries) {
    if (!P || !stats_out || n_entries < (int32_t)P->b.size()) return OMR_INVALID_ARGUMENT;
    for (size_t i = 0; i < P->b.size(); ++i) {
        const omr_status st = omr_batcher_stats(P->b[i], stats_out + 4 * i);
        if (st) return st;
    }
    return OMR_OK;
}

}  // extern "C"
