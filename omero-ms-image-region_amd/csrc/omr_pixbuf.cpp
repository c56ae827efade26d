// omr_pixbuf.cpp — the step before the path: ROMIO pixel buffer -> pinned staging -> device.
//
// Replaces pixelsService.getPixelBuffer(pixels, false) (ImageRegionRequestHandler.java:302-309)
// for repository-backed images, i.e. upstream ome.io.nio.RomioPixelBuffer: one file of
// big-endian planes in XYZCT order, plane (z, c, t) at ((t*sizeC + c)*sizeZ + z) * planeBytes,
// rows of sizeX pixels.  getTile(z, c, t, x, y, w, h) reads h row segments of that plane.
//
// omr_render_pixel_buffer_tiles is the host-fed render_image_region path for many tiles of one
// image at one setting (a viewer panning over a pyramid level).  The file is mapped read-only;
// when HIP accepts the mapping (hipHostRegister), the copy engine reads every tile's rows from
// the page cache into HBM with 2-D copies on a copy stream — no CPU byte copy.  Otherwise worker
// threads copy each group of tiles into a pinned slot that is then sent in one copy.  K1+K2
// render on the context's stream and the ARGB comes back (or stays in HBM for a JPEG batch);
// two slots are in flight so reads, PCIe copies and kernels overlap.
#include "omr_internal.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cerrno>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>

struct omr_pixel_buffer {
    int fd = -1;
    int32_t sx = 0, sy = 0, sz = 0, sc = 0, st = 0, pt = 0, bpp = 0;
    int64_t row_bytes = 0, plane_bytes = 0, total = 0;
    // Read-only shared mapping of the file, only for files up to kMaxRegisterBytes: once
    // registered with HIP (hipHostRegister, first pipelined render) the copy engines read tile
    // rows straight from it — no CPU copy at all.  Registration pins every page of the mapping
    // while the buffer is open, hence the cap; larger files (and getTile) use pread, which turns a
    // file truncated underneath us into an I/O error (the reference's IOException) rather than
    // a SIGBUS from a mapped read.  Requirement: a registered file is not truncated while open
    // (its pages stay pinned; the DMA then reads the old contents).
    const uint8_t* map = nullptr;
    std::mutex reg_m;
    int reg_state = 0;   // 0 untried, 1 registered, -1 not registrable (pread/memcpy path)
    uint64_t serial = 0; // process-unique id (a closed buffer's address may be reused by the next open)
};

static std::atomic<uint64_t> g_pixbuf_serial{0};

namespace omr {

// Fixed pool of reader threads (one per context, created on first use).
// run() hands out the indices of one generation through a single 64-bit ticket
// (generation << 32 | next index): a worker claims an index with a compare-and-swap that fails
// once the generation has moved on, so a straggler of generation k can never take (and run a
// second time) an index of generation k+1.  Exactly n claims succeed per generation, done_
// counts exactly n, and run() returns only after every claimed job of its generation finished.
class ReadPool {
public:
    explicit ReadPool(int n) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~ReadPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // Runs job(i) for i in [0, n) on the pool and the calling thread; returns when all are done.
    // One caller at a time (the owning context's thread).
    void run(int n, const std::function<void(int)>& job) {
        if (n <= 0) return;
        uint32_t gen;
        {
            std::lock_guard<std::mutex> g(m_);
            gen = ++gen_;
            job_ = &job;
            n_ = n;
            done_ = 0;
            ticket_.store((uint64_t)gen << 32);
        }
        cv_.notify_all();
        work(gen, n, &job);
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return done_ == n_; });
        job_ = nullptr;
    }
    int size() const { return (int)th_.size(); }

private:
    void work(uint32_t gen, int n, const std::function<void(int)>* job) {
        for (;;) {
            uint64_t t = ticket_.load();
            int i;
            for (;;) {
                if ((uint32_t)(t >> 32) != gen) return;          // generation over
                i = (int)(uint32_t)t;
                if (i >= n) return;
                if (ticket_.compare_exchange_weak(t, t + 1)) break;
            }
            (*job)(i);
            std::lock_guard<std::mutex> g(m_);
            if (++done_ == n_) done_cv_.notify_all();
        }
    }
    void loop() {
        uint32_t seen = 0;
        for (;;) {
            uint32_t gen;
            int n;
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || (gen_ != seen && job_); });
                if (stop_) return;
                seen = gen = gen_;
                n = n_;
                job = job_;
            }
            work(gen, n, job);
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* job_ = nullptr;
    std::atomic<uint64_t> ticket_{0};
    int n_ = 0, done_ = 0;
    uint32_t gen_ = 0;
    bool stop_ = false;
};

// Double-buffered staging of one context.
struct PixPipe {
    ReadPool pool;
    void* pin_in[2] = {nullptr, nullptr};
    void* pin_out[2] = {nullptr, nullptr};
    void* d_in[2] = {nullptr, nullptr};
    void* d_out[2] = {nullptr, nullptr};
    size_t in_cap = 0, out_cap = 0;
    hipEvent_t h2d[2] = {nullptr, nullptr}, rend[2] = {nullptr, nullptr}, d2h[2] = {nullptr, nullptr};
    hipEvent_t h2d_b[2] = {nullptr, nullptr};   // the second copy stream's part of a slot
    hipStream_t copy = nullptr;
    hipStream_t copy_b = nullptr;               // a second DMA queue (env OMR_PIXBUF_COPY_STREAMS=2)
    bool bands = true;                          // row-band copies (env OMR_PIXBUF_BANDS=0: per-tile rects)
    size_t group_bytes = (size_t)64 << 20;      // planes per staging slot (env OMR_PIXBUF_GROUP_MB)
    explicit PixPipe(int threads) : pool(threads) {}
    ~PixPipe() {
        if (copy) (void)hipStreamSynchronize(copy);
        for (int i = 0; i < 2; ++i) {
            if (pin_in[i]) (void)hipHostFree(pin_in[i]);
            if (pin_out[i]) (void)hipHostFree(pin_out[i]);
            if (d_in[i]) (void)hipFree(d_in[i]);
            if (d_out[i]) (void)hipFree(d_out[i]);
            for (hipEvent_t e : {h2d[i], rend[i], d2h[i], h2d_b[i]})
                if (e) (void)hipEventDestroy(e);
        }
        if (copy_b) (void)hipStreamSynchronize(copy_b);
        if (copy) (void)hipStreamDestroy(copy);
        if (copy_b) (void)hipStreamDestroy(copy_b);
    }
};

static void free_pipe(void* p) { delete static_cast<PixPipe*>(p); }

static omr_status get_pipe(Ctx* c, PixPipe*& out) {
    if (!c->pixbuf_state) {
        const unsigned hw = std::thread::hardware_concurrency();
        auto* p = new PixPipe((int)std::max(1u, std::min(hw ? hw : 4u, 16u) - 1));
        c->pixbuf_state = p;
        c->pixbuf_state_free = free_pipe;
        OMR_HIP(c, hipStreamCreateWithFlags(&p->copy, hipStreamNonBlocking));
        const char* ncs = std::getenv("OMR_PIXBUF_COPY_STREAMS");
        if (ncs && std::atoi(ncs) >= 2) OMR_HIP(c, hipStreamCreateWithFlags(&p->copy_b, hipStreamNonBlocking));
        const char* nb = std::getenv("OMR_PIXBUF_BANDS");
        if (nb && std::atoi(nb) == 0) p->bands = false;
        const char* gm = std::getenv("OMR_PIXBUF_GROUP_MB");
        if (gm && std::atoi(gm) >= 8) p->group_bytes = (size_t)std::atoi(gm) << 20;
        for (int i = 0; i < 2; ++i)
            for (hipEvent_t* e : {&p->h2d[i], &p->rend[i], &p->d2h[i], &p->h2d_b[i]})
                OMR_HIP(c, hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    out = static_cast<PixPipe*>(c->pixbuf_state);
    return OMR_OK;
}

static omr_status grow(Ctx* c, PixPipe* p, size_t in_bytes, size_t out_bytes, bool host_out) {
    if (in_bytes > p->in_cap) {
        for (int i = 0; i < 2; ++i) {
            if (p->pin_in[i]) OMR_HIP(c, hipHostFree(p->pin_in[i]));
            if (p->d_in[i]) OMR_HIP(c, hipFree(p->d_in[i]));
            p->pin_in[i] = p->d_in[i] = nullptr;
        }
        for (int i = 0; i < 2; ++i) {
            OMR_HIP(c, hipHostMalloc(&p->pin_in[i], in_bytes, hipHostMallocDefault));
            OMR_HIP(c, hipMalloc(&p->d_in[i], in_bytes));
        }
        p->in_cap = in_bytes;
    }
    if (out_bytes > p->out_cap) {
        for (int i = 0; i < 2; ++i) {
            if (p->pin_out[i]) OMR_HIP(c, hipHostFree(p->pin_out[i]));
            if (p->d_out[i]) OMR_HIP(c, hipFree(p->d_out[i]));
            p->pin_out[i] = p->d_out[i] = nullptr;
        }
        for (int i = 0; i < 2; ++i) {
            OMR_HIP(c, hipMalloc(&p->d_out[i], out_bytes));
            if (host_out) OMR_HIP(c, hipHostMalloc(&p->pin_out[i], out_bytes, hipHostMallocDefault));
        }
        p->out_cap = out_bytes;
    }
    if (host_out && !p->pin_out[0]) {
        for (int i = 0; i < 2; ++i) OMR_HIP(c, hipHostMalloc(&p->pin_out[i], p->out_cap, hipHostMallocDefault));
    }
    return OMR_OK;
}

// pread until done (short reads, EINTR).
static bool read_full(int fd, void* dst, size_t n, int64_t off) {
    uint8_t* d = static_cast<uint8_t*>(dst);
    while (n) {
        const ssize_t r = ::pread(fd, d, n, (off_t)off);
        if (r < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        if (r == 0) return false;
        d += r;
        n -= (size_t)r;
        off += r;
    }
    return true;
}

static bool tile_in_bounds(const omr_pixel_buffer* pb, int32_t z, int32_t c, int32_t t, int32_t x, int32_t y,
                           int32_t w, int32_t h) {
    return z >= 0 && z < pb->sz && c >= 0 && c < pb->sc && t >= 0 && t < pb->st && x >= 0 && y >= 0 && w >= 0 &&
           h >= 0 && (int64_t)x + w <= pb->sx && (int64_t)y + h <= pb->sy;
}

static int64_t plane_offset(const omr_pixel_buffer* pb, int32_t z, int32_t c, int32_t t) {
    return (((int64_t)t * pb->sc + c) * pb->sz + z) * pb->plane_bytes;
}

// Files above this size are never mapped or registered (see omr_pixel_buffer::map).
constexpr int64_t kMaxRegisterBytes = (int64_t)1 << 30;

// Rows y..y+h of the plane, columns x..x+w, packed into dst (pread: see omr_pixel_buffer::map).
static bool read_tile(const omr_pixel_buffer* pb, int32_t z, int32_t c, int32_t t, int32_t x, int32_t y, int32_t w,
                      int32_t h, uint8_t* dst) {
    const int64_t base = plane_offset(pb, z, c, t) + (int64_t)y * pb->row_bytes + (int64_t)x * pb->bpp;
    const size_t seg = (size_t)w * pb->bpp;
    if (w == pb->sx) return read_full(pb->fd, dst, seg * (size_t)h, base);   // one contiguous band
    for (int32_t r = 0; r < h; ++r)
        if (!read_full(pb->fd, dst + seg * r, seg, base + (int64_t)r * pb->row_bytes)) return false;
    return true;
}

// Register the file mapping with HIP once (portable, read-only): from then on tile rows are
// DMA'd from the page cache.  Returns false when the driver refuses (the pread path stays).
static bool ensure_registered(omr_pixel_buffer* pb) {
    if (!pb->map) return false;
    std::lock_guard<std::mutex> g(pb->reg_m);
    if (pb->reg_state == 0) {
        const hipError_t e = hipHostRegister(const_cast<uint8_t*>(pb->map), (size_t)pb->total,
                                             hipHostRegisterPortable | hipHostRegisterReadOnly);
        pb->reg_state = e == hipSuccess ? 1 : -1;
        if (e != hipSuccess) (void)hipGetLastError();
    }
    return pb->reg_state == 1;
}

}  // namespace omr

using namespace omr;

extern "C" {

omr_status omr_pixel_buffer_open(const char* path, int32_t size_x, int32_t size_y, int32_t size_z, int32_t size_c,
                                 int32_t size_t_, int32_t pixel_type, omr_pixel_buffer** out) {
    if (!out) return OMR_INVALID_ARGUMENT;
    *out = nullptr;
    const int bpp = bytes_per_pixel(pixel_type);
    if (!path || !bpp || size_x <= 0 || size_y <= 0 || size_z <= 0 || size_c <= 0 || size_t_ <= 0)
        return OMR_INVALID_ARGUMENT;
    // file size = x * y * z * c * t * bpp: reject dimensions whose product overflows int64
    // (a wrapped size could pass the file-size check below)
    int64_t total = bpp;
    for (const int32_t d : {size_x, size_y, size_z, size_c, size_t_})
        if (__builtin_mul_overflow(total, (int64_t)d, &total)) return OMR_INVALID_ARGUMENT;
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return OMR_NOT_FOUND;
    auto* pb = new omr_pixel_buffer;
    pb->serial = ++g_pixbuf_serial;
    pb->fd = fd;
    pb->sx = size_x; pb->sy = size_y; pb->sz = size_z; pb->sc = size_c; pb->st = size_t_;
    pb->pt = pixel_type;
    pb->bpp = bpp;
    pb->row_bytes = (int64_t)size_x * bpp;
    pb->plane_bytes = pb->row_bytes * size_y;
    pb->total = total;
    struct stat sb;
    if (::fstat(fd, &sb) != 0 || (int64_t)sb.st_size < pb->total) {   // RomioPixelBuffer size check
        ::close(fd);
        delete pb;
        return OMR_INVALID_ARGUMENT;
    }
    if (pb->total <= kMaxRegisterBytes) {
        void* m = ::mmap(nullptr, (size_t)pb->total, PROT_READ, MAP_SHARED, fd, 0);
        if (m != MAP_FAILED) pb->map = static_cast<const uint8_t*>(m);
    }
    *out = pb;
    return OMR_OK;
}

void omr_pixel_buffer_close(omr_pixel_buffer* pb) {
    if (!pb) return;
    if (pb->map) {
        if (pb->reg_state == 1) (void)hipHostUnregister(const_cast<uint8_t*>(pb->map));
        ::munmap(const_cast<uint8_t*>(pb->map), (size_t)pb->total);
    }
    if (pb->fd >= 0) ::close(pb->fd);
    delete pb;
}

int64_t omr_pixel_buffer_plane_offset(const omr_pixel_buffer* pb, int32_t z, int32_t c, int32_t t) {
    if (!pb || !tile_in_bounds(pb, z, c, t, 0, 0, 0, 0)) return -1;
    return plane_offset(pb, z, c, t);
}

omr_status omr_pixel_buffer_get_tile(const omr_pixel_buffer* pb, int32_t z, int32_t c, int32_t t, int32_t x,
                                     int32_t y, int32_t w, int32_t h, void* dst, size_t cap) {
    if (!pb || !dst) return OMR_INVALID_ARGUMENT;
    if (!tile_in_bounds(pb, z, c, t, x, y, w, h)) return OMR_INVALID_ARGUMENT;   // DimensionsOutOfBounds
    if (cap < (size_t)w * h * pb->bpp) return OMR_BUFFER_TOO_SMALL;
    return read_tile(pb, z, c, t, x, y, w, h, static_cast<uint8_t*>(dst)) ? OMR_OK : OMR_INTERNAL;
}

omr_status omr_ctx_set_pixel_buffer_dma(omr_ctx* ctx, int32_t enable) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    ctx->pixbuf_direct = enable != 0;
    return OMR_OK;
}

}  // extern "C"

namespace omr {

omr_status render_pixel_buffer_tiles(omr_ctx* ctx, const omr_pixel_buffer* pb, const omr_quantum_def* qdef,
                                     const omr_channel_binding* channels, int32_t size_c,
                                     const omr_tile_request* reqs, int32_t n, int32_t width, int32_t height,
                                     int32_t flip_h, int32_t flip_v, uint32_t* argb_out, int32_t out_on_device,
                                     int32_t* d_status) {
    if (!ctx) return OMR_INVALID_ARGUMENT;
    if (!pb || !qdef || !channels || !reqs || !argb_out || n < 0) return fail(ctx, OMR_INVALID_ARGUMENT, "null argument");
    if (size_c != pb->sc) return fail(ctx, OMR_INVALID_ARGUMENT, "channel bindings do not match the pixel buffer's sizeC");
    if (width <= 0 || height <= 0) return fail(ctx, OMR_INVALID_ARGUMENT, "bad tile size");
    if (n == 0) return OMR_OK;
    std::vector<int32_t> act;
    for (int c = 0; c < size_c; ++c)
        if (channels[c].active) {
            if (qdef->model == OMR_MODEL_GREYSCALE && !act.empty()) break;   // first active only
            act.push_back(c);
        }
    for (int i = 0; i < n; ++i)
        for (int32_t c : act)
            if (!tile_in_bounds(pb, reqs[i].z, c, reqs[i].t, reqs[i].x, reqs[i].y, width, height))
                return fail(ctx, OMR_INVALID_ARGUMENT, "tile request " + std::to_string(i) + " outside the image");
    OMR_HIP(ctx, hipSetDevice(ctx->device));
    PixPipe* P = nullptr;
    omr_status st = get_pipe(ctx, P);
    if (st) return st;
    const size_t plane = (size_t)width * height * pb->bpp;
    const size_t plane_al = align_up(plane, 256);
    const size_t tile_out = (size_t)width * height * 4;
    const int na = std::max<int>(1, (int)act.size());
    bool host_out = !out_on_device;
    bool out_pinned = false;
    if (host_out) {
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, argb_out) == hipSuccess && attr.type == hipMemoryTypeHost) out_pinned = true;
        (void)hipGetLastError();
    }
    const bool direct = ctx->pixbuf_direct && ensure_registered(const_cast<omr_pixel_buffer*>(pb));
    // Band mode: the tiles of a group that share a row band of one plane -- same z, c, t and y,
    // the neighbouring tiles a viewer asks for together -- come in as one band laid out at the
    // image's full row width: by DMA from the registered mapping, a single contiguous copy when
    // they cover the whole row, else one 2-D copy of their column span; staged, one pread per
    // chunk of rows (or per row of the span) into the pinned slot, then one copy of the slot.
    // K2 reads each tile in place with the image's row stride.  Per-tile mode: one 2-D copy (or
    // one pread per row) of width x height per tile and channel into a compact plane.
    const bool bands = P->bands && (int64_t)pb->sx * pb->bpp == pb->row_bytes;
    const size_t band_bytes = align_up((size_t)height * (size_t)pb->row_bytes, 256);
    const size_t budget = P->group_bytes;   // planes per slot
    struct Band {
        int32_t z, c, t, y, x0, x1;
    };
    // groups: [start, end) tile ranges, slot g & 1; per-tile-channel band index (band mode)
    std::vector<int> gstart;
    std::vector<int32_t> tile_band((size_t)n * na, -1);
    std::vector<std::vector<Band>> gbands;
    size_t in_need = 0;
    int gmax = 1;
    if (bands) {
        const size_t cap = std::max(budget, band_bytes * (size_t)na);
        std::vector<int32_t> hit(act.size());
        for (int i = 0; i < n;) {
            gstart.push_back(i);
            std::vector<Band> bl;
            const int i0 = i;
            for (; i < n; ++i) {
                const omr_tile_request& r = reqs[i];
                int fresh = 0;
                for (int a = 0; a < (int)act.size(); ++a) {
                    hit[a] = -1;
                    for (size_t k = 0; k < bl.size(); ++k)
                        if (bl[k].z == r.z && bl[k].c == act[a] && bl[k].t == r.t && bl[k].y == r.y) { hit[a] = (int32_t)k; break; }
                    fresh += hit[a] < 0;
                }
                if (i > i0 && (bl.size() + fresh) * band_bytes > cap) break;
                for (int a = 0; a < (int)act.size(); ++a) {
                    if (hit[a] < 0) {
                        hit[a] = (int32_t)bl.size();
                        bl.push_back(Band{r.z, act[a], r.t, r.y, r.x, r.x + width});
                    } else {
                        Band& b = bl[hit[a]];
                        b.x0 = std::min(b.x0, r.x);
                        b.x1 = std::max(b.x1, r.x + width);
                    }
                    tile_band[(size_t)i * na + a] = hit[a];
                }
            }
            // slots in file order, so bands adjacent in the file (the same plane's consecutive
            // row bands, or whole planes) are adjacent in the slot too and go as one copy
            std::vector<int32_t> ord(bl.size()), pos(bl.size());
            for (size_t k = 0; k < bl.size(); ++k) ord[k] = (int32_t)k;
            auto foff = [&](const Band& b) { return plane_offset(pb, b.z, b.c, b.t) + (int64_t)b.y * pb->row_bytes; };
            std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return foff(bl[a]) < foff(bl[b]); });
            std::vector<Band> sorted(bl.size());
            for (size_t k = 0; k < bl.size(); ++k) { sorted[k] = bl[ord[k]]; pos[ord[k]] = (int32_t)k; }
            for (int t = i0; t < i; ++t)
                for (int a = 0; a < (int)act.size(); ++a) tile_band[(size_t)t * na + a] = pos[tile_band[(size_t)t * na + a]];
            gmax = std::max(gmax, i - i0);
            in_need = std::max(in_need, sorted.size() * band_bytes);
            gbands.push_back(std::move(sorted));
        }
    } else {
        // ~64 MiB of compact planes per slot
        const int G = (int)std::max<size_t>(1, std::min<size_t>((size_t)n, budget / (plane_al * na)));
        for (int i = 0; i < n; i += G) gstart.push_back(i);
        gmax = G;
        in_need = plane_al * (size_t)G * na;
    }
    const int ngroups = (int)gstart.size();
    gstart.push_back(n);
    const size_t tab_bytes = align_up(sizeof(void*) * (size_t)gmax * size_c, 256);
    st = grow(ctx, P, tab_bytes + in_need, tile_out * gmax, host_out && !out_pinned);
    if (st) return st;
    std::atomic<bool> io_error{false};
    auto finish_host = [&](int g) -> omr_status {   // bounce slot -> caller (pageable output)
        const int s = g & 1, t0 = gstart[g], cnt = gstart[g + 1] - t0;
        OMR_HIP(ctx, hipEventSynchronize(P->d2h[s]));
        const uint8_t* src = static_cast<const uint8_t*>(P->pin_out[s]);
        uint8_t* dst = reinterpret_cast<uint8_t*>(argb_out) + (size_t)t0 * tile_out;
        const size_t total = tile_out * (size_t)cnt, piece = 1 << 20;
        const int pieces = (int)((total + piece - 1) / piece);
        P->pool.run(pieces, [&](int i) {
            const size_t o = (size_t)i * piece;
            std::memcpy(dst + o, src + o, std::min(piece, total - o));
        });
        return OMR_OK;
    };
    for (int g = 0; g < ngroups; ++g) {
        const int s = g & 1, t0 = gstart[g], cnt = gstart[g + 1] - t0;
        // pinned slot s is free again (also across calls: a call with per-tile statuses returns
        // without a final sync; an event never recorded completes at once)
        OMR_HIP(ctx, hipEventSynchronize(P->h2d[s]));
        uint8_t* hin = static_cast<uint8_t*>(P->pin_in[s]);
        uint8_t* din = static_cast<uint8_t*>(P->d_in[s]);
        const void** tab = reinterpret_cast<const void**>(hin);
        for (int i = 0; i < cnt; ++i)
            for (int c = 0; c < size_c; ++c) tab[(size_t)i * size_c + c] = nullptr;
        for (int i = 0; i < cnt; ++i)
            for (int a = 0; a < (int)act.size(); ++a)
                tab[(size_t)i * size_c + act[a]] =
                    bands ? din + tab_bytes + band_bytes * (size_t)tile_band[(size_t)(t0 + i) * na + a] +
                                (size_t)reqs[t0 + i].x * pb->bpp
                          : din + tab_bytes + plane_al * ((size_t)i * na + a);
        if (!direct && bands) {
            // file -> pinned, one job per 64 rows of a band: whole rows in one pread when the
            // band's tiles cover them, else one pread per row of the column span
            const std::vector<Band>& bl = gbands[g];
            constexpr int kRows = 64;
            const int chunks = (height + kRows - 1) / kRows;
            P->pool.run((int)bl.size() * chunks, [&](int j) {
                const Band& b = bl[j / chunks];
                const int r0 = (j % chunks) * kRows, r1 = std::min(height, r0 + kRows);
                const int64_t src = plane_offset(pb, b.z, b.c, b.t) + (int64_t)(b.y + r0) * pb->row_bytes;
                uint8_t* dst = hin + tab_bytes + band_bytes * (size_t)(j / chunks) + (size_t)r0 * pb->row_bytes;
                if (b.x0 == 0 && b.x1 == pb->sx) {
                    if (!read_full(pb->fd, dst, (size_t)(r1 - r0) * pb->row_bytes, src)) io_error = true;
                    return;
                }
                const size_t off = (size_t)b.x0 * pb->bpp, seg = (size_t)(b.x1 - b.x0) * pb->bpp;
                for (int r = 0; r < r1 - r0; ++r)
                    if (!read_full(pb->fd, dst + (size_t)r * pb->row_bytes + off, seg,
                                   src + (int64_t)r * pb->row_bytes + (int64_t)off)) { io_error = true; return; }
            });
            if (io_error) return fail(ctx, OMR_INTERNAL, "pixel buffer read failed");
        } else if (!direct) {
            P->pool.run(cnt * (int)act.size(), [&](int j) {   // file -> pinned, one tile-channel plane per job
                const int i = j / (int)act.size(), a = j % (int)act.size();
                const omr_tile_request& r = reqs[t0 + i];
                uint8_t* dst = hin + tab_bytes + plane_al * ((size_t)i * na + a);
                if (!read_tile(pb, r.z, act[a], r.t, r.x, r.y, width, height, dst)) io_error = true;
            });
            if (io_error) return fail(ctx, OMR_INTERNAL, "pixel buffer read failed");
        }
        OMR_HIP(ctx, hipStreamWaitEvent(P->copy, P->rend[s], 0));   // device slot s is free (this or a past call)
        if (P->copy_b) OMR_HIP(ctx, hipStreamWaitEvent(P->copy_b, P->rend[s], 0));
        if (bands && !direct) {
            OMR_HIP(ctx, hipMemcpyAsync(din, hin, tab_bytes + band_bytes * gbands[g].size(), hipMemcpyHostToDevice,
                                        P->copy));
        } else if (bands) {
            OMR_HIP(ctx, hipMemcpyAsync(din, hin, tab_bytes, hipMemcpyHostToDevice, P->copy));
            const std::vector<Band>& bl = gbands[g];
            const size_t hb = (size_t)height * pb->row_bytes;
            auto full = [&](const Band& b) { return b.x0 == 0 && b.x1 == pb->sx; };
            for (size_t k = 0; k < bl.size();) {
                const Band& b = bl[k];
                const int64_t fo = plane_offset(pb, b.z, b.c, b.t) + (int64_t)b.y * pb->row_bytes;
                const uint8_t* src = pb->map + fo;
                uint8_t* dst = din + tab_bytes + band_bytes * k;
                hipStream_t cs = (P->copy_b && (k & 1)) ? P->copy_b : P->copy;
                if (full(b)) {   // the tiles cover the row: the band is contiguous, and so is a run of
                                 // whole bands that follow each other in the file and in the slot
                    size_t e = k + 1;
                    while (e < bl.size() && band_bytes == hb && full(bl[e]) &&
                           plane_offset(pb, bl[e].z, bl[e].c, bl[e].t) + (int64_t)bl[e].y * pb->row_bytes ==
                               fo + (int64_t)(hb * (e - k)))
                        ++e;
                    OMR_HIP(ctx, hipMemcpyAsync(dst, src, hb * (e - k), hipMemcpyHostToDevice, cs));
                    k = e;
                    continue;
                } else
                    OMR_HIP(ctx, hipMemcpy2DAsync(dst + (size_t)b.x0 * pb->bpp, (size_t)pb->row_bytes,
                                                  src + (size_t)b.x0 * pb->bpp, (size_t)pb->row_bytes,
                                                  (size_t)(b.x1 - b.x0) * pb->bpp, (size_t)height,
                                                  hipMemcpyHostToDevice, cs));
                ++k;
            }
        } else if (direct) {
            // registered mapping: the copy engine reads each tile's rows from the page cache
            OMR_HIP(ctx, hipMemcpyAsync(din, hin, tab_bytes, hipMemcpyHostToDevice, P->copy));
            for (int i = 0; i < cnt; ++i) {
                const omr_tile_request& r = reqs[t0 + i];
                for (int a = 0; a < (int)act.size(); ++a) {
                    const uint8_t* src = pb->map + plane_offset(pb, r.z, act[a], r.t) + (int64_t)r.y * pb->row_bytes +
                                         (int64_t)r.x * pb->bpp;
                    // tile-channel planes alternate between the copy queues when there are two
                    hipStream_t cs = (P->copy_b && ((i * na + a) & 1)) ? P->copy_b : P->copy;
                    OMR_HIP(ctx, hipMemcpy2DAsync(din + tab_bytes + plane_al * ((size_t)i * na + a),
                                                  (size_t)width * pb->bpp, src, (size_t)pb->row_bytes,
                                                  (size_t)width * pb->bpp, (size_t)height, hipMemcpyHostToDevice,
                                                  cs));
                }
            }
        } else {
            OMR_HIP(ctx, hipMemcpyAsync(din, hin, tab_bytes + plane_al * (size_t)cnt * na, hipMemcpyHostToDevice,
                                        P->copy));
        }
        OMR_HIP(ctx, hipEventRecord(P->h2d[s], P->copy));
        OMR_HIP(ctx, hipStreamWaitEvent(ctx->stream, P->h2d[s], 0));
        if (P->copy_b) {
            OMR_HIP(ctx, hipEventRecord(P->h2d_b[s], P->copy_b));
            OMR_HIP(ctx, hipStreamWaitEvent(ctx->stream, P->h2d_b[s], 0));
        }
        uint32_t* dout = out_on_device ? argb_out + (size_t)t0 * width * height : static_cast<uint32_t*>(P->d_out[s]);
        st = omr_render_batch_device(ctx, qdef, channels, size_c, reinterpret_cast<const void* const*>(din), cnt,
                                     bands ? (int64_t)pb->sx : 0, pb->pt, 1, width, height, flip_h, flip_v, dout,
                                     d_status ? d_status + t0 : nullptr);
        if (st) return st;
        OMR_HIP(ctx, hipEventRecord(P->rend[s], ctx->stream));
        if (host_out) {
            void* dst = out_pinned ? static_cast<void*>(reinterpret_cast<uint8_t*>(argb_out) + (size_t)t0 * tile_out)
                                   : P->pin_out[s];
            OMR_HIP(ctx, hipMemcpyAsync(dst, dout, tile_out * (size_t)cnt, hipMemcpyDeviceToHost, ctx->stream));
            OMR_HIP(ctx, hipEventRecord(P->d2h[s], ctx->stream));
            if (!out_pinned && g >= 1) {
                st = finish_host(g - 1);
                if (st) return st;
            }
        }
    }
    if (host_out && !out_pinned) {
        st = finish_host(ngroups - 1);
        if (st) return st;
    }
    if (d_status && !host_out) {
        // per-tile statuses carry the QuantizationException; the caller (the batcher) encodes on
        // the same stream and syncs once after that.  The sticky flag is cleared behind the render.
        OMR_HIP(ctx, launch_flag_out(ctx->stream, ctx->d_flag, ctx->h_flag));
        return OMR_OK;
    }
    st = omr_ctx_synchronize(ctx);
    // with per-tile statuses the QuantizationException belongs to the flagged tiles only
    if (st == OMR_QUANTIZATION && d_status) st = OMR_OK;
    return st;
}

// Geometry of an open pixel buffer (the batcher's projection jobs render the full plane).
void pixel_buffer_dims(const omr_pixel_buffer* pb, int32_t dims[6]) {
    dims[0] = pb->sx; dims[1] = pb->sy; dims[2] = pb->sz; dims[3] = pb->sc; dims[4] = pb->st; dims[5] = pb->pt;
}

uint64_t pixel_buffer_serial(const omr_pixel_buffer* pb) { return pb->serial; }

// The whole Z-stack of (c, t) -- sizeZ planes, contiguous in the ROMIO layout -- into device memory
// at d_dst, on ctx's stream: a DMA from the registered mapping, else pread into pinned staging
// (synchronous).  What ProjectionService reads plane by plane (ProjectionService.java:176-291).
omr_status pixel_buffer_upload_stack(omr_ctx* ctx, const omr_pixel_buffer* pb, int32_t c, int32_t t, void* d_dst) {
    if (!tile_in_bounds(pb, 0, c, t, 0, 0, 0, 0)) return fail(ctx, OMR_INVALID_ARGUMENT, "stack outside the image");
    const int64_t off = plane_offset(pb, 0, c, t), bytes = pb->plane_bytes * pb->sz;
    if (ctx->pixbuf_direct && ensure_registered(const_cast<omr_pixel_buffer*>(pb))) {
        OMR_HIP(ctx, hipMemcpyAsync(d_dst, pb->map + off, (size_t)bytes, hipMemcpyHostToDevice, ctx->stream));
        return OMR_OK;
    }
    PixPipe* P = nullptr;
    omr_status st = get_pipe(ctx, P);
    if (st) return st;
    st = grow(ctx, P, (size_t)bytes, 0, false);
    if (st) return st;
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));          // the staging slot is free
    if (!read_full(pb->fd, P->pin_in[0], (size_t)bytes, off)) return fail(ctx, OMR_INTERNAL, "pixel buffer read failed");
    OMR_HIP(ctx, hipMemcpyAsync(d_dst, P->pin_in[0], (size_t)bytes, hipMemcpyHostToDevice, ctx->stream));
    OMR_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return OMR_OK;
}

}  // namespace omr

extern "C" omr_status omr_render_pixel_buffer_tiles(omr_ctx* ctx, const omr_pixel_buffer* pb,
                                                    const omr_quantum_def* qdef, const omr_channel_binding* channels,
                                                    int32_t size_c, const omr_tile_request* reqs, int32_t n,
                                                    int32_t width, int32_t height, int32_t flip_h, int32_t flip_v,
                                                    uint32_t* argb_out, int32_t out_on_device) {
    return omr::render_pixel_buffer_tiles(ctx, pb, qdef, channels, size_c, reqs, n, width, height, flip_h, flip_v,
                                          argb_out, out_on_device, nullptr);
}
