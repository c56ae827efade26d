// PCIe host -> HBM probe for the host-fed path: what the copy engines sustain for
// the transfer shapes omr_render_pixel_buffer_tiles issues.  Sources: pinned host memory
// (hipHostMalloc) and a tmpfs file mapped read-only and registered with HIP (the ROMIO path).
// Shapes: one contiguous copy; 2-D tile-channel rects (2 KiB rows of an 8 KiB image row, the C2
// tile of a 4096-wide u16 plane); full-width band rects (8 KiB rows).  One JSON line.
// Build: hipcc -O2 tools/pcie_probe.cpp -o tools/pcie_probe
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
            std::exit(1);                                                     \
        }                                                                     \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// GB/s of `reps` rounds of `fn` (each round moves `bytes`), after one warm round.
template <typename F>
static double rate(hipStream_t s, size_t bytes, int reps, F fn) {
    fn();
    CK(hipStreamSynchronize(s));
    const double t0 = now();
    for (int r = 0; r < reps; ++r) fn();
    CK(hipStreamSynchronize(s));
    return (double)bytes * reps / (now() - t0) / 1e9;
}

int main(int argc, char** argv) {
    const size_t W = 4096 * 2, H = 4096;            // one 4096 x 4096 u16 plane: 32 MiB
    const int planes = 4;                           // 128 MiB, the bench's ROMIO image
    const size_t total = W * H * planes;
    const char* dir = argc > 1 ? argv[1] : "/dev/shm";
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    void* dev = nullptr;
    CK(hipMalloc(&dev, total));
    void* pin = nullptr;
    CK(hipHostMalloc(&pin, total, hipHostMallocDefault));
    std::memset(pin, 1, total);
    // tmpfs file, mapped and registered as the pixel buffer does
    std::string path = std::string(dir) + "/omr_pcie_probe_XXXXXX";
    std::vector<char> p(path.begin(), path.end());
    p.push_back(0);
    const int fd = mkstemp(p.data());
    if (fd < 0) { std::perror("mkstemp"); return 1; }
    if (ftruncate(fd, (off_t)total) != 0) { std::perror("ftruncate"); return 1; }
    {
        std::vector<char> buf(1 << 20, 2);
        for (size_t o = 0; o < total; o += buf.size())
            if (pwrite(fd, buf.data(), buf.size(), (off_t)o) != (ssize_t)buf.size()) { std::perror("pwrite"); return 1; }
    }
    void* map = mmap(nullptr, total, PROT_READ, MAP_SHARED, fd, 0);
    if (map == MAP_FAILED) { std::perror("mmap"); return 1; }
    const bool reg = hipHostRegister(map, total, hipHostRegisterPortable | hipHostRegisterReadOnly) == hipSuccess;
    (void)hipGetLastError();
    std::printf("{\"bytes\": %zu", total);
    struct Src { const char* name; const uint8_t* p; };
    std::vector<Src> srcs = {{"pinned", (const uint8_t*)pin}};
    if (reg) srcs.push_back({"registered_tmpfs_mmap", (const uint8_t*)map});
    for (const Src& src : srcs) {
        const double contig = rate(s, total, 4, [&] { CK(hipMemcpyAsync(dev, src.p, total, hipMemcpyHostToDevice, s)); });
        // 2-D tile-channel rects: 1024 rows of 2 KiB (1024 u16 pixels) out of 8 KiB image rows
        const size_t tw = 1024 * 2, th = 1024;
        const int ntile = (int)(total / (tw * th));
        const double rect = rate(s, total, 4, [&] {
            for (int k = 0; k < ntile; ++k) {
                const int pl = k / 16, ty = (k % 16) / 4, tx = k % 4;
                const uint8_t* sp = src.p + (size_t)pl * W * H + (size_t)ty * th * W + (size_t)tx * tw;
                CK(hipMemcpy2DAsync((uint8_t*)dev + (size_t)k * tw * th, tw, sp, W, tw, th, hipMemcpyHostToDevice, s));
            }
        });
        // full-width bands: 1024 rows of 8 KiB (four tiles' rows at once)
        const int nband = (int)(total / (W * th));
        const double band = rate(s, total, 4, [&] {
            for (int k = 0; k < nband; ++k)
                CK(hipMemcpy2DAsync((uint8_t*)dev + (size_t)k * W * th, W, src.p + (size_t)k * W * th, W, W, th,
                                    hipMemcpyHostToDevice, s));
        });
        std::printf(", \"%s\": {\"contiguous_gbs\": %.2f, \"tile_rect_2KiB_rows_gbs\": %.2f, \"band_rect_8KiB_rows_gbs\": %.2f}",
                    src.name, contig, rect, band);
    }
    std::printf(", \"registered\": %s}\n", reg ? "true" : "false");
    if (reg) (void)hipHostUnregister(map);
    munmap(map, total);
    close(fd);
    unlink(p.data());
    (void)hipHostFree(pin);
    (void)hipFree(dev);
    return 0;
}
