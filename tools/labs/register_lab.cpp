// What page-locking the caller's own pageable array would cost, against the
// staging ring's two CPU copies (DESIGN.md §6 "Host-resident"): hipHostRegister
// / hipHostUnregister per chunk of an already-touched malloc'd array, and the
// DMA rate out of and into such chunks.  A host-only lab (no kernel).
//
//   register_lab [MiB per array, default 256]
#include <hip/hip_runtime.h>

#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 256;
    const size_t bytes = mib << 20;
    char *src = static_cast<char *>(std::aligned_alloc(4096, bytes));
    char *tgt = static_cast<char *>(std::aligned_alloc(4096, bytes));
    std::memset(src, 1, bytes);
    std::memset(tgt, 2, bytes);
    void *dev = nullptr;
    CK(hipMalloc(&dev, bytes));
    hipStream_t h2d, d2h;
    CK(hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking));

    for (size_t chunk_mib : {4, 16, 64, 256}) {
        const size_t chunk = std::min(bytes, chunk_mib << 20);
        for (int rep = 0; rep < 3; ++rep) {
            double reg = 0, unreg = 0;
            for (size_t off = 0; off < bytes; off += chunk) {
                const size_t n = std::min(chunk, bytes - off);
                double t0 = now_s();
                CK(hipHostRegister(src + off, n, hipHostRegisterDefault));
                double t1 = now_s();
                CK(hipHostUnregister(src + off));
                double t2 = now_s();
                reg += t1 - t0;
                unreg += t2 - t1;
            }
            std::printf("register chunk %4zu MiB: register %7.2f GB/s (%.2f ms per %zu MiB), unregister %7.2f GB/s\n",
                        chunk_mib, bytes / reg / 1e9, reg * 1e3, mib, bytes / unreg / 1e9);
        }
    }
    // DMA straight from / into registered chunks, one direction at a time and
    // both at once (the staging path's pinned rate is the bound)
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipHostRegister(src, bytes, hipHostRegisterDefault));
        CK(hipHostRegister(tgt, bytes, hipHostRegisterDefault));
        double t0 = now_s();
        CK(hipMemcpyAsync(dev, src, bytes, hipMemcpyHostToDevice, h2d));
        CK(hipStreamSynchronize(h2d));
        double t1 = now_s();
        CK(hipMemcpyAsync(tgt, dev, bytes, hipMemcpyDeviceToHost, d2h));
        CK(hipStreamSynchronize(d2h));
        double t2 = now_s();
        std::printf("registered whole: H2D %.1f GB/s, D2H %.1f GB/s\n", bytes / (t1 - t0) / 1e9,
                    bytes / (t2 - t1) / 1e9);
        CK(hipHostUnregister(src));
        CK(hipHostUnregister(tgt));
    }
    // the per-call scheme: register each 16 MiB chunk of source and target,
    // H2D, D2H behind it, unregister when its copies are done; end to end
    const size_t chunk = std::min(bytes, size_t(16) << 20);
    const size_t nch = (bytes + chunk - 1) / chunk;
    std::vector<hipEvent_t> ev(2 * nch);
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (int rep = 0; rep < 5; ++rep) {
        double t0 = now_s();
        for (size_t k = 0; k < nch; ++k) {
            const size_t off = k * chunk, n = std::min(chunk, bytes - off);
            CK(hipHostRegister(src + off, n, hipHostRegisterDefault));
            CK(hipHostRegister(tgt + off, n, hipHostRegisterDefault));
            CK(hipMemcpyAsync(static_cast<char *>(dev) + off, src + off, n, hipMemcpyHostToDevice, h2d));
            CK(hipEventRecord(ev[2 * k], h2d));
            CK(hipStreamWaitEvent(d2h, ev[2 * k], 0));
            CK(hipMemcpyAsync(tgt + off, static_cast<char *>(dev) + off, n, hipMemcpyDeviceToHost, d2h));
            CK(hipEventRecord(ev[2 * k + 1], d2h));
            if (k >= 2) {
                const size_t j = k - 2, oj = j * chunk;
                CK(hipEventSynchronize(ev[2 * j + 1]));
                CK(hipHostUnregister(src + oj));
                CK(hipHostUnregister(tgt + oj));
            }
        }
        for (size_t j = nch >= 2 ? nch - 2 : 0; j < nch; ++j) {
            CK(hipEventSynchronize(ev[2 * j + 1]));
            CK(hipHostUnregister(src + j * chunk));
            CK(hipHostUnregister(tgt + j * chunk));
        }
        double t1 = now_s();
        std::printf("register-per-chunk pipeline (16 MiB): %.2f ms, %.1f GiB/s of the array\n", (t1 - t0) * 1e3,
                    bytes / (t1 - t0) / (1 << 30));
    }
    // the per-call scheme with whole arrays: register source and target
    // (page-rounded), the chunked H2D / D2H pipeline, unregister; 8 calls on
    // the same arrays
    for (int rep = 0; rep < 8; ++rep) {
        double t0 = now_s();
        CK(hipHostRegister(src, bytes, hipHostRegisterDefault));
        CK(hipHostRegister(tgt, bytes, hipHostRegisterDefault));
        double t1 = now_s();
        for (size_t k = 0; k < nch; ++k) {
            const size_t off = k * chunk, n = std::min(chunk, bytes - off);
            CK(hipMemcpyAsync(static_cast<char *>(dev) + off, src + off, n, hipMemcpyHostToDevice, h2d));
            CK(hipEventRecord(ev[2 * k], h2d));
            CK(hipStreamWaitEvent(d2h, ev[2 * k], 0));
            CK(hipMemcpyAsync(tgt + off, static_cast<char *>(dev) + off, n, hipMemcpyDeviceToHost, d2h));
        }
        CK(hipStreamSynchronize(d2h));
        double t2 = now_s();
        CK(hipHostUnregister(src));
        CK(hipHostUnregister(tgt));
        double t3 = now_s();
        std::printf("register-whole per call: register %.3f ms, copies %.2f ms, unregister %.3f ms: %.1f GiB/s\n",
                    (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, bytes / (t3 - t0) / (1 << 30));
    }
    // stale pages: a registered, DMA'd, unregistered and unmapped array whose
    // address range a new mapping (other bytes) takes next must DMA the new
    // bytes, not the old pages'
    bool stale_ok = true;
    void *last = nullptr;
    int reused = 0;
    char *chk = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&chk), 4096, hipHostMallocDefault));
    for (int rep = 0; rep < 6; ++rep) {
        char *p = static_cast<char *>(mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
        if (p == MAP_FAILED) return 2;
        reused += p == last;
        std::memset(p, 0x40 + rep, bytes);
        CK(hipHostRegister(p, bytes, hipHostRegisterDefault));
        CK(hipMemcpyAsync(dev, p, bytes, hipMemcpyHostToDevice, h2d));
        CK(hipStreamSynchronize(h2d));
        CK(hipHostUnregister(p));
        for (size_t off : {size_t(0), bytes / 2, bytes - 4096}) {
            CK(hipMemcpy(chk, static_cast<char *>(dev) + off, 4096, hipMemcpyDeviceToHost));
            for (int i = 0; i < 4096; ++i) stale_ok &= chk[i] == (char)(0x40 + rep);
        }
        munmap(p, bytes);
        last = p;
    }
    std::printf("remapped ranges: %d of 5 at the same address; DMA read the new bytes: %s\n", reused,
                stale_ok ? "yes" : "NO (stale pages)");
    bool ok = stale_ok;
    for (size_t i = 0; i < bytes; i += 4093) ok &= tgt[i] == 1;
    std::printf("target holds the source: %s\n", ok ? "yes" : "NO");
    return ok ? 0 : 1;
}
