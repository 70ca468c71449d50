// What a blocking call on the mirrored heap pays for besides its kernel
// (the ISx round of profiles/r04_isx_mirror.txt): the page
// protection changes of a 64 KiB block, and the ways to move a host-written
// block to HBM ahead of a kernel on the same stream.  Medians over `reps`, us.
//
//   mprotect_*   one mprotect of a 64 KiB block of a 4 KiB-page mapping, in a
//                process whose HIP runtime is up (its threads share the mm,
//                so a permission cut costs a TLB shoot-down)
//   seq_*        one host-synchronised sequence on one stream:
//                kernel          a one-workgroup kernel, then hipStreamSynchronize
//                dma64k_kernel   hipMemcpyAsync H2D of a 64 KiB page-locked block, the kernel
//                copy64k_kernel  a one-workgroup kernel copying the block from its
//                                device-mapped host address (system-scope acquire
//                                first), the kernel
//                dma8_kernel     the same with an 8-byte DMA
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/mirror_cost_probe.hip -o tools/mirror_cost_probe
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void tiny_kernel(unsigned long long *p) {
    if (threadIdx.x == 0) p[0] += 1;
}

// 64 KiB = 4096 vectors, 16 per lane, all loads issued before any store
__global__ __launch_bounds__(256) void copy_from_host(u32x4 *dst, const u32x4 *src) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope: drop stale lines
    u32x4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = __builtin_nontemporal_load(src + threadIdx.x + k * 256);
#pragma unroll
    for (int k = 0; k < 16; ++k) dst[threadIdx.x + k * 256] = v[k];
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 2000;
    const size_t kBlk = 64 << 10;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned long long *dcount;
    CK(hipMalloc(&dcount, 64));
    CK(hipMemset(dcount, 0, 64));
    tiny_kernel<<<1, 256, 0, s>>>(dcount);
    CK(hipStreamSynchronize(s));

    // page-protection changes on a 64 KiB block
    char *view = static_cast<char *>(mmap(nullptr, 64 * kBlk, PROT_READ | PROT_WRITE,
                                          MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
    if (view == MAP_FAILED) return 1;
    std::memset(view, 1, 64 * kBlk);
    std::vector<double> t_none, t_read, t_rw;
    for (int r = 0; r < reps; ++r) {
        char *b = view + (r % 64) * kBlk;
        double t0 = now_us();
        mprotect(b, kBlk, PROT_READ);              // RW -> R: a cut
        double t1 = now_us();
        mprotect(b, kBlk, PROT_NONE);              // R -> none: a cut
        double t2 = now_us();
        mprotect(b, kBlk, PROT_READ | PROT_WRITE); // none -> RW: a grant
        double t3 = now_us();
        b[0] = (char)r;                             // the pages are touched again
        t_read.push_back(t1 - t0);
        t_none.push_back(t2 - t1);
        t_rw.push_back(t3 - t2);
    }
    std::printf("{\"probe\": \"mprotect_64KiB\", \"rw_to_read_us\": %.2f, \"read_to_none_us\": %.2f, "
                "\"none_to_rw_us\": %.2f}\n", median(t_read), median(t_none), median(t_rw));

    // host block, page-locked, and its device address
    char *host = static_cast<char *>(std::aligned_alloc(kBlk, 64 * kBlk));
    std::memset(host, 2, 64 * kBlk);
    CK(hipHostRegister(host, 64 * kBlk, hipHostRegisterDefault));
    void *host_dev = nullptr;
    CK(hipHostGetDevicePointer(&host_dev, host, 0));
    char *hbm;
    CK(hipMalloc(&hbm, 64 * kBlk));

    auto seq = [&](const char *name, int mode) {
        std::vector<double> t;
        for (int r = 0; r < reps + 20; ++r) {
            const size_t o = (r % 64) * kBlk;
            host[o] = (char)r;                     // the host's store into the block
            double t0 = now_us();
            if (mode == 1) CK(hipMemcpyAsync(hbm + o, host + o, kBlk, hipMemcpyHostToDevice, s));
            if (mode == 2)
                copy_from_host<<<1, 256, 0, s>>>(reinterpret_cast<u32x4 *>(hbm + o),
                                                  reinterpret_cast<const u32x4 *>(static_cast<char *>(host_dev) + o));
            if (mode == 3) CK(hipMemcpyAsync(hbm + o, host + o, 8, hipMemcpyHostToDevice, s));
            tiny_kernel<<<1, 256, 0, s>>>(dcount);
            CK(hipStreamSynchronize(s));
            double t1 = now_us();
            if (r >= 20) t.push_back(t1 - t0);
            if (mode && r % 97 == 0) {             // the block reached HBM with the host's byte
                char got = 0;
                CK(hipMemcpy(&got, hbm + o, 1, hipMemcpyDeviceToHost));
                if (got != (char)r) {
                    std::printf("{\"probe\": \"%s\", \"error\": \"stale byte at rep %d\"}\n", name, r);
                    std::exit(2);
                }
            }
        }
        std::printf("{\"probe\": \"seq_%s\", \"median_us\": %.2f}\n", name, median(t));
    };
    seq("kernel", 0);
    seq("dma64k_kernel", 1);
    seq("copy64k_kernel", 2);
    seq("dma8_kernel", 3);
    seq("kernel", 0);
    CK(hipHostUnregister(host));
    return 0;
}
