// Probe: can two processes on one GPU map each other's hipMalloc memory via
// hipIpc handles (dmabuf mode), and read/write it from kernels?
//   ./ipc_probe <pe> <npes> <shmfile>
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "pe %d: %s failed: %s\n", pe, #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Slot { hipIpcMemHandle_t h; std::atomic<long> ready; };
struct Shm { std::atomic<long> arrive; Slot slot[16]; };

__global__ void fill(double *p, size_t n, double v) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) p[i] = v + (double)i;
}
__global__ void sum_peers(double *out, double *const *ins, int nin, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    double r = ins[0][i];
    for (int j = 1; j < nin; ++j) r += ins[j][i];
    out[i] = r;
}

static void barrier(Shm *s, int npes, long &epoch) {
    epoch += npes;
    s->arrive.fetch_add(1);
    auto t0 = std::chrono::steady_clock::now();
    while (s->arrive.load() < epoch) {
        std::this_thread::yield();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) { fprintf(stderr, "barrier timeout\n"); exit(3); }
    }
}

int main(int argc, char **argv) {
    int pe = atoi(argv[1]), npes = atoi(argv[2]);
    int fd = open(argv[3], O_RDWR | O_CREAT, 0600);
    if (ftruncate(fd, sizeof(Shm)) != 0) return 2;
    Shm *s = (Shm *)mmap(nullptr, sizeof(Shm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    long epoch = 0;
    const size_t n = 1 << 24;
    double *buf;
    CK(hipSetDevice(0));
    CK(hipMalloc(&buf, n * 8));
    hipLaunchKernelGGL(fill, dim3(n / 256), dim3(256), 0, 0, buf, n, 1000.0 * pe);
    CK(hipDeviceSynchronize());
    CK(hipIpcGetMemHandle(&s->slot[pe].h, buf));
    s->slot[pe].ready.store(1);
    barrier(s, npes, epoch);
    double *peers[16];
    for (int q = 0; q < npes; ++q) {
        if (q == pe) { peers[q] = buf; continue; }
        void *p = nullptr;
        CK(hipIpcOpenMemHandle(&p, s->slot[q].h, hipIpcMemLazyEnablePeerAccess));
        peers[q] = (double *)p;
    }
    double **dpeers, *out;
    CK(hipMalloc(&dpeers, sizeof peers));
    CK(hipMemcpy(dpeers, peers, sizeof peers, hipMemcpyHostToDevice));
    CK(hipMalloc(&out, n * 8));
    auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(sum_peers, dim3(n / 256), dim3(256), 0, 0, out, dpeers, npes, n);
    CK(hipDeviceSynchronize());
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    double *h = (double *)malloc(n * 8);
    CK(hipMemcpy(h, out, n * 8, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) {
        double e = 0;
        for (int q = 0; q < npes; ++q) e += 1000.0 * q + (double)i;
        if (h[i] != e) ++bad;
    }
    barrier(s, npes, epoch);   // peers done reading my buffer
    for (int q = 0; q < npes; ++q) if (q != pe) CK(hipIpcCloseMemHandle(peers[q]));
    printf("pe %d/%d: bad=%zu kernel %.1f us\n", pe, npes, bad, us);
    barrier(s, npes, epoch);
    if (pe == 0) unlink(argv[3]);
    return bad ? 4 : 0;
}
