// Position-aware 64-bit checksum of a reduction result, on gfx950.
//
// Why: every member of an active set must end a reduction with the same
// target (A2A and RCCL algorithms), so a checksum per PE compared across the
// set verifies a whole multi-GPU result with 8 bytes of traffic per PE — the
// "checksum of checksums" property the parity tests use at full size, and an
// integrity check (SHMEM_LOG / shmemx_verify) where the reference has only a
// stub failure-detection story.
//
// Definition (host twin in tests/gpu_util.py::checksum64): the bytes of the
// n elements, long double slots reduced to their 10 value bytes and zero
// padded to 16, read as little-endian u64 words w_j (the last word zero
// padded), H = XOR_j mix(w_j + (j + 1) * 0x9E3779B97F4A7C15) with mix the
// splitmix64 finaliser.  XOR makes it order-free (any grid), the index makes
// it position-aware.
//
// Kernel shape: 16-byte loads per lane (2 words), a per-lane XOR, a wave XOR
// reduction by DPP within 16-lane rows and v_readlane across rows, the 4 wave
// partials combined in LDS, one partial per workgroup in its own slot, and the
// LAST workgroup to finish XORs the partials (same DPP + LDS reduction) and
// stores the result where the caller asked — host-mapped memory included, so
// the host reads it after the stream wait with no copy command.  One launch:
// round 2's separate one-workgroup finish kernel and the 8-byte D2H copy cost
// about 25 us per call over the 41 us of streaming.
//
// The hand-off of the partials to the last workgroup follows the guide's
// measured form (MI355X_MICROARCH.md, "inter-workgroup visibility", the sc1
// table): ONE lane per workgroup stores its partial with an agent-scope (sc1,
// write-through) store, waits for it (vmcnt(0)), then adds to an agent-scope
// arrival counter; the workgroup whose add returns the last count goes on.
// No per-workgroup release fence (an L2 write-back in each of 4096 blocks).
// The counter is sharded: 4096 adds to ONE address serialise at ~15 ns each
// (~60 us, measured in round 2 with atomicXor and again here with one
// counter: 89 us per call), so workgroup b adds to shard b % 16 (each on its
// own 128-B line), the last of each shard adds to a top counter, and the last
// of those (one agent acquire) reads every partial with sc1 loads.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "internal.h"
#include "shmem_reduce_mi355x.h"

namespace shmx {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kCkBlock = 256;

constexpr uint64_t kPhi = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t mix64(uint64_t w, uint64_t j) {
    uint64_t z = w + (j + 1) * kPhi;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// splitmix64's finaliser of z = w + (j + 1) * phi, the position term given.
__device__ __forceinline__ uint64_t fmix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// The two words of 16-byte vector i (words 2i and 2i + 1); c = (2i + 1) * phi.
template <bool LD>
__device__ __forceinline__ uint64_t mix_pair(u32x4 x, uint64_t c) {
    const uint64_t w0 = ((uint64_t)x[1] << 32) | x[0];
    uint64_t w1 = ((uint64_t)x[3] << 32) | x[2];
    if (LD) w1 &= 0xFFFFull;  // bytes 8-9 are sign/exponent, 10-15 padding
    return fmix(w0 + c) ^ fmix(w1 + c + kPhi);
}

// XOR over the 64 lanes with DPP inside each 16-lane row (quad_perm
// [1,0,3,2] and [2,3,0,1], row_half_mirror, row_mirror: every lane of a row
// ends with the row's XOR), then the four rows through v_readlane.
__device__ __forceinline__ unsigned wave_xor32(unsigned v) {
    v ^= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
    v ^= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
    v ^= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    v ^= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
    return (unsigned)(__builtin_amdgcn_readlane((int)v, 0) ^ __builtin_amdgcn_readlane((int)v, 16) ^
                      __builtin_amdgcn_readlane((int)v, 32) ^ __builtin_amdgcn_readlane((int)v, 48));
}

__device__ __forceinline__ uint64_t wave_xor(uint64_t v) {
    return ((uint64_t)wave_xor32((unsigned)(v >> 32)) << 32) | wave_xor32((unsigned)v);
}

// nwords full 8-byte words; `tail` bytes of a final partial word; LD: mask
// 16-byte long double slots down to their 10 value bytes.  work: the shard
// counters (kShards of them, kLine words apart), the top counter, then the
// per-workgroup partials (zero counters between launches: the last workgroup
// resets them); out[0] the result, then out[1] = epoch.
constexpr int kShards = 16;
constexpr int kLine = 16;                       // 128 B between counters
constexpr int kTop = kShards * kLine;           // the top counter's word
constexpr int kPartials = (kShards + 1) * kLine;   // first partial's word
template <bool LD>
__global__ __launch_bounds__(kCkBlock) void checksum_kernel(const unsigned char *data, size_t nwords,
                                                            size_t tail, unsigned long long *work,
                                                            unsigned long long *out,
                                                            unsigned long long epoch) {
    __shared__ unsigned long long part[kCkBlock / 64];
    __shared__ int is_last;
    const size_t tid = (size_t)blockIdx.x * kCkBlock + threadIdx.x;
    const size_t nthr = (size_t)gridDim.x * kCkBlock;
    uint64_t h = 0;
    const size_t npairs = nwords / 2;
    const u32x4 *v = reinterpret_cast<const u32x4 *>(data);
    // The position term (j + 1) * phi of word j = 2i (+1) advances by
    // 2 * nthr * phi per grid-stride step: carried, not multiplied (a 64-bit
    // multiply is several quarter-rate instructions on CDNA; the hash is
    // VALU-heavy enough to share the bound with HBM).
    uint64_t c = (2 * (uint64_t)tid + 1) * kPhi;
    const uint64_t dc = 2 * (uint64_t)nthr * kPhi;
    // (two vectors in flight per lane per trip measured no faster:
    // profiles/r03_checksum_mix_lab.txt)
    for (size_t i = tid; i < npairs; i += nthr, c += dc)
        h ^= mix_pair<LD>(__builtin_nontemporal_load(v + i), c);
    if (tid == 0) {
        if (nwords & 1) {  // odd word count (only when !LD)
            uint64_t w = 0;
            __builtin_memcpy(&w, data + (nwords - 1) * 8, 8);
            h ^= mix64(w, nwords - 1);
        }
        if (tail) {
            uint64_t w = 0;
            for (size_t b = 0; b < tail; ++b) w |= (uint64_t)data[nwords * 8 + b] << (8 * b);
            h ^= mix64(w, nwords);
        }
    }
    h = wave_xor(h);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) part[wave] = h;
    __syncthreads();
    unsigned long long *partials = work + kPartials;
    const unsigned nblocks = gridDim.x;
    const unsigned nshards = nblocks < (unsigned)kShards ? nblocks : (unsigned)kShards;
    if (threadIdx.x == 0) {
        unsigned long long b = 0;
#pragma unroll
        for (int w = 0; w < kCkBlock / 64; ++w) b ^= part[w];
        // one slot per block (no contended atomic on the result), written
        // through to memory, drained, then counted
        __hip_atomic_store(partials + blockIdx.x, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned sh = blockIdx.x % nshards;
        const unsigned in_shard = (nblocks - sh + nshards - 1) / nshards;
        unsigned *shard = reinterpret_cast<unsigned *>(work + sh * kLine);
        int last = __hip_atomic_fetch_add(shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   in_shard - 1;
        if (last) {
            unsigned *top = reinterpret_cast<unsigned *>(work + kTop);
            last = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nshards - 1;
        }
        is_last = last;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!is_last) return;
    // the last workgroup: every partial, with sc1 loads, all issued before
    // any is used (a load per loop trip would wait out each one's latency:
    // 16 round trips to memory per lane at 4096 blocks); slots past the grid
    // are loaded from a valid address and masked, so no load is guarded
    constexpr int kPer = kChecksumMaxBlocks / kCkBlock;
    uint64_t pv[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const unsigned i = threadIdx.x + k * kCkBlock;
        pv[k] = __hip_atomic_load(partials + (i < nblocks ? i : nblocks - 1), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    }
    uint64_t x = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) x ^= threadIdx.x + k * kCkBlock < nblocks ? pv[k] : 0;
    x = wave_xor(x);
    __syncthreads();   // part[] is reused
    if (lane == 0) part[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long r = 0;
#pragma unroll
        for (int w = 0; w < kCkBlock / 64; ++w) r ^= part[w];
        // the result, then (ordered behind it: one lane, drained) the call's
        // epoch, which the host polls instead of waiting for the stream
        __hip_atomic_store(out, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(out + 1, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        // zero counters for the next launch (stream-ordered after this one)
        for (unsigned k = 0; k < nshards; ++k)
            __hip_atomic_store(reinterpret_cast<unsigned *>(work + k * kLine), 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(reinterpret_cast<unsigned *>(work + kTop), 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The counter + partials: device memory of this process, the counter zeroed
// once here and by every launch's last workgroup after that.
unsigned long long *checksum_work() {
    static unsigned long long *w = [] {
        void *p = nullptr;
        const size_t words = kPartials + (size_t)kChecksumMaxBlocks;
        if (hipMalloc(&p, sizeof(unsigned long long) * words) != hipSuccess) return
            static_cast<unsigned long long *>(nullptr);
        if (hipMemset(p, 0, sizeof(unsigned long long) * kPartials) != hipSuccess ||
            hipDeviceSynchronize() != hipSuccess) return static_cast<unsigned long long *>(nullptr);
        return static_cast<unsigned long long *>(p);
    }();
    return w;
}

}  // namespace

hipError_t launch_checksum(int type, const void *ptr, size_t n, unsigned long long *out,
                           unsigned long long epoch, hipStream_t stream) {
    const size_t sz = type_size(type);
    if (!sz || !out) return hipErrorInvalidValue;
    unsigned long long *work = checksum_work();
    if (!work) return hipErrorOutOfMemory;
    const size_t bytes = n * sz;
    const bool ld = type == SHMEMX_TYPE_LONGDOUBLE;
    const size_t nwords = bytes / 8, tail = bytes % 8;
    // 16-byte loads need a 16-byte aligned base; otherwise hash bytewise
    // through the tail path is too slow, so require it (hipMalloc gives 256).
    if (n && (reinterpret_cast<uintptr_t>(ptr) & 15u) != 0) return hipErrorInvalidValue;
    size_t blocks = (nwords / 2 + kCkBlock - 1) / kCkBlock;
    // 2048 workgroups: 44.6 us at 32 Mi doubles against 45.3 at 4096 (fewer
    // arrivals); 1024 and fewer lose bytes in flight (profiles/r03_checksum.txt)
    constexpr size_t kCap = 2048;
    if (blocks > kCap) blocks = kCap;
    if (blocks < 1) blocks = 1;
    const unsigned char *p = static_cast<const unsigned char *>(ptr);
    if (ld)
        hipLaunchKernelGGL(checksum_kernel<true>, dim3((unsigned)blocks), dim3(kCkBlock), 0, stream, p,
                           nwords, tail, work, out, epoch);
    else
        hipLaunchKernelGGL(checksum_kernel<false>, dim3((unsigned)blocks), dim3(kCkBlock), 0, stream, p,
                           nwords, tail, work, out, epoch);
    return hipGetLastError();
}

}  // namespace shmx
