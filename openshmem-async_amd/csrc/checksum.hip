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
// partials combined in LDS, one partial per workgroup in its own slot, and a
// one-workgroup kernel XORing the partials (same DPP + LDS reduction).
#include <hip/hip_runtime.h>

#include <cstdint>

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
// 16-byte long double slots down to their 10 value bytes.
template <bool LD>
__global__ __launch_bounds__(kCkBlock) void checksum_kernel(const unsigned char *data, size_t nwords,
                                                            size_t tail, unsigned long long *partials) {
    __shared__ unsigned long long part[kCkBlock / 64];
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
    if (threadIdx.x == 0) {
        unsigned long long b = 0;
#pragma unroll
        for (int w = 0; w < kCkBlock / 64; ++w) b ^= part[w];
        partials[blockIdx.x] = b;   // one slot per block: no contended atomic
    }
}

// The block partials XORed by one workgroup (DPP wave reduction + LDS), the
// result in *out.  A same-address atomic per block cost ~15 ns each, 60 us
// for 4096 blocks: more than streaming the 256 MiB (profiles/r02_checksum_lab.txt).
__global__ __launch_bounds__(kCkBlock) void checksum_finish_kernel(const unsigned long long *partials,
                                                                   int nparts, unsigned long long *out) {
    __shared__ unsigned long long part[kCkBlock / 64];
    uint64_t h = 0;
    for (int i = threadIdx.x; i < nparts; i += kCkBlock) h ^= partials[i];
    h = wave_xor(h);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = h;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = 0;
#pragma unroll
        for (int w = 0; w < kCkBlock / 64; ++w) b ^= part[w];
        *out = b;
    }
}

}  // namespace

hipError_t launch_checksum(int type, const void *ptr, size_t n, unsigned long long *out,
                           hipStream_t stream) {
    const size_t sz = type_size(type);
    if (!sz || !out) return hipErrorInvalidValue;
    if (n == 0) return hipMemsetAsync(out, 0, sizeof *out, stream);
    const size_t bytes = n * sz;
    const bool ld = type == SHMEMX_TYPE_LONGDOUBLE;
    const size_t nwords = bytes / 8, tail = bytes % 8;
    // 16-byte loads need a 16-byte aligned base; otherwise hash bytewise
    // through the tail path is too slow, so require it (hipMalloc gives 256).
    if ((reinterpret_cast<uintptr_t>(ptr) & 15u) != 0) return hipErrorInvalidValue;
    size_t blocks = (nwords / 2 + kCkBlock - 1) / kCkBlock;
    if (blocks > (size_t)kChecksumMaxBlocks) blocks = kChecksumMaxBlocks;
    if (blocks < 1) blocks = 1;
    const unsigned char *p = static_cast<const unsigned char *>(ptr);
    unsigned long long *partials = out + 1;
    if (ld)
        hipLaunchKernelGGL(checksum_kernel<true>, dim3((unsigned)blocks), dim3(kCkBlock), 0, stream, p,
                           nwords, tail, partials);
    else
        hipLaunchKernelGGL(checksum_kernel<false>, dim3((unsigned)blocks), dim3(kCkBlock), 0, stream, p,
                           nwords, tail, partials);
    hipLaunchKernelGGL(checksum_finish_kernel, dim3(1), dim3(kCkBlock), 0, stream, partials, (int)blocks,
                       out);
    return hipGetLastError();
}

}  // namespace shmx
