// slk_codec.hip — lossless sparse codec for the cut exchange of the multi-GPU topologies (K3 Pipeline,
// K4 Hub): the reference ships the dense fp32 cut activations and the dense fp32 cut gradient over
// HTTP (src/client_part.py:117-125, src/server_part.py:57-58); here they travel over RCCL/xGMI, which
// bounds those configurations (354 MB per direction per step at B = 4096). The cut is a ReLU output,
// about half zeros, so a micro-batch travels as
//   mask : one bit per element, set where the element's bit pattern is nonzero (uint32 words), and
//   vals : the set elements in element order (f32, bit for bit),
// and the cut GRADIENT travels as the values at the same set positions only: the client multiplies
// the gradient by its own ReLU mask (act > 0, a subset of the set bits) before using it
// (src/client_part.py:132 through ReLU's backward), so the positions left out never matter. Both
// directions are then ~ (density + 1/32) of the dense bytes, and every result downstream is bit-identical
// to the dense exchange.
// Layout: elements in blocks of 2048 (one 256-thread workgroup; 32 mask words of 64 bits); per block
// the count of set bits, an exclusive scan of the counts gives each block's offset into vals.
#include "slk_common.h"

namespace {
constexpr int CB = 2048;            // elements per block
constexpr int CB_WORDS = CB / 32;   // uint32 mask words per block
}  // namespace

// mask + per-block counts from the dense tensor
__global__ __launch_bounds__(256) void cut_mask_kernel(const uint32_t* __restrict__ x, long n,
                                                       uint32_t* __restrict__ mask, int* __restrict__ counts) {
    __shared__ int wsum[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long b0 = (long)blockIdx.x * CB;
    int cnt = 0;
#pragma unroll
    for (int it = 0; it < CB / 256; ++it) {             // wave w: elements b0 + 512 w + 64 it + lane
        const long i = b0 + wave * (CB / 4) + it * 64 + lane;
        const bool set = i < n && x[i] != 0u;
        const unsigned long long bal = __ballot(set);
        cnt += __popcll(bal);
        if (lane < 2) {
            const long w = (b0 + wave * (CB / 4) + it * 64) / 32 + lane;
            if (w * 32 < n) mask[w] = (uint32_t)(bal >> (32 * lane));
        }
    }
    if (lane == 0) wsum[wave] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
}

// per-block counts from a mask (the receiving side)
__global__ __launch_bounds__(256) void cut_count_kernel(const uint32_t* __restrict__ mask, long n, int nblk,
                                                        int* __restrict__ counts) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= nblk) return;
    const long nw = (n + 31) / 32;
    int c = 0;
    for (int k = 0; k < CB_WORDS; ++k) {
        const long w = (long)b * CB_WORDS + k;
        if (w < nw) c += __popc(mask[w]);
    }
    counts[b] = c;
}

// exclusive scan of the block counts (one workgroup) -> offsets; total -> total[0]
__global__ __launch_bounds__(1024) void cut_scan_kernel(const int* __restrict__ counts, int nblk,
                                                        int* __restrict__ offsets, int* __restrict__ total) {
    __shared__ int part[1024];
    const int t = threadIdx.x;
    const int per = (nblk + 1023) / 1024;
    const int lo = min(nblk, t * per), hi = min(nblk, lo + per);
    int s = 0;
    for (int b = lo; b < hi; ++b) s += counts[b];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {   // Hillis-Steele inclusive scan of the thread sums
        const int v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = part[t] - s;                 // exclusive prefix of this thread's range
    for (int b = lo; b < hi; ++b) {
        offsets[b] = run;
        run += counts[b];
    }
    if (t == 1023) total[0] = part[1023];
}

// vals[offset + rank] = x[i] for the set elements (pack) or x[i] = set ? vals[...] : 0 (unpack).
// Wave w of block b covers elements b*2048 + 512 w .. +511: its start offset is the block offset plus
// the set bits of the block's earlier words.
template <bool PACK>
__global__ __launch_bounds__(256) void cut_move_kernel(uint32_t* __restrict__ x, long n, const uint32_t* __restrict__ mask,
                                                       const int* __restrict__ offsets, uint32_t* __restrict__ vals) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long b0 = (long)blockIdx.x * CB;
    const long nw = (n + 31) / 32;
    const long w0 = b0 / 32;
    int off = offsets[blockIdx.x];
    for (int k = 0; k < wave * (CB_WORDS / 4); ++k) off += w0 + k < nw ? __popc(mask[w0 + k]) : 0;
#pragma unroll
    for (int it = 0; it < CB / 256; ++it) {
        const long e0 = b0 + wave * (CB / 4) + it * 64;
        const long w = e0 / 32;
        const uint32_t lo = w < nw ? mask[w] : 0u, hi = w + 1 < nw ? mask[w + 1] : 0u;
        const unsigned long long m = (unsigned long long)lo | ((unsigned long long)hi << 32);
        const bool set = (m >> lane) & 1ull;
        const int rank = __popcll(m & ((1ull << lane) - 1ull));
        const long i = e0 + lane;
        if (PACK) {
            if (set) vals[off + rank] = x[i];
        } else if (i < n) {
            x[i] = set ? vals[off + rank] : 0u;
        }
        off += __popcll(m);
    }
}

// int32 offsets: one micro-batch of at most 2^31 - 1 elements (99,273 reference cut samples)
constexpr int64_t CUT_NMAX = 2147483647;

static inline int cut_blocks(int64_t n) { return (int)((n + CB - 1) / CB); }

extern "C" int slk_cut_blocks(int64_t n) { return n > 0 && n <= CUT_NMAX ? cut_blocks(n) : 0; }

extern "C" int slk_cut_encode(const float* x, int64_t n, uint32_t* mask, int* counts, int* offsets, int* total,
                              float* vals, void* stream) {
    SLK_CHECK_ARG(n >= 0 && n <= CUT_NMAX);  // offsets, counts and the total are int32
    if (n == 0) return 0;   // empty tensors carry null pointers
    SLK_CHECK_ARG(x && mask && counts && offsets && total && vals);
    const int nb = cut_blocks(n);
    hipStream_t st = slk_stream(stream);
    hipLaunchKernelGGL(cut_mask_kernel, dim3(nb), dim3(256), 0, st, reinterpret_cast<const uint32_t*>(x), n, mask, counts);
    hipLaunchKernelGGL(cut_scan_kernel, dim3(1), dim3(1024), 0, st, counts, nb, offsets, total);
    hipLaunchKernelGGL(cut_move_kernel<true>, dim3(nb), dim3(256), 0, st, const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(x)),
                       n, mask, offsets, reinterpret_cast<uint32_t*>(vals));
    return slk_launch_status();
}

extern "C" int slk_cut_offsets(const uint32_t* mask, int64_t n, int* counts, int* offsets, int* total, void* stream) {
    SLK_CHECK_ARG(n >= 0 && n <= CUT_NMAX);  // offsets, counts and the total are int32
    if (n == 0) return 0;   // empty tensors carry null pointers
    SLK_CHECK_ARG(mask && counts && offsets && total);
    const int nb = cut_blocks(n);
    hipStream_t st = slk_stream(stream);
    hipLaunchKernelGGL(cut_count_kernel, dim3((nb + 255) / 256), dim3(256), 0, st, mask, n, nb, counts);
    hipLaunchKernelGGL(cut_scan_kernel, dim3(1), dim3(1024), 0, st, counts, nb, offsets, total);
    return slk_launch_status();
}

extern "C" int slk_cut_pack(const float* x, int64_t n, const uint32_t* mask, const int* offsets, float* vals, void* stream) {
    SLK_CHECK_ARG(n >= 0 && n <= CUT_NMAX);  // offsets, counts and the total are int32
    if (n == 0) return 0;   // empty tensors carry null pointers
    SLK_CHECK_ARG(x && mask && offsets && vals);
    hipLaunchKernelGGL(cut_move_kernel<true>, dim3(cut_blocks(n)), dim3(256), 0, slk_stream(stream),
                       const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(x)), n, mask, offsets,
                       reinterpret_cast<uint32_t*>(vals));
    return slk_launch_status();
}

extern "C" int slk_cut_unpack(const float* vals, int64_t n, const uint32_t* mask, const int* offsets, float* x, void* stream) {
    SLK_CHECK_ARG(n >= 0 && n <= CUT_NMAX);  // offsets, counts and the total are int32
    if (n == 0) return 0;   // empty tensors carry null pointers
    SLK_CHECK_ARG(x && mask && offsets && vals);
    hipLaunchKernelGGL(cut_move_kernel<false>, dim3(cut_blocks(n)), dim3(256), 0, slk_stream(stream),
                       reinterpret_cast<uint32_t*>(x), n, mask, offsets,
                       const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(vals)));
    return slk_launch_status();
}
