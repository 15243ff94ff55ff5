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
// Layout: elements in blocks of 2048 (one 256-thread workgroup; 64 mask words of 32 bits); per block
// the count of set bits, an exclusive scan of the counts gives each block's offset into vals.
#include "slk_common.h"

namespace {
constexpr int CB = 2048;            // elements per block
constexpr int CB_WORDS = CB / 32;   // uint32 mask words per block
constexpr int CS_LDS = 12288;       // block counts the scan stages in LDS
}  // namespace

// Thread t of a block owns elements 8t .. 8t+7 of the block (bits 8 (t & 3) .. +7 of mask word t / 4):
// the dense side moves as two 16-B accesses per thread, the sparse side through LDS so that every global
// access of the packed values is a contiguous run of the block's own values (coalesced both ways).
constexpr int CT = 256;                  // threads per block
constexpr int CE = CB / CT;              // 8 elements per thread
static_assert(CE == 8, "a thread's elements are one byte of a mask word");

// the thread's 8 elements (bit patterns) -> v; zeros past n
__device__ __forceinline__ void cut_load8(const uint32_t* __restrict__ x, long e0, long n, bool vec, uint32_t v[8]) {
    if (vec && e0 + 8 <= n) {
        const uint4 a = *reinterpret_cast<const uint4*>(x + e0), b = *reinterpret_cast<const uint4*>(x + e0 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = e0 + j < n ? x[e0 + j] : 0u;
    }
}

// exclusive prefix of c over the block's threads (in thread order) and the block total
__device__ __forceinline__ int cut_block_prefix(int c, int* wtot, int& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int inc = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    int base = 0;
#pragma unroll
    for (int w = 0; w < CT / 64; ++w) base += w < wave ? wtot[w] : 0;
    total = ((wtot[0] + wtot[1]) + wtot[2]) + wtot[3];
    return base + inc - c;
}

// mask + per-block counts from the dense tensor
__global__ __launch_bounds__(CT) void cut_mask_kernel(const uint32_t* __restrict__ x, long n,
                                                      uint32_t* __restrict__ mask, int* __restrict__ counts) {
    __shared__ int wsum[CT / 64];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const long e0 = (long)blockIdx.x * CB + CE * t;
    const bool vec = (reinterpret_cast<size_t>(x) & 15) == 0;
    uint32_t v[8];
    cut_load8(x, e0, n, vec, v);
    uint32_t byte = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) byte |= (v[j] != 0u ? 1u : 0u) << j;
    // the 4 threads of a mask word OR their bytes together (lanes 4q .. 4q+3)
    uint32_t w = byte << (8 * (t & 3));
    w |= __shfl_xor(w, 1, 64);
    w |= __shfl_xor(w, 2, 64);
    const long wi = (long)blockIdx.x * (CB / 32) + t / 4;
    if ((t & 3) == 0 && wi * 32 < n) mask[wi] = w;
    int c = __popc(byte);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) wsum[wave] = c;
    __syncthreads();
    if (t == 0) counts[blockIdx.x] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
}

// per-block counts from a mask (the receiving side): one wave per block, lane = mask word
__device__ __forceinline__ void cut_count_body(const uint32_t* __restrict__ mask, long n, int nblk, int* __restrict__ counts) {
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (b >= nblk) return;  // wave-uniform
    const long nw = (n + 31) / 32;
    const long w = (long)b * CB_WORDS + lane;
    int c = w < nw ? __popc(mask[w]) : 0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) counts[b] = c;
}
__global__ __launch_bounds__(256) void cut_count_kernel(const uint32_t* __restrict__ mask, long n, int nblk,
                                                        int* __restrict__ counts) {
    cut_count_body(mask, n, nblk, counts);
}

// word ranks (the fused consumers, slk_cut_unpack_x3 / slk_conv2_dgrad_x3_pack): ranks[w] = the vals index of
// the first set element of mask word w = offsets[block] + the set bits of the block's earlier words. One
// wave per block, lane = mask word: an element's rank is then ranks[e / 32] + popc(mask[e / 32] below e % 32)
__device__ __forceinline__ void cut_ranks_body(const uint32_t* __restrict__ mask, long n, int nblk,
                                               const int* __restrict__ offsets, int* __restrict__ ranks) {
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (b >= nblk) return;  // wave-uniform
    const long nw = (n + 31) / 32;
    const long w = (long)b * CB_WORDS + lane;
    const int c = w < nw ? __popc(mask[w]) : 0;
    int inc = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (w < nw) ranks[w] = offsets[b] + inc - c;
}
__global__ __launch_bounds__(256) void cut_ranks_kernel(const uint32_t* __restrict__ mask, long n, int nblk,
                                                        const int* __restrict__ offsets, int* __restrict__ ranks) {
    cut_ranks_body(mask, n, nblk, offsets, ranks);
}

__device__ void cut_scan_body(const int* __restrict__ counts, int nblk, int* __restrict__ offsets,
                              int* __restrict__ total, int* part, int* cs);

// The same three passes over the np parts of a chunk in one launch each (dist.Hub: one part per client):
// parts = device table [np][5] of (mask, counts, offsets, total, ranks) pointers, every part n elements;
// blockIdx.y (count, ranks) / blockIdx.x (scan) = the part
__global__ __launch_bounds__(256) void cut_count_parts_kernel(const uint64_t* __restrict__ parts, long n, int nblk) {
    const uint64_t* e = parts + 5 * blockIdx.y;
    cut_count_body(reinterpret_cast<const uint32_t*>(e[0]), n, nblk, reinterpret_cast<int*>(e[1]));
}
__global__ __launch_bounds__(1024) void cut_scan_parts_kernel(const uint64_t* __restrict__ parts, int nblk) {
    __shared__ int part[1024];
    __shared__ int cs[CS_LDS];
    const uint64_t* e = parts + 5 * blockIdx.x;
    cut_scan_body(reinterpret_cast<const int*>(e[1]), nblk, reinterpret_cast<int*>(e[2]), reinterpret_cast<int*>(e[3]),
                  part, cs);
}
__global__ __launch_bounds__(256) void cut_ranks_parts_kernel(const uint64_t* __restrict__ parts, long n, int nblk) {
    const uint64_t* e = parts + 5 * blockIdx.y;
    cut_ranks_body(reinterpret_cast<const uint32_t*>(e[0]), n, nblk, reinterpret_cast<const int*>(e[2]),
                   reinterpret_cast<int*>(e[4]));
}

// exclusive scan of the block counts (one workgroup) -> offsets; total -> total[0]. Up to CS_LDS counts
// are staged in LDS by coalesced loads (each thread then scans a contiguous range from LDS).
__device__ void cut_scan_body(const int* __restrict__ counts, int nblk, int* __restrict__ offsets,
                              int* __restrict__ total, int* part, int* cs) {
    const int t = threadIdx.x;
    const bool staged = nblk <= CS_LDS;
    if (staged) {
        for (int i = t; i < nblk; i += 1024) cs[i] = counts[i];
        __syncthreads();
    }
    const int* src = staged ? cs : counts;
    const int per = (nblk + 1023) / 1024;
    const int lo = min(nblk, t * per), hi = min(nblk, lo + per);
    int s = 0;
    for (int b = lo; b < hi; ++b) s += src[b];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {   // Hillis-Steele inclusive scan of the thread sums
        const int v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = part[t] - s;                 // exclusive prefix of this thread's range
    if (staged) {
        for (int b = lo; b < hi; ++b) {    // in place, then coalesced stores
            const int c = cs[b];
            cs[b] = run;
            run += c;
        }
        __syncthreads();
        for (int i = t; i < nblk; i += 1024) offsets[i] = cs[i];
    } else {
        for (int b = lo; b < hi; ++b) {
            offsets[b] = run;
            run += counts[b];
        }
    }
    if (t == 1023) total[0] = part[1023];
}
__global__ __launch_bounds__(1024) void cut_scan_kernel(const int* __restrict__ counts, int nblk,
                                                        int* __restrict__ offsets, int* __restrict__ total) {
    __shared__ int part[1024];
    __shared__ int cs[CS_LDS];
    cut_scan_body(counts, nblk, offsets, total, part, cs);
}

// PACK: vals[offset + rank] = x[i] for the set elements; UNPACK: x[i] = set ? vals[...] : 0. The block's
// values pass through LDS (staged in element order), so the vals side moves as one contiguous run.
template <bool PACK>
__global__ __launch_bounds__(CT) void cut_move_kernel(uint32_t* __restrict__ x, long n, const uint32_t* __restrict__ mask,
                                                      const int* __restrict__ offsets, uint32_t* __restrict__ vals) {
    __shared__ uint32_t sv[CB];
    __shared__ int wtot[CT / 64];
    const int t = threadIdx.x;
    const long e0 = (long)blockIdx.x * CB + CE * t;
    const long nw = (n + 31) / 32;
    const long wi = (long)blockIdx.x * (CB / 32) + t / 4;
    const uint32_t byte = wi < nw ? (mask[wi] >> (8 * (t & 3))) & 0xFFu : 0u;
    int cnt;
    const int pre = cut_block_prefix(__popc(byte), wtot, cnt);
    const int off = offsets[blockIdx.x];
    const bool vec = (reinterpret_cast<size_t>(x) & 15) == 0;
    if (PACK) {
        uint32_t v[8];
        cut_load8(x, e0, n, vec, v);
        int r = pre;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if ((byte >> j) & 1u) sv[r++] = v[j];
        __syncthreads();
        for (int i = t; i < cnt; i += CT) vals[off + i] = sv[i];
    } else {
        for (int i = t; i < cnt; i += CT) sv[i] = vals[off + i];
        __syncthreads();
        uint32_t v[8];
        int r = pre;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = ((byte >> j) & 1u) ? sv[r++] : 0u;
        if (vec && e0 + 8 <= n) {
            *reinterpret_cast<uint4*>(x + e0) = make_uint4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<uint4*>(x + e0 + 4) = make_uint4(v[4], v[5], v[6], v[7]);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (e0 + j < n) x[e0 + j] = v[j];
        }
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
    hipLaunchKernelGGL(cut_mask_kernel, dim3(nb), dim3(CT), 0, st, reinterpret_cast<const uint32_t*>(x), n, mask, counts);
    hipLaunchKernelGGL(cut_scan_kernel, dim3(1), dim3(1024), 0, st, counts, nb, offsets, total);
    hipLaunchKernelGGL(cut_move_kernel<true>, dim3(nb), dim3(CT), 0, st, const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(x)),
                       n, mask, offsets, reinterpret_cast<uint32_t*>(vals));
    return slk_launch_status();
}

extern "C" int slk_cut_offsets(const uint32_t* mask, int64_t n, int* counts, int* offsets, int* total, void* stream) {
    SLK_CHECK_ARG(n >= 0 && n <= CUT_NMAX);  // offsets, counts and the total are int32
    if (n == 0) return 0;   // empty tensors carry null pointers
    SLK_CHECK_ARG(mask && counts && offsets && total);
    const int nb = cut_blocks(n);
    hipStream_t st = slk_stream(stream);
    hipLaunchKernelGGL(cut_count_kernel, dim3((nb + 3) / 4), dim3(256), 0, st, mask, n, nb, counts);
    hipLaunchKernelGGL(cut_scan_kernel, dim3(1), dim3(1024), 0, st, counts, nb, offsets, total);
    return slk_launch_status();
}

extern "C" int slk_cut_ranks(const uint32_t* mask, int64_t n, const int* offsets, int* ranks, void* stream) {
    SLK_CHECK_ARG(n >= 0 && n <= CUT_NMAX);
    if (n == 0) return 0;
    SLK_CHECK_ARG(mask && offsets && ranks);
    const int nb = cut_blocks(n);
    hipLaunchKernelGGL(cut_ranks_kernel, dim3((nb + 3) / 4), dim3(256), 0, slk_stream(stream), mask, n, nb, offsets, ranks);
    return slk_launch_status();
}

extern "C" int slk_cut_offsets_ranks_parts(const uint64_t* parts, int np, int64_t n, void* stream) {
    SLK_CHECK_ARG(n >= 0 && n <= CUT_NMAX && np >= 0 && np <= 65535);
    if (n == 0 || np == 0) return 0;
    SLK_CHECK_ARG(parts);
    const int nb = cut_blocks(n);
    hipStream_t st = slk_stream(stream);
    hipLaunchKernelGGL(cut_count_parts_kernel, dim3((nb + 3) / 4, np), dim3(256), 0, st, parts, n, nb);
    hipLaunchKernelGGL(cut_scan_parts_kernel, dim3(np), dim3(1024), 0, st, parts, nb);
    hipLaunchKernelGGL(cut_ranks_parts_kernel, dim3((nb + 3) / 4, np), dim3(256), 0, st, parts, n, nb);
    return slk_launch_status();
}

extern "C" int slk_cut_pack(const float* x, int64_t n, const uint32_t* mask, const int* offsets, float* vals, void* stream) {
    SLK_CHECK_ARG(n >= 0 && n <= CUT_NMAX);  // offsets, counts and the total are int32
    if (n == 0) return 0;   // empty tensors carry null pointers
    SLK_CHECK_ARG(x && mask && offsets && vals);
    hipLaunchKernelGGL(cut_move_kernel<true>, dim3(cut_blocks(n)), dim3(CT), 0, slk_stream(stream),
                       const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(x)), n, mask, offsets,
                       reinterpret_cast<uint32_t*>(vals));
    return slk_launch_status();
}

extern "C" int slk_cut_unpack(const float* vals, int64_t n, const uint32_t* mask, const int* offsets, float* x, void* stream) {
    SLK_CHECK_ARG(n >= 0 && n <= CUT_NMAX);  // offsets, counts and the total are int32
    if (n == 0) return 0;   // empty tensors carry null pointers
    SLK_CHECK_ARG(x && mask && offsets && vals);
    hipLaunchKernelGGL(cut_move_kernel<false>, dim3(cut_blocks(n)), dim3(CT), 0, slk_stream(stream),
                       reinterpret_cast<uint32_t*>(x), n, mask, offsets,
                       const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(vals)));
    return slk_launch_status();
}
