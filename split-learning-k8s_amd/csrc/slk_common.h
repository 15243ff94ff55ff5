// slk_common.h — shared helpers for the gfx950 split-CNN kernels (internal; not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/slk.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Fixed model geometry (src/model_def.py:8,18,20,22).
namespace slk {
constexpr int IN_HW = 28;            // x: 1 x 28 x 28
constexpr int C1 = 32;               // conv1 out channels
constexpr int A_HW = 26;             // cut activation spatial size
constexpr int A_PIX = A_HW * A_HW;   // 676
constexpr int A_SAMPLE = C1 * A_PIX; // 21632 floats per sample (86,528 B)
constexpr int C2 = 64;               // conv2 out channels
constexpr int O_HW = 24;             // conv2 output spatial size
constexpr int P_HW = 12;             // pooled spatial size
constexpr int P_WIN = P_HW * P_HW;   // 144 pooling windows per channel
constexpr int P_SAMPLE = C2 * P_WIN; // 9216 = fc1 in_features
constexpr int NCLS = 10;
constexpr int K2 = C1 * 9;           // conv2 reduction length per output (288)
constexpr int W2_N = C2 * K2;        // 18432
constexpr int W3_N = NCLS * P_SAMPLE;// 92160
constexpr int CODE_NONE = 4;         // pooled value <= 0: ReLU blocks the gradient
}  // namespace slk

// Pin gather-then-MFMA phases in the conv2 main loops with sched_barrier (A/B switch).
#ifndef SLK_PIN_PHASES
#define SLK_PIN_PHASES 0
#endif

template <typename T>
__device__ __forceinline__ void slk_keep(T& v) { asm volatile("" : "+v"(v)); }

#define SLK_CHECK_ARG(cond)                 \
    do {                                    \
        if (!(cond)) return (int)hipErrorInvalidValue; \
    } while (0)

static inline int slk_launch_status() { return (int)hipGetLastError(); }

static inline hipStream_t slk_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// f32-input MFMA wrappers (exact f32, k-ordered fma chain; cdna_hip_programming.md §3).
// 32x32x2: lane l supplies A[i=l&31][k=l>>5] and B[k=l>>5][j=l&31];
//          D: col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5), r in [0,16).
// 16x16x4: lane l supplies A[i=l&15][k=l>>4] and B[k=l>>4][j=l&15];
//          D: col = l&15, row = 4*(l>>4) + r, r in [0,4).
__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// Butterfly sum over the 64 lanes: every lane ends with the total, bit-identically (each step adds
// the same two partial sums, commutatively, in both partner lanes). Inside a 16-lane row by DPP
// (quad_perm 1032 / 2301, row_half_mirror, row_mirror: no LDS traffic), then across rows by
// ds_swizzle/bpermute.
__device__ __forceinline__ float wave_sum(float v) {
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));  // row_half_mirror
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));  // row_mirror
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// The x3 scale value of the cut a = relu(conv1(x) + b1) of one sample, computed by the client's conv1
// kernels (round 5): an upper bound of max a from the image's max |x| alone,
//     bound = max_c fma(sum_k |W1[c][k]| (taps in order), max|x|, max(b1[c], 0)),
// the same float expression in every kernel that emits it, so their act_amax outputs agree bit for bit.
// Only the scale's power of two is derived from it (x3_exp: the bound lands in [2^13, 2^14)), so the
// image writer needs no first pass over its own outputs. How far the cut's max sits below the bound depends
// on the data and the weights (mixed-sign W1 or cancelling inputs make it loose): every factor of 2 of
// slack moves the whole split one bit lower, so elements ~2^-24 of the bound and below lose lo-part bits to
// f16's subnormal range — the absolute error stays ~2^-24 of the bound (tests/test_x3_gpu.py checks x3 vs the
// f32 path with a bound 2^4-2^6 x the max). Block-wide: every thread calls it after xs
// (the 28 x 28 image in LDS) is complete; red holds >= 8 floats of scratch; returns the bound to all.
__device__ __forceinline__ float conv1_cut_bound(const float* xs, const float* __restrict__ W1,
                                                 const float* __restrict__ b1, float* red) {
    const int tid = threadIdx.x, nw = (blockDim.x + 63) >> 6;
    float m = 0.f;
    for (int i = tid; i < slk::IN_HW * slk::IN_HW; i += blockDim.x) m = fmaxf(m, fabsf(xs[i]));
    m = wave_max(m);
    if ((tid & 63) == 0) red[tid >> 6] = m;
    __syncthreads();
    float xmax = red[0];
    for (int w = 1; w < nw; ++w) xmax = fmaxf(xmax, red[w]);
    float bc = 0.f;
    if (tid < 64) {
        if (tid < slk::C1) {
            float ws = 0.f;
#pragma unroll
            for (int k = 0; k < 9; ++k) ws += fabsf(W1[tid * 9 + k]);
            bc = fmaf(ws, xmax, fmaxf(b1[tid], 0.f));
        }
        bc = wave_max(bc);
    }
    __syncthreads();  // every wave has read red[]
    if (tid == 0) red[0] = bc;
    __syncthreads();
    return red[0];
}

// ---------------------------------------------------------------------------- LDS-DMA as inline asm
// global_load_lds issued through asm: hipcc then neither counts it nor inserts its own vmcnt(0) in
// front of LDS reads and writes it cannot prove disjoint from a DMA in flight (it cannot tell a
// prefetch buffer from the one being read, so the prefetch would drain before every use). The kernel
// retires the DMA with its own counted `s_waitcnt vmcnt` + barrier. lds_dst is wave-uniform.
typedef __attribute__((address_space(3))) void* slk_lds_ptr;
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(slk_lds_ptr)(const_cast<void*>(p)));
}
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
// Scalar base + per-lane 32-bit byte offset (saddr form): with the lane offsets computed once per
// launch, a piece costs no VALU address arithmetic at all (sbase is wave-uniform).
__device__ __forceinline__ void glds16_so(const void* sbase, uint32_t voff, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void glds4(const void* gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
