// slk_wide_head.hip — server stage of the widened split CNN (K5) and the Adam optimizer.
//
// Server (oracle/wide_step.py server_step): Dropout(0.25) -> flatten (c*64 + y*8 + x) ->
// Linear(16384, 10) -> CrossEntropyLoss(mean) forward and backward, i.e. server_part.py:47-57's
// step for the widened model. 0.1 % of the step's FLOPs and HBM-bound: VALU kernels that read the cut
// (bf16, C8 layout) once for the logits and once for the weight gradient. The dropout mask is a
// counter-based hash of (seed, step, sample, feature) recomputed wherever it is needed, so no mask
// tensor exists and a HIP-graph replay draws a fresh mask from the device step counter.
//
// Adam (torch.optim.Adam, default flags: `_single_tensor_adam` of torch/optim/adam.py) fused with the
// fixed-order reduction of the wgrad slabs, plus the kernels that rebuild the bf16 weight shadows the
// MFMA convolutions read and the C8-ordered f32 copy of the fc weight the head reads.
#include "slk_common.h"

namespace {
constexpr int CUTF = 16384;       // features per sample
constexpr int NCH = CUTF / 8;     // 2048 chunks of 8 channels (C8 order: chunk = plane*64 + pixel)
constexpr int NC = 10;
}  // namespace

__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

// keep bits of the 8 features of chunk fc (C8 order) of sample b: feature index (torch flatten) of
// element k is (plane*8 + k)*64 + pixel.
__device__ __forceinline__ uint32_t keep_bits(uint32_t b, int fc, uint32_t step, uint32_t seed, uint32_t thresh) {
    const uint32_t plane = fc >> 6, pix = fc & 63;
    const uint32_t base = step * 0x85EBCA77u + seed * 0xC2B2AE3Du;
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t e = b * (uint32_t)CUTF + (plane * 8 + k) * 64 + pix;
        bits |= (lowbias32(e * 0x9E3779B1u + base) >= thresh ? 1u : 0u) << k;
    }
    return bits;
}

__device__ __forceinline__ void unpack8(const uint4 v, float (&f)[8]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f[2 * k] = __uint_as_float(w[k] << 16);
        f[2 * k + 1] = __uint_as_float(w[k] & 0xFFFF0000u);
    }
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
    const __bf16 x = (__bf16)a, y = (__bf16)b;
    return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

// The head as three launches over a (feature slice x sample group) grid, so every fc weight is read
// into registers once per workgroup and reused over 64 samples (the weight matrix is 655 KB: re-read
// per handful of samples it, not the cut, was the traffic):
//   head_logits : thread = one 8-feature chunk of a 2048-feature slice, weights in registers; per
//                 sample: dropout, 80 FMAs, wave reduction -> partial logits [B][32][10] (workspace)
//   head_ce     : thread = sample; fixed-order sum of the 32 partials + bias, cross-entropy fwd/bwd
//   head_back   : same grid; per sample the cut gradient chunk (bf16) and the fc weight-gradient
//                 accumulation (80 registers) -> one slab per sample group [dWf | dbf]
constexpr int HSLICE = 8;            // 2048-feature slices (256 chunks each)
#ifndef SLK_HSG
#define SLK_HSG 64
#endif
constexpr int HSG = SLK_HSG;         // samples per group (= per fc weight-gradient slab)
constexpr int HPART = HSLICE * 4;    // partial logits per sample (slices x waves)
#ifndef SLK_HSG_L
#define SLK_HSG_L 32
#endif
#ifndef SLK_HEAD_PF
#define SLK_HEAD_PF 1
#endif
constexpr int HPF = SLK_HEAD_PF;     // samples' cut chunks in flight ahead of the one in use (A/B: 2 and 4 no gain)
constexpr int HSG_L = SLK_HSG_L;     // samples per group of the logits pass (no slab: free to differ;
                                     // A/B via bench: 64 -> 0.193 ms head, 32 -> 0.177, 16 -> 0.175 but a slower step)

__device__ __forceinline__ void load_w(const float* __restrict__ wf8, int fc, float (&w)[NC][8]) {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        const float4 lo = *reinterpret_cast<const float4*>(wf8 + (size_t)j * CUTF + fc * 8);
        const float4 hi = *reinterpret_cast<const float4*>(wf8 + (size_t)j * CUTF + fc * 8 + 4);
        w[j][0] = lo.x; w[j][1] = lo.y; w[j][2] = lo.z; w[j][3] = lo.w;
        w[j][4] = hi.x; w[j][5] = hi.y; w[j][6] = hi.z; w[j][7] = hi.w;
    }
}

// dropout applied to a loaded cut chunk v of sample b; returns the keep bits
__device__ __forceinline__ uint32_t dropped(uint4 v, int b, int fc, uint32_t step, uint32_t seed, uint32_t thresh,
                                            float keep_scale, float (&d)[8]) {
    const uint32_t kb = keep_bits((uint32_t)b, fc, step, seed, thresh);
    unpack8(v, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = (kb >> k) & 1 ? d[k] * keep_scale : 0.f;
    return kb;
}
__device__ __forceinline__ uint4 cut_chunk(const uint16_t* __restrict__ cut, int b, int fc, int B) {
    return b < B ? *reinterpret_cast<const uint4*>(cut + ((size_t)b * NCH + fc) * 8) : make_uint4(0, 0, 0, 0);
}

__global__ __launch_bounds__(256) void wide_head_logits_kernel(const uint16_t* __restrict__ cut, const float* __restrict__ wf8,
                                                               const int* __restrict__ step_ptr, uint32_t seed,
                                                               uint32_t thresh, float keep_scale,
                                                               float* __restrict__ part, int b0, int B) {
    const int slice = blockIdx.x % HSLICE, grp = blockIdx.x / HSLICE;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int fc = slice * 256 + threadIdx.x;
    const uint32_t step = (uint32_t)*step_ptr;
    float w[NC][8];
    load_w(wf8, fc, w);
    const int b1 = min(B, (grp + 1) * HSG_L);
    uint4 ring[HPF];
#pragma unroll
    for (int i = 0; i < HPF; ++i) ring[i] = cut_chunk(cut, grp * HSG_L + i, fc, b1);
#pragma unroll 1
    for (int b = grp * HSG_L; b < b1; ++b) {
        const uint4 v = ring[0];
#pragma unroll
        for (int i = 0; i + 1 < HPF; ++i) ring[i] = ring[i + 1];
        ring[HPF - 1] = cut_chunk(cut, b + HPF, fc, b1);  // later samples' chunks in flight during this one
        float d[8];
        dropped(v, b0 + b, fc, step, seed, thresh, keep_scale, d);
        float pj[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            float a = 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k) a = __builtin_fmaf(d[k], w[j][k], a);
            pj[j] = wave_sum(a);
        }
        if (lane < NC) {
            float v = pj[0];
#pragma unroll
            for (int j = 1; j < NC; ++j) v = lane == j ? pj[j] : v;
            part[((size_t)b * HPART + slice * 4 + wave) * NC + lane] = v;
        }
    }
}

__global__ __launch_bounds__(256) void wide_head_ce_kernel(const float* __restrict__ part, const float* __restrict__ bf,
                                                           const int64_t* __restrict__ labels, float grad_scale,
                                                           float* __restrict__ logits, float* __restrict__ loss_i,
                                                           float* __restrict__ dlogits, int* __restrict__ err_flag, int B) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    // partials of this sample: 32 x 10 contiguous floats, read 8 partials (20 float4) at a time so
    // the loads are in flight together; summed per logit in partial order q = 0..31 from 0, then + bias
    float z[NC], m = -__builtin_inff();
#pragma unroll
    for (int j = 0; j < NC; ++j) z[j] = 0.f;
    const float4* p4 = reinterpret_cast<const float4*>(part + (size_t)b * HPART * NC);
#pragma unroll
    for (int q0 = 0; q0 < HPART; q0 += 8) {
        float pv[8 * NC];
#pragma unroll
        for (int i = 0; i < 2 * NC; ++i) {
            const float4 t = p4[q0 * NC / 4 + i];
            pv[4 * i] = t.x; pv[4 * i + 1] = t.y; pv[4 * i + 2] = t.z; pv[4 * i + 3] = t.w;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int j = 0; j < NC; ++j) z[j] += pv[q * NC + j];
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        z[j] = z[j] + bf[j];
        m = fmaxf(m, z[j]);
    }
    float se = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j) se += expf(z[j] - m);
    const float lse = m + logf(se);
    if (!labels) {  // forward only (the module path: WideModelPartB.forward, the loss comes later)
#pragma unroll
        for (int j = 0; j < NC; ++j) logits[(size_t)b * NC + j] = z[j];
        return;
    }
    const int64_t y = labels[b];
    const bool ok = y >= 0 && y < NC;
    if (!ok && err_flag) atomicOr(err_flag, 1);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        logits[(size_t)b * NC + j] = z[j];
        dlogits[(size_t)b * NC + j] = ok ? (expf(z[j] - lse) - (j == y ? 1.f : 0.f)) * grad_scale : __builtin_nanf("");
    }
    loss_i[b] = ok ? lse - z[(int)y] : __builtin_nanf("");
}

__global__ __launch_bounds__(256) void wide_head_back_kernel(const uint16_t* __restrict__ cut, const float* __restrict__ wf8,
                                                             const float* __restrict__ dlogits,
                                                             const int* __restrict__ step_ptr, uint32_t seed,
                                                             uint32_t thresh, float keep_scale,
                                                             uint16_t* __restrict__ dcut, float* __restrict__ slabs, int b0,
                                                             int B) {
    const int slice = blockIdx.x % HSLICE, grp = blockIdx.x / HSLICE;
    const int fc = slice * 256 + threadIdx.x;
    const uint32_t step = (uint32_t)*step_ptr;
    float w[NC][8], acc[NC][8];
    load_w(wf8, fc, w);
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[j][k] = 0.f;
    float accb = 0.f;
    const int b1 = min(B, (grp + 1) * HSG);
    uint4 ring[HPF];
#pragma unroll
    for (int i = 0; i < HPF; ++i) ring[i] = cut_chunk(cut, grp * HSG + i, fc, b1);
#pragma unroll 1
    for (int b = grp * HSG; b < b1; ++b) {
        const uint4 v = ring[0];
#pragma unroll
        for (int i = 0; i + 1 < HPF; ++i) ring[i] = ring[i + 1];
        ring[HPF - 1] = cut_chunk(cut, b + HPF, fc, b1);
        float d[8];
        const uint32_t kb = dropped(v, b0 + b, fc, step, seed, thresh, keep_scale, d);
        const float* dl = dlogits + (size_t)b * NC;
        float dlr[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) dlr[j] = dl[j];
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float a = 0.f;
#pragma unroll
            for (int j = 0; j < NC; ++j) a = __builtin_fmaf(dlr[j], w[j][k], a);
            o[k] = (kb >> k) & 1 ? a * keep_scale : 0.f;
        }
#pragma unroll
        for (int j = 0; j < NC; ++j)
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[j][k] = __builtin_fmaf(dlr[j], d[k], acc[j][k]);
        if (slice == 0 && threadIdx.x < NC) accb += dl[threadIdx.x];
        const uint32_t ow[4] = {pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7])};
        *reinterpret_cast<uint4*>(dcut + ((size_t)b * NCH + fc) * 8) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    }
    float* slab = slabs + (size_t)grp * (NC * CUTF + NC);
    const int plane = fc >> 6, pix = fc & 63;
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
        for (int k = 0; k < 8; ++k) slab[(size_t)j * CUTF + (plane * 8 + k) * 64 + pix] = acc[j][k];
    if (slice == 0 && threadIdx.x < NC) slab[NC * CUTF + threadIdx.x] = accb;
}

// Fixed-order slab reduction + Adam (torch.optim.Adam, amsgrad=False, maximize=False, no weight
// decay). t = *step + 1; bias corrections in double like torch's Python floats; tensor math in f32:
//   m = m + (1-b1)(g - m)  [lerp]; v = v*b2 + (1-b2) g*g  [mul_ + addcmul_];
//   p = p - (lr / (1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)  [addcdiv_].
constexpr int AD_WAVES = 16;
// Few slabs (<= AD_COLS_MAX, the conv2/conv3/fc wgrad slab sets): thread = column, the slabs summed
// in ascending order with 8 loads in flight, 1024 columns per block (coalesced rows); many slabs
// (the conv1 set): 64 columns per block, 16 waves over the slab range, partials added in wave order.
constexpr int AD_COLS_MAX = 64;
__host__ __device__ constexpr int adam_cols_per_block(int nslab) { return nslab <= AD_COLS_MAX ? 1024 : 64; }

__device__ __forceinline__ void adam_slab_block_rows(float* __restrict__ param, float* __restrict__ grad,
                                                float* __restrict__ m_, float* __restrict__ v_,
                                                const float* __restrict__ slabs, int nslab, int n, float lr,
                                                float b1, float b2, float eps, const int* __restrict__ step_ptr,
                                                int blk) {
    __shared__ float part[AD_WAVES][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i = blk * 64 + lane;
    float g = 0.f;
    if (i < n) {
        const float* s = slabs + i;
        int k = wave;
        for (; k + 7 * AD_WAVES < nslab; k += 8 * AD_WAVES) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = s[(size_t)(k + u * AD_WAVES) * n];
#pragma unroll
            for (int u = 0; u < 8; ++u) g += v[u];
        }
        for (; k < nslab; k += AD_WAVES) g += s[(size_t)k * n];
    }
    part[wave][lane] = g;
    __syncthreads();
    if (wave == 0 && i < n) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < AD_WAVES; ++w) t += part[w][lane];
        if (grad) grad[i] = t;
        const double tt = (double)(*step_ptr + 1);
        const double bc1 = 1.0 - pow((double)b1, tt);
        const float step_size = (float)((double)lr / bc1);
        const float bc2s = (float)sqrt(1.0 - pow((double)b2, tt));
        float m = m_[i], v = v_[i];
        m = m + (1.f - b1) * (t - m);
        v = v * b2 + t * t * (1.f - b2);
        const float denom = sqrtf(v) / bc2s + eps;
        param[i] = param[i] + (-step_size) * (m / denom);
        m_[i] = m;
        v_[i] = v;
    }
}

__device__ __forceinline__ void adam_slab_block_cols(float* __restrict__ param, float* __restrict__ grad,
                                                     float* __restrict__ m_, float* __restrict__ v_,
                                                     const float* __restrict__ slabs, int nslab, int n, float lr,
                                                     float b1, float b2, float eps, const int* __restrict__ step_ptr,
                                                     int blk) {
    const int i = blk * 1024 + threadIdx.x;
    if (i >= n) return;
    const float* s = slabs + i;
    float t = 0.f;
    int k = 0;
    for (; k + 8 <= nslab; k += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = s[(size_t)(k + u) * n];
#pragma unroll
        for (int u = 0; u < 8; ++u) t += v[u];
    }
    for (; k < nslab; ++k) t += s[(size_t)k * n];
    if (grad) grad[i] = t;
    const double tt = (double)(*step_ptr + 1);
    const double bc1 = 1.0 - pow((double)b1, tt);
    const float step_size = (float)((double)lr / bc1);
    const float bc2s = (float)sqrt(1.0 - pow((double)b2, tt));
    float m = m_[i], v = v_[i];
    m = m + (1.f - b1) * (t - m);
    v = v * b2 + t * t * (1.f - b2);
    const float denom = sqrtf(v) / bc2s + eps;
    param[i] = param[i] + (-step_size) * (m / denom);
    m_[i] = m;
    v_[i] = v;
}

__device__ __forceinline__ void adam_slab_block(float* __restrict__ param, float* __restrict__ grad,
                                                float* __restrict__ m_, float* __restrict__ v_,
                                                const float* __restrict__ slabs, int nslab, int n, float lr,
                                                float b1, float b2, float eps, const int* __restrict__ step_ptr,
                                                int blk) {
    if (adam_cols_per_block(nslab) == 1024)
        adam_slab_block_cols(param, grad, m_, v_, slabs, nslab, n, lr, b1, b2, eps, step_ptr, blk);
    else
        adam_slab_block_rows(param, grad, m_, v_, slabs, nslab, n, lr, b1, b2, eps, step_ptr, blk);
}

__global__ __launch_bounds__(1024) void adam_from_slabs_kernel(float* __restrict__ param, float* __restrict__ grad,
                                                               float* __restrict__ m_, float* __restrict__ v_,
                                                               const float* __restrict__ slabs, int nslab, int n,
                                                               float lr, float b1, float b2, float eps,
                                                               const int* __restrict__ step_ptr) {
    adam_slab_block(param, grad, m_, v_, slabs, nslab, n, lr, b1, b2, eps, step_ptr, blockIdx.x);
}

// Several parameter segments (each with its own slab set) in ONE launch: consecutive block ranges,
// each running adam_from_slabs_kernel's code on its segment — bit-identical to separate launches.
constexpr int AD_MAXSEG = 4;
struct AdamSeg {
    float* param;
    float* grad;
    float* m;
    float* v;
    const float* slabs;
    int nslab, n, nblk;
};
struct AdamMulti {
    AdamSeg seg[AD_MAXSEG];
    int nseg;
    float lr, b1, b2, eps;
    const int* step;
};
__global__ __launch_bounds__(1024) void adam_multi_kernel(const AdamMulti a) {
    int blk = blockIdx.x;
#pragma unroll
    for (int s = 0; s < AD_MAXSEG; ++s) {
        if (s < a.nseg) {
            const AdamSeg& g = a.seg[s];
            if (blk < g.nblk) {
                adam_slab_block(g.param, g.grad, g.m, g.v, g.slabs, g.nslab, g.n, a.lr, a.b1, a.b2, a.eps, a.step, blk);
                return;
            }
            blk -= g.nblk;
        }
    }
}

// bf16 shadows of the client conv weights (torch layout [co][ci][3][3] f32 masters) in the layouts
// slk_wide.hip's implicit GEMMs stream: forward [co/128][tap][ci/8][co%128][8]; dgrad (roles
// swapped, taps flipped) [ci/MT][8-tap][co/8][ci%MT][8] with MT = 64 (conv2) / 128 (conv3).
// Also the bf16 conv1 weight w1b [64][32] = W1[co] (27, order ci, ky, kx) | 5 zeros: conv1's MFMA A operand.
__global__ __launch_bounds__(256) void wide_shadows_kernel(const float* __restrict__ W1, const float* __restrict__ W2,
                                                           const float* __restrict__ W3, uint16_t* __restrict__ w1b,
                                                           uint16_t* __restrict__ w2f, uint16_t* __restrict__ w2d,
                                                           uint16_t* __restrict__ w3f, uint16_t* __restrict__ w3d) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    constexpr int N2 = 128 * 64 * 9, N3 = 256 * 128 * 9;
    if (e < 64 * 32) {
        const int co = e >> 5, i = e & 31;
        const __bf16 h = (__bf16)(i < 27 ? W1[co * 27 + i] : 0.f);
        w1b[e] = __builtin_bit_cast(uint16_t, h);
    }
    if (e < N2) {
        const int co = e / (64 * 9), r = e - co * 64 * 9, ci = r / 9, tap = r - ci * 9;
        const __bf16 h = (__bf16)W2[e];
        const uint16_t u = __builtin_bit_cast(uint16_t, h);
        w2f[((tap * 8 + (ci >> 3)) * 128 + co) * 8 + (ci & 7)] = u;
        w2d[(((8 - tap) * 16 + (co >> 3)) * 64 + ci) * 8 + (co & 7)] = u;
    } else if (e < N2 + N3) {
        const int f = e - N2;
        const int co = f / (128 * 9), r = f - co * 128 * 9, ci = r / 9, tap = r - ci * 9;
        const __bf16 h = (__bf16)W3[f];
        const uint16_t u = __builtin_bit_cast(uint16_t, h);
        w3f[((((co >> 7) * 9 + tap) * 16 + (ci >> 3)) * 128 + (co & 127)) * 8 + (ci & 7)] = u;
        w3d[(((8 - tap) * 32 + (co >> 3)) * 128 + ci) * 8 + (co & 7)] = u;
    }
}

// fc weight in the cut's C8 order: wf8[j][(plane*64 + pix)*8 + k] = Wf[j][(plane*8 + k)*64 + pix]
__global__ __launch_bounds__(256) void wide_fc_shadow_kernel(const float* __restrict__ wf, float* __restrict__ wf8) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= NC * CUTF) return;
    const int j = e / CUTF, f = e - j * CUTF;
    const int k = f & 7, fc = f >> 3, plane = fc >> 6, pix = fc & 63;
    wf8[e] = wf[(size_t)j * CUTF + (plane * 8 + k) * 64 + pix];
}

__global__ void tick_kernel(int* __restrict__ ctr) { *ctr += 1; }

extern "C" int slk_wide_head_nslab(int B) { return B > 0 ? (B + HSG - 1) / HSG : 0; }
extern "C" int slk_wide_head_work(int B) { return B > 0 ? B * HPART * NC : 0; }
// CE: one sample per thread in 64-thread blocks, so B = 4096 spreads over 64 CUs instead of 16
// (0.0168 -> 0.0074 ms per launch, rocprofv3). (Storing the forward's dropout bits for the backward
// instead of re-hashing: back -8.7 us, logits +5 us — not kept.)
constexpr int HCE_T = 64;
extern "C" int slk_wide_head(const uint16_t* cut, const float* wf8, const float* bf, const int64_t* labels,
                             const int* step, unsigned seed, unsigned keep_threshold, float keep_scale,
                             float grad_scale, float* logits, float* loss_i, float* dlogits, uint16_t* dcut,
                             float* slabs, float* work, int* err_flag, int b0, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && b0 >= 0 && cut && wf8 && bf && labels && step && logits && loss_i && dlogits && dcut &&
                  slabs && work);
    SLK_CHECK_ARG(((uintptr_t)work & 15) == 0);  // the CE kernel reads the partials as float4
    if (B == 0) return 0;
    const int ng = slk_wide_head_nslab(B);
    hipStream_t st = slk_stream(stream);
    hipLaunchKernelGGL(wide_head_logits_kernel, dim3(HSLICE * ((B + HSG_L - 1) / HSG_L)), dim3(256), 0, st, cut, wf8, step, seed,
                       keep_threshold, keep_scale, work, b0, B);
    hipLaunchKernelGGL(wide_head_ce_kernel, dim3((B + HCE_T - 1) / HCE_T), dim3(HCE_T), 0, st, work, bf, labels, grad_scale,
                       logits, loss_i, dlogits, err_flag, B);
    hipLaunchKernelGGL(wide_head_back_kernel, dim3(HSLICE * ng), dim3(256), 0, st, cut, wf8, dlogits, step, seed,
                       keep_threshold, keep_scale, dcut, slabs, b0, B);
    return slk_launch_status();
}
extern "C" int slk_wide_head_fwd(const uint16_t* cut, const float* wf8, const float* bf, const int* step,
                                 unsigned seed, unsigned keep_threshold, float keep_scale, float* logits, float* work,
                                 int b0, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && b0 >= 0 && cut && wf8 && bf && step && logits && work);
    SLK_CHECK_ARG(((uintptr_t)work & 15) == 0);
    if (B == 0) return 0;
    hipStream_t st = slk_stream(stream);
    hipLaunchKernelGGL(wide_head_logits_kernel, dim3(HSLICE * ((B + HSG_L - 1) / HSG_L)), dim3(256), 0, st, cut, wf8, step, seed,
                       keep_threshold, keep_scale, work, b0, B);
    hipLaunchKernelGGL(wide_head_ce_kernel, dim3((B + HCE_T - 1) / HCE_T), dim3(HCE_T), 0, st, work, bf, nullptr, 0.f, logits,
                       nullptr, nullptr, nullptr, B);
    return slk_launch_status();
}

extern "C" int slk_wide_head_bwd(const uint16_t* cut, const float* wf8, const float* dlogits, const int* step,
                                 unsigned seed, unsigned keep_threshold, float keep_scale, uint16_t* dcut, float* slabs,
                                 int b0, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && b0 >= 0 && cut && wf8 && dlogits && step && dcut && slabs);
    if (B == 0) return 0;
    hipLaunchKernelGGL(wide_head_back_kernel, dim3(HSLICE * slk_wide_head_nslab(B)), dim3(256), 0, slk_stream(stream), cut,
                       wf8, dlogits, step, seed, keep_threshold, keep_scale, dcut, slabs, b0, B);
    return slk_launch_status();
}

extern "C" int slk_adam_from_slabs(float* param, float* grad, float* m, float* v, const float* slabs, int nslab,
                                   int n, float lr, float beta1, float beta2, float eps, const int* step,
                                   void* stream) {
    SLK_CHECK_ARG(param && m && v && slabs && step && nslab > 0 && n >= 0);
    if (n == 0) return 0;
    hipLaunchKernelGGL(adam_from_slabs_kernel, dim3((n + adam_cols_per_block(nslab) - 1) / adam_cols_per_block(nslab)), dim3(1024), 0, slk_stream(stream), param, grad, m, v,
                       slabs, nslab, n, lr, beta1, beta2, eps, step);
    return slk_launch_status();
}
extern "C" int slk_adam_multi_from_slabs(float* const* params, float* const* grads, float* const* m, float* const* v,
                                         const float* const* slabs, const int* nslab, const int* n, int nseg,
                                         float lr, float beta1, float beta2, float eps, const int* step,
                                         void* stream) {
    SLK_CHECK_ARG(nseg >= 0 && nseg <= AD_MAXSEG && step);
    SLK_CHECK_ARG(nseg == 0 || (params && m && v && slabs && nslab && n));
    AdamMulti a{};
    int nblk = 0;
    for (int s = 0; s < nseg; ++s) {
        SLK_CHECK_ARG(params[s] && m[s] && v[s] && slabs[s] && nslab[s] > 0 && n[s] >= 0);
        a.seg[s] = AdamSeg{params[s], grads ? grads[s] : nullptr, m[s], v[s], slabs[s], nslab[s], n[s], (n[s] + adam_cols_per_block(nslab[s]) - 1) / adam_cols_per_block(nslab[s])};
        nblk += a.seg[s].nblk;
    }
    a.nseg = nseg;
    a.lr = lr;
    a.b1 = beta1;
    a.b2 = beta2;
    a.eps = eps;
    a.step = step;
    if (nblk == 0) return 0;
    hipLaunchKernelGGL(adam_multi_kernel, dim3(nblk), dim3(1024), 0, slk_stream(stream), a);
    return slk_launch_status();
}
extern "C" int slk_wide_shadows(const float* W1, const float* W2, const float* W3, uint16_t* w1b, uint16_t* w2f,
                                uint16_t* w2d, uint16_t* w3f, uint16_t* w3d, void* stream) {
    SLK_CHECK_ARG(W1 && W2 && W3 && w1b && w2f && w2d && w3f && w3d);
    constexpr int N = 128 * 64 * 9 + 256 * 128 * 9;
    hipLaunchKernelGGL(wide_shadows_kernel, dim3((N + 255) / 256), dim3(256), 0, slk_stream(stream), W1, W2, W3, w1b,
                       w2f, w2d, w3f, w3d);
    return slk_launch_status();
}
extern "C" int slk_wide_fc_shadow(const float* wf, float* wf8, void* stream) {
    SLK_CHECK_ARG(wf && wf8);
    hipLaunchKernelGGL(wide_fc_shadow_kernel, dim3((NC * CUTF + 255) / 256), dim3(256), 0, slk_stream(stream), wf, wf8);
    return slk_launch_status();
}
extern "C" int slk_tick(int* counter, void* stream) {
    SLK_CHECK_ARG(counter);
    hipLaunchKernelGGL(tick_kernel, dim3(1), dim3(1), 0, slk_stream(stream), counter);
    return slk_launch_status();
}
