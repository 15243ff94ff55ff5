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

// The training step's head is two launches: wide_head16_kernel (logits on the f32 MFMA, cross-entropy
// and the cut gradient, 16 samples per workgroup) and wide_head_back_kernel<false> (the fc weight
// gradient over a (feature slice x sample group) grid: thread = one 8-feature chunk of a 2048-feature
// slice accumulating 80 products over HSG samples -> one slab per sample group [dWf | dbf]).
// The module path's backward (slk_wide_head_bwd) is wide_head_back_kernel<true>, which also writes
// the cut gradient with the same per-element formula (dcut_chunk).
constexpr int HSLICE = 8;            // 2048-feature slices (256 chunks each)
#ifndef SLK_HSG
#define SLK_HSG 64
#endif
constexpr int HSG = SLK_HSG;         // samples per group (= per fc weight-gradient slab)
#ifndef SLK_HEAD_PF
#define SLK_HEAD_PF 1
#endif
constexpr int HPF = SLK_HEAD_PF;     // samples' cut chunks in flight ahead of the one in use (A/B: 2 and 4 no gain)

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

// cut gradient of one 8-feature chunk: (dlogits @ Wf) masked and scaled like the forward's dropout
__device__ __forceinline__ uint4 dcut_chunk(const float (&w)[NC][8], const float (&dlr)[NC], uint32_t kb, float keep_scale) {
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < NC; ++j) a = __builtin_fmaf(dlr[j], w[j][k], a);
        o[k] = (kb >> k) & 1 ? a * keep_scale : 0.f;
    }
    return make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
}

// The training step's head in ONE pass over the cut for 16 samples per workgroup (then
// wide_head_back_kernel<false> for the fc weight gradient): logits on v_mfma_f32_16x16x4_f32
// (A = 16 samples x 4 features, B = 4 features x 16 classes, 10 used), cross-entropy, and the cut
// gradient from the dropout bits the logits phase left in LDS. Replaces head_logits (10 wave
// reductions per sample and chunk slice) + head_ce + the cut-gradient half of head_back.
// Wave w owns chunks [256 w, 256 w + 256); lane (s16, kg) loads chunk 256 w + 4 blk + kg of sample
// s16 (16 contiguous bytes; 4 kg lanes = 64 B of a row) and the same chunk of Wf row min(s16, 9) (an
// L2 hit: Wf is 655 KB for all workgroups); MFMA i of a block takes feature i of each lane's chunk.
constexpr int WH_S = 16, WH_T = 512, WH_W = WH_T / 64;
constexpr int WH_CPW = NCH / WH_W;  // 256 chunks per wave = 64 blocks of 4
constexpr int WH_KBS = NCH + 16;    // LDS row stride of the dropout bits (16 rows x 4 dwords: 64 distinct banks)
#ifndef SLK_WH_PF
#define SLK_WH_PF 8
#endif
constexpr int WH_PF = SLK_WH_PF;    // blocks in flight per lane (cut + Wf registers)
static_assert(NCH % WH_W == 0 && (WH_CPW / 4) % WH_PF == 0 && NCH % WH_T == 0, "head16 tiling");

template <bool TRAIN>  // false: logits only (WideModelPartB.forward; labels .. dcut unused)
__global__ __launch_bounds__(WH_T) void wide_head16_kernel(
    const uint16_t* __restrict__ cut, const float* __restrict__ wf8, const float* __restrict__ bf,
    const int64_t* __restrict__ labels, const int* __restrict__ step_ptr, uint32_t seed, uint32_t thresh,
    float keep_scale, float grad_scale, float* __restrict__ logits, float* __restrict__ loss_i,
    float* __restrict__ dlogits, uint16_t* __restrict__ dcut, uint8_t* __restrict__ kbits, int* __restrict__ err_flag,
    int b0, int B) {
    __shared__ __attribute__((aligned(16))) uint8_t kbl[WH_S * WH_KBS];
    __shared__ __attribute__((aligned(16))) f32x4 red[WH_W * 64];
    __shared__ float zl[WH_S][NC];
    __shared__ float dls[WH_S][NC];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int s0 = blockIdx.x * WH_S, ns = min(WH_S, B - s0);
    const uint32_t step = (uint32_t)*step_ptr;
    {
        const int s16 = lane & 15, kg = lane >> 4, sl = min(s16, ns - 1);  // rows past the batch: never stored
        const uint4* crow = reinterpret_cast<const uint4*>(cut + (size_t)(s0 + sl) * CUTF);
        const float4* wrow = reinterpret_cast<const float4*>(wf8 + (size_t)min(s16, NC - 1) * CUTF);
        const int cb = wave * WH_CPW + kg;
        const int bs = b0 + s0 + sl;
        uint4 cv[WH_PF];
        float4 wv[WH_PF][2];
#pragma unroll
        for (int p = 0; p < WH_PF; ++p) {
            cv[p] = crow[cb + 4 * p];
            wv[p][0] = wrow[2 * (cb + 4 * p)];
            wv[p][1] = wrow[2 * (cb + 4 * p) + 1];
        }
        f32x4 acc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
            slk_keep(acc[q]);
        }
#pragma unroll 1
        for (int blk = 0; blk < WH_CPW / 4; blk += WH_PF) {
#pragma unroll
            for (int p = 0; p < WH_PF; ++p) {
                const int ch = cb + 4 * (blk + p);
                const uint4 v = cv[p];
                const float wf[8] = {wv[p][0].x, wv[p][0].y, wv[p][0].z, wv[p][0].w,
                                     wv[p][1].x, wv[p][1].y, wv[p][1].z, wv[p][1].w};
                if (blk + WH_PF < WH_CPW / 4) {
                    cv[p] = crow[ch + 4 * WH_PF];
                    wv[p][0] = wrow[2 * (ch + 4 * WH_PF)];
                    wv[p][1] = wrow[2 * (ch + 4 * WH_PF) + 1];
                }
                float d[8];
                const uint32_t kb = dropped(v, bs, ch, step, seed, thresh, keep_scale, d);
                if constexpr (TRAIN) kbl[s16 * WH_KBS + ch] = (uint8_t)kb;
#pragma unroll
                for (int i = 0; i < 8; ++i) acc[i & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(d[i], wf[i], acc[i & 3], 0, 0, 0);
            }
        }
        // D[4 (lane >> 4) + r][lane & 15] = (sample, class) partial over this wave's chunks
        red[wave * 64 + lane] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    }
    __syncthreads();
    if (tid < 256) {
        const int l = tid & 63, r = tid >> 6, n = l & 15, s = 4 * (l >> 4) + r;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < WH_W; ++w) v += red[w * 64 + l][r];
        if (n < NC) {
            zl[s][n] = v + bf[n];
            if (!TRAIN && s < ns) logits[(size_t)(s0 + s) * NC + n] = v + bf[n];
        }
    }
    if constexpr (!TRAIN) return;
    __syncthreads();
    if (tid < WH_S) {  // cross-entropy of sample tid (wide_head_ce_kernel's formula)
        const int s = tid;
        if (s < ns) {
            const int b = s0 + s;
            float z[NC], m = -__builtin_inff();
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                z[j] = zl[s][j];
                m = fmaxf(m, z[j]);
            }
            float se = 0.f;
#pragma unroll
            for (int j = 0; j < NC; ++j) se += expf(z[j] - m);
            const float lse = m + logf(se);
            const int64_t y = labels[b];
            const bool ok = y >= 0 && y < NC;
            if (!ok && err_flag) atomicOr(err_flag, 1);
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                const float g = ok ? (expf(z[j] - lse) - (j == y ? 1.f : 0.f)) * grad_scale : __builtin_nanf("");
                logits[(size_t)b * NC + j] = z[j];
                dlogits[(size_t)b * NC + j] = g;
                dls[s][j] = g;
            }
            loss_i[b] = ok ? lse - z[(int)y] : __builtin_nanf("");
        }
    }
    __syncthreads();
    // the dropout bits for wide_head_back_kernel<false> (kbits [B][2048]: 8 MB at B = 4096, so the
    // weight-gradient pass reads them instead of re-hashing 8 features per chunk)
#pragma unroll
    for (int i = tid; i < WH_S * NCH / 16; i += WH_T) {
        const int s = i / (NCH / 16), q = i - s * (NCH / 16);
        if (s < ns)
            reinterpret_cast<uint4*>(kbits + (size_t)(s0 + s) * NCH)[q] =
                *reinterpret_cast<const uint4*>(kbl + s * WH_KBS + 16 * q);
    }
    // cut gradient: thread = chunk (4 per thread), Wf's 80 floats of it in registers, every sample's
    // chunk stored as 1-KiB-contiguous wave stores
#pragma unroll 1
    for (int ch = tid; ch < NCH; ch += WH_T) {
        float w[NC][8];
        load_w(wf8, ch, w);
#pragma unroll 1
        for (int s = 0; s < ns; ++s) {
            asm volatile("" ::: "memory");  // keeps the 16 x 10 dls reads from being hoisted out of the chunk loop
            float dlr[NC];
#pragma unroll
            for (int j = 0; j < NC; ++j) dlr[j] = dls[s][j];
            *reinterpret_cast<uint4*>(dcut + ((size_t)(s0 + s) * NCH + ch) * 8) =
                dcut_chunk(w, dlr, kbl[s * WH_KBS + ch], keep_scale);
        }
    }
}

template <bool DCUT>
__global__ __launch_bounds__(256) void wide_head_back_kernel(const uint16_t* __restrict__ cut, const float* __restrict__ wf8,
                                                             const float* __restrict__ dlogits,
                                                             const int* __restrict__ step_ptr, uint32_t seed,
                                                             uint32_t thresh, float keep_scale,
                                                             uint16_t* __restrict__ dcut, float* __restrict__ slabs,
                                                             const uint8_t* __restrict__ kbits, int b0, int B) {
    const int slice = blockIdx.x % HSLICE, grp = blockIdx.x / HSLICE;
    const int fc = slice * 256 + threadIdx.x;
    const uint32_t step = (uint32_t)*step_ptr;
    float w[NC][8], acc[NC][8];
    if constexpr (DCUT) load_w(wf8, fc, w);
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
        uint32_t kb;
        if constexpr (DCUT) {
            kb = dropped(v, b0 + b, fc, step, seed, thresh, keep_scale, d);
        } else {  // the forward's bits (wide_head16_kernel<true>), same formula as dropped()
            kb = kbits[(size_t)b * NCH + fc];
            unpack8(v, d);
#pragma unroll
            for (int k = 0; k < 8; ++k) d[k] = (kb >> k) & 1 ? d[k] * keep_scale : 0.f;
        }
        const float* dl = dlogits + (size_t)b * NC;
        float dlr[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) dlr[j] = dl[j];
#pragma unroll
        for (int j = 0; j < NC; ++j)
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[j][k] = __builtin_fmaf(dlr[j], d[k], acc[j][k]);
        if (slice == 0 && threadIdx.x < NC) accb += dl[threadIdx.x];
        if constexpr (DCUT) *reinterpret_cast<uint4*>(dcut + ((size_t)b * NCH + fc) * 8) = dcut_chunk(w, dlr, kb, keep_scale);
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
// Few slabs (<= AD_COLS_MAX): thread = column, the slabs summed in ascending order with 8 loads in flight,
// 1024 columns per block (coalesced rows); many slabs (the conv1 and conv2 sets): 64 columns per block, 16
// waves over the slab range, partials added in wave order.
// Round 6: 17-64 slabs (the conv3 and fc sets at B = 4096) as 4 waves per 64 columns, each summing every 4th
// slab, partials added in order, 256 columns per block (a thread per column walked 64 slabs in 8 dependent rounds).
#ifndef SLK_AD_MID
#define SLK_AD_MID 1
#endif
constexpr int AD_COLS_MAX = SLK_AD_MID ? 16 : 64, AD_MID_MAX = 64;
__host__ __device__ constexpr int adam_cols_per_block(int nslab) {
    return nslab <= AD_COLS_MAX ? 1024 : (nslab <= AD_MID_MAX ? 256 : 64);
}

// the Adam update of element i from its summed gradient t (shared by the reduction forms below)
__device__ __forceinline__ void adam_apply(int i, float t, float* __restrict__ param, float* __restrict__ grad,
                                           float* __restrict__ m_, float* __restrict__ v_, float lr, float b1,
                                           float b2, float eps, const int* __restrict__ step_ptr) {
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

__device__ __forceinline__ void adam_slab_block_mid(float* __restrict__ param, float* __restrict__ grad,
                                                    float* __restrict__ m_, float* __restrict__ v_,
                                                    const float* __restrict__ slabs, int nslab, int n, float lr,
                                                    float b1, float b2, float eps, const int* __restrict__ step_ptr,
                                                    int blk) {
    __shared__ float part[4][256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = (wave & 3) * 64 + lane, sg = wave >> 2;  // column within the block, slab group
    const int i = blk * 256 + c;
    float g = 0.f;
    if (i < n) {
        const float* s = slabs + i;
        int k = sg;
        for (; k + 7 * 4 < nslab; k += 8 * 4) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = s[(size_t)(k + 4 * u) * n];
#pragma unroll
            for (int u = 0; u < 8; ++u) g += v[u];
        }
        for (; k < nslab; k += 4) g += s[(size_t)k * n];
    }
    part[sg][c] = g;
    __syncthreads();
    if (sg == 0 && i < n) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) t += part[q][c];
        adam_apply(i, t, param, grad, m_, v_, lr, b1, b2, eps, step_ptr);
    }
}

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
    else if (adam_cols_per_block(nslab) == 256)
        adam_slab_block_mid(param, grad, m_, v_, slabs, nslab, n, lr, b1, b2, eps, step_ptr, blk);
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
extern "C" int slk_wide_head_work(int B) { return B > 0 ? B * (NCH / 4) : 0; }  // the dropout bits, B x 2048 B
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
    hipLaunchKernelGGL(wide_head16_kernel<true>, dim3((B + WH_S - 1) / WH_S), dim3(WH_T), 0, st, cut, wf8, bf, labels, step, seed,
                       keep_threshold, keep_scale, grad_scale, logits, loss_i, dlogits, dcut, (uint8_t*)work, err_flag,
                       b0, B);
    hipLaunchKernelGGL(wide_head_back_kernel<false>, dim3(HSLICE * ng), dim3(256), 0, st, cut, wf8, dlogits, step, seed,
                       keep_threshold, keep_scale, dcut, slabs, (const uint8_t*)work, b0, B);
    return slk_launch_status();
}
extern "C" int slk_wide_head_fwd(const uint16_t* cut, const float* wf8, const float* bf, const int* step,
                                 unsigned seed, unsigned keep_threshold, float keep_scale, float* logits,
                                 int b0, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && b0 >= 0 && cut && wf8 && bf && step && logits);
    if (B == 0) return 0;
    hipStream_t st = slk_stream(stream);
    hipLaunchKernelGGL(wide_head16_kernel<false>, dim3((B + WH_S - 1) / WH_S), dim3(WH_T), 0, st, cut, wf8, bf, nullptr, step,
                       seed, keep_threshold, keep_scale, 0.f, logits, nullptr, nullptr, nullptr, nullptr, nullptr, b0, B);
    return slk_launch_status();
}

extern "C" int slk_wide_head_bwd(const uint16_t* cut, const float* wf8, const float* dlogits, const int* step,
                                 unsigned seed, unsigned keep_threshold, float keep_scale, uint16_t* dcut, float* slabs,
                                 int b0, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && b0 >= 0 && cut && wf8 && dlogits && step && dcut && slabs);
    if (B == 0) return 0;
    hipLaunchKernelGGL(wide_head_back_kernel<true>, dim3(HSLICE * slk_wide_head_nslab(B)), dim3(256), 0, slk_stream(stream), cut,
                       wf8, dlogits, step, seed, keep_threshold, keep_scale, dcut, slabs, nullptr, b0, B);
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
