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
constexpr int HSB = 4;            // samples per head workgroup
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

// One 256-thread workgroup per HSB samples; thread t owns chunks t + 256 i (i < 8).
__global__ __launch_bounds__(256) void wide_head_kernel(
    const uint16_t* __restrict__ cut, const float* __restrict__ wf8, const float* __restrict__ bf,
    const int64_t* __restrict__ labels, const int* __restrict__ step_ptr, uint32_t seed, uint32_t thresh,
    float keep_scale, float grad_scale, float* __restrict__ logits, float* __restrict__ loss_i,
    float* __restrict__ dlogits, uint16_t* __restrict__ dcut, int* __restrict__ err_flag, int B) {
    __shared__ float red[4][HSB * NC];
    __shared__ float dl_s[HSB * NC];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b0 = blockIdx.x * HSB;
    const int nb = min(HSB, B - b0);
    const uint32_t step = (uint32_t)*step_ptr;

    float acc[HSB][NC];
#pragma unroll
    for (int s = 0; s < HSB; ++s)
#pragma unroll
        for (int j = 0; j < NC; ++j) acc[s][j] = 0.f;
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
        const int fc = tid + 256 * i;
        float w[NC][8];
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const float4 lo = *reinterpret_cast<const float4*>(wf8 + (size_t)j * CUTF + fc * 8);
            const float4 hi = *reinterpret_cast<const float4*>(wf8 + (size_t)j * CUTF + fc * 8 + 4);
            w[j][0] = lo.x; w[j][1] = lo.y; w[j][2] = lo.z; w[j][3] = lo.w;
            w[j][4] = hi.x; w[j][5] = hi.y; w[j][6] = hi.z; w[j][7] = hi.w;
        }
#pragma unroll
        for (int s = 0; s < HSB; ++s) {
            if (s >= nb) break;
            const uint32_t kb = keep_bits((uint32_t)(b0 + s), fc, step, seed, thresh);
            float v[8];
            unpack8(*reinterpret_cast<const uint4*>(cut + ((size_t)(b0 + s) * NCH + fc) * 8), v);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = (kb >> k) & 1 ? v[k] * keep_scale : 0.f;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                float a = acc[s][j];
#pragma unroll
                for (int k = 0; k < 8; ++k) a = __builtin_fmaf(v[k], w[j][k], a);
                acc[s][j] = a;
            }
        }
    }
#pragma unroll
    for (int s = 0; s < HSB; ++s)
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const float t = wave_sum(acc[s][j]);
            if (lane == 0) red[wave][s * NC + j] = t;
        }
    __syncthreads();
    if (tid < nb) {
        const int s = tid, b = b0 + s;
        float z[NC], m = -__builtin_inff();
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            z[j] = (((red[0][s * NC + j] + red[1][s * NC + j]) + red[2][s * NC + j]) + red[3][s * NC + j]) + bf[j];
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
            logits[(size_t)b * NC + j] = z[j];
            const float d = ok ? (expf(z[j] - lse) - (j == y ? 1.f : 0.f)) * grad_scale : __builtin_nanf("");
            dlogits[(size_t)b * NC + j] = d;
            dl_s[s * NC + j] = d;
        }
        loss_i[b] = ok ? lse - z[(int)y] : __builtin_nanf("");
    }
    __syncthreads();
    // dcut = keep * scale * (dlogits @ Wf)   (bf16, C8)
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
        const int fc = tid + 256 * i;
        float w[NC][8];
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const float4 lo = *reinterpret_cast<const float4*>(wf8 + (size_t)j * CUTF + fc * 8);
            const float4 hi = *reinterpret_cast<const float4*>(wf8 + (size_t)j * CUTF + fc * 8 + 4);
            w[j][0] = lo.x; w[j][1] = lo.y; w[j][2] = lo.z; w[j][3] = lo.w;
            w[j][4] = hi.x; w[j][5] = hi.y; w[j][6] = hi.z; w[j][7] = hi.w;
        }
#pragma unroll
        for (int s = 0; s < HSB; ++s) {
            if (s >= nb) break;
            const uint32_t kb = keep_bits((uint32_t)(b0 + s), fc, step, seed, thresh);  // recomputed: no mask storage
            float o[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                float a = 0.f;
#pragma unroll
                for (int j = 0; j < NC; ++j) a = __builtin_fmaf(dl_s[s * NC + j], w[j][k], a);
                o[k] = (kb >> k) & 1 ? a * keep_scale : 0.f;
            }
            *reinterpret_cast<uint4*>(dcut + ((size_t)(b0 + s) * NCH + fc) * 8) =
                make_uint4(pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7]));
        }
    }
}

// fc weight gradient: slab[slice] = [dWf (torch layout [10][16384]) | dbf]. Thread = chunk (8
// features x 10 classes = 80 accumulators), workgroup = 256 chunks x one batch slice.
constexpr int FCW_SLICES = 64;
__global__ __launch_bounds__(256) void wide_fc_wgrad_kernel(const uint16_t* __restrict__ cut, const float* __restrict__ dlogits,
                                                            const int* __restrict__ step_ptr, uint32_t seed, uint32_t thresh,
                                                            float keep_scale, float* __restrict__ slabs, int B) {
    const int cb = blockIdx.x & 7, slice = blockIdx.x >> 3;
    const int fc = cb * 256 + threadIdx.x;
    const uint32_t step = (uint32_t)*step_ptr;
    const int per = (B + FCW_SLICES - 1) / FCW_SLICES;
    const int s0 = slice * per, s1 = min(B, s0 + per);
    float acc[NC][8];
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[j][k] = 0.f;
    float accb = 0.f;
#pragma unroll 1
    for (int b = s0; b < s1; ++b) {
        const uint32_t kb = keep_bits((uint32_t)b, fc, step, seed, thresh);
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(cut + ((size_t)b * NCH + fc) * 8), v);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = (kb >> k) & 1 ? v[k] * keep_scale : 0.f;
        const float* dl = dlogits + (size_t)b * NC;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const float d = dl[j];
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[j][k] = __builtin_fmaf(d, v[k], acc[j][k]);
        }
        if (cb == 0 && threadIdx.x < NC) accb += dl[threadIdx.x];
    }
    float* slab = slabs + (size_t)slice * (NC * CUTF + NC);
    const int plane = fc >> 6, pix = fc & 63;
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
        for (int k = 0; k < 8; ++k) slab[(size_t)j * CUTF + (plane * 8 + k) * 64 + pix] = acc[j][k];
    if (cb == 0 && threadIdx.x < NC) slab[NC * CUTF + threadIdx.x] = accb;
}

// Fixed-order slab reduction + Adam (torch.optim.Adam, amsgrad=False, maximize=False, no weight
// decay). t = *step + 1; bias corrections in double like torch's Python floats; tensor math in f32:
//   m = m + (1-b1)(g - m)  [lerp]; v = v*b2 + (1-b2) g*g  [mul_ + addcmul_];
//   p = p - (lr / (1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)  [addcdiv_].
constexpr int AD_WAVES = 16;
__global__ __launch_bounds__(1024) void adam_from_slabs_kernel(float* __restrict__ param, float* __restrict__ grad,
                                                               float* __restrict__ m_, float* __restrict__ v_,
                                                               const float* __restrict__ slabs, int nslab, int n,
                                                               float lr, float b1, float b2, float eps,
                                                               const int* __restrict__ step_ptr) {
    __shared__ float part[AD_WAVES][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + lane;
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

extern "C" int slk_wide_head(const uint16_t* cut, const float* wf8, const float* bf, const int64_t* labels,
                             const int* step, unsigned seed, unsigned keep_threshold, float keep_scale,
                             float grad_scale, float* logits, float* loss_i, float* dlogits, uint16_t* dcut,
                             int* err_flag, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && cut && wf8 && bf && labels && step && logits && loss_i && dlogits && dcut);
    if (B == 0) return 0;
    hipLaunchKernelGGL(wide_head_kernel, dim3((B + HSB - 1) / HSB), dim3(256), 0, slk_stream(stream), cut, wf8, bf,
                       labels, step, seed, keep_threshold, keep_scale, grad_scale, logits, loss_i, dlogits, dcut,
                       err_flag, B);
    return slk_launch_status();
}
extern "C" int slk_wide_fc_wgrad_nslab(int B) { return B >= 0 ? FCW_SLICES : 0; }
extern "C" int slk_wide_fc_wgrad(const uint16_t* cut, const float* dlogits, const int* step, unsigned seed,
                                 unsigned keep_threshold, float keep_scale, float* slabs, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && cut && dlogits && step && slabs);
    hipLaunchKernelGGL(wide_fc_wgrad_kernel, dim3(8 * FCW_SLICES), dim3(256), 0, slk_stream(stream), cut, dlogits,
                       step, seed, keep_threshold, keep_scale, slabs, B);
    return slk_launch_status();
}
extern "C" int slk_adam_from_slabs(float* param, float* grad, float* m, float* v, const float* slabs, int nslab,
                                   int n, float lr, float beta1, float beta2, float eps, const int* step,
                                   void* stream) {
    SLK_CHECK_ARG(param && m && v && slabs && step && nslab > 0 && n >= 0);
    if (n == 0) return 0;
    hipLaunchKernelGGL(adam_from_slabs_kernel, dim3((n + 63) / 64), dim3(1024), 0, slk_stream(stream), param, grad, m, v,
                       slabs, nslab, n, lr, beta1, beta2, eps, step);
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
