// slk_client.hip — client stage (ModelPartA, src/model_def.py:5-12) for gfx950.
//
//   conv1_fwd   : act = relu(conv2d(x, W1, b1))          (client_part.py:114)
//   conv1_wgrad : relu-bwd + conv1 weight/bias gradient   (client_part.py:132)
//
// Both are HBM-bound (conv1 is 9 MACs per output): the fwd writes 86,528 B per sample, the wgrad
// reads 2 x 86,528 B per sample. Neither is a GEMM worth MFMA (K = 9), so both are coalesced
// float4 VALU kernels with the tiny per-sample image and the weights staged in LDS.
#include "slk_common.h"

using namespace slk;

// One workgroup per sample: thread t < 169 owns the 4 consecutive pixels 4t .. 4t+3 of every channel
// plane (676 = 169 x 4; a group may straddle two rows), reads their 3x3 windows once from the
// LDS-staged image, then walks the 32 channels with wave-uniform (broadcast) weights and stores one
// float4 per channel: 2.7 KB contiguous per channel plane per workgroup. 192 threads (3 waves), 169
// active. HBM-bound on the 86,528-B/sample write; 16-B stores measured 8% faster than a
// pixel-per-thread layout with 4-B stores (0.079 vs 0.085 ms, tools/ablate.py), non-temporal
// stores 18% slower.
constexpr int C1F4_T = 192;
constexpr int C1F4_G = A_PIX / 4;  // 169
__global__ __launch_bounds__(C1F4_T) void conv1_fwd_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ W1,
                                                             const float* __restrict__ b1,
                                                             float* __restrict__ act,
                                                             float* __restrict__ act_amax) {
    __shared__ float xs[IN_HW * IN_HW];
    __shared__ float amx[8];
    __shared__ float ws[C1 * 10];  // [c][9 taps | bias]
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const float* xb = x + (size_t)b * IN_HW * IN_HW;
    for (int i = tid; i < IN_HW * IN_HW / 4; i += C1F4_T)
        reinterpret_cast<float4*>(xs)[i] = reinterpret_cast<const float4*>(xb)[i];
    for (int i = tid; i < C1 * 9; i += C1F4_T) ws[(i / 9) * 10 + i % 9] = W1[i];
    if (tid < C1) ws[tid * 10 + 9] = b1[tid];
    __syncthreads();
    // act_amax (optional): the x3 conv2 kernels' per-sample scale value of the cut — the bound of its max
    // from max|x| (conv1_cut_bound, slk_common.h), as slk_conv1_fwd_x3 emits it; without it the idle
    // threads leave here
    const bool active = tid < C1F4_G;
    if (act_amax) {
        const float bnd = conv1_cut_bound(xs, W1, b1, amx);
        if (tid == 0) act_amax[b] = bnd;
    }
    if (!active) return;
    if (active) {
        float xv[4][9];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int p = 4 * tid + u;
            const int y = p / A_HW, xx = p - (p / A_HW) * A_HW;
#pragma unroll
            for (int k = 0; k < 9; ++k) xv[u][k] = xs[(y + k / 3) * IN_HW + xx + k % 3];
        }
        float4* out = reinterpret_cast<float4*>(act + (size_t)b * A_SAMPLE) + tid;
#pragma unroll 4
        for (int c = 0; c < C1; ++c) {
            const float* w = ws + c * 10;
            float wk[10];
#pragma unroll
            for (int k = 0; k < 10; ++k) wk[k] = w[k];
            float o[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                // tap order (ky, kx) row-major, bias added last — as conv1_fwd_kernel
                float s = 0.f;
#pragma unroll
                for (int k = 0; k < 9; ++k) s = fmaf(xv[u][k], wk[k], s);
                s += wk[9];
                o[u] = s > 0.f ? s : 0.f;
            }
            out[c * C1F4_G] = make_float4(o[0], o[1], o[2], o[3]);
        }
    }
}

#ifndef SLK_C1W_NG
#define SLK_C1W_NG 128
#endif
#ifndef SLK_C1W_U
#define SLK_C1W_U 1
#endif
constexpr int C1W_NG = SLK_C1W_NG;  // sample ranges: x 8 channel groups = 1024 workgroups = 4 per CU
#ifndef SLK_C1W_CG
#define SLK_C1W_CG 4
#endif
constexpr int C1W_CG = SLK_C1W_CG;
// conv1 weight gradient (ReLU backward + dW1, db1). Grid (G = min(B, 128) contiguous sample ranges of
// B/G (+-1) samples, 8 channel groups of 4) = one round of workgroups (no tail round), 256 threads,
// one item per thread in flight (measured at B = 4096, tools/ablate.py: G = 128 / 1 item 0.077 ms,
// G = 96 / 2 items 0.080, G = 256 / 1 0.082, G = 64 / 4 0.090, G = 192 / 1 0.096); each workgroup writes its group's slab row [dW1 c*9+tap (288) | db1 c (32)] (the
// client flat layout) for its 4 channels after a fixed-order block reduction. The work of a group
// (B/G samples x 338 horizontal pixel PAIRS per channel plane; 26 is even, so a pair never straddles a
// row) is flattened over the threads: item = (sample, pair). A pair's operands are float2 loads (cut
// gradient of 4 channels, the 3x4 input window as 3 row loads) and every FMA is a v_pk_fma_f32 over
// the two pixels: ~150 VALU instructions per pair x 4 channels instead of ~350 pixel-at-a-time.
// REMASK = true: the ReLU mask is recomputed from x, W1, b1 with conv1_fwd_kernel's exact per-pixel
// FMA order (fma over taps from 0, then + bias; act > 0 <=> s > 0), so act is never read (89.6 KB
// moved per sample instead of 176 KB). Valid whenever W1/b1 are the weights of the forward (true
// inside a split step: the client's SGD comes after its backward). REMASK = false reads act.
// Both produce bit-identical slabs (same summation order; tested).
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int C1W_PAIRS = A_PIX / 2;     // 338
constexpr int C1W_PROW = A_HW / 2;       // 13 pairs per row
template <bool REMASK>
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ act,
                                                             const float* __restrict__ W1,
                                                             const float* __restrict__ b1,
                                                             const float* __restrict__ gcut,
                                                             float* __restrict__ slabs, int B) {
    __shared__ float red[4][C1W_CG * 10];
    const int grp = blockIdx.x;
    const int c0 = blockIdx.y * C1W_CG;
    const int tid = threadIdx.x;
    const int G = gridDim.x;
    const int b0 = (int)((long long)grp * B / G);
    const int nb = (int)((long long)(grp + 1) * B / G) - b0;
    const int nitem = nb * C1W_PAIRS;

    float w[C1W_CG][10];  // wave-uniform: scalar loads
#pragma unroll
    for (int c = 0; c < C1W_CG; ++c) {
#pragma unroll
        for (int k = 0; k < 9; ++k) w[c][k] = REMASK ? W1[(c0 + c) * 9 + k] : 0.f;
        w[c][9] = REMASK ? b1[c0 + c] : 0.f;
    }
    f32x2 acc[C1W_CG][10];
#pragma unroll
    for (int c = 0; c < C1W_CG; ++c)
#pragma unroll
        for (int k = 0; k < 10; ++k) acc[c][k] = f32x2{0.f, 0.f};

    constexpr int U = SLK_C1W_U;  // items in flight per thread
#pragma unroll 1
    for (int base = tid; base < nitem; base += 256 * U) {
        f32x2 gv[U][C1W_CG], av[U][C1W_CG], xr[U][3][2];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int it0 = base + 256 * u;
            ok[u] = it0 < nitem;
            const int it = ok[u] ? it0 : nitem - 1;
            const int sl = it / C1W_PAIRS, q = it - sl * C1W_PAIRS;
            const int row = q / C1W_PROW, col = 2 * (q - row * C1W_PROW);
            const int bb = b0 + sl;
            const float* gb = gcut + ((size_t)bb * C1 + c0) * A_PIX + row * A_HW + col;
            const float* xi = x + (size_t)bb * IN_HW * IN_HW + row * IN_HW + col;
#pragma unroll
            for (int c = 0; c < C1W_CG; ++c) gv[u][c] = *reinterpret_cast<const f32x2*>(gb + c * A_PIX);
            if (!REMASK) {
                const float* ab = act + ((size_t)bb * C1 + c0) * A_PIX + row * A_HW + col;
#pragma unroll
                for (int c = 0; c < C1W_CG; ++c) av[u][c] = *reinterpret_cast<const f32x2*>(ab + c * A_PIX);
            }
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                xr[u][r][0] = *reinterpret_cast<const f32x2*>(xi + r * IN_HW);
                xr[u][r][1] = *reinterpret_cast<const f32x2*>(xi + r * IN_HW + 2);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            f32x2 xp[9];  // tap (r, k) operand pair: pixels (col, col+1) -> x[row+r][col+k], x[row+r][col+1+k]
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                xp[3 * r + 0] = xr[u][r][0];
                xp[3 * r + 1] = f32x2{xr[u][r][0].y, xr[u][r][1].x};
                xp[3 * r + 2] = xr[u][r][1];
            }
#pragma unroll
            for (int c = 0; c < C1W_CG; ++c) {
                f32x2 t = f32x2{0.f, 0.f};
                if (REMASK) {
#pragma unroll
                    for (int k = 0; k < 9; ++k) t = __builtin_elementwise_fma(xp[k], f32x2{w[c][k], w[c][k]}, t);
                    t = t + f32x2{w[c][9], w[c][9]};
                } else {
                    t = av[u][c];
                }
                f32x2 gm;
                gm.x = (ok[u] && t.x > 0.f) ? gv[u][c].x : 0.f;  // threshold_backward mask
                gm.y = (ok[u] && t.y > 0.f) ? gv[u][c].y : 0.f;
#pragma unroll
                for (int k = 0; k < 9; ++k) acc[c][k] = __builtin_elementwise_fma(gm, xp[k], acc[c][k]);
                acc[c][9] = acc[c][9] + gm;
            }
        }
    }
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int c = 0; c < C1W_CG; ++c)
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            const float v = wave_sum(acc[c][k].x + acc[c][k].y);
            if (lane == 0) red[wave][c * 10 + k] = v;
        }
    __syncthreads();
    if (tid < C1W_CG * 10) {
        const int c = tid / 10, k = tid - c * 10;
        const float v = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
        float* slab = slabs + (size_t)grp * SLK_CLIENT_NPARAM;
        if (k < 9) slab[(c0 + c) * 9 + k] = v;
        else slab[C1 * 9 + c0 + c] = v;
    }
}

extern "C" int slk_conv1_wgrad_nslab(int B) { return B > 0 ? (B < C1W_NG ? B : C1W_NG) : 0; }

extern "C" int slk_conv1_fwd(const float* x, const float* W1, const float* b1, float* act, int B,
                             void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(x && W1 && b1 && act);
    conv1_fwd_kernel<<<B, C1F4_T, 0, slk_stream(stream)>>>(x, W1, b1, act, nullptr);
    return slk_launch_status();
}

extern "C" int slk_conv1_fwd_amax(const float* x, const float* W1, const float* b1, float* act, float* act_amax,
                                  int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(x && W1 && b1 && act && act_amax);
    conv1_fwd_kernel<<<B, C1F4_T, 0, slk_stream(stream)>>>(x, W1, b1, act, act_amax);
    return slk_launch_status();
}

extern "C" int slk_conv1_wgrad(const float* x, const float* act, const float* cut_grad,
                               float* slabs, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(x && act && cut_grad && slabs);
    dim3 grid(slk_conv1_wgrad_nslab(B), C1 / C1W_CG);
    conv1_wgrad_kernel<false><<<grid, 256, 0, slk_stream(stream)>>>(x, act, nullptr, nullptr, cut_grad, slabs, B);
    return slk_launch_status();
}

extern "C" int slk_conv1_wgrad_remask(const float* x, const float* W1, const float* b1, const float* cut_grad,
                                      float* slabs, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(x && W1 && b1 && cut_grad && slabs);
    dim3 grid(slk_conv1_wgrad_nslab(B), C1 / C1W_CG);
    conv1_wgrad_kernel<true><<<grid, 256, 0, slk_stream(stream)>>>(x, nullptr, W1, b1, cut_grad, slabs, B);
    return slk_launch_status();
}
