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

// One workgroup per sample. Thread t produces float4 chunks of the NCHW output; 676 % 4 == 0, so a
// chunk never straddles two channels.
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ W1,
                                                        const float* __restrict__ b1,
                                                        float* __restrict__ act) {
    __shared__ float xs[IN_HW * IN_HW];
    __shared__ float ws[C1 * 9];
    __shared__ float bs[C1];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const float* xb = x + (size_t)b * IN_HW * IN_HW;
    for (int i = tid; i < IN_HW * IN_HW / 4; i += 256)
        reinterpret_cast<float4*>(xs)[i] = reinterpret_cast<const float4*>(xb)[i];
    for (int i = tid; i < C1 * 9; i += 256) ws[i] = W1[i];
    if (tid < C1) bs[tid] = b1[tid];
    __syncthreads();

    float4* out = reinterpret_cast<float4*>(act + (size_t)b * A_SAMPLE);
    for (int i4 = tid; i4 < A_SAMPLE / 4; i4 += 256) {
        const int e = i4 * 4;
        const int c = e / A_PIX;
        const int p0 = e - c * A_PIX;
        const float* w = ws + c * 9;
        float r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int p = p0 + u;
            const int y = p / A_HW, xx = p - (p / A_HW) * A_HW;
            const float* src = xs + y * IN_HW + xx;
            // same tap order as the reference conv (ky, kx row-major), bias added last
            float s = 0.f;
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) s = fmaf(src[ky * IN_HW + kx], w[ky * 3 + kx], s);
            s += bs[c];
            r[u] = s > 0.f ? s : 0.f;
        }
        out[i4] = make_float4(r[0], r[1], r[2], r[3]);
    }
}

// conv1 weight gradient. Grid (ngroups, 32 channels); a workgroup owns one channel c and a group of
// G samples, so its 676*G-long reduction stays in registers + one LDS tree: fixed order, bit-stable.
// Output slab row (per group): [dW1 c*9+tap (288) | db1 c (32)] = the client flat layout.
constexpr int C1W_G = 8;
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ act,
                                                          const float* __restrict__ gcut,
                                                          float* __restrict__ slabs, int B) {
    __shared__ float xs[C1W_G * IN_HW * IN_HW];
    __shared__ float red[4][10];
    const int grp = blockIdx.x;
    const int c = blockIdx.y;
    const int tid = threadIdx.x;
    const int b0 = grp * C1W_G;
    const int nb = min(C1W_G, B - b0);
    for (int i = tid; i < nb * IN_HW * IN_HW / 4; i += 256)
        reinterpret_cast<float4*>(xs)[i] =
            reinterpret_cast<const float4*>(x + (size_t)b0 * IN_HW * IN_HW)[i];
    __syncthreads();

    float acc[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) acc[k] = 0.f;
    constexpr int P4 = A_PIX / 4;  // 169 float4 per channel plane
    for (int i4 = tid; i4 < nb * P4; i4 += 256) {
        const int bl = i4 / P4;
        const int p0 = (i4 - bl * P4) * 4;
        const size_t off = ((size_t)(b0 + bl) * C1 + c) * A_PIX + p0;
        const float4 g4 = *reinterpret_cast<const float4*>(gcut + off);
        const float4 a4 = *reinterpret_cast<const float4*>(act + off);
        const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
        const float av[4] = {a4.x, a4.y, a4.z, a4.w};
        const float* xi = xs + bl * IN_HW * IN_HW;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float gm = av[u] > 0.f ? gv[u] : 0.f;  // threshold_backward: grad where relu out > 0
            const int p = p0 + u;
            const int y = p / A_HW, xx = p - (p / A_HW) * A_HW;
            const float* src = xi + y * IN_HW + xx;
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) acc[ky * 3 + kx] = fmaf(gm, src[ky * IN_HW + kx], acc[ky * 3 + kx]);
            acc[9] += gm;
        }
    }
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const float v = wave_sum(acc[k]);
        if (lane == 0) red[wave][k] = v;
    }
    __syncthreads();
    if (tid < 10) {
        const float v = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
        float* slab = slabs + (size_t)grp * SLK_CLIENT_NPARAM;
        if (tid < 9) slab[c * 9 + tid] = v;
        else slab[C1 * 9 + c] = v;
    }
}

extern "C" int slk_conv1_wgrad_nslab(int B) { return B > 0 ? (B + C1W_G - 1) / C1W_G : 0; }

extern "C" int slk_conv1_fwd(const float* x, const float* W1, const float* b1, float* act, int B,
                             void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(x && W1 && b1 && act);
    conv1_fwd_kernel<<<B, 256, 0, slk_stream(stream)>>>(x, W1, b1, act);
    return slk_launch_status();
}

extern "C" int slk_conv1_wgrad(const float* x, const float* act, const float* cut_grad,
                               float* slabs, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(x && act && cut_grad && slabs);
    dim3 grid(slk_conv1_wgrad_nslab(B), C1);
    conv1_wgrad_kernel<<<grid, 256, 0, slk_stream(stream)>>>(x, act, cut_grad, slabs, B);
    return slk_launch_status();
}
