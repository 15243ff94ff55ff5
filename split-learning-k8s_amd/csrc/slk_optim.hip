// slk_optim.hip — deterministic reductions, fused SGD and the device-side loss log.
//
// optim.SGD(lr=0.01) on both sides (client_part.py:17,133; server_part.py:15,52) is
// `p.add_(g, alpha=-lr)` per parameter. Here the parameters of a stage live in one flat block, so
// one launch updates all of them, and the weight-gradient slabs written by the wgrad kernels are
// summed (fixed order, bit-stable) in the same pass that applies the update.
#include "slk_common.h"

// Deterministic slab reduction (+ optional SGD). A 1024-thread block owns 64 columns; wave w sums
// slabs w, w+16, w+32, ... of those columns in order (8 loads in flight), then wave 0 adds the 16
// partials in wave order. The result is a fixed function of the inputs (no atomics).
constexpr int RS_WAVES = 16;
__global__ __launch_bounds__(1024) void sgd_from_slabs_kernel(float* __restrict__ param,
                                                              float* __restrict__ grad,
                                                              const float* __restrict__ slabs,
                                                              int nslab, int n, float lr, int acc) {
    __shared__ float part[RS_WAVES][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + lane;
    float g = 0.f;
    if (i < n) {
        const float* s = slabs + i;
        int k = wave;
        for (; k + 7 * RS_WAVES < nslab; k += 8 * RS_WAVES) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = s[(size_t)(k + u * RS_WAVES) * n];
#pragma unroll
            for (int u = 0; u < 8; ++u) g += v[u];
        }
        for (; k < nslab; k += RS_WAVES) g += s[(size_t)k * n];
    }
    part[wave][lane] = g;
    __syncthreads();
    if (wave == 0 && i < n) {
        float t = acc ? grad[i] : 0.f;
#pragma unroll
        for (int w = 0; w < RS_WAVES; ++w) t += part[w][lane];
        if (grad) grad[i] = t;
        if (param) param[i] = param[i] - lr * t;
    }
}

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ param,
                                                  const float* __restrict__ grad, int n, float lr) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
        param[i] = param[i] - lr * grad[i];
}

__device__ __forceinline__ float block_sum_256(const float* __restrict__ v, int n) {
    __shared__ float red[4];
    float s = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) s += v[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    return ((red[0] + red[1]) + red[2]) + red[3];
}

__global__ __launch_bounds__(256) void loss_sum_kernel(const float* __restrict__ v, int n, float scale,
                                                       float* __restrict__ out) {
    const float s = block_sum_256(v, n);
    if (threadIdx.x == 0) out[0] = s * scale;
}

__global__ __launch_bounds__(256) void loss_log_kernel(const float* __restrict__ v, int n, float scale,
                                                       float* __restrict__ ring, int capacity,
                                                       int* __restrict__ counter) {
    const float s = block_sum_256(v, n);
    if (threadIdx.x == 0) {
        const int c = *counter;
        ring[c % capacity] = s * scale;
        *counter = c + 1;
    }
}

static inline int grid_for(int n) {
    int g = (n + 255) / 256;
    return g > 2048 ? 2048 : (g < 1 ? 1 : g);
}

extern "C" int slk_reduce_slabs(const float* slabs, int nslab, int n, float* out, int accumulate,
                                void* stream) {
    SLK_CHECK_ARG(nslab >= 0 && n >= 0);
    if (n == 0) return 0;
    SLK_CHECK_ARG(out && (slabs || nslab == 0));
    sgd_from_slabs_kernel<<<(n + 63) / 64, 1024, 0, slk_stream(stream)>>>(nullptr, out, slabs, nslab, n, 0.f,
                                                                           accumulate ? 1 : 0);
    return slk_launch_status();
}

extern "C" int slk_sgd_from_slabs(float* param, float* grad, const float* slabs, int nslab, int n,
                                  float lr, void* stream) {
    SLK_CHECK_ARG(nslab >= 0 && n >= 0);
    if (n == 0) return 0;
    SLK_CHECK_ARG(param && (slabs || nslab == 0));
    sgd_from_slabs_kernel<<<(n + 63) / 64, 1024, 0, slk_stream(stream)>>>(param, grad, slabs, nslab, n, lr, 0);
    return slk_launch_status();
}

extern "C" int slk_sgd(float* param, const float* grad, int n, float lr, void* stream) {
    SLK_CHECK_ARG(n >= 0);
    if (n == 0) return 0;
    SLK_CHECK_ARG(param && grad);
    sgd_kernel<<<grid_for(n), 256, 0, slk_stream(stream)>>>(param, grad, n, lr);
    return slk_launch_status();
}

extern "C" int slk_loss_sum(const float* values, int n, float scale, float* out, void* stream) {
    SLK_CHECK_ARG(n > 0);
    SLK_CHECK_ARG(values && out);
    loss_sum_kernel<<<1, 256, 0, slk_stream(stream)>>>(values, n, scale, out);
    return slk_launch_status();
}

extern "C" int slk_loss_log(const float* values, int n, float scale, float* ring, int capacity,
                            int* counter, void* stream) {
    SLK_CHECK_ARG(n > 0 && capacity > 0);
    SLK_CHECK_ARG(values && ring && counter);
    loss_log_kernel<<<1, 256, 0, slk_stream(stream)>>>(values, n, scale, ring, capacity, counter);
    return slk_launch_status();
}

extern "C" int slk_abi_version(void) { return SLK_ABI_VERSION; }

extern "C" const char* slk_error_string(int err) {
    return hipGetErrorString(static_cast<hipError_t>(err));
}
