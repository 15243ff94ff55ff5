// slk_optim.hip — deterministic reductions, fused SGD and the device-side loss log.
//
// optim.SGD(lr=0.01) on both sides (client_part.py:17,133; server_part.py:15,52) is
// `p.add_(g, alpha=-lr)` per parameter. Here the parameters of a stage live in one flat block, so
// one launch updates all of them, and the weight-gradient slabs written by the wgrad kernels are
// summed (fixed order, bit-stable) in the same pass that applies the update.
#include "slk_common.h"

__global__ __launch_bounds__(256) void sgd_from_slabs_kernel(float* __restrict__ param,
                                                             float* __restrict__ grad,
                                                             const float* __restrict__ slabs,
                                                             int nslab, int n, float lr, int acc) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        float g = acc ? grad[i] : 0.f;
        const float* s = slabs + i;
        int k = 0;
        for (; k + 4 <= nslab; k += 4) {  // 4 loads in flight, summed in slab order
            const float a0 = s[(size_t)k * n], a1 = s[(size_t)(k + 1) * n];
            const float a2 = s[(size_t)(k + 2) * n], a3 = s[(size_t)(k + 3) * n];
            g += a0; g += a1; g += a2; g += a3;
        }
        for (; k < nslab; ++k) g += s[(size_t)k * n];
        if (grad) grad[i] = g;
        if (param) param[i] = param[i] - lr * g;
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
    sgd_from_slabs_kernel<<<grid_for(n), 256, 0, slk_stream(stream)>>>(nullptr, out, slabs, nslab, n, 0.f,
                                                                        accumulate ? 1 : 0);
    return slk_launch_status();
}

extern "C" int slk_sgd_from_slabs(float* param, float* grad, const float* slabs, int nslab, int n,
                                  float lr, void* stream) {
    SLK_CHECK_ARG(nslab >= 0 && n >= 0);
    if (n == 0) return 0;
    SLK_CHECK_ARG(param && (slabs || nslab == 0));
    sgd_from_slabs_kernel<<<grid_for(n), 256, 0, slk_stream(stream)>>>(param, grad, slabs, nslab, n, lr, 0);
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
