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
// Few slabs (<= RS_COLS_MAX) -> thread = column, slabs summed in ascending order with 8 loads in flight,
// 1024 columns per block; up to RS_MID_MAX (the fc wgrad set, 64 at B = 4096) -> 256 columns per block,
// 4 waves per 64 columns each summing every 4th slab, the 4 partials added in order (round 6: one thread
// per column walked 64 slabs in 8 dependent rounds on 91 blocks; 64-column blocks over 92,170 columns
// were ~1,400 dispatch-bound blocks); many slabs -> 64 columns per block, 16 waves over the slab range.
#ifndef SLK_RS_MID
#define SLK_RS_MID 1  // 0: the round-5 forms (<= 64 slabs thread per column), kept for the A/B
#endif
constexpr int RS_COLS_MAX = SLK_RS_MID ? 16 : 64, RS_MID_MAX = 64;
__host__ __device__ constexpr int rs_cols_per_block(int nslab) {
    return nslab <= RS_COLS_MAX ? 1024 : (nslab <= RS_MID_MAX ? 256 : 64);
}
static inline int rs_blocks(int n, int nslab) { return (n + rs_cols_per_block(nslab) - 1) / rs_cols_per_block(nslab); }

__device__ __forceinline__ void slab_reduce_sgd_cols(float* __restrict__ param, float* __restrict__ grad,
                                                     const float* __restrict__ slabs, int nslab, int n, float lr,
                                                     int acc, int blk) {
    const int i = blk * 1024 + threadIdx.x;
    if (i >= n) return;
    const float* s = slabs + i;
    float g = 0.f;
    int k = 0;
    for (; k + 8 <= nslab; k += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = s[(size_t)(k + u) * n];
#pragma unroll
        for (int u = 0; u < 8; ++u) g += v[u];
    }
    for (; k < nslab; ++k) g += s[(size_t)k * n];
    const float t = acc ? grad[i] + g : g;
    if (grad) grad[i] = t;
    if (param) param[i] = param[i] - lr * t;
}

__device__ __forceinline__ void slab_reduce_sgd_rows(float* __restrict__ param, float* __restrict__ grad,
                                                     const float* __restrict__ slabs, int nslab, int n, float lr,
                                                     int acc, int blk) {
    __shared__ float part[RS_WAVES][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i = blk * 64 + lane;
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

__device__ __forceinline__ void slab_reduce_sgd_mid(float* __restrict__ param, float* __restrict__ grad,
                                                    const float* __restrict__ slabs, int nslab, int n, float lr,
                                                    int acc, int blk) {
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
        float t = acc ? grad[i] : 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) t += part[q][c];
        if (grad) grad[i] = t;
        if (param) param[i] = param[i] - lr * t;
    }
}

__device__ __forceinline__ void slab_reduce_sgd(float* __restrict__ param, float* __restrict__ grad,
                                                const float* __restrict__ slabs, int nslab, int n, float lr,
                                                int acc, int blk) {
    if (rs_cols_per_block(nslab) == 1024)
        slab_reduce_sgd_cols(param, grad, slabs, nslab, n, lr, acc, blk);
    else if (rs_cols_per_block(nslab) == 256)
        slab_reduce_sgd_mid(param, grad, slabs, nslab, n, lr, acc, blk);
    else
        slab_reduce_sgd_rows(param, grad, slabs, nslab, n, lr, acc, blk);
}

__global__ __launch_bounds__(1024) void sgd_from_slabs_kernel(float* __restrict__ param,
                                                              float* __restrict__ grad,
                                                              const float* __restrict__ slabs,
                                                              int nslab, int n, float lr, int acc) {
    slab_reduce_sgd(param, grad, slabs, nslab, n, lr, acc, blockIdx.x);
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

// Every optimizer step of one split step in ONE launch (the last launches of the step are latency,
// not bandwidth): block 0 (if loss_v) logs the loss, the next nblk0 blocks reduce + step segment 0,
// the next nblk1 segment 1, .... Each block runs exactly the code of sgd_from_slabs_kernel /
// loss_log_kernel on its slice, so the results are bit-identical to the separate launches.
struct SgdSeg {
    float* param;
    float* grad;
    const float* slabs;
    int nslab, n, nblk;
};
constexpr int SGD_MAXSEG = 4;
struct SgdMulti {
    SgdSeg seg[SGD_MAXSEG];
    int nseg;
    float lr;
    const float* loss_v;
    int loss_n;
    float loss_scale;
    float* ring;
    int capacity;
    int* counter;
};

__global__ __launch_bounds__(1024) void sgd_multi_kernel(const SgdMulti a) {
    int blk = blockIdx.x;
    if (a.loss_v) {
        // block 0 logs the loss (dispatched first: its serial sum overlaps the segments' blocks);
        // threads 0..255 sum exactly as block_sum_256 (the other waves add nothing)
        if (blk == 0) {
            __shared__ float red[4];
            float v = 0.f;
            if (threadIdx.x < 256)
                for (int i = threadIdx.x; i < a.loss_n; i += 256) v += a.loss_v[i];
            v = wave_sum(v);
            if (threadIdx.x < 256 && (threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
            __syncthreads();
            if (threadIdx.x == 0) {
                const float tot = ((red[0] + red[1]) + red[2]) + red[3];
                const int c = *a.counter;
                a.ring[c % a.capacity] = tot * a.loss_scale;
                *a.counter = c + 1;
            }
            return;
        }
        --blk;
    }
#pragma unroll
    for (int s = 0; s < SGD_MAXSEG; ++s) {
        if (s < a.nseg) {
            if (blk < a.seg[s].nblk) {
                slab_reduce_sgd(a.seg[s].param, a.seg[s].grad, a.seg[s].slabs, a.seg[s].nslab, a.seg[s].n, a.lr, 0, blk);
                return;
            }
            blk -= a.seg[s].nblk;
        }
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
    sgd_from_slabs_kernel<<<rs_blocks(n, nslab), 1024, 0, slk_stream(stream)>>>(nullptr, out, slabs, nslab, n, 0.f,
                                                                           accumulate ? 1 : 0);
    return slk_launch_status();
}

extern "C" int slk_sgd_from_slabs(float* param, float* grad, const float* slabs, int nslab, int n,
                                  float lr, void* stream) {
    SLK_CHECK_ARG(nslab >= 0 && n >= 0);
    if (n == 0) return 0;
    SLK_CHECK_ARG(param && (slabs || nslab == 0));
    sgd_from_slabs_kernel<<<rs_blocks(n, nslab), 1024, 0, slk_stream(stream)>>>(param, grad, slabs, nslab, n, lr, 0);
    return slk_launch_status();
}

extern "C" int slk_sgd_multi_from_slabs(float* const* params, float* const* grads, const float* const* slabs,
                                        const int* nslab, const int* n, int nseg, float lr,
                                        const float* loss_values, int loss_n, float loss_scale, float* ring,
                                        int capacity, int* counter, void* stream) {
    SLK_CHECK_ARG(nseg >= 0 && nseg <= SGD_MAXSEG && (nseg == 0 || (params && slabs && nslab && n)));
    SLK_CHECK_ARG(!loss_values || (loss_n > 0 && capacity > 0 && ring && counter));
    SgdMulti a{};
    int nblk = 0;
    for (int s = 0; s < nseg; ++s) {
        // a segment with no param is a reduce only (grad = sum of slabs): the all-reduce bucket fill
        SLK_CHECK_ARG(n[s] >= 0 && nslab[s] >= 0 && (params[s] || (grads && grads[s])) && (slabs[s] || nslab[s] == 0));
        a.seg[s] = SgdSeg{params[s], grads ? grads[s] : nullptr, slabs[s], nslab[s], n[s], rs_blocks(n[s], nslab[s])};
        nblk += a.seg[s].nblk;
    }
    a.nseg = nseg;
    a.lr = lr;
    a.loss_v = loss_values;
    a.loss_n = loss_n;
    a.loss_scale = loss_scale;
    a.ring = ring;
    a.capacity = capacity;
    a.counter = counter;
    if (loss_values) ++nblk;
    if (nblk == 0) return 0;
    sgd_multi_kernel<<<nblk, 1024, 0, slk_stream(stream)>>>(a);
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

// sha256 of the library's sources (splitcnn/build.py source_hash), baked in at compile time so the
// loader can refuse a binary built from other sources; the tag is also searchable in the file.
#ifndef SLK_BUILD_ID
#define SLK_BUILD_ID "unknown"
#endif
extern "C" __attribute__((used, visibility("default"))) const char slk_build_id_tag[] = "SLK_BUILD_ID:" SLK_BUILD_ID;
extern "C" const char* slk_build_id(void) { return slk_build_id_tag + 13; }

extern "C" const char* slk_error_string(int err) {
    return hipGetErrorString(static_cast<hipError_t>(err));
}
