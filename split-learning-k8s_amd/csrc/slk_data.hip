// slk_data.hip — the MNIST batch loader as one HBM-resident gather.
//
// The reference builds batches with DataLoader(train_dataset, batch_size=64, shuffle=True)
// (client_part.py:98) over torchvision MNIST with ToTensor() + Normalize((0.1307,), (0.3081,))
// (client_part.py:61-64): per sample, u8 -> float32 /255, then (v - mean) / std, all in float32.
// Here the whole u8 dataset (47 MB for the 60k training set) stays resident in HBM, and a batch
// is one launch: gather the shuffled rows, normalise, write x [B,1,28,28] f32 and y [B] i64.
// Division is IEEE-correct (hipcc's default for f32 '/'), so x is bit-identical to the torchvision
// transform. HBM-bound: 784 B read + 3,136 B written per sample.
#include "slk_common.h"

namespace {
constexpr int IMG = 28 * 28;        // bytes per image
constexpr int CHUNKS = IMG / 4;     // 196 u32 words per image
}

__global__ __launch_bounds__(256) void mnist_batch_kernel(const uint32_t* __restrict__ images,
                                                          const uint8_t* __restrict__ labels,
                                                          int n_images, const int64_t* __restrict__ idx,
                                                          int B, float mean, float stdv,
                                                          float4* __restrict__ x, int64_t* __restrict__ y,
                                                          int* __restrict__ err) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= B * CHUNKS) return;
    const int s = g / CHUNKS, c = g - s * CHUNKS;
    int64_t i = idx[s];
    if (i < 0 || i >= n_images) {     // out-of-range index: flag it, read row 0 instead of faulting
        if (c == 0 && err) *err = 1;
        i = 0;
    }
    const uint32_t w = images[(size_t)i * CHUNKS + c];
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float t = (float)((w >> (8 * k)) & 0xffu) / 255.0f;   // ToTensor
        v[k] = (t - mean) / stdv;                                     // Normalize
    }
    x[g] = make_float4(v[0], v[1], v[2], v[3]);
    if (c == 0) y[s] = (int64_t)labels[i];
}

extern "C" int slk_mnist_batch(const uint8_t* images, const uint8_t* labels, int n_images,
                               const int64_t* idx, int B, float mean, float stdv, float* x,
                               int64_t* y, int* err_flag, void* stream) {
    SLK_CHECK_ARG(B >= 0 && n_images > 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(images && labels && idx && x && y);
    SLK_CHECK_ARG(((uintptr_t)images & 3) == 0 && ((uintptr_t)x & 15) == 0);
    const int total = B * CHUNKS;
    mnist_batch_kernel<<<(total + 255) / 256, 256, 0, slk_stream(stream)>>>(
        reinterpret_cast<const uint32_t*>(images), labels, n_images, idx, B, mean, stdv,
        reinterpret_cast<float4*>(x), y, err_flag);
    return slk_launch_status();
}
