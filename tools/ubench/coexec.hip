// Microbenchmark: do v_mfma_f32_16x16x4_f32 and independent VALU (v_pk_add_f32) execute concurrently
// on gfx950? Times K iterations of {16 MFMAs on 16 independent accumulators} with 0 / 16 / 32 / 64
// packed adds per iteration on independent registers, one wave per SIMD and two waves per SIMD.
// Also the bf16 16x16x32 MFMA for contrast. Prints ns per iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef short bf8 __attribute__((ext_vector_type(8)));

template <int NV, bool BF>
__global__ void kern(float* out, int iters, float seed) {
    f32x4 acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = f32x4{seed, 0, 0, 0};
    f2 v[8];
    for (int i = 0; i < 8; ++i) v[i] = f2{seed * i, seed + i};
    const float a = seed * threadIdx.x, b = seed + threadIdx.x;
    bf8 ab;
    for (int i = 0; i < 8; ++i) ab[i] = (short)(threadIdx.x + i);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if constexpr (BF) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, acc[i], 0, 0, 0);
            else acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < NV / 16; ++j) {
                f2& x = v[(i * (NV / 16) + j) & 7];
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x) : "v"(v[(i + j + 1) & 7]));
            }
        }
    }
    float s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    for (int i = 0; i < 8; ++i) s += v[i].x + v[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NV, bool BF>
float run(float* out, int threads, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<NV, BF><<<256, threads>>>(out, iters, 1e-3f);
    hipEventRecord(e0);
    kern<NV, BF><<<256, threads>>>(out, iters, 1e-3f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e6f / iters;
}

int main() {
    float* out;
    hipMalloc(&out, 256 * 512 * 4);
    const int iters = 20000;
    for (int threads : {256, 512}) {
        printf("waves/SIMD=%d f32: nv0 %.1f nv16 %.1f nv32 %.1f nv64 %.1f | bf16: nv0 %.1f nv32 %.1f nv64 %.1f ns/iter\n",
               threads / 256, run<0, false>(out, threads, iters), run<16, false>(out, threads, iters),
               run<32, false>(out, threads, iters), run<64, false>(out, threads, iters),
               run<0, true>(out, threads, iters), run<32, true>(out, threads, iters), run<64, true>(out, threads, iters));
    }
    return 0;
}
