// Microbenchmark: how many independent SCALAR f32 VALU instructions (v_add_f32) hide between
// back-to-back v_mfma_f32_16x16x4_f32 on gfx950 (one wave per SIMD), vs packed v_pk_add_f32.
// Prints ns per MFMA for 0..8 scalar fillers per MFMA and 2/4 packed fillers per MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <int NS, int NP, int NL = 0, int NL4 = 0>
__global__ void kern(float* out, int iters, float seed) {
    __shared__ float lds[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = seed * i;
    __syncthreads();
    float lv[8];
    float4 lv4[4];
    for (int i = 0; i < 8; ++i) lv[i] = 0.f;
    for (int i = 0; i < 4; ++i) lv4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int lbase = (threadIdx.x & 63) * 4;
    f32x4 acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = f32x4{seed, 0, 0, 0};
    float s[8];
    f2 p[4];
    for (int i = 0; i < 8; ++i) s[i] = seed * (i + 1);
    for (int i = 0; i < 4; ++i) p[i] = f2{seed * i, seed + i};
    const float a = seed * threadIdx.x, b = seed + threadIdx.x, c = seed * 3.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
            // 8 independent chains: filler k of this gap advances chain k (latency never exposed)
#pragma unroll
            for (int k = 0; k < NS; ++k) asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[k]) : "v"(c));
#pragma unroll
            for (int k = 0; k < NP; ++k) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[k]) : "v"(p[(k + 1) & 3]));
#pragma unroll
            for (int k = 0; k < NL; ++k) asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(lv[k]) : "v"(lbase * 4), "i"(k * 1024));
#pragma unroll
            for (int k = 0; k < NL4; ++k) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(lv4[k]) : "v"(lbase * 4), "i"(k * 1024));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    for (int i = 0; i < 8; ++i) s[i] += lv[i];
    for (int i = 0; i < 4; ++i) s[i] += lv4[i].x + lv4[i].w;
    float r = 0;
    for (int i = 0; i < 16; ++i) r += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    for (int i = 0; i < 8; ++i) r += s[i];
    for (int i = 0; i < 4; ++i) r += p[i].x + p[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int NS, int NP, int NL = 0, int NL4 = 0>
float run(float* out, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<NS, NP, NL, NL4><<<256, 256>>>(out, iters, 1e-3f);
    (void)hipEventRecord(e0);
    kern<NS, NP, NL, NL4><<<256, 256>>>(out, iters, 1e-3f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e6f / (iters * 16.f);
}

int main() {
    float* out;
    (void)hipMalloc(&out, 256 * 256 * 4);
    const int it = 20000;
    printf("ns per f32 16x16x4 MFMA, scalar fillers/gap 0,1,2,3,4,6,8: %.2f %.2f %.2f %.2f %.2f %.2f %.2f | packed 2: %.2f packed 4: %.2f\n",
           run<0, 0>(out, it), run<1, 0>(out, it), run<2, 0>(out, it), run<3, 0>(out, it), run<4, 0>(out, it),
           run<6, 0>(out, it), run<8, 0>(out, it), run<0, 2>(out, it), run<0, 4>(out, it));
    printf("ds_read_b32 fillers/gap 1,2,4: %.2f %.2f %.2f | ds_read_b128 fillers/gap 1,2: %.2f %.2f ns per MFMA\n",
           run<0, 0, 1, 0>(out, it), run<0, 0, 2, 0>(out, it), run<0, 0, 4, 0>(out, it), run<0, 0, 0, 1>(out, it),
           run<0, 0, 0, 2>(out, it));
    return 0;
}
