// Profiling-only microbenchmark: sustained v_mfma_f32_32x32x2_f32 rate and in-kernel clock.
// Each wave runs NCHAIN independent accumulator chains for ITERS steps on random-ish operands.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NCHAIN>
__global__ __launch_bounds__(256) void mfma_loop(const float* in, float* out, int iters, unsigned long long* clk) {
    float a = in[threadIdx.x], b = in[threadIdx.x + 256];
    f32x16 acc[NCHAIN];
    for (int c = 0; c < NCHAIN; ++c)
        for (int r = 0; r < 16; ++r) acc[c][r] = in[(c * 16 + r) & 511];
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < NCHAIN; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int c = 0; c < NCHAIN; ++c)
        for (int r = 0; r < 16; ++r) s += acc[c][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) { clk[blockIdx.x * 2] = t1 - t0; clk[blockIdx.x * 2 + 1] = r1 - r0; }
}

template <int NCHAIN>
void run(int blocks, int iters, float* in, float* out, unsigned long long* clk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    mfma_loop<NCHAIN><<<blocks, 256>>>(in, out, iters, clk);
    hipEventRecord(e0);
    for (int rep = 0; rep < 5; ++rep) mfma_loop<NCHAIN><<<blocks, 256>>>(in, out, iters, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
    std::vector<unsigned long long> h(blocks * 2);
    hipMemcpy(h.data(), clk, blocks * 16, hipMemcpyDeviceToHost);
    double ghz = 0; for (int i = 0; i < blocks; ++i) ghz += (double)h[2*i] / (double)h[2*i+1] * 0.1; ghz /= blocks;
    double flops = (double)blocks * 4 /*waves*/ * iters * NCHAIN * 32.0 * 32 * 2 * 2;
    printf("{\"chains\": %d, \"blocks\": %d, \"waves_per_simd\": %.2f, \"ms\": %.4f, \"tflops\": %.1f, \"clock_ghz\": %.3f}\n",
           NCHAIN, blocks, blocks * 4.0 / 1024, ms, flops / ms / 1e9, ghz);
}

int main() {
    float *in, *out; unsigned long long* clk;
    hipMalloc(&in, 4096); hipMalloc(&out, 1 << 24); hipMalloc(&clk, 1 << 16);
    std::vector<float> h(1024); for (int i = 0; i < 1024; ++i) h[i] = (i * 7919 % 1000) / 1000.f - 0.5f;
    hipMemcpy(in, h.data(), 4096, hipMemcpyHostToDevice);
    for (int bpc : {1, 2, 3}) { run<3>(256 * bpc, 20000, in, out, clk); run<1>(256 * bpc, 20000, in, out, clk); }
    return 0;
}
