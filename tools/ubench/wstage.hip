// Microbenchmark: the cost of streaming a weight slice into LDS beside bf16 MFMAs, the K5 conv loop's
// regime (2 workgroups x 4 waves per CU = 2 waves per SIMD; per step and wave 16
// v_mfma_f32_16x16x32_bf16, 8 ds_read_b128 fragment reads, one s_barrier) — per step and wave the
// slice arrives as
//   V0: nothing (MFMA + fragment reads + barrier only)
//   V1: NP LDS-DMA pieces (global_load_lds_dwordx4, 1 KiB each per wave), counted vmcnt waits
//   V2: NP global_load_dwordx4 into registers two steps ahead + NP ds_write_b128 (register staging)
// from an L2-resident 2 MiB buffer. Prints ns per step. build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(size_t)(lds_ptr_t)(const_cast<void*>(p)); }

template <int V, int NP, bool F32 = false>
__global__ __launch_bounds__(256, F32 ? 1 : 2) void kern(const char* __restrict__ src, float* out, int iters) {
    __shared__ __attribute__((aligned(1024))) char lds[32768];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    f32x4 acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf8 F[2][8];
    for (int k = 0; k < 2; ++k) for (int i = 0; i < 8; ++i) for (int j = 0; j < 8; ++j) F[k][i][j] = (short)(lane + i + j + k);
    const uint32_t rbase = lds_addr(lds) + lane * 16;
    const char* gbase = src + ((blockIdx.x * 4 + wave) & 127) * 16384 + lane * 16;
    u32x4 stage[3][NP];
    for (int k = 0; k < 3; ++k) for (int p = 0; p < NP; ++p) stage[k][p] = u32x4{0u, 0u, 0u, 0u};
    for (int it = 0; it < iters; it += 6) {
#pragma unroll
        for (int u = 0; u < 6; ++u) {
            const int step = it + u;
            // weight ring: 2 slots x 4 waves x 3 KiB above the 8 KiB fragment area
            const uint32_t wslot = lds_addr(lds) + 8192 + (u & 1) * 12288 + wave * 3072;
            if constexpr (V == 1) {
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NP) : "memory");
            } else if constexpr (V == 2) {
                // the loads of two steps ago have landed -> LDS
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NP) : "memory");
#pragma unroll
                for (int p = 0; p < NP; ++p)
                    asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(wslot + (uint32_t)(lane * 16)), "v"(stage[(u + 1) % 3][p]), "i"(p * 1024) : "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            const char* g = gbase + (step & 7) * 2048;
            if constexpr (V == 1) {
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    uint32_t keep;
                    const uint32_t dst = __builtin_amdgcn_readfirstlane(wslot + p * 1024);
                    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                                 : "=&s"(keep) : "v"(g + p * 1024), "s"(dst) : "memory");
                }
            } else if constexpr (V == 2) {
#pragma unroll
                for (int p = 0; p < NP; ++p)
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(stage[u % 3][p]) : "v"(g + p * 1024) : "memory");
            }
            // fragments of the next step (waited by the next step's lgkmcnt before its barrier)
#pragma unroll
            for (int i = 0; i < 8; ++i)
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(F[(u + 1) & 1][i]) : "v"(rbase), "i"(i * 1024) : "memory");
            if constexpr (F32) {
                // the fp32 Winograd kernels' regime: one wave per SIMD, 32 v_mfma_f32_16x16x4_f32 per step
#pragma unroll
                for (int j = 0; j < 32; ++j)
                    acc[j & 15] = __builtin_amdgcn_mfma_f32_16x16x4f32(__builtin_bit_cast(float, (int)F[u & 1][j & 7][0] | ((int)F[u & 1][j & 7][1] << 16)),
                                                                        __builtin_bit_cast(float, (int)F[u & 1][(j >> 3) + 4][2]), acc[j & 15], 0, 0, 0);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int f = 0; f < 4; ++f)
                        acc[4 * i + f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F[u & 1][i], F[u & 1][4 + f], acc[4 * i + f], 0, 0, 0);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    for (int k = 0; k < 3; ++k) for (int p = 0; p < NP; ++p) s += (float)stage[k][p][0];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int V, int NP, bool F32 = false>
float run(const char* src, float* out, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    kern<V, NP, F32><<<F32 ? 256 : 512, 256>>>(src, out, iters);
    hipEventRecord(e0);
    kern<V, NP, F32><<<F32 ? 256 : 512, 256>>>(src, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e6f / iters;
}

int main() {
    char* src;
    float* out;
    hipMalloc(&src, 4 << 20);  // max offset 127*16 KiB + 7*2 KiB + 3 KiB
    hipMemset(src, 0, 4 << 20);
    hipMalloc(&out, 512 * 256 * 4);
    const int iters = 30000;  // multiple of 6
    for (int rep = 0; rep < 2; ++rep)
        printf("ns/step: none %.1f | NP=1: dma %.1f regs %.1f | NP=2: dma %.1f regs %.1f | NP=3: dma %.1f regs %.1f\n",
               run<0, 1>(src, out, iters), run<1, 1>(src, out, iters), run<2, 1>(src, out, iters),
               run<1, 2>(src, out, iters), run<2, 2>(src, out, iters), run<1, 3>(src, out, iters),
               run<2, 3>(src, out, iters));
    for (int rep = 0; rep < 2; ++rep)
        printf("f32 MFMA, 1 wave/SIMD, ns/step: none %.1f | NP=1: dma %.1f regs %.1f | NP=2: dma %.1f regs %.1f | NP=3: dma %.1f regs %.1f\n",
               run<0, 1, true>(src, out, iters), run<1, 1, true>(src, out, iters), run<2, 1, true>(src, out, iters),
               run<1, 2, true>(src, out, iters), run<2, 2, true>(src, out, iters), run<1, 3, true>(src, out, iters),
               run<2, 3, true>(src, out, iters));
    return 0;
}
