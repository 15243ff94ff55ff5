// Probe of gfx950's 2:4-sparse f16 MFMA, v_smfmac_f32_16x16x64_f16 (no public ISA table here): which dense K
// each lane's compressed A values and dense B values stand for, how the per-lane index word is read, and the
// issue cost against the dense v_mfma_f32_16x16x32_f16 — before any kernel is built on it.
//   semantics: one wave, random small-integer operands (exact in f32), random valid indices (two distinct
//              positions per group of 4, ascending); the host checks the output against candidate layouts.
//   timing:    one 256-thread workgroup per CU x 256 CUs, 4 or 8 independent accumulator chains per wave,
//              s_memtime cycles per instruction per wave (1 or 2 waves per SIMD), dense vs sparse.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void sem(const _Float16* a, const _Float16* b, const int* idx, float* d, int abid1) {
    const int l = threadIdx.x;
    f16x8 av;
    f16x16 bv;
    for (int i = 0; i < 8; ++i) av[i] = a[l * 8 + i];
    for (int i = 0; i < 16; ++i) bv[i] = b[l * 16 + i];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (abid1) acc = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av, bv, acc, idx[l], 0, 1);
    else acc = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av, bv, acc, idx[l], 0, 0);
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = acc[r];
}

// one-hot decode: wave w sets compressed A value (lane la = 16 (w / 8), value i = w % 8) to 1 (row m = 0), all
// other A values 0; B[lane][j] = 1 + 16 (lane / 16) + j + 64 (lane % 16) (distinct, exact in f16); index word
// per lane = idxw. D[0][n] then reads the B value (lane 16 g + n, j) that A's value meets: g and j decoded on the host.
__global__ void onehot(float* d, int idxw) {
    const int l = threadIdx.x, w = blockIdx.x;
    const int la = 16 * (w / 8), i1 = w % 8;
    f16x8 av;
    f16x16 bv;
    for (int i = 0; i < 8; ++i) av[i] = (_Float16)((l == la && i == i1) ? 1.f : 0.f);
    for (int j = 0; j < 16; ++j) bv[j] = (_Float16)(float)(1 + 16 * (l / 16) + j + 64 * (l % 16));
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av, bv, acc, idxw, 0, 0);
    for (int r = 0; r < 4; ++r) d[(w * 64 + l) * 4 + r] = acc[r];
}

template <bool SPARSE, int NCH>
__global__ __launch_bounds__(512) void timing(float* out, unsigned long long* cyc, int iters) {
    const int l = threadIdx.x & 63;
    f16x8 a;
    f16x16 b;
    for (int i = 0; i < 8; ++i) a[i] = (_Float16)(0.001f * ((l * 7 + i * 3) % 13));
    for (int i = 0; i < 16; ++i) b[i] = (_Float16)(0.001f * ((l * 5 + i * 11) % 17));
    const f16x8 b8 = __builtin_shufflevector(b, b, 0, 1, 2, 3, 4, 5, 6, 7);
    const int ix = 0x4E4E4E4E & 0xFFFF;  // (0,1),(2,3)... valid ascending pairs: 0b01001110 per byte -> (2,3),(0,1)
    f32x4 acc[NCH];
    for (int c = 0; c < NCH; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, (float)c};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if (SPARSE) acc[c] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(a, b, acc[c], ix, 0, 0);
            else acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b8, acc[c], 0, 0, 0);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int c = 0; c < NCH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (l == 0) cyc[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}

static int rnd(int n) { return rand() % n; }

int main() {
    const int L = 64;
    _Float16 ha[L * 8], hb[L * 16];
    float fa[L * 8], fb[L * 16], hd[L * 4];
    int hidx[L];
    srand(7);
    for (int i = 0; i < L * 8; ++i) { fa[i] = (float)(rnd(9) - 4); ha[i] = (_Float16)fa[i]; }
    for (int i = 0; i < L * 16; ++i) { fb[i] = (float)(rnd(9) - 4); hb[i] = (_Float16)fb[i]; }
    const int pairs[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};
    for (int l = 0; l < L; ++l) {
        int w = 0;
        for (int g = 0; g < 4; ++g) {
            const int p = rnd(6);
            w |= (pairs[p][0] | (pairs[p][1] << 2)) << (4 * g);
        }
        hidx[l] = w | (rnd(65536) << 16);  // upper half random: must not matter at abid 0
    }
    _Float16 *da, *db;
    int* didx;
    float* dd;
    hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&didx, sizeof hidx); hipMalloc(&dd, sizeof hd);
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    hipMemcpy(didx, hidx, sizeof hidx, hipMemcpyHostToDevice);
    for (int abid = 0; abid < 2; ++abid) {
        hipLaunchKernelGGL(sem, dim3(1), dim3(64), 0, 0, da, db, didx, dd, abid);
        hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost);
        // candidate layouts. D: lane l holds D[4 (l / 16) + r][l % 16] (as the dense 16x16x32).
        // B lane l (col n = l % 16) value j stands for dense K = kb(l, j):
        //   HB0: 16 (l / 16) + j            HB1: j < 8 ? 8 (l / 16) + j : 32 + 8 (l / 16) + j - 8
        // A lane l (row m = l % 16) compressed value i: group i / 2 of the SAME lane's K list (the lane's 16 K
        // in 4 groups of 4), position idx_i = (index word >> (2 i + 16 abid)) & 3
        for (int hb = 0; hb < 2; ++hb) {
            double err = 0.0, mx = 0.0;
            for (int m = 0; m < 16; ++m)
                for (int n = 0; n < 16; ++n) {
                    double A[64] = {0}, Bk[64];
                    for (int lg = 0; lg < 4; ++lg) {
                        const int la = 16 * lg + m, lb = 16 * lg + n;
                        int kl[16];
                        for (int j = 0; j < 16; ++j) kl[j] = hb == 0 ? 16 * lg + j : (j < 8 ? 8 * lg + j : 32 + 8 * lg + j - 8);
                        for (int j = 0; j < 16; ++j) Bk[kl[j]] = fb[lb * 16 + j];
                        const unsigned w = (unsigned)hidx[la] >> (16 * abid);
                        for (int i = 0; i < 8; ++i) {
                            const int pos = (w >> (2 * i)) & 3;
                            A[kl[4 * (i / 2) + pos]] += fa[la * 8 + i];
                        }
                    }
                    double s = 0.0;
                    for (int k = 0; k < 64; ++k) s += A[k] * Bk[k];
                    const int lo = 16 * (m / 4) + n, r = m % 4;
                    err = fmax(err, fabs(s - hd[lo * 4 + r]));
                    mx = fmax(mx, fabs(s));
                }
            printf("abid %d layout HB%d: max |err| %.3g (max |D| %.3g)%s\n", abid, hb, err, mx, err == 0.0 ? "  <== MATCH" : "");
        }
    }
    // one-hot decode, for several index words
    {
        float* d1;
        hipMalloc(&d1, 32 * 64 * 4 * 4);
        static float h1[32 * 64 * 4];
        const int words[4] = {0x0000, 0xE4E4 /* 0b11100100: (0,1),(2,3) */, 0x4E4E, 0xD8D8};
        for (int wi = 0; wi < 4; ++wi) {
            const int iw = words[wi] | (words[wi] << 16);
            hipLaunchKernelGGL(onehot, dim3(32), dim3(64), 0, 0, d1, iw);
            hipMemcpy(h1, d1, sizeof h1, hipMemcpyDeviceToHost);
            printf("index word 0x%04x:\n", words[wi]);
            for (int w = 0; w < 32; ++w) {
                printf("  A lane %2d value %d ->", 16 * (w / 8), w % 8);
                int hits = 0;
                for (int l = 0; l < 64; ++l)
                    for (int r = 0; r < 4; ++r) {
                        const float v = h1[(w * 64 + l) * 4 + r];
                        if (v != 0.f) {
                            const int m = 4 * (l / 16) + r, n = l % 16, bv = (int)v - 1;
                            if (hits < 3) printf(" D[%d][%d] = B(lane %d, j %d)", m, n, 16 * ((bv % 64) / 16) + bv / 64, bv % 16);
                            ++hits;
                        }
                    }
                printf("  (%d nonzero)\n", hits);
            }
        }
    }
    // timing
    const int NB = 256, T = 256, IT = 2000;
    float* o;
    unsigned long long* cy;
    hipMalloc(&o, NB * 512 * 4);
    hipMalloc(&cy, NB * 8 * 8);
    unsigned long long hc[NB * 8];
    for (int rep = 0; rep < 2; ++rep) {
        for (int v = 0; v < 4; ++v) {
            for (int wps = 1; wps <= 2; ++wps) {
                const int threads = T * wps;
                auto run = [&](void (*k)(float*, unsigned long long*, int), int nch, const char* name) {
                    hipLaunchKernelGGL(k, dim3(NB), dim3(threads), 0, 0, o, cy, IT);
                    hipDeviceSynchronize();
                    hipMemcpy(hc, cy, NB * (threads / 64) * 8, hipMemcpyDeviceToHost);
                    double s = 0;
                    for (int i = 0; i < NB * threads / 64; ++i) s += hc[i];
                    s /= NB * threads / 64;
                    if (rep == 1) printf("%-7s chains %d waves/SIMD %d: %.2f cycles per instruction per wave\n", name, nch, wps, s / (IT * nch));
                };
                if (v == 0) run(timing<false, 4>, 4, "dense");
                if (v == 1) run(timing<true, 4>, 4, "sparse");
                if (v == 2) run(timing<false, 8>, 8, "dense");
                if (v == 3) run(timing<true, 8>, 8, "sparse");
            }
        }
    }
    return 0;
}
