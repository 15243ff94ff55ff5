// Accumulation-bias probe for the x3 scheme (f32 operands split hi/lo, products hh + hl + lh on
// v_mfma_f32_16x16x32_f16): dot products of K = 576 random f32 pairs (the conv2 dgrad's K: 64 co x 9 taps)
// per output, 16 x 16 outputs per wave, 256 waves. Variants:
//   0: all three products of every K-step into ONE accumulator (the shipped kernels)
//   1: hh into acc A, hl + lh into acc B, A + B at the end (VALU add)
//   2: as 0, but every K-step's 3 MFMAs into a zeroed accumulator, added to the running sum by VALU
//   3: as 0, alternate K-steps accumulate -(products) into a second accumulator (operand a negated), acc0 - acc1
//   4: as 1, plus 3's negation on the hh accumulator
// Output: per variant, mean signed error / mean |exact| and max |err| / max |exact| against a float64 sum.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int K = 576, NW = 256;
__device__ inline void split(float v, _Float16& h, _Float16& l) { h = (_Float16)v; l = (_Float16)(v - (float)h); }
__device__ inline f32x4 mf(const f16x8& a, const f16x8& b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
// A [NW][16][K] (scaled so max ~ 2^13), B [NW][K][16]
__global__ void dots(const float* A, const float* Bm, float* D, int variant) {
    const int lane = threadIdx.x, w = blockIdx.x;
    const float* a0 = A + (size_t)w * 16 * K;
    const float* b0 = Bm + (size_t)w * K * 16;
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    for (int s = 0; s < K / 32; ++s) {
        f16x8 ah, al, bh, bl, nah, nal;
        for (int j = 0; j < 8; ++j) {
            const int k = 32 * s + 8 * (lane >> 4) + j;
            _Float16 h, l;
            split(a0[(lane & 15) * K + k], h, l); ah[j] = h; al[j] = l; nah[j] = -h; nal[j] = -l;
            split(b0[k * 16 + (lane & 15)], h, l); bh[j] = h; bl[j] = l;
        }
        if (variant == 0) {
            acc0 = mf(ah, bh, acc0); acc0 = mf(ah, bl, acc0); acc0 = mf(al, bh, acc0);
        } else if (variant == 1) {
            acc0 = mf(ah, bh, acc0); acc1 = mf(ah, bl, acc1); acc1 = mf(al, bh, acc1);
        } else if (variant == 2) {
            f32x4 t = {0, 0, 0, 0};
            t = mf(ah, bh, t); t = mf(ah, bl, t); t = mf(al, bh, t);
            for (int r = 0; r < 4; ++r) acc0[r] += t[r];
        } else if (variant == 3) {
            if (s & 1) { acc1 = mf(nah, bh, acc1); acc1 = mf(nah, bl, acc1); acc1 = mf(nal, bh, acc1); }
            else { acc0 = mf(ah, bh, acc0); acc0 = mf(ah, bl, acc0); acc0 = mf(al, bh, acc0); }
        } else {
            f32x4* hh = (s & 1) ? &acc1 : &acc0;
            // hh: alternate sign per step between two accumulators; cross terms into a third (kept in acc1.. no: use D scratch)
            if (s & 1) *hh = mf(nah, bh, *hh); else *hh = mf(ah, bh, *hh);
        }
    }
    for (int r = 0; r < 4; ++r) {
        float v = acc0[r];
        if (variant == 1) v = acc0[r] + acc1[r];
        if (variant == 3) v = acc0[r] - acc1[r];
        if (variant == 4) v = acc0[r] - acc1[r];
        D[((size_t)w * 16 + 4 * (lane >> 4) + r) * 16 + (lane & 15)] = v;
    }
}
static double gauss() { double u = (rand() + 1.0) / (RAND_MAX + 2.0), v = rand() / (RAND_MAX + 1.0); return sqrt(-2 * log(u)) * cos(6.283185307 * v); }
int main() {
    float *A, *Bm, *D;
    const size_t na = (size_t)NW * 16 * K, nb = (size_t)NW * K * 16;
    hipMallocManaged(&A, na * 4); hipMallocManaged(&Bm, nb * 4); hipMallocManaged(&D, (size_t)NW * 256 * 4);
    srand(7);
    // data like the dgrad: weights ~ U(+-0.06) scaled to max 2^13; dY sparse (3/4 zeros: pool routing), gaussian, scaled
    for (size_t i = 0; i < na; ++i) A[i] = (float)((rand() % 4 == 0) ? gauss() * 2000.0 : 0.0);
    for (size_t i = 0; i < nb; ++i) Bm[i] = (float)((2.0 * rand() / RAND_MAX - 1.0) * 8000.0);
    double* ex = (double*)malloc(NW * 256 * sizeof(double));
    for (int w = 0; w < NW; ++w)
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                double s = 0;
                for (int k = 0; k < K; ++k) s += (double)A[((size_t)w * 16 + i) * K + k] * (double)Bm[((size_t)w * K + k) * 16 + j];
                ex[(w * 16 + i) * 16 + j] = s;
            }
    const char* names[] = {"one acc (shipped)", "hh | cross split", "per-step zero acc + VALU add", "sign-alternating acc pair", "hh only, sign-alternating"};
    for (int v = 0; v < 5; ++v) {
        dots<<<NW, 64>>>(A, Bm, D, v);
        hipDeviceSynchronize();
        double se = 0, sa = 0, me = 0, mx = 0;
        for (int i = 0; i < NW * 256; ++i) {
            double e = D[i] - ex[i];
            if (v == 4) {  // reference for hh-only: exact sum of hh products
                continue;
            }
            se += e; sa += fabs(ex[i]); me = fmax(me, fabs(e)); mx = fmax(mx, fabs(ex[i]));
        }
        if (v < 4) printf("%-32s mean signed err / mean|exact| %+.3e   max|err| / max|exact| %.3e\n", names[v], se / sa, me / mx);
    }
    return 0;
}
