// Statistical probe of v_mfma_f32_16x16x32_f16's accumulation: D = C + sum_k A[i][k] B[k][j] for random
// f16 A, B and f32 C, against the exact sum (double) and its single RNE rounding to f32. Reports how often
// the MFMA differs from RNE(exact), the mean signed error in ulps of the result, and whether the errors lean
// to -inf (truncating alignment) or toward zero.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void mm(const _Float16* A, const _Float16* Bm, const float* C, float* D) {
    const int lane = threadIdx.x;
    f16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * (lane >> 4) + j;
        a[j] = A[(lane & 15) * 32 + k];   // A[i][k], i = lane & 15
        b[j] = Bm[k * 16 + (lane & 15)];  // B[k][j], j = lane & 15
    }
    f32x4 c;
    for (int r = 0; r < 4; ++r) c[r] = C[(4 * (lane >> 4) + r) * 16 + (lane & 15)];
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) D[(4 * (lane >> 4) + r) * 16 + (lane & 15)] = c[r];
}
static double urand() { return rand() / (RAND_MAX + 1.0); }
int main() {
    _Float16 *A, *Bm; float *C, *D;
    hipMallocManaged(&A, 16 * 32 * 2); hipMallocManaged(&Bm, 32 * 16 * 2); hipMallocManaged(&C, 1024); hipMallocManaged(&D, 1024);
    srand(1);
    const char* names[] = {"uniform +-1, C=0", "uniform +-1, C +-4", "exp spread 2^-10..2^0, C=0", "exp spread, C +-1",
                           "positive only, C=0", "x3-like hi*lo (small terms)"};
    for (int mode = 0; mode < 6; ++mode) {
        long n = 0, diff = 0, below = 0, above = 0; double sum_err = 0, sum_abs = 0;
        for (int it = 0; it < 400; ++it) {
            for (int i = 0; i < 16 * 32; ++i) {
                double va = 2 * urand() - 1, vb = 2 * urand() - 1;
                if (mode == 2 || mode == 3) { va = ldexp(va, -(rand() % 11)); vb = ldexp(vb, -(rand() % 11)); }
                if (mode == 4) { va = fabs(va); vb = fabs(vb); }
                if (mode == 5) { if (i % 3 == 1) vb = ldexp(vb, -11); if (i % 3 == 2) va = ldexp(va, -11); }
                A[i] = (_Float16)va; Bm[i] = (_Float16)vb;
            }
            for (int i = 0; i < 256; ++i) C[i] = (mode == 1) ? (float)(8 * urand() - 4) : (mode == 3 ? (float)(2 * urand() - 1) : 0.f);
            mm<<<1, 64>>>(A, Bm, C, D);
            hipDeviceSynchronize();
            for (int i = 0; i < 16; ++i)
                for (int j = 0; j < 16; ++j) {
                    double ex = C[i * 16 + j];
                    for (int k = 0; k < 32; ++k) ex += (double)(float)A[i * 32 + k] * (double)(float)Bm[k * 16 + j];
                    const float rne = (float)ex;
                    const float got = D[i * 16 + j];
                    const double ulp = ldexp(1.0, ilogb(fabs((double)rne) > 0 ? (double)rne : 1e-30) - 23);
                    ++n;
                    if (got != rne) ++diff;
                    if (got < rne) ++below;
                    if (got > rne) ++above;
                    sum_err += (got - ex) / ulp;
                    sum_abs += fabs(got - ex) / ulp;
                }
        }
        printf("%-30s n=%ld  mfma!=RNE(exact): %.4f  below %.4f above %.4f  mean signed err %.4f ulp  mean |err| %.4f ulp\n",
               names[mode], n, (double)diff / n, (double)below / n, (double)above / n, sum_err / n, sum_abs / n);
    }
    return 0;
}
