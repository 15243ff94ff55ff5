// Probe of the f16 MFMA's f32 accumulation rounding (v_mfma_f32_16x16x32_f16): is C + sum(a*b) rounded
// once (RNE / RZ) or per product? Lane 0's column carries the probe products, all others zero.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void probe(const float* c0, const float* av, const float* bv, float* out) {
    const int lane = threadIdx.x;
    // A: row i = lane&15, k = 8*(lane>>4)+j ; B: col j = lane&15, k = 8*(lane>>4)+j
    f16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * (lane >> 4) + j;
        a[j] = (lane & 15) == 0 ? (_Float16)av[k] : (_Float16)0.f;
        b[j] = (lane & 15) == 0 ? (_Float16)bv[k] : (_Float16)0.f;
    }
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    if (lane == 0) c[0] = c0[0];  // D row 4*(lane>>4)+r, col lane&15: lane 0, r 0 = (0,0)
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    if (lane == 0) out[0] = c[0];
}
int main() {
    float *c0, *av, *bv, *out;
    hipMallocManaged(&c0, 4); hipMallocManaged(&av, 128); hipMallocManaged(&bv, 128); hipMallocManaged(&out, 4);
    const float ulp = ldexpf(1.f, -23);
    struct Case { const char* name; float c; int n; float prod[4]; } cases[] = {
        {"+0.75ulp", 1.f, 1, {0.75f * ulp}},
        {"-0.75ulp", 1.f, 1, {-0.375f * ulp}},   // below 1.0 the ulp is 2^-24: -0.75 of it
        {"+0.25ulp", 1.f, 1, {0.25f * ulp}},
        {"+0.5ulp tie", 1.f, 1, {0.5f * ulp}},
        {"+1.5ulp tie", 1.f, 1, {1.5f * ulp}},
        {"2 x +0.6ulp", 1.f, 2, {0.6f * ulp, 0.6f * ulp}},
        {"3 x +0.4ulp", 1.f, 3, {0.4f * ulp, 0.4f * ulp, 0.4f * ulp}},
        {"-1 +0.75ulp (neg c)", -1.f, 1, {-0.75f * ulp}},
    };
    for (auto& cs : cases) {
        for (int k = 0; k < 32; ++k) { av[k] = 0.f; bv[k] = 0.f; }
        for (int i = 0; i < cs.n; ++i) {
            // product p = a*b with a = 2^-12 (exact f16), b = p * 2^12 (must be an exact f16)
            av[i] = ldexpf(1.f, -12); bv[i] = cs.prod[i] * ldexpf(1.f, 12);
            if ((float)(_Float16)bv[i] != bv[i]) printf("warning: b not exact for %s\n", cs.name);
        }
        c0[0] = cs.c;
        probe<<<1, 64>>>(c0, av, bv, out);
        hipDeviceSynchronize();
        double exact = cs.c; for (int i = 0; i < cs.n; ++i) exact += (double)cs.prod[i];
        float rne = (float)exact;
        printf("%-22s c=%g exact-c=%+.3f ulp  mfma-c=%+.3f ulp  rne(exact)-c=%+.3f ulp\n", cs.name, cs.c,
               (exact - cs.c) / ulp, ((double)out[0] - cs.c) / ulp, ((double)rne - cs.c) / ulp);
    }
    return 0;
}
