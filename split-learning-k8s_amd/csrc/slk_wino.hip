// slk_wino.hip — conv2 (32 -> 64 channels, 3x3, 26x26 -> 24x24; src/model_def.py:18) as Winograd
// F(2x2, 3x3) on the f32-input MFMA, for gfx950 / MI355X.
//
// Why: conv2's three products are 97.95 % of the step's FLOPs and f32 has no faster
// matrix path on gfx950 than v_mfma_f32_16x16x4_f32 (= the f32 vector peak, no xf32). F(2x2,3x3)
// turns every 2x2 block of outputs into 16 element-wise products in a 4x4 transform domain instead of
// 36 direct MACs: 2.25x fewer MFMA FLOPs, exact f32 arithmetic throughout (the transforms only use
// 0, +-1, +-1/2; simulated error vs fp64 3e-7 relative, direct f32 1.6e-7 — far inside the 1e-4 / 1e-5
// parity bars).
//
// Transform matrices (Lavin & Gray 2016, correlation form, which is torch's conv2d):
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]   (input tile 4x4 -> V = B^T d B)
//   G   = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1] (filter 3x3 -> U = G g G^T)
//   A^T = [1 1 1 0; 0 1 -1 -1]                     (product 4x4 -> Y = A^T M A, 2x2 outputs)
//
// The 2x2 output tile of F(2,3) is exactly one 2x2 max-pool window of conv2's output, so the
// forward epilogue (bias + ReLU + pool + routing code) consumes one transformed tile per lane.
#include "slk_common.h"

using namespace slk;

// Profiling-only ablation bits (tools/build_variant.sh -DSLK_WINO_ABL=...): 1 = skip the input
// transform (B operand = raw patch), 2 = skip the output transform (y = 4 raw accumulators).
#ifndef SLK_WINO_ABL
#define SLK_WINO_ABL 0
#endif

typedef __attribute__((address_space(3))) void* lds_ptr_t;

typedef float f2 __attribute__((ext_vector_type(2)));

namespace {

// ---------------------------------------------------------------- packed (v_pk_add_f32) transforms
// A 4x4 tile is held as 8 register pairs: row r = {lo = (c0, c1), hi = (c2, c3)}. Steps that combine
// rows are plain element-wise pair ops; the step that combines columns inside a row needs lane-half
// selects, which hipcc does not emit (it moves halves around with v_mov instead), so it is written
// with op_sel / neg modifiers: per row
//   (v0, v1) = (a0 - a2, a1 + a2) = lo + (-a2, a2)         op_sel_hi:[1,0] neg_lo:[0,1]
//   (v2, v3) = (-a1 + a2, a1 - a3) = (a1, a1)·(-,+) + (a2, a3)·(+,-)
// 8 packed adds per tile instead of 16 scalar ones. The trailing s_nop 1 is the VALU-write ->
// MFMA-operand wait state (the outputs feed MFMAs directly).
__device__ __forceinline__ void pk_colstep4(const f2 (&lo)[4], const f2 (&hi)[4], f2 (&v01)[4], f2 (&v23)[4]) {
    asm("v_pk_add_f32 %0, %8, %12 op_sel_hi:[1,0] neg_lo:[0,1]\n\t"
        "v_pk_add_f32 %4, %8, %12 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[1,0] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %1, %9, %13 op_sel_hi:[1,0] neg_lo:[0,1]\n\t"
        "v_pk_add_f32 %5, %9, %13 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[1,0] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %2, %10, %14 op_sel_hi:[1,0] neg_lo:[0,1]\n\t"
        "v_pk_add_f32 %6, %10, %14 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[1,0] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %3, %11, %15 op_sel_hi:[1,0] neg_lo:[0,1]\n\t"
        "v_pk_add_f32 %7, %11, %15 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[1,0] neg_hi:[0,1]\n\t"
        "s_nop 1"
        : "=&v"(v01[0]), "=&v"(v01[1]), "=&v"(v01[2]), "=&v"(v01[3]),
          "=&v"(v23[0]), "=&v"(v23[1]), "=&v"(v23[2]), "=&v"(v23[3])
        : "v"(lo[0]), "v"(lo[1]), "v"(lo[2]), "v"(lo[3]), "v"(hi[0]), "v"(hi[1]), "v"(hi[2]), "v"(hi[3]));
}

// V = B^T d B from the 4 rows of a patch (R[r] = {lo, hi}); out v[i][j] = {v01[i].x, v01[i].y,
// v23[i].x, v23[i].y}.
__device__ __forceinline__ void pk_wino_in(const f2 (&Rlo)[4], const f2 (&Rhi)[4], f2 (&v01)[4], f2 (&v23)[4]) {
    f2 Tlo[4], Thi[4];
    Tlo[0] = Rlo[0] - Rlo[2]; Thi[0] = Rhi[0] - Rhi[2];
    Tlo[1] = Rlo[1] + Rlo[2]; Thi[1] = Rhi[1] + Rhi[2];
    Tlo[2] = Rlo[2] - Rlo[1]; Thi[2] = Rhi[2] - Rhi[1];
    Tlo[3] = Rlo[1] - Rlo[3]; Thi[3] = Rhi[1] - Rhi[3];
    pk_colstep4(Tlo, Thi, v01, v23);
}

// Y = A^T m A for two output channels at once (pairs = 2 accumulator rows r, r+1 of the same
// (i,j)): y[q] for q = 00, 01, 10, 11.
__device__ __forceinline__ void pk_wino_out(const f2 (&m)[16], f2 (&y)[4]) {
    f2 s0[4], s1[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        s0[c] = (m[0 * 4 + c] + m[1 * 4 + c]) + m[2 * 4 + c];
        s1[c] = (m[1 * 4 + c] - m[2 * 4 + c]) - m[3 * 4 + c];
    }
    y[0] = (s0[0] + s0[1]) + s0[2];
    y[1] = (s0[1] - s0[2]) - s0[3];
    y[2] = (s1[0] + s1[1]) + s1[2];
    y[3] = (s1[1] - s1[2]) - s1[3];
}

// ---------------------------------------------------------------- 4x4 transforms (in registers)
// V = B^T d B, d row-major d[4*r + c].
__device__ __forceinline__ void wino_in(const float (&d)[16], float (&v)[16]) {
    float t[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        t[0 * 4 + c] = d[0 * 4 + c] - d[2 * 4 + c];
        t[1 * 4 + c] = d[1 * 4 + c] + d[2 * 4 + c];
        t[2 * 4 + c] = d[2 * 4 + c] - d[1 * 4 + c];
        t[3 * 4 + c] = d[1 * 4 + c] - d[3 * 4 + c];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        v[r * 4 + 0] = t[r * 4 + 0] - t[r * 4 + 2];
        v[r * 4 + 1] = t[r * 4 + 1] + t[r * 4 + 2];
        v[r * 4 + 2] = t[r * 4 + 2] - t[r * 4 + 1];
        v[r * 4 + 3] = t[r * 4 + 1] - t[r * 4 + 3];
    }
}

// U = G g G^T, g row-major g[3*r + c].
__device__ __forceinline__ void wino_filter(const float (&g)[9], float (&u)[16]) {
    float t[12];  // t = G g : 4 x 3
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        t[0 * 3 + c] = g[0 * 3 + c];
        t[1 * 3 + c] = 0.5f * ((g[0 * 3 + c] + g[1 * 3 + c]) + g[2 * 3 + c]);
        t[2 * 3 + c] = 0.5f * ((g[0 * 3 + c] - g[1 * 3 + c]) + g[2 * 3 + c]);
        t[3 * 3 + c] = g[2 * 3 + c];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        u[r * 4 + 0] = t[r * 3 + 0];
        u[r * 4 + 1] = 0.5f * ((t[r * 3 + 0] + t[r * 3 + 1]) + t[r * 3 + 2]);
        u[r * 4 + 2] = 0.5f * ((t[r * 3 + 0] - t[r * 3 + 1]) + t[r * 3 + 2]);
        u[r * 4 + 3] = t[r * 3 + 2];
    }
}

// Y = A^T m A -> y[0..3] = y00, y01, y10, y11 (row-major = torch's pool scan order q).
__device__ __forceinline__ void wino_out(const float (&m)[16], float (&y)[4]) {
    float s[8];  // s = A^T m : 2 x 4
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        s[0 * 4 + c] = (m[0 * 4 + c] + m[1 * 4 + c]) + m[2 * 4 + c];
        s[1 * 4 + c] = (m[1 * 4 + c] - m[2 * 4 + c]) - m[3 * 4 + c];
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        y[r * 2 + 0] = (s[r * 4 + 0] + s[r * 4 + 1]) + s[r * 4 + 2];
        y[r * 2 + 1] = (s[r * 4 + 1] - s[r * 4 + 2]) - s[r * 4 + 3];
    }
}

}  // namespace

// ============================================================================ LDS-DMA helpers
// 16-byte LDS-DMA issued as inline asm: hipcc then neither counts it nor inserts its own vmcnt(0) in
// front of every LDS read (it cannot tell a prefetch buffer from the one being read), so the next
// band stays in flight under the current band's MFMAs and is retired by a counted wait.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

template <int N>
__device__ __forceinline__ void wg_wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// barrier that retires this wave's LDS traffic but leaves VMEM (LDS-DMA prefetch, stores) in flight
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// ============================================================================ forward + pool
// M[ij][co][tile] = sum_ci U[ij][co][ci] * V[ij][ci][tile] : 16 GEMMs of 64 x 144 x 32 per sample.
// Persistent, one 8-wave workgroup per CU (two waves per SIMD). Wave w owns output channels
// 16*(w&3) .. +15 and input-channel half kh = w>>2 (ci 16kh .. 16kh+15), and keeps their transformed
// filters in registers for the whole launch: A operand of v_mfma_f32_16x16x4_f32, lane l holds
// U[ij][16(w&3) + (l&15)][16kh + 4s + (l>>4)] for k step s = 0..3 (64 VGPRs).
// Work unit = (sample, band of 4 tile rows = 48 tiles = 3 groups of 16): input rows 8*band ..
// 8*band+9 of all 32 channels (33,280 B) double-buffered in LDS by 16-byte LDS-DMA.
// Per group and k step a lane (ci, tile = l&15) reads its 4x4 input patch from LDS (8 ds_read_b64),
// transforms it in registers (B operand of 16 MFMAs, one per (i,j)); the 16 accumulators of a
// (co, tile) pair sit in one lane and register slot, so the output transform is in-register.
// K halves: both waves of a pair apply the (linear) output transform to their partial sums; one parks
// its 2x2 partials in LDS, the other adds them (always y_kh0 + y_kh1), then bias, ReLU, the 2x2 max-pool
// (first max wins) and the routing code, and stores. The finishing role alternates per group; the
// two waves of a pair share a SIMD (waves w, w+4), so the parking wave's MFMAs for the next group run
// under its partner's epilogue.
constexpr int WF_WAVES = 8;
constexpr int WF_THREADS = WF_WAVES * 64;
constexpr int WF_ROWS = 10;                    // input rows per band
constexpr int WF_CSTR = WF_ROWS * A_HW;        // 260 floats per channel in LDS (contiguous)
constexpr int WF_BUF = C1 * WF_CSTR;           // 8320 floats = 33,280 B
constexpr int WF_PIECES = WF_BUF / 4;          // 2080 sixteen-byte pieces
constexpr int WF_CHUNKS = (WF_PIECES + 63) / 64;
constexpr int WF_BSTR = WF_CHUNKS * 256;       // buffer stride: the last chunk writes a full KiB
constexpr int WF_XCH = 4 * 16 * 64;            // parked partials per parity: [co block][r*4+q][lane]
constexpr int WF_GRID = 256;                   // one workgroup per CU

__device__ __forceinline__ void wf_dma_band(const float* __restrict__ act, int u, const float* dst, int wave, int lane) {
    const int b = u / 3, band = u - 3 * (u / 3);
    const float* src = act + (size_t)b * A_SAMPLE + band * 8 * A_HW;
    const uint32_t base = (uint32_t)(uintptr_t)dst;
#pragma unroll 1
    for (int c = wave; c < WF_CHUNKS; c += WF_WAVES) {
        // lanes past the band end (last chunk) re-read the band's last piece into the pad
        const int p = min(c * 64 + lane, WF_PIECES - 1);
        const int ci = p / 65, k = p - 65 * (p / 65);
        glds16(src + ci * A_PIX + 4 * k, __builtin_amdgcn_readfirstlane(base + c * 1024));
    }
}

__global__ __launch_bounds__(WF_THREADS, 1) void conv2_fwd_pool_wino_kernel(
    const float* __restrict__ act, const float* __restrict__ W2, const float* __restrict__ b2,
    float* __restrict__ pooled, uint8_t* __restrict__ code, int B) {
    __shared__ __attribute__((aligned(16))) float smem[2 * WF_BSTR + 2 * WF_XCH + C2];
    float* xch = smem + 2 * WF_BSTR;
    float* bias_s = xch + 2 * WF_XCH;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int cb = wave & 3, kh = wave >> 2;
    const int nunit = 3 * B;

    int u = blockIdx.x;
    if (u < nunit) wf_dma_band(act, u, smem, wave, lane);

    // transformed filters of this lane's (co, ci) pairs
    float uw[4][16];
    {
        const int co = 16 * cb + li;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const float* gp = W2 + (size_t)co * K2 + (16 * kh + 4 * s + lk) * 9;
            float g[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) g[k] = gp[k];
            wino_filter(g, uw[s]);
        }
    }
    if (tid < C2) bias_s[tid] = b2[tid];
    wg_wait_vmcnt<0>();  // first band + filters landed

    int buf = 0;
#pragma unroll 1
    for (; u < nunit; u += gridDim.x) {
        // this unit's band has landed: its DMA was issued before the previous unit's epilogue
        // stores (>= 8 per wave) — and every wave is done reading the other buffer
        wg_wait_vmcnt<8>();
        lds_barrier();
        const int nu = u + gridDim.x;
        if (nu < nunit) wf_dma_band(act, nu, smem + (buf ^ 1) * WF_BSTR, wave, lane);
        const float* img = smem + buf * WF_BSTR;
        const int b = u / 3, band = u - 3 * (u / 3);
        const auto prs = __builtin_amdgcn_make_buffer_rsrc(pooled + (size_t)b * P_SAMPLE, 0, P_SAMPLE * 4, 0x00020000);
        const auto crs = __builtin_amdgcn_make_buffer_rsrc(code + (size_t)b * P_SAMPLE, 0, P_SAMPLE, 0x00020000);
#pragma unroll 1
        for (int g = 0; g < 3; ++g) {
            const int t = 48 * band + 16 * g + li;       // tile = pooling window index
            const int ty = t / P_HW, tx = t - P_HW * (t / P_HW);
            const float* pp = img + (16 * kh + lk) * WF_CSTR + (2 * ty - 8 * band) * A_HW + 2 * tx;
            f32x4 acc[16];
#pragma unroll
            for (int ij = 0; ij < 16; ++ij) acc[ij] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float* ps = pp + 4 * s * WF_CSTR;
                f2 Rlo[4], Rhi[4], v01[4], v23[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    Rlo[r] = *reinterpret_cast<const f2*>(ps + r * A_HW);
                    Rhi[r] = *reinterpret_cast<const f2*>(ps + r * A_HW + 2);
                }
                if (SLK_WINO_ABL & 1) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) { v01[r] = Rlo[r]; v23[r] = Rhi[r]; }
                } else {
                    pk_wino_in(Rlo, Rhi, v01, v23);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    acc[4 * i + 0] = mfma16x16x4(uw[s][4 * i + 0], v01[i].x, acc[4 * i + 0]);
                    acc[4 * i + 1] = mfma16x16x4(uw[s][4 * i + 1], v01[i].y, acc[4 * i + 1]);
                    acc[4 * i + 2] = mfma16x16x4(uw[s][4 * i + 2], v23[i].x, acc[4 * i + 2]);
                    acc[4 * i + 3] = mfma16x16x4(uw[s][4 * i + 3], v23[i].y, acc[4 * i + 3]);
                }
            }
            // partial output transform, two rows (co = 16cb + 4lk + r, r = 2h, 2h+1) per packed op;
            // column = tile t
            f2 y[2][4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                f2 m[16];
#pragma unroll
                for (int ij = 0; ij < 16; ++ij) m[ij] = h ? acc[ij].zw : acc[ij].xy;
                pk_wino_out(m, y[h]);
            }
            // parked partials: [q][lane][r] (16 B per lane and q: ds_write_b128 / ds_read_b128)
            float4* xp = reinterpret_cast<float4*>(xch + (g & 1) * WF_XCH + cb * 16 * 64) + lane;
            const bool fin = kh == (g & 1);
            if (!fin) {
#pragma unroll
                for (int q = 0; q < 4; ++q) xp[q * 64] = make_float4(y[0][q].x, y[0][q].y, y[1][q].x, y[1][q].y);
            }
            lds_barrier();
            if (fin) {
                const float4 bv = reinterpret_cast<const float4*>(bias_s)[4 * cb + lk];
                f2 z[2][4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 o4 = xp[q * 64];
                    const f2 olo = {o4.x, o4.y}, ohi = {o4.z, o4.w};
                    // fixed order: K half 0 + K half 1, then bias
                    z[0][q] = (kh == 0 ? y[0][q] + olo : olo + y[0][q]) + f2{bv.x, bv.y};
                    z[1][q] = (kh == 0 ? y[1][q] + ohi : ohi + y[1][q]) + f2{bv.z, bv.w};
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int h = r >> 1;
                    float yq[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) yq[q] = (r & 1) ? z[h][q].y : z[h][q].x;
                    // max over the raw window, first max wins; = torch's relu-then-pool scan
                    const float mx = fmaxf(fmaxf(yq[0], yq[1]), fmaxf(yq[2], yq[3]));
                    const int idx = yq[0] == mx ? 0 : yq[1] == mx ? 1 : yq[2] == mx ? 2 : 3;
                    const bool pos = mx > 0.f;
                    const int co = 16 * cb + 4 * lk + r;
                    const int o = co * P_WIN + t;
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(pos ? mx : 0.f), prs, 4 * o, 0, 0);
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(pos ? idx : CODE_NONE), crs, o, 0, 0);
                }
            }
        }
        buf ^= 1;
    }
}

extern "C" int slk_conv2_fwd_pool(const float* act, const float* W2, const float* b2, float* pooled,
                                  uint8_t* code, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(act && W2 && b2 && pooled && code);
    const int nunit = 3 * B;
    conv2_fwd_pool_wino_kernel<<<nunit < WF_GRID ? nunit : WF_GRID, WF_THREADS, 0, slk_stream(stream)>>>(
        act, W2, b2, pooled, code, B);
    return slk_launch_status();
}
