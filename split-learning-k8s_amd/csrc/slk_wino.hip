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
// a - b as ONE v_pk_add_f32 (hipcc splits a packed subtraction into two scalar v_sub_f32)
__device__ __forceinline__ f2 pk_sub(f2 a, f2 b) {
    f2 d;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
__device__ __forceinline__ void pk_wino_out(const f2 (&m)[16], f2 (&y)[4]) {
    f2 s0[4], s1[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        s0[c] = (m[0 * 4 + c] + m[1 * 4 + c]) + m[2 * 4 + c];
        s1[c] = pk_sub(pk_sub(m[1 * 4 + c], m[2 * 4 + c]), m[3 * 4 + c]);
    }
    y[0] = (s0[0] + s0[1]) + s0[2];
    y[1] = pk_sub(pk_sub(s0[1], s0[2]), s0[3]);
    y[2] = (s1[0] + s1[1]) + s1[2];
    y[3] = pk_sub(pk_sub(s1[1], s1[2]), s1[3]);
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

// LDS-DMA helpers (glds16): slk_common.h

template <int N>
__device__ __forceinline__ void wg_wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// v_mfma_f32_16x16x4_f32 with the A operand read straight from an AGPR (legal on gfx950, but hipcc
// copies AGPR-resident operands to a VGPR first — one v_accvgpr_read + s_nop per MFMA, and every
// VALU instruction costs its issue cycles on top of the f32 MFMA stream). B and C/D in VGPRs.
// Wait states: B comes from the colstep asm (ends with s_nop 1); the accumulators are read by VALU only
// after mfma_drain(); AGPRs are written once per launch, long before the first MFMA.
__device__ __forceinline__ void mfma_a(f32x4& acc, float a, float b) {
    asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc) : "a"(a), "v"(b));
}
// first k step: C = 0 (an inline constant), so the accumulators need no zeroing instructions
__device__ __forceinline__ void mfma_a0(f32x4& acc, float a, float b) {
    asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, 0" : "=v"(acc) : "a"(a), "v"(b));
}
// accumulators kept in AGPRs (A, B in VGPRs): the weight gradient's 256 accumulator registers
__device__ __forceinline__ void mfma_acc(f32x4& acc, float a, float b) {
    asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_acc0(f32x4& acc, float a, float b) {
    asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}
// MFMA result -> VALU read: the 8-pass XDL op needs >= 11 wait states before hipcc's code reads acc
__device__ __forceinline__ void mfma_drain() { asm volatile("s_nop 15" ::: "memory"); }

// barrier that retires this wave's LDS traffic but leaves VMEM (LDS-DMA prefetch, stores) in flight
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// ============================================================================ forward + pool
// M[ij][co][tile] = sum_ci U[ij][co][ci] * V[ij][ci][tile] : 16 GEMMs of 64 x 144 x 32 per sample.
// On gfx950 the f32 MFMA and the VALU do not execute concurrently (tools/ubench/coexec.hip: every
// packed add issued between MFMAs adds ~4-5 cycles, from one wave per SIMD or two), so the design
// minimises VALU instructions per MFMA rather than relying on overlap:
// Persistent, one 4-wave workgroup per CU (one wave per SIMD, 512 registers each). Wave w owns output
// channels 16w .. 16w+15 over the FULL reduction (32 input channels): their transformed filters stay
// in registers for the whole launch (A operand of v_mfma_f32_16x16x4_f32: lane l holds
// U[ij][16w + (l&15)][4s + (l>>4)] for k step s = 0..7, 128 VGPRs), so no partial sums cross waves and
// there is no barrier inside a band.
// Work unit = (sample, band of 4 tile rows = 48 tiles = 3 groups of 16): input rows 8*band ..
// 8*band+9 of all 32 channels (33,280 B) double-buffered in LDS by 16-byte LDS-DMA (inline asm, so the
// next band stays in flight under the current band's MFMAs; one counted vmcnt + barrier per band).
// Per group and k step a lane (ci = 4s + (l>>4), tile = l&15) reads its 4x4 input patch (8
// ds_read_b64), transforms it with 8 packed adds (B operand of 16 MFMAs, one per (i,j)); the 16
// accumulators of a (co, tile) pair sit in one lane and register slot, so the output transform (two
// channels per packed op), bias, ReLU, the 2x2 max-pool (first max wins) and the routing code are
// in-register and pooled/code leave by buffer stores.
constexpr int WF_WAVES = 4;
constexpr int WF_THREADS = WF_WAVES * 64;
constexpr int WF_ROWS = 10;                    // input rows per band
constexpr int WF_CSTR = WF_ROWS * A_HW;        // 260 floats per channel in LDS (contiguous)
constexpr int WF_BUF = C1 * WF_CSTR;           // 8320 floats = 33,280 B
constexpr int WF_PIECES = WF_BUF / 4;          // 2080 sixteen-byte pieces
constexpr int WF_CHUNKS = (WF_PIECES + 63) / 64;
constexpr int WF_BSTR = WF_CHUNKS * 256;       // buffer stride: the last chunk writes a full KiB
constexpr int WF_GRID = 256;                   // one workgroup per CU

// ============================================================================ shared helpers
// 4x4 patch of a row-major LDS image (row stride A_HW floats) as 8 ds_read_b64, as row pairs
__device__ __forceinline__ void lds_patch_pk(const float* ps, f2 (&lo)[4], f2 (&hi)[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        lo[r] = *reinterpret_cast<const f2*>(ps + r * A_HW);
        hi[r] = *reinterpret_cast<const f2*>(ps + r * A_HW + 2);
    }
}

// ---------------------------------------------------------------------------- forward, v2
// Same transform-domain GEMMs, but wave w owns 32 output channels (2 M blocks: co 32*(w&1) .. +31)
// instead of 16, so one transformed input patch feeds 32 MFMAs instead of 16: the input transform
// (16 packed adds + 8 ds_read_b64 per k step) is paid half as often per MFMA, and on gfx950 every
// VALU instruction between f32 MFMAs costs its issue cycles (tools/ubench/fillers.hip). The two
// wave pairs (w>>1) each run their own band stream (2 bands in flight per workgroup, 4 LDS buffers
// = 135 KB); transformed filters of both M blocks stay AGPR-resident (256 AGPRs, the MFMA A operand).
// The bias rides in the C operand of the first MFMA of transform position (1,1): A^T E11 A = all
// ones, so it reaches all four outputs of the window with coefficient +1 (no bias adds in the
// epilogue).
__device__ __forceinline__ void mfma_ac(f32x4& acc, float a, float b, const f32x4& c) {
    asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %3" : "=v"(acc) : "a"(a), "v"(b), "v"(c));
}

// A band's staging DMA: wave pair half h moves chunks c = h, h+2, ... (< WF_CHUNKS) of 64 sixteen-byte
// pieces; piece (c, lane) = channel p / 65, 16-byte column p % 65 of the band (p = 64 c + lane). The
// per-lane byte offsets from the band's first float are the same for every band, so they are computed
// once per launch and each piece is one saddr-form DMA (no VALU address arithmetic, no loop branch:
// the per-piece division, address and branch code had cost ~150 cycles per piece beside the MFMAs).
constexpr int WF_PPW = (WF_CHUNKS + 1) / 2;   // pieces per wave and band (17 for half 0, 16 for half 1)
__device__ __forceinline__ void wf2_dma_offsets(int half, int lane, uint32_t (&off)[WF_PPW]) {
#pragma unroll
    for (int i = 0; i < WF_PPW; ++i) {
        const int p = min((half + 2 * i) * 64 + lane, WF_PIECES - 1);
        const int ci = p / 65, k = p - 65 * (p / 65);
        off[i] = (uint32_t)(ci * A_PIX + 4 * k) * 4u;
    }
}
__device__ __forceinline__ void wf2_dma_band(const float* __restrict__ act, int band, const float* dst, int half,
                                             const uint32_t (&off)[WF_PPW]) {
    const int b = band / 3, bs = band - 3 * (band / 3);
    const float* src = act + (size_t)b * A_SAMPLE + bs * 8 * A_HW;
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
#pragma unroll
    for (int i = 0; i < WF_PPW; ++i) {
        const int c = half + 2 * i;
        if (c < WF_CHUNKS) glds16_so(src, off[i], base + c * 1024);
    }
}

__global__ __launch_bounds__(WF_THREADS, 1) void conv2_fwd_pool_wino2_kernel(
    const float* __restrict__ act, const float* __restrict__ W2, const float* __restrict__ b2,
    float* __restrict__ pooled, uint8_t* __restrict__ code, int B) {
    __shared__ __attribute__((aligned(16))) float smem[4 * WF_BSTR];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int wu = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform (buffer descriptors, DMA bases)
    const int mh = wu & 1, pr = wu >> 1;
    const int nband = 3 * B, nsu = (nband + 1) >> 1;
    float* bufs = smem + 2 * pr * WF_BSTR;

    uint32_t doff[WF_PPW];
    wf2_dma_offsets(mh, lane, doff);
    int su = blockIdx.x;
    if (2 * su + pr < nband) wf2_dma_band(act, 2 * su + pr, bufs, mh, doff);

    // transformed filters (co = 32mh + 16m + li, ci = 4s + lk) and the bias of this lane's rows
    float uw[2][8][16];
    f32x4 bias4[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int co = 32 * mh + 16 * m + li;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const float* gp = W2 + (size_t)co * K2 + (4 * s + lk) * 9;
            float g[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) g[k] = gp[k];
            float u[16];
            wino_filter(g, u);
#pragma unroll
            for (int k = 0; k < 16; ++k) asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(uw[m][s][k]) : "v"(u[k]));
        }
        const float* bp = b2 + 32 * mh + 16 * m + 4 * lk;  // (a view into the flat parameters: no
        bias4[m] = f32x4{bp[0], bp[1], bp[2], bp[3]};        //  16-byte alignment assumed)
    }
    wg_wait_vmcnt<0>();  // first band + filters landed

    int buf = 0;
#pragma unroll 1
    for (; su < nsu; su += gridDim.x) {
        // this band landed: its DMA was issued before the previous band's 48 epilogue stores of this
        // wave — and every wave is done reading the other buffers
        wg_wait_vmcnt<48>();
        lds_barrier();
        const int nb = 2 * (su + gridDim.x) + pr;
        if (nb < nband) wf2_dma_band(act, nb, bufs + (buf ^ 1) * WF_BSTR, mh, doff);
        const int band = 2 * su + pr;
        if (band < nband) {
            const float* img = bufs + buf * WF_BSTR;
            const int b = band / 3, bs = band - 3 * (band / 3);
            const auto prs = __builtin_amdgcn_make_buffer_rsrc(pooled + (size_t)b * P_SAMPLE, 0, P_SAMPLE * 4, 0x00020000);
            const auto crs = __builtin_amdgcn_make_buffer_rsrc(code + (size_t)b * P_SAMPLE, 0, P_SAMPLE, 0x00020000);
#pragma unroll 1
            for (int g = 0; g < 3; ++g) {
                const int t = 48 * bs + 16 * g + li;  // tile = pooling window index
                const int ty = t / P_HW, tx = t - P_HW * (t / P_HW);
                const float* pp = img + lk * WF_CSTR + (2 * ty - 8 * bs) * A_HW + 2 * tx;
                f32x4 acc[2][16];  // written first by the k step 0 MFMAs (C = 0, or the bias at (1,1))
                f2 Rlo[4], Rhi[4];
                lds_patch_pk(pp, Rlo, Rhi);
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    f2 v01[4], v23[4];
                    pk_wino_in(Rlo, Rhi, v01, v23);
                    if (s < 7) lds_patch_pk(pp + 4 * (s + 1) * WF_CSTR, Rlo, Rhi);  // under these MFMAs
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int m = 0; m < 2; ++m)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            if (s == 0) {
                                mfma_a0(acc[m][4 * i + 0], uw[m][s][4 * i + 0], v01[i].x);
                                if (i == 1) mfma_ac(acc[m][4 * i + 1], uw[m][s][4 * i + 1], v01[i].y, bias4[m]);
                                else mfma_a0(acc[m][4 * i + 1], uw[m][s][4 * i + 1], v01[i].y);
                                mfma_a0(acc[m][4 * i + 2], uw[m][s][4 * i + 2], v23[i].x);
                                mfma_a0(acc[m][4 * i + 3], uw[m][s][4 * i + 3], v23[i].y);
                            } else {
                                mfma_a(acc[m][4 * i + 0], uw[m][s][4 * i + 0], v01[i].x);
                                mfma_a(acc[m][4 * i + 1], uw[m][s][4 * i + 1], v01[i].y);
                                mfma_a(acc[m][4 * i + 2], uw[m][s][4 * i + 2], v23[i].x);
                                mfma_a(acc[m][4 * i + 3], uw[m][s][4 * i + 3], v23[i].y);
                            }
                        }
                    __builtin_amdgcn_sched_barrier(0);
                }
                mfma_drain();
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    // output transform, two rows (co = 32mh + 16m + 4lk + r, r = 2h, 2h+1) per packed op
                    f2 z[2][4];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        f2 mm[16];
#pragma unroll
                        for (int ij = 0; ij < 16; ++ij) mm[ij] = h ? acc[m][ij].zw : acc[m][ij].xy;
                        pk_wino_out(mm, z[h]);
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int h = r >> 1;
                        float yq[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) yq[q] = (r & 1) ? z[h][q].y : z[h][q].x;
                        // max over the raw window, first max wins; = torch's relu-then-pool scan.
                        // Branch-free (hipcc turns the ternary chain into exec-mask branches): the
                        // max as v_max3 + v_max (no NaN-quieting copies), the index as selects.
                        float mx;
                        asm("v_max3_f32 %0, %1, %2, %3\n\tv_max_f32 %0, %0, %4"
                            : "=&v"(mx) : "v"(yq[0]), "v"(yq[1]), "v"(yq[2]), "v"(yq[3]));
                        int idx = yq[2] == mx ? 2 : 3;
                        idx = yq[1] == mx ? 1 : idx;
                        idx = yq[0] == mx ? 0 : idx;
                        const bool pos = mx > 0.f;
                        const int o = (32 * mh + 16 * m + 4 * lk + r) * P_WIN + t;
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(pos ? mx : 0.f), prs, 4 * o, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(pos ? idx : CODE_NONE), crs, o, 0, 0);
                    }
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
    const int nsu = (3 * B + 1) / 2;
    conv2_fwd_pool_wino2_kernel<<<nsu < WF_GRID ? nsu : WF_GRID, WF_THREADS, 0, slk_stream(stream)>>>(
        act, W2, b2, pooled, code, B);
    return slk_launch_status();
}

// Routing lookup tables, built once per workgroup in LDS (float4 entries, code c = 0..4):
//   dgrad  EXP[c] = (c==0, c==1, c==2, c==3): the 2x2 block of a window whose gradient sits at c;
//   wgrad  ZT[c][16] = A[i][c>>1] * A[j][c&1] (A = [1 0; 1 1; 1 -1; 0 -1]): Z = A dY A^T of that block.
// Code 4 (ReLU-blocked window) maps to zeros. A lookup + packed multiplies replaces per-element
// compares and selects: on gfx950 every VALU instruction costs its issue cycles on top of the f32
// MFMA stream (tools/ubench/fillers.hip), packed or not, so the count of instructions is what matters.
__device__ __forceinline__ void build_luts(float* lut_exp, float* lut_z, int tid) {
    if (tid < 5 * 4) {
        const int c = tid >> 2, k = tid & 3;
        lut_exp[tid] = (c == k) ? 1.f : 0.f;
    }
    if (tid < 5 * 16) {
        const int c = tid >> 4, i = (tid >> 2) & 3, j = tid & 3;
        const float a0[4] = {1.f, 1.f, 1.f, 0.f}, a1[4] = {0.f, 1.f, -1.f, -1.f};
        const float ai = (c & 2) ? a1[i] : a0[i];
        const float aj = (c & 1) ? a1[j] : a0[j];
        lut_z[tid] = c < 4 ? ai * aj : 0.f;
    }
}

// ============================================================================ dgrad (cut gradient)
// g[ci][y][x] = sum_co sum_{a,b} dcpad[co][y+a][x+b] * W2[co][ci][2-a][2-b]: a "full" correlation of
// the pool/ReLU-routed conv2 output gradient dc (24x24, zero border of 2 -> 28x28) with the flipped
// filter. Winograd F(2x2,3x3): 13 x 13 = 169 output tiles per sample (11 groups of 16, the last one
// 9 wide), M[ij][ci][tile] = sum_co U'[ij][ci][co] * V[ij][co][tile]: 16 GEMMs of 32 x 169 x 64.
// The 4x4 input patch of tile (ty, tx) is dcpad rows 2ty .. 2ty+3 = pooling windows (ty-1 .. ty,
// tx-1 .. tx): each quadrant holds at most ONE nonzero, dpooled at the window's routing code, so the
// patch is expanded in registers straight from (dpooled, code) staged in LDS (lookup + 2 packed
// multiplies per window) — dc never exists.
// Persistent, one 4-wave workgroup per CU (one wave per SIMD, 512 registers): wave w owns the K half
// kh = w&1 (co 32kh .. 32kh+31, 8 k steps) for BOTH 16-row M blocks (all 32 ci), so one expanded
// patch feeds 32 MFMAs, and group slot gs = w>>1 (groups 2p + gs, p = 0..5; slot 12 is empty). The
// transformed flipped filters stay in registers for the launch (A operand: lane l holds
// U'[ij][16m + (l&15)][32kh + 4s + (l>>4)], 256 VGPRs). Unit = one sample: dpooled (36,864 B) + code
// (9,216 B) by LDS-DMA, double-buffered. Per group the two K halves meet once: each wave parks the
// 2x2 partial outputs of the M block its partner finishes (ds_write_b128), one barrier, then finishes
// its own M block (mine + partner's: commutative, so bitwise reproducible) and stores the cut gradient.
constexpr int WD_WAVES = 4;
constexpr int WD_THREADS = WD_WAVES * 64;
constexpr int WD_PAIRS = 6;                    // group pairs per sample: groups 0..10 (+ an empty 11th)
constexpr int WD_NT = 13 * 13;
constexpr int WD_DP_CH = P_SAMPLE / 256;       // 36 KiB chunks of dpooled
constexpr int WD_CD_OFF = P_SAMPLE + 64;       // float offset of the code bytes in a buffer
constexpr int WD_CD_CH = P_SAMPLE / 1024;      // 9 KiB chunks of code
constexpr int WD_BSTR = WD_CD_OFF + P_SAMPLE / 4 + 64;   // 11648 floats = 46,592 B per buffer
constexpr int WD_XCH = 2 * 2 * 4 * 64 * 4;     // per parity: [group slot][writer kh][r][lane] float4
constexpr int WD_GRID = 256;

__device__ __forceinline__ void wd_dma_sample(const float* __restrict__ dpool, const uint8_t* __restrict__ code, int b,
                                              const float* dst, int wave, int lane) {
    const uint32_t base = (uint32_t)(uintptr_t)dst;
    const float* dsrc = dpool + (size_t)b * P_SAMPLE;
    const uint8_t* csrc = code + (size_t)b * P_SAMPLE;
#pragma unroll 1
    for (int c = wave; c < WD_DP_CH + WD_CD_CH; c += WD_WAVES) {
        if (c < WD_DP_CH)
            glds16(dsrc + c * 256 + lane * 4, __builtin_amdgcn_readfirstlane(base + c * 1024));
        else
            glds16(csrc + (c - WD_DP_CH) * 1024 + lane * 16,
                   __builtin_amdgcn_readfirstlane(base + WD_CD_OFF * 4 + (c - WD_DP_CH) * 1024));
    }
}

__global__ __launch_bounds__(WD_THREADS, 1) void conv2_dgrad_wino_kernel(
    const float* __restrict__ dpool, const uint8_t* __restrict__ code, const float* __restrict__ W2,
    float* __restrict__ gcut, int B) {
    __shared__ __attribute__((aligned(16))) float smem[2 * WD_BSTR + 2 * WD_XCH + 40];
    float* xch = smem + 2 * WD_BSTR;
    float* lut = xch + 2 * WD_XCH;  // EXP table, 5 float4, then 5 zero float4 (out-of-range windows)
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int wu = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: scalar branches on kh
    const int kh = wu & 1, gs = wu >> 1;

    int b = blockIdx.x;
    if (b < B) wd_dma_sample(dpool, code, b, smem, wu, lane);
    if (tid < 40) lut[tid] = (tid < 20 && (tid >> 2) == (tid & 3)) ? 1.f : 0.f;

    // transformed flipped filters: lane (ci = 16(m ^ kh) + li, co = 32kh + 4s + lk); slot m = 0 is the
    // ci block this wave finishes, m = 1 the one it hands to its partner
    float uw[2][8][16];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const float* gp = W2 + (size_t)(32 * kh + 4 * s + lk) * K2 + (16 * (m ^ kh) + li) * 9;
            float g[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) g[k] = gp[8 - k];
            wino_filter(g, uw[m][s]);
        }
    wg_wait_vmcnt<0>();

    // Rolling tile stream: this workgroup's samples k = 0 .. nloc-1 (b = blockIdx.x + k * gridDim.x)
    // are one stream of 169-tile blocks; iteration i gives group slot gs the 16 tiles
    // T = 32 i + 16 gs + li (a group may straddle two samples: a lane reads the buffer of ITS sample),
    // so no group slot computes padding: ceil(169 nloc / 32) iterations instead of 6 nloc.
    // Sample k lives in buffer k & 1; its DMA is issued once every tile of sample k - 2 is done (a
    // whole iteration ahead of any use: >= 4 iterations, >= 32 stores of this wave, before it).
    const int nloc = b < B ? (B - 1 - b) / (int)gridDim.x + 1 : 0;
    if (nloc > 1) wd_dma_sample(dpool, code, b + gridDim.x, smem + WD_BSTR, wu, lane);
    wg_wait_vmcnt<0>();  // samples 0 and 1 + filters landed
    lds_barrier();
    const int ntile = WD_NT * nloc;
    const int nit = (ntile + 31) >> 5;
    int next_dma = 2, resident = nloc > 1 ? 1 : 0;
#pragma unroll 1
    for (int it = 0; it < nit; ++it) {
        // a new sample enters this iteration: its DMA (>= 32 stores of this wave ago) has landed
        const int khi = min((32 * it + 31) / WD_NT, nloc - 1);
        if (khi > resident) {
            wg_wait_vmcnt<8>();
            lds_barrier();
            resident = khi;
        }
        // every tile before this iteration was read before the previous iteration's exchange
        // barrier: sample next_dma - 2 is free once its last tile is behind us
        if (next_dma < nloc && WD_NT * (next_dma - 1) <= 32 * it) {
            wd_dma_sample(dpool, code, b + next_dma * (int)gridDim.x, smem + (next_dma & 1) * WD_BSTR, wu, lane);
            ++next_dma;
        }
        const int p = it;
        const int T = 32 * it + 16 * gs + li;
        const bool valid = T < ntile;
        const int Tc = valid ? T : ntile - 1;
        const int k = Tc / WD_NT;
        const int tc = Tc - WD_NT * k;
        const float* dps = smem + (k & 1) * WD_BSTR + (32 * kh + lk) * P_WIN;
        const uint8_t* cds = reinterpret_cast<const uint8_t*>(smem + (k & 1) * WD_BSTR + WD_CD_OFF) + (32 * kh + lk) * P_WIN;
        float* gsm = gcut + (size_t)(b + k * (int)gridDim.x) * A_SAMPLE;
        {
            const int ty = tc / 13, tx = tc - 13 * (tc / 13);
            // windows (ty-1+wy, tx-1+wx), clamped in range; an out-of-range window reads the zero
            // half of the table (no per-step select)
            int woff[4];
            const float4* lutw[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const int py = ty - 1 + (w >> 1), px = tx - 1 + (w & 1);
                const bool ok = py >= 0 && py < P_HW && px >= 0 && px < P_HW;
                woff[w] = min(max(py, 0), P_HW - 1) * P_HW + min(max(px, 0), P_HW - 1);
                lutw[w] = reinterpret_cast<const float4*>(lut) + (ok ? 0 : 5);
            }
            f32x4 acc[2][16];  // written first by the C = 0 MFMAs of k step 0

            // k step s = channel co = 32kh + 4s + lk: raw (value, code) of the 4 windows
            float dv[2][4];
            int cd[2][4];
            auto load = [&](int s, float (&v)[4], int (&c)[4]) {
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    v[w] = dps[s * 4 * P_WIN + woff[w]];
                    c[w] = cds[s * 4 * P_WIN + woff[w]];  // clamped address: always a valid read
                }
            };
            // table rows of a step's 4 windows: issued one step ahead (the code arrived a step
            // earlier), so the dependent LDS read is not exposed in front of the expansion
            auto lutload = [&](const int (&c)[4], float4 (&E)[4]) {
#pragma unroll
                for (int w = 0; w < 4; ++w) E[w] = lutw[w][c[w]];
            };
            auto expand = [&](const float (&v)[4], const float4 (&E)[4], f2 (&v01)[4], f2 (&v23)[4]) {
                f2 Rlo[4], Rhi[4];
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const float4 e = E[w];
                    const f2 vv = {v[w], v[w]};
                    const f2 r0 = vv * f2{e.x, e.y}, r1 = vv * f2{e.z, e.w};
                    const int wy = w >> 1;
                    if (w & 1) { Rhi[2 * wy] = r0; Rhi[2 * wy + 1] = r1; }
                    else { Rlo[2 * wy] = r0; Rlo[2 * wy + 1] = r1; }
                }
                pk_wino_in(Rlo, Rhi, v01, v23);
            };
            load(0, dv[0], cd[0]);
            load(1, dv[1], cd[1]);
            f2 v01[4], v23[4];
            float4 E[4];
            lutload(cd[0], E);
            expand(dv[0], E, v01, v23);
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                if (s < 7) lutload(cd[(s + 1) & 1], E);        // in flight under this step's MFMAs
                if (s < 6) load(s + 2, dv[s & 1], cd[s & 1]);  // likewise
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int m = 0; m < 2; ++m)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if (s == 0) {
                            mfma_a0(acc[m][4 * i + 0], uw[m][s][4 * i + 0], v01[i].x);
                            mfma_a0(acc[m][4 * i + 1], uw[m][s][4 * i + 1], v01[i].y);
                            mfma_a0(acc[m][4 * i + 2], uw[m][s][4 * i + 2], v23[i].x);
                            mfma_a0(acc[m][4 * i + 3], uw[m][s][4 * i + 3], v23[i].y);
                        } else {
                            mfma_a(acc[m][4 * i + 0], uw[m][s][4 * i + 0], v01[i].x);
                            mfma_a(acc[m][4 * i + 1], uw[m][s][4 * i + 1], v01[i].y);
                            mfma_a(acc[m][4 * i + 2], uw[m][s][4 * i + 2], v23[i].x);
                            mfma_a(acc[m][4 * i + 3], uw[m][s][4 * i + 3], v23[i].y);
                        }
                    }
                __builtin_amdgcn_sched_barrier(0);
                if (s < 7) expand(dv[(s + 1) & 1], E, v01, v23);
            }
            mfma_drain();
            // partial output transform (rows ci = 16(m ^ kh) + 4lk + r, pairs r = 2h, 2h+1)
            f2 y[2][2][4];
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    f2 mm[16];
#pragma unroll
                    for (int ij = 0; ij < 16; ++ij) mm[ij] = h ? acc[m][ij].zw : acc[m][ij].xy;
                    pk_wino_out(mm, y[m][h]);
                }
            auto row = [&](const f2 (&ym)[2][4], int r) -> float4 {
                const int h = r >> 1;
                return (r & 1) ? make_float4(ym[h][0].y, ym[h][1].y, ym[h][2].y, ym[h][3].y)
                               : make_float4(ym[h][0].x, ym[h][1].x, ym[h][2].x, ym[h][3].x);
            };
            float4* xw = reinterpret_cast<float4*>(xch + (p & 1) * WD_XCH) + (gs * 2 + kh) * 4 * 64 + lane;
            const float4* xr = reinterpret_cast<const float4*>(xch + (p & 1) * WD_XCH) + (gs * 2 + (kh ^ 1)) * 4 * 64 + lane;
            // park the M block the partner finishes (slot 1 = ci block 1 - kh; kh = 0 finishes ci 0..15,
            // kh = 1 ci 16..31 — slot 0 is always the wave's own block: no selects on kh)
#pragma unroll
            for (int r = 0; r < 4; ++r) xw[r * 64] = row(y[1], r);
            lds_barrier();
            auto finish = [&](const f2 (&ym)[2][4], int mb) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float4 a = row(ym, r), o = xr[r * 64];
                    const float4 tot = make_float4(a.x + o.x, a.y + o.y, a.z + o.z, a.w + o.w);
                    const int ci = 16 * mb + 4 * lk + r;
                    float* op = gsm + ci * A_PIX + 2 * ty * A_HW + 2 * tx;
                    if (valid) {
                        *reinterpret_cast<f2*>(op) = f2{tot.x, tot.y};
                        *reinterpret_cast<f2*>(op + A_HW) = f2{tot.z, tot.w};
                    }
                }
            };
            finish(y[0], kh);
        }
    }
}

extern "C" int slk_conv2_dgrad(const float* dpooled, const uint8_t* code, const float* W2,
                               float* cut_grad, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(dpooled && code && W2 && cut_grad);
    conv2_dgrad_wino_kernel<<<B < WD_GRID ? B : WD_GRID, WD_THREADS, 0, slk_stream(stream)>>>(
        dpooled, code, W2, cut_grad, B);
    return slk_launch_status();
}

// ============================================================================ wgrad (conv2 weights)
// dW2[co][ci][a][b] = sum_{b,y,x} dc[co][y][x] * act[ci][y+a][x+b];  db2[co] = sum dc.
// Winograd F(2x2,3x3) filter gradient: with U = G g G^T linear in g, per 2x2 output tile t (= one
// pool window)  dU[ij][co][ci] += Z_t[ij][co] * V_t[ij][ci],  Z_t = A dY_t A^T (the routed window:
// one nonzero, so Z_t = v * ZT[code], a lookup and 8 packed multiplies), V_t = B^T d_t B (the
// forward's input transform of the act patch), and dW = G^T dU G once per workgroup slab (linear, so
// the slabs keep the [dW2 | db2] layout slk_sgd_from_slabs sums in fixed order).
// GEMM per (i,j): M = 64 co, N = 32 ci, K = tiles x samples; v_mfma_f32_16x16x4_f32 with A = Z
// (lane: co = l&15, tile = l>>4) and B = V (tile = l>>4, ci = l&15); no filter registers.
// Persistent, one 4-wave workgroup per CU: wave w owns the output channels 32*(w&1) .. +31 (2 M
// blocks) x all 32 input channels (2 N blocks) = 64 accumulator tiles (256 AGPRs), and the K steps
// (4 tiles each) of parity w>>1. Unit = (sample, band of 4 tile rows = 48 tiles = 12 K steps): the
// act band (as the forward) + the dpooled/code band of the same windows, double-buffered by LDS-DMA.
// At the end the two K-parity waves of each M half meet in LDS (fixed order), apply G^T . G and
// write the workgroup's slab; db2 rides along as ZT[c][1][1] = 1 for every routed window.
constexpr int WW_WAVES = 4;
constexpr int WW_THREADS = WW_WAVES * 64;
constexpr int WW_DSTR = 52;                           // dpooled band row stride (48 used; 2-way banks)
constexpr int WW_DP_OFF = WF_BSTR;                    // float offset of the dpooled band in a buffer
constexpr int WW_DP_CH = 64 * 13 / 64;                // 13 chunks (13 sixteen-byte pieces per row)
// Code band rows are 48 bytes (the band's 48 windows, 3 DMA pieces): lanes li = 0..15 (one co each)
// then read bytes 12 dwords apart, 2-way at worst on ds_read_u8's 32 banks (a 64-byte stride put 8
// lanes on each of 2 banks: 8-way). The ZT table rows are 20 floats apart so that the five codes'
// float4 reads sit on five distinct 16-byte slots of the 256-byte bank row (at 16 floats, code 4 —
// ReLU-blocked, the commonest — shared a slot with code 0). A/B knobs: SLK_WW_CSTR, SLK_WW_LUTS.
#ifndef SLK_WW_CSTR
#define SLK_WW_CSTR 48
#endif
#ifndef SLK_WW_LUTS
#define SLK_WW_LUTS 20
#endif
constexpr int WW_CSTR = SLK_WW_CSTR;                  // code band row stride in bytes (48 used)
constexpr int WW_LUTS = SLK_WW_LUTS;                  // ZT row stride in floats (16 used)
constexpr int WW_CD_OFF = WW_DP_OFF + 64 * WW_DSTR;   // float offset of the code band
constexpr int WW_CD_PC = WW_CSTR / 16;                // DMA pieces per code row (3 used)
constexpr int WW_CD_CH = 64 * WW_CD_PC / 64;          // chunks of the code band
constexpr int WW_NCH = WF_CHUNKS + WW_DP_CH + WW_CD_CH;
constexpr int WW_BSTR = WW_CD_OFF + 64 * WW_CSTR / 4; // 12800 floats = 51,200 B per buffer
constexpr int WW_GRID = 256;
constexpr int WW_SLAB = W2_N + C2;
// Staging buffers (2: a unit's DMA is issued one unit ahead). Removing DMA + wait + barrier saves
// 0.085 of 0.413 ms (a round-1 ablation build), but 3 buffers (DMA two units ahead) gain
// nothing (0.422 vs 0.417 ms): not DMA latency. Knob kept for A/B.
#ifndef SLK_WW_NBUF
#define SLK_WW_NBUF 2
#endif
constexpr int WW_NBUF = SLK_WW_NBUF;
// SLK_WW_SPREAD = 1 issues the next unit's DMA two or three pieces per K step instead of all at the
// unit start. With the per-piece address code of round 1 it gained nothing (0.4175 vs 0.4153 ms; 3
// buffers 0.4286) — that code, not the DMA's latency or burst, was the cost (dropping the issue
// entirely: 0.414 -> 0.346 ms at an unchanged 2.31 GHz in-kernel clock). With the offset table the
// spread form is the faster one (0.3808 vs 0.3859 ms, same box, profiles/r02_ab_dma_offsets.txt).
// (3 buffers no longer fit beside the table.)
#ifndef SLK_WW_SPREAD
#define SLK_WW_SPREAD 1
#endif
constexpr bool WW_SPREAD = SLK_WW_SPREAD;
// glds16 instructions of wave w per unit (chunks w, w+4, ...): the counted wait leaves the newer
// unit's batch in flight
template <int W>
__device__ __forceinline__ void ww_wait_newest_batch() { wg_wait_vmcnt<(WW_NCH - W + WW_WAVES - 1) / WW_WAVES>(); }
static_assert(WW_DP_OFF * 4 == WF_CHUNKS * 1024 && WW_CD_OFF * 4 == (WF_CHUNKS + WW_DP_CH) * 1024,
              "the three staging regions are consecutive KiB chunks");

// chunks i0 .. i1-1 of this wave's share (chunk c = wave + 4i) of unit u's staging DMA. Piece (c, lane)'s
// byte offset from its region's first element (act band, dpooled band or code band of the unit) is
// the same for every unit: the offsets are computed once per launch into an LDS table (this kernel has
// no VGPRs to spare) and a piece is one saddr-form DMA from a scalar region base — the per-piece
// divisions, 64-bit address arithmetic and region branches had cost ~200 cycles per piece beside the
// MFMAs (16 % of the kernel: dropping the DMA issue took it from 0.414 to 0.346 ms).
constexpr int WW_PPW = (WW_NCH + WW_WAVES - 1) / WW_WAVES;   // 13 pieces per wave and unit
constexpr int WW_TQ = (WW_PPW + 3) / 4;                      // uint4 table entries per lane
__device__ __forceinline__ uint32_t ww_piece_offset(int c, int lane) {
    if (c < WF_CHUNKS) {
        const int p = min(c * 64 + lane, WF_PIECES - 1);
        const int ci = p / 65, k = p - 65 * (p / 65);
        return (uint32_t)(ci * A_PIX + 4 * k) * 4u;
    } else if (c < WF_CHUNKS + WW_DP_CH) {
        const int p = (c - WF_CHUNKS) * 64 + lane;
        const int co = p / 13, k = min(p - 13 * (p / 13), 11);
        return (uint32_t)(co * P_WIN + 4 * k) * 4u;
    }
    const int p = (c - WF_CHUNKS - WW_DP_CH) * 64 + lane;
    const int co = p / WW_CD_PC, k = min(p - WW_CD_PC * (p / WW_CD_PC), 2);
    return (uint32_t)(co * P_WIN + 16 * k);
}
__device__ __forceinline__ void ww_dma_table(uint4* tab, int wave, int lane) {
#pragma unroll
    for (int q = 0; q < WW_TQ; ++q) {
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = wave + WW_WAVES * (4 * q + j);
            o[j] = c < WW_NCH ? ww_piece_offset(c, lane) : 0u;
        }
        tab[(wave * WW_TQ + q) * 64 + lane] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}
__device__ __forceinline__ void ww_dma_unit(const float* __restrict__ act, const float* __restrict__ dpool,
                                            const uint8_t* __restrict__ code, int u, const float* dst, int wave,
                                            int lane, const uint4* tab, int i0 = 0, int i1 = 1 << 20) {
    const int b = u / 3, band = u - 3 * (u / 3);
    wave &= WW_WAVES - 1;   // (known range: the chunk bound below folds away for i < WW_PPW - 1)
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)dst);
    const void* asrc = act + (size_t)b * A_SAMPLE + band * 8 * A_HW;
    const void* dsrc = dpool + (size_t)b * P_SAMPLE + band * 48;
    const void* csrc = code + (size_t)b * P_SAMPLE + band * 48;
    uint4 o[WW_TQ];
#pragma unroll
    for (int q = 0; q < WW_TQ; ++q) o[q] = tab[(wave * WW_TQ + q) * 64 + lane];
#pragma unroll
    for (int i = 0; i < WW_PPW; ++i) {
        const int c = wave + WW_WAVES * i;
        if (c >= WW_NCH || i < i0 || i >= i1) continue;
        const uint4 oq = o[i >> 2];
        const uint32_t off = (i & 3) == 0 ? oq.x : (i & 3) == 1 ? oq.y : (i & 3) == 2 ? oq.z : oq.w;
        const void* src = c < WF_CHUNKS ? asrc : (c < WF_CHUNKS + WW_DP_CH ? dsrc : csrc);
        glds16_so(src, off, base + c * 1024);
    }
}

// dW = G^T dU G (adjoint of wino_filter), dw row-major dw[3*k + l]
__device__ __forceinline__ void wino_filter_grad(const float (&du)[16], float (&dw)[9]) {
    float t[12];  // t = G^T dU : 3 x 4
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float s = du[4 + j] + du[8 + j];
        t[0 * 4 + j] = du[j] + 0.5f * s;
        t[1 * 4 + j] = 0.5f * (du[4 + j] - du[8 + j]);
        t[2 * 4 + j] = 0.5f * s + du[12 + j];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float s = t[k * 4 + 1] + t[k * 4 + 2];
        dw[k * 3 + 0] = t[k * 4 + 0] + 0.5f * s;
        dw[k * 3 + 1] = 0.5f * (t[k * 4 + 1] - t[k * 4 + 2]);
        dw[k * 3 + 2] = 0.5f * s + t[k * 4 + 3];
    }
}

__global__ __launch_bounds__(WW_THREADS, 1) void conv2_wgrad_wino_kernel(
    const float* __restrict__ act, const float* __restrict__ dpool, const uint8_t* __restrict__ code,
    float* __restrict__ slabs, int B) {
    __shared__ __attribute__((aligned(16))) float smem[WW_NBUF * WW_BSTR + 5 * WW_LUTS + WW_WAVES * WW_TQ * 64 * 4];
    float* lutz = smem + WW_NBUF * WW_BSTR;  // ZT[c][16], rows WW_LUTS floats apart
    uint4* dtab = reinterpret_cast<uint4*>(lutz + ((5 * WW_LUTS + 3) & ~3));  // DMA piece offsets
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int wu = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform: scalar branches on tp
    const int mh = wu & 1, tp = wu >> 1;
    const int nunit = 3 * B;

    int u = blockIdx.x;
    ww_dma_table(dtab, wu, lane);   // read back only by the same lane: no barrier
    if (u < nunit) ww_dma_unit(act, dpool, code, u, smem, wu, lane, dtab);
    if (tid < 5 * 16) {
        const int c = tid >> 4, i = (tid >> 2) & 3, j = tid & 3;
        const float ai = (c & 2) ? (i == 0 ? 0.f : (i == 1 ? 1.f : -1.f)) : (i == 3 ? 0.f : 1.f);
        const float aj = (c & 1) ? (j == 0 ? 0.f : (j == 1 ? 1.f : -1.f)) : (j == 3 ? 0.f : 1.f);
        lutz[c * WW_LUTS + (tid & 15)] = c < 4 ? ai * aj : 0.f;
    }
    f32x4 acc[2][2][16];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int ij = 0; ij < 16; ++ij) acc[m][n][ij] = f32x4{0.f, 0.f, 0.f, 0.f};
    float dbp[2] = {0.f, 0.f};
    if (WW_NBUF > 2 && u + (int)gridDim.x < nunit)
        ww_dma_unit(act, dpool, code, u + gridDim.x, smem + WW_BSTR, wu, lane, dtab);

    int buf = 0;
#pragma unroll 1
    for (; u < nunit; u += gridDim.x) {
        // this unit's DMA landed (no other vector memory ops in this loop: only the next unit's batch
        // may stay in flight) and every wave is done with the buffer refilled next
        const int nu = u + (WW_NBUF - 1) * (int)gridDim.x;
        {
            if (WW_NBUF > 2 && u + (int)gridDim.x < nunit) {
                switch (wu) {
                    case 0: ww_wait_newest_batch<0>(); break;
                    case 1: ww_wait_newest_batch<1>(); break;
                    case 2: ww_wait_newest_batch<2>(); break;
                    default: ww_wait_newest_batch<3>(); break;
                }
            } else {
                wg_wait_vmcnt<0>();
            }
            lds_barrier();
            if (nu < nunit && !WW_SPREAD) {
                const int nb = buf + WW_NBUF - 1 >= WW_NBUF ? buf - 1 : buf + WW_NBUF - 1;
                ww_dma_unit(act, dpool, code, nu, smem + nb * WW_BSTR, wu, lane, dtab);
            }
        }
        const float* img = smem + buf * WW_BSTR;
        const float* dpb = img + WW_DP_OFF + (32 * mh + li) * WW_DSTR;
        const uint8_t* cdb = reinterpret_cast<const uint8_t*>(img + WW_CD_OFF) + (32 * mh + li) * WW_CSTR;
        const int band = u - 3 * (u / 3);

        // K step j (tiles 4ks + lk of the band, ks = tp + 2j): raw act patches of ci = li, 16 + li
        // and the routed windows of co = 32mh + li, 32mh + 16 + li
        f2 Rlo[2][2][4], Rhi[2][2][4];
        float dv[2][2];
        int cd[2][2];
        auto load = [&](int j, f2 (&lo)[2][4], f2 (&hi)[2][4], float (&v)[2], int (&c)[2]) {
            // band-local tile tl = 12 qy + qx (< 48): patch at rows 2qy, cols 2qx of the band image,
            // i.e. 2 tl + 28 qy floats; qy = tl / 12 = (43 tl) >> 9 exactly for tl < 128
            const int tl = 4 * (tp + 2 * j) + lk;
            const int qy = (tl * 43) >> 9;
            const float* pa = img + li * WF_CSTR + 2 * tl + 28 * qy;
            lds_patch_pk(pa, lo[0], hi[0]);
            lds_patch_pk(pa + 16 * WF_CSTR, lo[1], hi[1]);
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                v[m] = dpb[m * 16 * WW_DSTR + tl];
                c[m] = cdb[m * 16 * WW_CSTR + tl];
            }
        };
        f2 v01[2][4], v23[2][4], z01[2][4], z23[2][4];
        // ZT rows of a step's two windows, issued one step ahead (the codes arrived a step earlier)
        // so the dependent LDS read is not exposed in front of the multiplies
        auto zload = [&](const int (&c)[2], float4 (&E)[2][4]) {
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const float4* zt = reinterpret_cast<const float4*>(lutz + WW_LUTS * c[m]);
#pragma unroll
                for (int i = 0; i < 4; ++i) E[m][i] = zt[i];
            }
        };
        auto xform = [&](const f2 (&lo)[2][4], const f2 (&hi)[2][4], const float (&v)[2], const float4 (&E)[2][4]) {
            pk_wino_in(lo[0], hi[0], v01[0], v23[0]);
            pk_wino_in(lo[1], hi[1], v01[1], v23[1]);
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const f2 vv = {v[m], v[m]};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float4 e = E[m][i];
                    z01[m][i] = vv * f2{e.x, e.y};
                    z23[m][i] = vv * f2{e.z, e.w};
                }
                dbp[m] += z01[m][1].y;  // ZT[c][1][1] = 1 for a routed window, 0 for code 4
            }
        };
        float4 E[2][4];
        load(0, Rlo[0], Rhi[0], dv[0], cd[0]);
        load(1, Rlo[1], Rhi[1], dv[1], cd[1]);
        zload(cd[0], E);
        xform(Rlo[0], Rhi[0], dv[0], E);
        const float* dma_dst = smem + (buf + WW_NBUF - 1 >= WW_NBUF ? buf - 1 : buf + WW_NBUF - 1) * WW_BSTR;
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            // (SLK_WW_SPREAD) the next unit's staging DMA, two or three pieces per K step
            if (WW_SPREAD && nu < nunit)
                ww_dma_unit(act, dpool, code, nu, dma_dst, wu, lane, dtab, 2 * j, j == 5 ? 1 << 20 : 2 * j + 2);
            if (j < 5) zload(cd[(j + 1) & 1], E);                                  // under these MFMAs
            if (j < 4) load(j + 2, Rlo[j & 1], Rhi[j & 1], dv[j & 1], cd[j & 1]);  // likewise
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int n = 0; n < 2; ++n)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        mfma_acc(acc[m][n][4 * i + 0], z01[m][i].x, v01[n][i].x);
                        mfma_acc(acc[m][n][4 * i + 1], z01[m][i].y, v01[n][i].y);
                        mfma_acc(acc[m][n][4 * i + 2], z23[m][i].x, v23[n][i].x);
                        mfma_acc(acc[m][n][4 * i + 3], z23[m][i].y, v23[n][i].y);
                    }
            __builtin_amdgcn_sched_barrier(0);
            if (j < 5) xform(Rlo[(j + 1) & 1], Rhi[(j + 1) & 1], dv[(j + 1) & 1], E);
        }
        buf = buf + 1 == WW_NBUF ? 0 : buf + 1;
    }

    mfma_drain();
    // ---- combine the K parities, transform, write this workgroup's [dW2 | db2] slab
    float* slab = slabs + (size_t)blockIdx.x * WW_SLAB;
    float* park = smem;  // [mh][n][ij][r][lane] for one M block m at a time (16384 floats)
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        lds_barrier();  // previous readers of `park` (or of the staging buffers) are done
        if (tp == 1) {
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int ij = 0; ij < 16; ++ij)
#pragma unroll
                    for (int r = 0; r < 4; ++r) park[(((mh * 2 + n) * 16 + ij) * 4 + r) * 64 + lane] = acc[m][n][ij][r];
        }
        lds_barrier();
        if (tp == 0) {
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float du[16], dw[9];
#pragma unroll
                    for (int ij = 0; ij < 16; ++ij) du[ij] = acc[m][n][ij][r] + park[(((mh * 2 + n) * 16 + ij) * 4 + r) * 64 + lane];
                    wino_filter_grad(du, dw);
                    const int co = 32 * mh + 16 * m + 4 * lk + r, ci = 16 * n + li;
#pragma unroll
                    for (int k = 0; k < 9; ++k) slab[co * K2 + ci * 9 + k] = dw[k];
                }
        }
    }
    // db2: lanes of one co hold partials over tiles (lk) -> butterfly, then K parity 0 + 1
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        dbp[m] += __shfl_xor(dbp[m], 16, 64);
        dbp[m] += __shfl_xor(dbp[m], 32, 64);
    }
    lds_barrier();
    if (tp == 1 && lk == 0) {
        park[(mh * 2 + 0) * 16 + li] = dbp[0];
        park[(mh * 2 + 1) * 16 + li] = dbp[1];
    }
    lds_barrier();
    if (tp == 0 && lk == 0) {
#pragma unroll
        for (int m = 0; m < 2; ++m) slab[W2_N + 32 * mh + 16 * m + li] = dbp[m] + park[(mh * 2 + m) * 16 + li];
    }
}

extern "C" int slk_conv2_wgrad_nslab(int B) { return B > 0 ? (3 * B < WW_GRID ? 3 * B : WW_GRID) : 0; }

extern "C" int slk_conv2_wgrad(const float* act, const float* dpooled, const uint8_t* code,
                               float* slabs, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(act && dpooled && code && slabs);
    conv2_wgrad_wino_kernel<<<slk_conv2_wgrad_nslab(B), WW_THREADS, 0, slk_stream(stream)>>>(act, dpooled, code, slabs, B);
    return slk_launch_status();
}
