// slk_x3.hip — conv2 of the reference split CNN (src/model_def.py:18,25-27) as a direct implicit GEMM
// on the f16 MFMA with fp32-grade operands ("x3"): every f32 operand v is split, after an exact
// power-of-two scale 2^s, into v*2^s = h + l + r with h = f16(v*2^s), l = f16(v*2^s - h) (both RNE),
// |r| <= 2^-22 |v*2^s|, and each product is formed as h_a*h_b + h_a*l_b + l_a*h_b by three
// v_mfma_f32_16x16x32_f16 into one f32 accumulator (dropped: l_a*l_b <= 2^-22 |ab|). Per product that is
// a relative error of at most ~3 * 2^-22 = 7e-7 — an order of the f32 MFMA's own 2^-24 rounding per
// accumulation step, and below the error the Winograd F(2x2,3x3) transforms add to the f32 path — at
// 3 f16 MFMAs (48 cycles) per 16x16x32 block instead of 8 f32 MFMAs (256 cycles).
//
// Scales (exact powers of two, so unscaling the f32 accumulator is exact):
//   - weights: one per launch, from max|W2| (every workgroup reduces W2 itself in its prologue);
//   - data operands: one per SAMPLE, from a per-sample max |.| array (slk_row_amax, or fused into the
//     producer), so that the largest element lands in [2^13, 2^14): nothing overflows f16's 65504 and
//     nothing that matters reaches f16's subnormal range (values 2^-38 below a sample's max lose
//     relative precision, which is below f32's own resolution of that sum).
// Routing/pool/ReLU semantics are those of the f32 kernels (torch CPU: first max wins, strict >).
#include "slk_common.h"

#include <type_traits>

using namespace slk;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

namespace {

// s such that amax * 2^s < 2^14 (amax in [2^13, 2^14) after scaling); 0 for zero / non-finite amax.
// Clamped to X3_SMAX so that 2^s and 2^-s are both normal floats: a sample whose max is below
// 2^(14 - X3_SMAX) (~2^-112, e.g. the subnormal dpooled of a confidently-correct sample) lands lower in
// f16's range instead of being scaled by inf. Every unscale multiplies by 2^-s of each operand in turn
// (x3_unscale), never by 2^-(s1 + s2), so it stays finite and exact.
constexpr int X3_SMAX = 126;
__device__ __forceinline__ int x3_exp(float amax) {
    if (!(amax > 0.f) || !__builtin_isfinite(amax)) return 0;
    int e;
    (void)frexpf(amax, &e);  // amax = m * 2^e, m in [0.5, 1)
    return min(14 - e, X3_SMAX);
}
// 2^-s1 * 2^-s2 applied as two exact power-of-two multiplies (each factor a normal float)
__device__ __forceinline__ float x3_unscale(float v, float u1, float u2) { return (v * u1) * u2; }

// 8 scaled f32 values -> 8 f16 hi + 8 f16 lo (v_cvt_pk_f16_f32, RNE).
__device__ __forceinline__ void x3_split8(const float* v, float sc, f16x8& h, f16x8& l) {
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
        const float a = v[k] * sc, b = v[k + 1] * sc;
        const _Float16 ha = (_Float16)a, hb = (_Float16)b;
        h[k] = ha;
        h[k + 1] = hb;
        l[k] = (_Float16)(a - (float)ha);
        l[k + 1] = (_Float16)(b - (float)hb);
    }
}

__device__ __forceinline__ f32x4 mfma_f16(const f16x8& a, const f16x8& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// acc += (ah + al)(bh + bl) - al*bl
__device__ __forceinline__ f32x4 mfma_x3(const f16x8& ah, const f16x8& al, const f16x8& bh, const f16x8& bl, f32x4 c) {
    c = mfma_f16(ah, bh, c);
    c = mfma_f16(ah, bl, c);
    return mfma_f16(al, bh, c);
}

// max over the wave: within 16-lane rows by DPP, then across rows (2 LDS-path shuffles instead of 6)
__device__ __forceinline__ float wave_max_dpp(float v) {
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false)));   // quad_perm 1,0,3,2
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false)));   // quad_perm 2,3,0,1
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false)));  // row_half_mirror
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false)));  // row_mirror
    v = fmaxf(v, __shfl_xor(v, 16, 64));
    return fmaxf(v, __shfl_xor(v, 32, 64));
}

}  // namespace

// ============================================================================ per-row max |x|
// amax[r] = max_i |x[r*n + i]| (NaNs ignored). The x3 kernels' per-sample operand scales.
__global__ __launch_bounds__(256) void row_amax_kernel(const float* __restrict__ x, int n, float* __restrict__ amax) {
    __shared__ float red[4];
    const float* row = x + (size_t)blockIdx.x * n;
    float m = 0.f;
    if ((n & 3) == 0 && ((reinterpret_cast<size_t>(x) & 15) == 0)) {
        const float4* r4 = reinterpret_cast<const float4*>(row);
        const int n4 = n / 4;
        int i = threadIdx.x;
        // 8 independent float4 loads in flight per thread (one at a time left the kernel latency-bound
        // at ~3.9 TB/s over a 354 MB cut); max is order-independent, so the result is unchanged
        for (; i + 7 * 256 < n4; i += 8 * 256) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = r4[i + 256 * u];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
        }
        for (; i < n4; i += 256) {
            const float4 v = r4[i];
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        }
    } else {
        for (int i = threadIdx.x; i < n; i += 256) m = fmaxf(m, fabsf(row[i]));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) amax[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// ============================================================================ conv2 forward + pool
// Unit = (sample, third): output rows 8t..8t+7 (window rows 4t..4t+3), input rows 8t..8t+9 (the
// unit's 32 channel segments of 260 floats are contiguous runs of act). Staging, two units ahead:
//   1. LDS-DMA copies the unit's raw f32 rows into a raw buffer [ci][260] (2,080 16-byte pieces, the
//      per-lane source offsets computed once per launch), issued at the top of unit u for unit u+2;
//   2. during unit u+1's MFMAs each thread reads its items (pixel, 8-ci chunk) from the raw buffer
//      (8 conflict-free ds_read_b32), scales, splits and writes them as two f16 planes [pixel][ci]
//      (64 B per pixel; chunk slot kc ^ (x & 2) makes every ds_read_b128 of the MFMA loop
//      conflict-free, tools-checked for all 9 taps).
// One `s_waitcnt vmcnt` (allowing the previous epilogue's 12 stores to stay in flight) + barrier per
// unit. 8 waves (2 per SIMD): wave = (co half ch, window row wr); its 2 x 9 taps x (h, l) weight
// fragments (144 VGPRs) stay in registers for the launch. Tried and slower: 4 waves (one per SIMD)
// holding all 64 co — weights copied back from AGPRs per MFMA by hipcc 0.375 ms; taps 0-7 in AGPRs as
// asm MFMA operands + tap 8 in VGPRs, A reads 2 steps ahead 0.342 ms (vs 0.254): one wave per SIMD
// leaves the split/epilogue VALU and the LDS latency uncovered. A = input (M = 16 pixels = 4 pool windows x
// 4 positions), B = weights (N = 16 co), K = 32 ci of one tap; the C/D layout puts the 4 positions of
// one window in one lane's 4 accumulators, so ReLU + 2x2 max-pool + routing code are in-register.
constexpr int X3F_WAVES = 8;
constexpr int X3F_THREADS = 64 * X3F_WAVES;
constexpr int X3F_NT = 2;                        // co tiles per wave
constexpr int X3F_ROWS = 10;
constexpr int X3F_PIX = X3F_ROWS * A_HW;          // 260 pixels per unit
constexpr int X3F_PLANE = X3F_PIX * 64;           // 16,640 B per f16 plane
constexpr int X3F_BUF = 2 * X3F_PLANE;            // h + l
constexpr int X3F_RAW = C1 * X3F_PIX * 4;         // 33,280 B raw f32 rows
constexpr int X3F_PIECES16 = X3F_RAW / 16;        // 2,080 16-byte DMA pieces per unit
constexpr int X3F_WPIECES = (X3F_PIECES16 / 64 + 1 + X3F_WAVES - 1) / X3F_WAVES;  // DMA wave-instructions per wave
constexpr int X3F_ITEMS = X3F_PIX * 4;            // (pixel, 8-ci chunk) split items
constexpr int X3F_IPT = (X3F_ITEMS + X3F_THREADS - 1) / X3F_THREADS;  // 3
constexpr int X3F_GRID = 256;
constexpr int X3F_STORES = 2 * X3F_NT;            // epilogue global stores per wave and unit (x3f_store_row)
static_assert(X3F_RAW % 1024 == 512, "the last DMA wave-instruction is a half piece");
// AMX (f32 rows in, the drop-in module path): the kernel computes each sample's max |act| itself instead of a
// separate row_amax pass over the cut. A sample's 5,408 16-B pieces are read in 3 contiguous chunks by
// LDS-DMA into one chunk buffer — chunk j of sample b in unit 3b - 5 + j, at the wave's split point;
// folded into a per-lane running max in the next unit (its top wait has retired the DMA) by the lanes that
// DMA'd it; reduced across the waves through red_amx in unit 3b - 1, just before its split of unit 3b,
// the sample's first use of its scale. The chunk reads add the cut's bytes once more to the kernel's
// traffic: 0.257 -> 0.306 ms at B = 4096, against a 0.06-0.09 ms row_amax pass it replaces.
constexpr int X3F_SP16 = A_SAMPLE * 4 / 16;                        // 5,408 pieces per sample
constexpr int X3F_CP = (X3F_SP16 + 2) / 3;                         // 1,803 pieces per chunk
constexpr int X3F_CI = (X3F_CP + 63) / 64;                         // 29 wave-instructions per chunk
constexpr int X3F_CIW = (X3F_CI + X3F_WAVES - 1) / X3F_WAVES;      // per wave (max)
// act16 images in HBM: per SAMPLE, the whole 26 x 26 cut as an h plane then an l plane ([pixel][32 ci]
// f16, 64-B pixels, chunk slot c8 ^ (x & 2)), 86,528 B a sample: a unit (sample, third t3) is rows
// 8 t3 .. 8 t3 + 9 of each plane — two contiguous 16,640-B runs — so no row is stored twice
constexpr int X3S_PLANE = A_PIX * 64;             // 43,264 B
constexpr int X3S_SAMPLE = 2 * X3S_PLANE;         // 86,528 B
constexpr int X3S_UNIT_OFF = 8 * A_HW * 64;       // 13,312 B between consecutive thirds
static_assert(X3F_PLANE == X3F_ROWS * A_HW * 64 && X3F_PLANE % 1024 == 256, "unit run = 16 KiB + 256 B");

// LDS-DMA of unit uu's image (h run -> lds, l run -> lds + X3F_PLANE) by an 8-wave workgroup: 2 x
// (16 full 1-KiB wave-instructions + one 256-B quarter), pieces spread over the waves (4 or 5 each)
__device__ __forceinline__ void x3_issue_unit_img(const uint16_t* act16, int uu, int wave, int lane, uint32_t lds) {
    const int b = uu / 3, t3 = uu - (uu / 3) * 3;
    const char* srch = reinterpret_cast<const char*>(act16) + (size_t)b * X3S_SAMPLE + t3 * X3S_UNIT_OFF;
    constexpr int PP = X3F_PLANE / 1024 + 1;  // 17 pieces per plane
#pragma unroll
    for (int r = 0; r < 5; ++r) {
        const int piece = wave + 8 * r;
        if (piece < 2 * PP) {
            const int pl = piece >= PP ? 1 : 0, pp = piece - PP * pl;
            const char* src = srch + pl * X3S_PLANE;
            if (pp < PP - 1 || lane < 16) glds16_so(src, (uint32_t)(pp * 1024 + lane * 16), lds + pl * X3F_PLANE + pp * 1024);
        }
    }
}

// the same image as separate pieces for issue inside the MFMA stream: full piece r (0-3) of wave w is
// piece w + 8r of the 32 full 1-KiB pieces (plane = piece >> 4); the two 256-B quarters go to waves 0-1
__device__ __forceinline__ const char* x3_unit_img_src(const uint16_t* act16, int uu) {
    const int b = uu / 3, t3 = uu - (uu / 3) * 3;
    return reinterpret_cast<const char*>(act16) + (size_t)b * X3S_SAMPLE + t3 * X3S_UNIT_OFF;
}
__device__ __forceinline__ void x3_issue_img_full(const char* srch, int wave, int lane, uint32_t lds, int r) {
    const int piece = wave + 8 * r, pl = piece >> 4, pp = piece & 15;
    glds16_so(srch + pl * X3S_PLANE, (uint32_t)(pp * 1024 + lane * 16), lds + pl * X3F_PLANE + pp * 1024);
}
__device__ __forceinline__ void x3_issue_img_quarter(const char* srch, int wave, int lane, uint32_t lds) {
    if (lane < 16) glds16_so(srch + wave * X3S_PLANE, (uint32_t)(16 * 1024 + lane * 16), lds + wave * X3F_PLANE + 16 * 1024);
}

__device__ __forceinline__ void x3f_issue_raw(const float* act, int uu, int wave, int lane, const uint32_t* voff,
                                              uint32_t raw_lds) {
    const int b = uu / 3, t3 = uu - (uu / 3) * 3;
    const char* base = reinterpret_cast<const char*>(act + (size_t)b * A_SAMPLE + t3 * 8 * A_HW);
#pragma unroll
    for (int k = 0; k < X3F_WPIECES; ++k) {
        const int piece = wave + X3F_WAVES * k;
        if (piece < X3F_PIECES16 / 64) {
            glds16_so(base, voff[k], raw_lds + piece * 1024);
        } else if (piece == X3F_PIECES16 / 64 && lane < 32) {
            glds16_so(base, voff[k], raw_lds + piece * 1024);
        }
    }
}

// pooled / code of one (unit, co) output row (12 windows). Lane (n16, kc) holds windows kc, 4 + kc, 8 + kc
// (M tiles 0-2); a 4 x 4 transpose across the four 16-lane groups (two v_permlane32_swap + two
// v_permlane16_swap per value) gives lane kc' windows 4 kc' .. 4 kc' + 3: one float4 + one u32 store on
// lanes kc' < 3 instead of three 4-B and three 1-B stores per lane (16 scattered pieces each; the six
// stores cost ~15 % of the kernel, interleaved A/B)
__device__ __forceinline__ void x3f_t4(uint32_t& r0, uint32_t& r1, uint32_t& r2, uint32_t& r3) {
    auto s = __builtin_amdgcn_permlane32_swap(r0, r2, false, false);  // r0 lanes 32-63 <-> r2 lanes 0-31
    r0 = s[0];
    r2 = s[1];
    s = __builtin_amdgcn_permlane32_swap(r1, r3, false, false);
    r1 = s[0];
    r3 = s[1];
    s = __builtin_amdgcn_permlane16_swap(r0, r1, false, false);  // r0 odd 16-lane rows <-> r1 even rows
    r0 = s[0];
    r1 = s[1];
    s = __builtin_amdgcn_permlane16_swap(r2, r3, false, false);
    r2 = s[0];
    r3 = s[1];
}
__device__ __forceinline__ void x3f_store_row(float m0, float m1, float m2, uint32_t c0, uint32_t c1, uint32_t c2,
                                              int kc, float* __restrict__ prow, uint8_t* __restrict__ crow) {
    uint32_t v0 = __float_as_uint(m0), v1 = __float_as_uint(m1), v2 = __float_as_uint(m2), v3 = 0u;
    uint32_t q3 = 0u;
    x3f_t4(v0, v1, v2, v3);
    x3f_t4(c0, c1, c2, q3);
    if (kc < 3) {
        *reinterpret_cast<float4*>(prow + 4 * kc) =
            make_float4(__uint_as_float(v0), __uint_as_float(v1), __uint_as_float(v2), __uint_as_float(v3));
        *reinterpret_cast<uint32_t*>(crow + 4 * kc) = c0 | (c1 << 8) | (c2 << 16) | (q3 << 24);
    }
}

// act16 (optional): every unit's f16 image (the layout above, the sample's own scale) is also written
// to the per-sample act16 image (X3S_*) for conv2_wgrad_x3's input operand.
// IN16 = true: the input IS such an image array (slk_conv1_fwd_x3 wrote it): each unit's image is moved
// by LDS-DMA two units ahead into a 3-deep ring of f16 buffers — no f32 rows, no split.
// AMX = true (IN16 false, act16 required): amax is not read; the per-sample max |act| is computed here
// (layout above X3F_SP16) and written to amax_out.
template <bool IN16, bool AMX = false>
__global__ __launch_bounds__(X3F_THREADS, 1) void conv2_fwd_pool_x3_kernel(
    const float* __restrict__ act, const float* __restrict__ amax, const float* __restrict__ W2,
    const float* __restrict__ b2, float* __restrict__ pooled, uint8_t* __restrict__ code, int B,
    uint16_t* __restrict__ act16 = nullptr, float* __restrict__ amax_out = nullptr) {
    static_assert(3 * X3F_BUF <= 2 * X3F_BUF + 2 * X3F_RAW, "IN16 ring fits");
    static_assert(!(IN16 && AMX), "AMX reads f32 rows");
    constexpr int SMEM = 2 * X3F_BUF + 2 * X3F_RAW + (AMX ? X3F_CI * 1024 : 0);
    static_assert(SMEM + 64 <= 163840, "LDS");
    __shared__ __attribute__((aligned(1024))) char smem[SMEM];
    __shared__ float red[X3F_WAVES];
    __shared__ float red_amx[X3F_WAVES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ch = wave & 1, wr = wave >> 1;
    const int n16 = lane & 15, kc = lane >> 4;
    char* const raw0 = smem + 2 * X3F_BUF;

    const int U = 3 * B;
    const int G = gridDim.x;
    // a contiguous range of units per workgroup: the three thirds of a sample run back to back on one
    // CU, so the 2 halo rows each shares with the next come from that XCD's L2, not HBM (AMX: whole
    // samples per workgroup)
    const int per = AMX ? 3 * ((B + G - 1) / G) : (U + G - 1) / G;
    const int u0 = min((int)blockIdx.x * per, U), u1 = min(u0 + per, U);
    int u = u0;
    // AMX state: the running max of the sample being read (per lane), the current unit's sample max and
    // the next sample's (wave-uniform)
    float run = 0.f, am_cur = 0.f, am_nxt = 0.f;
    char* const cbuf = smem + 2 * X3F_BUF + 2 * X3F_RAW;
    auto amx_chunk = [&](int v, int& sb, int& lim) {  // unit v reads chunk (v + 2) % 3 of sample (v + 5) / 3
        sb = __builtin_amdgcn_readfirstlane((v + 5) / 3);
        const int j = __builtin_amdgcn_readfirstlane((v + 2) - 3 * ((v + 2) / 3));
        lim = j == 2 ? X3F_SP16 - 2 * X3F_CP : X3F_CP;
        return reinterpret_cast<const char*>(act + (size_t)sb * A_SAMPLE) + j * X3F_CP * 16;
    };
    auto amx_issue = [&](int v) {
        int sb, lim;
        const char* src = amx_chunk(v, sb, lim);
        if (3 * sb >= u1) return;
        const uint32_t dst = lds_u32(cbuf);
#pragma unroll
        for (int r = 0; r < X3F_CIW; ++r) {
            const int i = wave + X3F_WAVES * r, q = 64 * i + lane;
            if (i < X3F_CI && q < lim) glds16_so(src, (uint32_t)(q * 16), dst + i * 1024);
        }
    };
    auto amx_fold = [&](int v) {  // at the top of unit v + 1, after its barrier: unit v's chunk has landed
        int sb, lim;
        amx_chunk(v, sb, lim);
        if (3 * sb >= u1) return;
#pragma unroll
        for (int r = 0; r < X3F_CIW; ++r) {
            const int i = wave + X3F_WAVES * r, q = 64 * i + lane;
            if (i < X3F_CI && q < lim) {
                const float4 v4 = *reinterpret_cast<const float4*>(cbuf + i * 1024 + lane * 16);
                run = fmaxf(run, fmaxf(fmaxf(fabsf(v4.x), fabsf(v4.y)), fmaxf(fabsf(v4.z), fabsf(v4.w))));
            }
        }
    };
    // DMA source offsets (bytes within a unit): piece g = 64k' + lane -> channel g / 65, 16-B run g % 65
    uint32_t voff[X3F_WPIECES];
#pragma unroll
    for (int k = 0; k < X3F_WPIECES; ++k) {
        const int g = (wave + X3F_WAVES * k) * 64 + lane;
        const int c = g / 65, r = g - (g / 65) * 65;
        voff[k] = (uint32_t)(c * A_PIX * 4 + r * 16);
    }
    // IN16: unit uu's image -> ring slot
    auto issue_img = [&](int uu, char* dstp) { x3_issue_unit_img(act16, uu, wave, lane, lds_u32(dstp)); };
    if constexpr (IN16) {
        if (u < u1) issue_img(u, smem);
        if (u + 1 < u1) issue_img(u + 1, smem + X3F_BUF);
    } else {
        if (u < u1) x3f_issue_raw(act, u, wave, lane, voff, lds_u32(raw0));
        if (u + 1 < u1) x3f_issue_raw(act, u + 1, wave, lane, voff, lds_u32(raw0 + X3F_RAW));
    }
    if constexpr (AMX) {  // sample u0 / 3 whole and chunks 0-1 of the next one, by plain loads
        float m0 = 0.f;
        if (u0 < u1) {
            // all loads in flight at once (11 + 8 per lane), then the maxima
            const float4* s4 = reinterpret_cast<const float4*>(act + (size_t)(u0 / 3) * A_SAMPLE);
            constexpr int NS = (X3F_SP16 + X3F_THREADS - 1) / X3F_THREADS;
            constexpr int NC = (2 * X3F_CP + X3F_THREADS - 1) / X3F_THREADS;
            const bool nxt = u0 + 3 < u1;
            float4 v4[NS + NC];
#pragma unroll
            for (int r = 0; r < NS + NC; ++r) {
                const int i = tid + X3F_THREADS * (r < NS ? r : r - NS);
                const bool ok = r < NS ? i < X3F_SP16 : (nxt && i < 2 * X3F_CP);
                v4[r] = ok ? s4[(r < NS ? 0 : X3F_SP16) + i] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int r = 0; r < NS + NC; ++r) {
                const float m = fmaxf(fmaxf(fabsf(v4[r].x), fabsf(v4[r].y)), fmaxf(fabsf(v4[r].z), fabsf(v4[r].w)));
                if (r < NS) m0 = fmaxf(m0, m);
                else run = fmaxf(run, m);
            }
        }
        m0 = wave_max(m0);
        if (lane == 0) red_amx[wave] = m0;
    }

    // weight scale: max |W2| over the whole tensor
    float wm = 0.f;
    for (int e = tid; e < W2_N; e += X3F_THREADS) wm = fmaxf(wm, fabsf(W2[e]));
    wm = wave_max(wm);
    if (lane == 0) red[wave] = wm;
    __syncthreads();
    wm = red[0];
#pragma unroll
    for (int i = 1; i < X3F_WAVES; ++i) wm = fmaxf(wm, red[i]);
    const int sw = x3_exp(wm);
    const float wsc = ldexpf(1.f, sw);
    auto red_amx_max = [&]() {
        float m = red_amx[0];
#pragma unroll
        for (int i = 1; i < X3F_WAVES; ++i) m = fmaxf(m, red_amx[i]);
        return m;
    };
    if constexpr (AMX) {
        am_cur = red_amx_max();
        if (tid == 0 && u0 < u1) amax_out[u0 / 3] = am_cur;
    }
    // AMX, once per unit at the wave's split point (before the split; at the unit's top instead — after the
    // barrier, before the MFMA stream — the LDS latencies were on the critical path: 0.328 vs 0.306 ms):
    // the next sample's max from the partials, the fold of the chunk unit u - 1 read (its DMA retired by
    // this unit's top wait), this wave's partial after a sample's last chunk, the DMA of this unit's chunk
    auto amx_step = [&](int r3) {
        if (r3 == 2) {  // the next sample's partials (written by unit u - 1, a barrier ago)
            am_nxt = red_amx_max();
            if (tid == 0 && u + 1 < u1) amax_out[u / 3 + 1] = am_nxt;
        }
        if (u > u0) amx_fold(u - 1);
        if (r3 == 1) {  // unit u - 1 read the next sample's last chunk: this wave's partial
            const float m = wave_max_dpp(run);
            if (lane == 0) red_amx[wave] = m;
            run = 0.f;
        }
        amx_issue(u);
    };
    // data scale: per sample (AMX: sample b is the current unit's or the next one)
    auto sexp = [&](int b) {
        if constexpr (AMX) return x3_exp(b == u / 3 ? am_cur : am_nxt);
        else return x3_exp(amax[b]);
    };

    // B fragments: lane (n16, kc) holds W2[co][8kc .. 8kc+7][tap], co = 16nt + n16
    f16x8 wh[X3F_NT][9], wl[X3F_NT][9];
    float bias[X3F_NT];
#pragma unroll
    for (int nt = 0; nt < X3F_NT; ++nt) {
        const int co = 32 * ch + 16 * nt + n16;
        bias[nt] = b2[co];
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = W2[(co * C1 + 8 * kc + j) * 9 + tap];
            x3_split8(v, wsc, wh[nt][tap], wl[nt][tap]);
        }
    }
    // A fragment bases per (mt, kx): M row m = n16 -> window wx = 4mt + (m >> 2), position q = m & 3;
    // the pixel's chunk slot is kc ^ (x & 2) (x = its column in the unit)
    int abase[3][3];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int q = n16 & 3, wx = 4 * mt + (n16 >> 2);
            const int x = 2 * wx + (q & 1) + kx;
            abase[mt][kx] = ((2 * wr + (q >> 1)) * A_HW + x) * 64 + ((kc ^ (x & 2)) * 16);
        }
    // split items: (pixel p, chunk c8) -> raw read offset, f16 write offset; threads past the last item
    // redo it (identical stores): the split has no branch and shares a basic block with the MFMAs
    int rd[X3F_IPT], wo[X3F_IPT];
#pragma unroll
    for (int it = 0; it < X3F_IPT; ++it) {
        const int i = min(tid + it * X3F_THREADS, X3F_ITEMS - 1);
        const int c8 = i / X3F_PIX, p = i - (i / X3F_PIX) * X3F_PIX;
        const int x = p % A_HW;
        rd[it] = (8 * c8 * X3F_PIX + p) * 4;
        wo[it] = p * 64 + ((c8 ^ (x & 2)) * 16);
    }
    auto split_unit = [&](int uu, const char* raw, char* buf) {
        const float sc = ldexpf(1.f, sexp(uu / 3));
#pragma unroll
        for (int it = 0; it < X3F_IPT; ++it) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const float*>(raw + rd[it] + j * X3F_PIX * 4);
            f16x8 h, l;
            x3_split8(v, sc, h, l);
            *reinterpret_cast<f16x8*>(buf + wo[it]) = h;
            *reinterpret_cast<f16x8*>(buf + X3F_PLANE + wo[it]) = l;
        }
    };

    // prologue: unit u's raw rows landed -> split into f16 buffer 0 (IN16: its image is there)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (!IN16 && u < u1) split_unit(u, raw0, smem);
    int k = 0;
    const int sph = wave >= 4 ? 0 : 1;
    // Epilogue of one (M tile, co tile) window group: the first max of the raw accumulators (the unscale
    // is monotone, so this is the max of the outputs; the index is the first-equal one up to ties that
    // only rounding creates), then unscale (exact: 2^-(s_b + sw) as pre * us, pre = 1 unless that power
    // is not a normal float) + bias + ReLU on the max alone. IN16 runs it in pieces inside the MFMA
    // stream — the previous unit's M tile 2 during M tile 0, M tile 0 during M tile 1, M tile 1 during M
    // tile 2 — so its VALU issues between MFMAs instead of after them (0.226 -> 0.218 ms interleaved
    // A/B; an epilogue after the stream with a rare-case scale branch: 0.237).
    // The pooled value + code of a lane's window in M tiles 0 and 1 are held (hm / hc) until the row's
    // tile 2 is done, then the row is stored by x3f_store_row.
    f32x4 pend[X3F_NT];
    float hm[2][X3F_NT];
    uint32_t hc[2][X3F_NT];
    size_t p_o = 0;  // output row of the pending tile 2 (window 0 of co 32 ch + n16)
    float p_pre = 1.f, p_us = 1.f;
    auto pool_piece = [&](const f32x4& a, float pre, float us, float bs, float& m, uint32_t& c) {
        float am = a[0];
        int idx = 0;
#pragma unroll
        for (int q = 1; q < 4; ++q)
            if (a[q] > am) { am = a[q]; idx = q; }
        m = fmaf(am * pre, us, bs);
        m = m > 0.f ? m : 0.f;
        c = m > 0.f ? (uint32_t)idx : (uint32_t)CODE_NONE;
    };
#pragma unroll 1
    for (; u < u1; ++u, ++k) {
        const int cb = k & 1;
        // unit u+G's raw rows (issued one unit ago) have landed; the previous epilogue's stores may stay
        // IN16: unit u's image (issued two units ago) has landed; unit u+G's DMA (at most 5 wave-
        // instructions, issued one unit ago) and the previous epilogue's stores may stay in flight
        if constexpr (IN16) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X3F_STORES + 4) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(X3F_STORES) : "memory");
        __syncthreads();
        const int kr = k % 3;  // IN16 ring slot of unit u
        if constexpr (AMX) {
            if (u - 3 * (u / 3) == 0 && u > u0) am_cur = am_nxt;

        }
        // IN16: unit u+2's image (past the range: a clamped unit into the free slot, never read) — the
        // quarters now, the 4 full pieces of each wave spread over the first MFMA steps (one burst here
        // measured 0.2456 vs 0.2336 ms, interleaved A/B)
        const char* nsrc = x3_unit_img_src(act16, min(u + 2, u1 - 1));
        const uint32_t nlds = lds_u32(smem + (kr == 0 ? 2 : kr - 1) * X3F_BUF);
        if (IN16 && wave < 2) x3_issue_img_quarter(nsrc, wave, lane, nlds);
        if constexpr (!IN16) {
            if (u + 2 < u1) x3f_issue_raw(act, u + 2, wave, lane, voff, lds_u32(raw0 + cb * X3F_RAW));
        }
        const char* cur = smem + (IN16 ? kr : cb) * X3F_BUF;
        f32x4 acc[3][X3F_NT];
        if constexpr (IN16) {
            // no staging in the loop: all 27 (M tile, tap) steps in one stream
#pragma unroll
            for (int mt = 0; mt < 3; ++mt)
#pragma unroll
                for (int nt = 0; nt < X3F_NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
            // A fragments read RA steps ahead through a ring of RA + 1 (interleaved A/B: RA = 1 0.2287 ms,
            // 2 0.2333, 3 0.2339 — the epilogue pieces and DMA pieces now fill the gaps the deeper ring hid)
            constexpr int RA = 1;
            f16x8 fh[RA + 1], fl[RA + 1];
            auto rdA = [&](int st) {
                const int mt = st / 9, tap = st % 9, ky = tap / 3, kx = tap % 3;
                fh[st % (RA + 1)] = *reinterpret_cast<const f16x8*>(cur + abase[mt][kx] + ky * A_HW * 64);
                fl[st % (RA + 1)] = *reinterpret_cast<const f16x8*>(cur + X3F_PLANE + abase[mt][kx] + ky * A_HW * 64);
            };
#pragma unroll
            for (int q = 0; q < RA; ++q) rdA(q);
            // this unit's scales and output offsets (for the pieces of its epilogue issued in-stream)
            const int b_ = u / 3, t3_ = u - (u / 3) * 3, se_ = sexp(b_) + sw;
            const float pre_ = ldexpf(1.f, min(126 - se_, 0)), us_ = ldexpf(1.f, -min(se_, 126));
            const size_t o_ = (size_t)b_ * P_SAMPLE + (32 * ch + n16) * P_WIN + (4 * t3_ + wr) * P_HW;
            if (k == 0) {  // no pending row yet: a zero row aimed at this unit's outputs (rewritten later)
#pragma unroll
                for (int nt = 0; nt < X3F_NT; ++nt) {
                    pend[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
                    hm[0][nt] = hm[1][nt] = 0.f;
                    hc[0][nt] = hc[1][nt] = 0u;
                }
                p_o = o_;
                p_pre = 1.f;
                p_us = 1.f;
            }
#pragma unroll
            for (int st = 0; st < 27; ++st) {
                if (st < 8 && (st & 1) == 0) x3_issue_img_full(nsrc, wave, lane, nlds, st >> 1);
                if (st + RA < 27) rdA(st + RA);
                const int mt = st / 9, tap = st % 9;
#pragma unroll
                for (int nt = 0; nt < X3F_NT; ++nt)
                    acc[mt][nt] = mfma_x3(fh[st % (RA + 1)], fl[st % (RA + 1)], wh[nt][tap], wl[nt][tap], acc[mt][nt]);
                if (tap == 3 || tap == 6) {
                    const int nt = tap == 3 ? 0 : 1;
                    if (mt == 0) {  // the previous unit's tile 2 completes its row
                        float m2;
                        uint32_t c2;
                        pool_piece(pend[nt], p_pre, p_us, bias[nt], m2, c2);
                        const size_t ro = p_o + nt * 16 * P_WIN;
                        x3f_store_row(hm[0][nt], hm[1][nt], m2, hc[0][nt], hc[1][nt], c2, kc, pooled + ro, code + ro);
                    } else {
                        pool_piece(acc[mt - 1][nt], pre_, us_, bias[nt], hm[mt - 1][nt], hc[mt - 1][nt]);
                    }
                }
            }
            pend[0] = acc[2][0];
            pend[1] = acc[2][1];
            p_o = o_;
            p_pre = pre_;
            p_us = us_;
            // (measured: leaving the order to the compiler beats pinning it with sched_group_barrier,
            // 0.243 vs 0.275 ms, and the pre-ring loop 0.260)
        } else
#pragma unroll
        for (int mt = 0; mt < 3; ++mt) {
#pragma unroll
            for (int nt = 0; nt < X3F_NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int ky = tap / 3, kx = tap % 3;
                const f16x8 ah = *reinterpret_cast<const f16x8*>(cur + abase[mt][kx] + ky * A_HW * 64);
                const f16x8 al = *reinterpret_cast<const f16x8*>(cur + X3F_PLANE + abase[mt][kx] + ky * A_HW * 64);
#pragma unroll
                for (int nt = 0; nt < X3F_NT; ++nt) acc[mt][nt] = mfma_x3(ah, al, wh[nt][tap], wl[nt][tap], acc[mt][nt]);
            }
            // staging after M tile 0 on waves 4-7 and after M tile 1 on waves 0-3 (waves w and w + 4
            // share a SIMD; measured: 0/1 beats 0/0 and 0/2). Past the last unit this splits a clamped
            // unit's stale raw rows into a buffer nobody reads
            if constexpr (AMX) {
                if (mt == sph) amx_step(u - 3 * (u / 3));
            }
            if (!IN16 && mt == sph) split_unit(min(u + 1, u1 - 1), raw0 + (cb ^ 1) * X3F_RAW, smem + (cb ^ 1) * X3F_BUF);
            if (!IN16 && mt == sph && act16) {
                // this unit's f16 image -> HBM for the wgrad (2,080 16-B pieces)
                // (rows 8-9 of a third are rows 0-1 of the next: both units store the same values there)
                char* dst = reinterpret_cast<char*>(act16) + (size_t)(u / 3) * X3S_SAMPLE + (u - (u / 3) * 3) * X3S_UNIT_OFF;
#pragma unroll
                for (int r = 0; r < (X3F_BUF / 16 + X3F_THREADS - 1) / X3F_THREADS; ++r) {
                    const int i = min(tid + r * X3F_THREADS, X3F_BUF / 16 - 1);
                    const int pl = i >= X3F_PLANE / 16 ? 1 : 0;
                    *reinterpret_cast<uint4*>(dst + pl * (X3S_PLANE - X3F_PLANE) + i * 16) =
                        *reinterpret_cast<const uint4*>(cur + i * 16);
                }
            }
        }
        if constexpr (!IN16) {  // epilogue after the stream (the f32-cut path stages mid-stream)
            const int b = u / 3, t3 = u - (u / 3) * 3, se = sexp(b) + sw;
            const float pre = ldexpf(1.f, min(126 - se, 0)), us = ldexpf(1.f, -min(se, 126));
            const size_t o = (size_t)b * P_SAMPLE + (32 * ch + n16) * P_WIN + (4 * t3 + wr) * P_HW;
#pragma unroll
            for (int nt = 0; nt < X3F_NT; ++nt) {
                float m[3];
                uint32_t c[3];
#pragma unroll
                for (int mt = 0; mt < 3; ++mt) pool_piece(acc[mt][nt], pre, us, bias[nt], m[mt], c[mt]);
                const size_t ro = o + nt * 16 * P_WIN;
                x3f_store_row(m[0], m[1], m[2], c[0], c[1], c[2], kc, pooled + ro, code + ro);
            }
        }
    }
    if (IN16 && k > 0) {  // the last unit's M tile 2
#pragma unroll
        for (int nt = 0; nt < X3F_NT; ++nt) {
            float m2;
            uint32_t c2;
            pool_piece(pend[nt], p_pre, p_us, bias[nt], m2, c2);
            const size_t ro = p_o + nt * 16 * P_WIN;
            x3f_store_row(hm[0][nt], hm[1][nt], m2, hc[0][nt], hc[1][nt], c2, kc, pooled + ro, code + ro);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
}

// ============================================================================ conv2 dgrad (cut gradient)
// g[ci][y][x] = sum_{co,ky,kx} W2[co][ci][ky][kx] * dY[co][y-ky][x-kx], dY = the max-pool/ReLU routing of
// dpooled by `code` (src/server_part.py:51 through model_def.py:25-27). GEMM per sample: M = output
// pixels (676 -> 43 tiles of 16 consecutive linear pixels p = 26y + x, so a lane's 4 accumulators are 4
// consecutive pixels = one float4 store), N = 32 ci, K = 64 co x 9 taps (K-step = 32 co of one tap).
// Unit = (sample, pixel part pt (tiles 0-14 / 15-28 / 29-42), co half h): the routed dY rows the part's
// taps reach are expanded into an LDS image with row stride 26: dY(Y, X) at image pixel
// 2 + 26 (Y - Ybase) + X, columns 24-25 and the 2 leading pixels zero (written once) — the 24-wide dY in
// the 26-wide grid carries exactly the 2-column halo a 3x3 tap needs, so tap (ky, kx) of output pixel p
// reads image pixel p + 2 - 26 Ybase - 26 ky - kx: a per-tile base + an immediate. Pixel records are
// [4 h chunks | 4 l chunks | 32 B pad] = 160 B: conflict-free ds_read_b128 for every tap (64-B records
// are 2-way). Images are double-buffered (2 x 58.6 KB): unit u+1's pooled gradient + codes are loaded to
// registers at the top of unit u and routed / split / stored into the other image mid-unit (items
// (window, 4 co), co group fastest across lanes: the ds_write_b64 of 16 lanes cover 128 distinct
// bytes); one barrier per unit. 8 waves: wave = (ci tile nt, tile group g: tiles T0 + g + 4i); its weight
// fragments for both co halves (2 x 9 x (h, l) = 144 VGPRs) stay in registers, its <= 4 accumulators live
// across the part's two co halves.
// ReLU bitmap of the cut (written by conv1_fwd_x3_kernel, layout there): u32 words per (ci, u), per sample
#ifndef SLK_X3W_ROUND4
#define SLK_X3W_ROUND4 0
#endif
#ifndef SLK_X3W_SPARSE
#define SLK_X3W_SPARSE 1
#endif
constexpr int RB_SAMPLE = 4 * (A_PIX / 4);  // 676 u32 = 2,704 B per sample: [channel group 4][169]
constexpr int X3D_THREADS = 512;
constexpr int X3D_REC = 160;                       // bytes per image pixel: h 64 | l 64 | pad 32
constexpr int X3D_NRMAX = 14;                      // image rows (dY rows) of the largest part
constexpr int X3D_PIX = 2 + X3D_NRMAX * A_HW;      // 366 image pixels
constexpr int X3D_IMG = X3D_PIX * X3D_REC;         // 58,560 B
constexpr int X3D_MT = 43;                         // M tiles per sample
constexpr int X3D_MPW = 4;                         // M tiles per wave and part (max)
constexpr int X3D_GRID = 256;
constexpr int X3D_ITEMS_MAX = 7 * P_HW * 8;        // (window, 4-co group) items of the largest part (672)
static_assert(2 * X3D_IMG <= 163840, "LDS");
#ifndef SLK_X3D_TRACE
#define SLK_X3D_TRACE 0
#endif
// the fused dgrad's client epilogue on the f16 MFMA (split operands) instead of the f32 MFMA
#ifndef SLK_X3D_EPI16
#define SLK_X3D_EPI16 0
#endif
// profiling only (wrong results): bit 1 no dY staging, bit 2 no client epilogue, bit 4 its f32 MFMAs as one fma,
// bit 8 no dY global loads (the staging stores kept)
#ifndef SLK_X3D_ABL
#define SLK_X3D_ABL 0
#endif
#if SLK_X3D_TRACE
// profiling probe: per (workgroup, wave, unit) shader-clock stamps of the dgrad's phases (lane 0, vector stores)
__device__ unsigned long long g_x3d_trace[256 * 8 * 128 * 8];
#define X3_TS(buf, u, slot)                                                                                 \
    do {                                                                                                   \
        unsigned long long _t;                                                                             \
        asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                          \
        if (lane == 0 && (u) < 128) buf[(((size_t)blockIdx.x * 8 + wave) * 128 + (u)) * 8 + (slot)] = _t;  \
    } while (0)
#define X3D_TS(u, slot) X3_TS(g_x3d_trace, u, slot)
#define X3Q_TS(u, slot) X3_TS(g_x3q_trace, u, slot)
__device__ unsigned long long g_x3q_trace[256 * 8 * 128 * 8];
extern "C" int slk_x3q_trace_read(void* dst) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_x3q_trace), sizeof(g_x3q_trace)) == hipSuccess ? 0 : 1;
}
extern "C" int slk_x3d_trace_read(void* dst) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_x3d_trace), sizeof(g_x3d_trace)) == hipSuccess ? 0 : 1;
}
#else
#define X3D_TS(u, slot)
#define X3Q_TS(u, slot)
#endif

__device__ __forceinline__ int x3d_t0(int pt) { return pt == 0 ? 0 : (pt == 1 ? 15 : 29); }
__device__ __forceinline__ int x3d_ybase(int pt) { return pt == 0 ? -2 : (pt == 1 ? 6 : 14); }
__device__ __forceinline__ int x3d_nwr(int pt) { return pt == 2 ? 7 : 6; }  // image window rows

// Accumulation: per (tile, unit) the hi*hi products go into the tile's accumulator and the two cross
// products (hi*lo, lo*hi) into a separate chain started from zero, added to the accumulator by one f32
// add at the end of the tile's 9 taps. The f16 MFMA's internal alignment truncates (toward -inf) at the
// unit of its largest addend; cross products added straight onto the large accumulator lost their low
// bits there, a bias of ~-1.5e-8 of sum |a b| per output that the client gradient (a sum over 2.8 M cut
// elements) turned into ~1e-6 of db1 (tools/ubench/x3_bias.hip: 17x less bias this way).
// C1W = true (the fused single-GPU step): the cut gradient is not stored; the epilogue applies the
// client's ReLU mask (the 1-bit map conv1_fwd_x3 wrote) and accumulates the conv1 weight gradient
// dW1[ci][tap] = sum_p g[ci][p] x[p + tap], db1[ci] = sum_p g[ci][p] as a GEMM on the f32 MFMA
// (v_mfma_f32_16x16x4_f32, an exact fmaf chain): A = the masked, unscaled accumulators as they sit in
// the lanes (row = ci, k = the lane's 4-pixel group), B = x at each lane's (pixel, tap) (col = tap 0-8,
// 9 = bias -> 1.0), one 16 ci x 16 col accumulator per wave for the whole launch; each workgroup writes
// one 320-float client slab (src/client_part.py:132 — the client's act.backward(cut_grad) without the
// cut gradient ever reaching HBM). x and the bit map of the next pair are loaded a unit ahead into LDS.
// PACK (C1W = false, pvals != nullptr): the cut gradient leaves in the codec's packed form (slk_codec.hip)
// instead of dense: only the elements set in the received cut's mask, each at its rank (pranks[e / 32] +
// the set bits of its word below it) — what slk_cut_pack would extract from the dense gradient, without
// the 354 MB (B = 4096) dense write and re-read. Sample 0 of the launch is element 0 of the mask.
template <bool C1W>
__global__ __launch_bounds__(X3D_THREADS, 1) void conv2_dgrad_x3_kernel(
    const float* __restrict__ dpooled, const float* __restrict__ amax, const uint8_t* __restrict__ code,
    const float* __restrict__ W2, float* __restrict__ cut_grad, int B, const float* __restrict__ xin = nullptr,
    const uint32_t* __restrict__ relu_bits = nullptr, float* __restrict__ c1slabs = nullptr,
    const uint32_t* __restrict__ pmask = nullptr, const int* __restrict__ pranks = nullptr,
    float* __restrict__ pvals = nullptr, const uint64_t* __restrict__ pparts = nullptr, int ppart_b = 0) {
    __shared__ __attribute__((aligned(1024))) char smem[2 * X3D_IMG];
    // C1W: per pair, x (3,136 B), a second copy of x, then its ReLU bits (2,704 B), double-buffered
    // (XB_BYTES apart, a multiple of 128 B), moved by LDS-DMA; after both buffers the plane of ones (below).
    // The epilogue's x reads (ds_read2_b32: banks = dword % 32 over 32-lane halves) of lane groups kc and
    // kc + 1 collided 2-way (taps 28-30 / 56-58 dwords over the other's 0-2 / 24-26 after the +4 pixel
    // shift); odd kc reads the copy, 812 dwords (12 banks) further, and the ones plane sits 7 banks off
    // both x planes (at 0 its lanes collided with tap 0's): 680 -> 4 modelled conflict cycles per sample
    // and co tile (the guide's LDS bank table over every tile, tap and row-crossing case; a copy 16 banks
    // over left 54, the row-crossing groups)
    constexpr int XB_X = IN_HW * IN_HW * 4, XB_COPY = XB_X + 112, XB_BITS = XB_COPY + XB_X, XB_ONES = 28;
    constexpr int XB_BYTES = (XB_BITS + RB_SAMPLE * 4 + 127) / 128 * 128;
    static_assert(XB_X > 3072 && XB_X <= 4096 && XB_X % 16 == 0 && RB_SAMPLE * 4 > 2048 && RB_SAMPLE * 4 <= 3072 &&
                  RB_SAMPLE % 4 == 0 && XB_COPY % 16 == 0 && XB_BITS % 16 == 0, "DMA pieces of issue_xb");
    static_assert((XB_COPY / 4) % 32 == 12 && XB_BYTES % 128 == 0, "x copy 12 banks over");
    // PACK (C1W = false): per pair, the mask words and word ranks its epilogue needs — [ci 32][PKW words] of
    // each, from the pair's first pixel — double-buffered like C1W's x / bits (2 x 2,560 B)
    constexpr int PKW = 10, PK_BYTES = 2 * C1 * PKW * 4;
    __shared__ __attribute__((aligned(1024))) char xbm[C1W ? 2 * XB_BYTES + 32 + XB_X : 2 * PK_BYTES];
    // C1W: each wave's conv1-gradient accumulator D1[ci 16 nt + 4 (lane >> 4) + r][col lane & 15] (col =
    // tap 0-8, 9 = bias), kept here between epilogues (not in the MFMA loop's registers)
    __shared__ __attribute__((aligned(16))) f32x4 d1s[C1W ? X3D_THREADS : 1];
    // C1W: an x-shaped plane of 1.0 that the bias column's lanes (col 9) read in place of x, so the B
    // operand needs no per-element select (cols 10-15 read x: their D1 columns are never stored); 4 banks
    // off both x planes (above)
    float* const ones = reinterpret_cast<float*>(xbm + (C1W ? 2 * XB_BYTES + XB_ONES : 0));
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nt = wave & 1, g = wave >> 1;
    const int n16 = lane & 15, kc = lane >> 4;
    const int G = gridDim.x;
    X3D_TS(0, 7);

    // zero both images once: the leading pixels and columns 24-25 are never written again
    for (int o = tid * 16; o < 2 * X3D_IMG; o += X3D_THREADS * 16) *reinterpret_cast<uint4*>(smem + o) = make_uint4(0, 0, 0, 0);

    // weight scale (max |W2|), reduced through the tail of image 1 (outside every image pixel's h|l)
    float* red = reinterpret_cast<float*>(smem + X3D_IMG + 128);  // pixel 0's pad is never read
    float wm = 0.f;
    for (int e = tid; e < W2_N; e += X3D_THREADS) wm = fmaxf(wm, fabsf(W2[e]));
    wm = wave_max(wm);
    __syncthreads();  // zeroing done before red[] is written into image 1
    if (lane == 0) red[wave] = wm;
    __syncthreads();
    wm = red[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) wm = fmaxf(wm, red[i]);
    __syncthreads();
    if (tid < 8) red[tid] = 0.f;  // restore the zero image
    const int sw = x3_exp(wm);
    const float wsc = ldexpf(1.f, sw);
    // B fragments: lane (n16, kc) holds W2[32h + 8kc + j][ci][tap], ci = 16nt + n16
    f16x8 wh[2][9], wl[2][9];
    {
        const int ci = 16 * nt + n16;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = W2[((32 * h + 8 * kc + j) * C1 + ci) * 9 + tap];
                x3_split8(v, wsc, wh[h][tap], wl[h][tap]);
            }
    }

    X3D_TS(1, 7);
    // expansion items of a unit: i = tid + 512 r -> 4-co group c4 = i & 7, window wi = i >> 3 (row-major
    // over the part's image window rows); rows outside 0..11 expand to zeros
    constexpr int NR = 2, SSTR = X3D_THREADS;
    static_assert(NR * SSTR >= X3D_ITEMS_MAX, "staging items");
    const int stid = tid;
    float dv[NR][4];
    uint32_t dcb[NR][4];
    float ld_amax = 0.f;
    auto load_dy = [&](int uu) {
        const int b = uu / 6, rr = uu - (uu / 6) * 6, pt = rr >> 1, h = rr & 1;
        ld_amax = amax[b];  // used by the store_dy of this unit (one unit later)
        const int wr0 = x3d_ybase(pt) / 2, nwr = x3d_nwr(pt);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int i = stid + r * SSTR;
            const int c4 = i & 7, wi = i >> 3;
            const int wr = wr0 + wi / P_HW, wx = wi - (wi / P_HW) * P_HW;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                dv[r][j] = 0.f;
                dcb[r][j] = CODE_NONE;  // routes nothing
            }
            if (i < nwr * P_HW * 8 && wr >= 0 && wr < P_HW) {
                const size_t o = (size_t)b * P_SAMPLE + (32 * h + 4 * c4) * P_WIN + wr * P_HW + wx;
                // code bytes stay one per register until store_dy: combining them here made the
                // compiler wait for the loads on the spot (a full memory latency per unit)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
#if SLK_X3D_ABL & 8
                    dv[r][j] = (float)((o + j) & 255) * 1e-3f;  // no global loads
                    dcb[r][j] = (uint32_t)(o + j) & 3u;
#else
                    dv[r][j] = dpooled[o + j * P_WIN];
                    dcb[r][j] = code[o + j * P_WIN];
#endif
                }
            }
        }
    };
    auto store_dy = [&](int uu, char* img) {
        const int pt = (uu - (uu / 6) * 6) >> 1;
        const int nwr = x3d_nwr(pt);
        const float sc = ldexpf(1.f, x3_exp(ld_amax));
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int i = stid + r * SSTR;
            if (r == 0 || i < nwr * P_HW * 8) {
                const int c4 = i & 7, wi = i >> 3;
                const int wrl = wi / P_HW, wx = wi - (wi / P_HW) * P_HW;
                uint32_t hv[2], lv[2];
#pragma unroll
                for (int j = 0; j < 4; j += 2) {
                    const float a = dv[r][j] * sc, c = dv[r][j + 1] * sc;
                    const _Float16 ha = (_Float16)a, hc = (_Float16)c;
                    const _Float16 la = (_Float16)(a - (float)ha), lc = (_Float16)(c - (float)hc);
                    hv[j / 2] = __builtin_bit_cast(uint32_t, f16x2{ha, hc});
                    lv[j / 2] = __builtin_bit_cast(uint32_t, f16x2{la, lc});
                }
                const uint32_t dcw = dcb[r][0] | (dcb[r][1] << 8) | (dcb[r][2] << 16) | (dcb[r][3] << 24);
                const uint32_t cA = __builtin_amdgcn_perm(0u, dcw, 0x01010000u), cB = __builtin_amdgcn_perm(0u, dcw, 0x03030202u);
                char* rec = img + (2 + (2 * wrl) * A_HW + 2 * wx) * X3D_REC + c4 * 8;
#pragma unroll
                for (int pos = 0; pos < 4; ++pos) {
                    const uint32_t T = 0xFFu << (8 * pos);
                    const uint32_t mA = __builtin_amdgcn_perm(0u, T, cA), mB = __builtin_amdgcn_perm(0u, T, cB);
                    char* o = rec + ((pos >> 1) * A_HW + (pos & 1)) * X3D_REC;
                    *reinterpret_cast<uint2*>(o) = make_uint2(hv[0] & mA, hv[1] & mB);
                    *reinterpret_cast<uint2*>(o + 64) = make_uint2(lv[0] & mA, lv[1] & mB);
                }
            }
        }
    };

    f32x4 acc[X3D_MPW];
    // a workgroup walks PAIRS (pair = (sample, part); unit index = 2 * pair + h: the two co halves of a
    // part are consecutive for the accumulators) over a CONTIGUOUS range, so the three parts of a sample
    // run back to back on one CU: the dpooled window rows that neighbouring parts share (19 rows read
    // per 12) and the sample's x / bit map come from that XCD's L2 the second time (a stride of G put
    // them on different XCDs: HBM re-reads)
    const int P = 3 * B;  // pairs
    const int per = (P + G - 1) / G;
    const int p0 = min((int)blockIdx.x * per, P), p1 = min(p0 + per, P);
    int pr = p0;
    // pair pp's x, x copy and bits -> buffer buf: waves 0-3 move x, waves 4-7 its copy (3 x 1 KiB + 64 B
    // each), waves 0-2 the bits (2 x 1 KiB + 656 B), one 16-B piece per lane (retired by the s_waitcnt before
    // the barrier that opens the next pair)
    auto issue_xb = [&](int pp, int buf) {
        const size_t b = (size_t)(pp / 3);
        const uint32_t dst = lds_u32(xbm) + buf * XB_BYTES;
        const int w4 = wave & 3;
        if (w4 < 3 || lane < (XB_X % 1024) / 16)
            glds16_so(reinterpret_cast<const char*>(xin + b * IN_HW * IN_HW) + w4 * 1024, (uint32_t)lane * 16,
                      dst + (wave >= 4 ? XB_COPY : 0) + w4 * 1024);
        if (wave < 2 || (wave == 2 && lane < (RB_SAMPLE * 4 - 2048) / 16))
            glds16_so(reinterpret_cast<const char*>(relu_bits + b * RB_SAMPLE) + wave * 1024, (uint32_t)lane * 16,
                      dst + XB_BITS + wave * 1024);
    };
    // PACK: sample bb's (mask, ranks, vals) and its index within them (pparts: its part's, else the launch's)
    const bool pack = !C1W && (pvals != nullptr || pparts != nullptr);
    auto pack_ptrs = [&](int bb, const uint32_t*& mk, const int*& rk, float*& vl, int& lb, int& nsb) {
        mk = pmask;
        rk = pranks;
        vl = pvals;
        lb = bb;
        nsb = B;
        if (pparts != nullptr) {
            const int part = bb / ppart_b;
            lb = bb - part * ppart_b;
            nsb = ppart_b;
            mk = reinterpret_cast<const uint32_t*>(pparts[3 * part]);
            rk = reinterpret_cast<const int*>(pparts[3 * part + 1]);
            vl = reinterpret_cast<float*>(pparts[3 * part + 2]);
        }
    };
    // PACK: pair pp's words -> buffer buf: 640 words (mask then ranks, [ci][PKW] each) in 10 glds4 pieces of 64
    // lanes (waves 0-7 one each, waves 0-1 a second); words past the part's last read its last word (unused)
    auto issue_pk = [&](int pp, int buf) {
        const int bb = pp / 3, pt = pp - (pp / 3) * 3;
        const uint32_t* mk;
        const int* rk;
        float* vl;
        int lb, nsb;
        pack_ptrs(bb, mk, rk, vl, lb, nsb);
        const int q0 = 16 * x3d_t0(pt);
        const uint32_t dst = lds_u32(xbm) + buf * PK_BYTES;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int piece = wave + 8 * r;
            if (piece < 2 * C1 * PKW / 64) {
                const int idx = piece * 64 + lane, arr = idx >= C1 * PKW ? 1 : 0, j = idx - arr * C1 * PKW;
                const int ci = j / PKW, jj = j - (j / PKW) * PKW;
                const int w = min(((((lb * C1 + ci) * A_PIX) + q0) >> 5) + jj, nsb * (A_SAMPLE / 32) - 1);
                glds4(arr ? reinterpret_cast<const void*>(rk + w) : reinterpret_cast<const void*>(mk + w),
                      dst + piece * 256);
            }
        }
    };
    if (pack && pr < p1) issue_pk(pr, 0);
    if constexpr (C1W) {
        d1s[tid] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int e = tid; e < IN_HW * IN_HW; e += X3D_THREADS) ones[e] = 1.f;
        if (pr < p1) issue_xb(pr, 0);
    }
    if (pr < p1) {
        load_dy(2 * pr);
        __syncthreads();  // zeroing / red restore done before the first expansion
        store_dy(2 * pr, smem);
        load_dy(2 * pr + 1);
    }
    int k = 0, q = 0;
    X3D_TS(2, 7);
    // C1W epilogue of one pair: client ReLU backward + conv1 wgrad (the cut gradient g is the value the
    // C1W = false store would write): for each tile and r, one f32 MFMA over k = the 4 lane groups' pixels
    // 16 t + 4 kc + r. All of the pair's x / bit-map reads are issued first; the ReLU mask is an integer
    // AND of the accumulator bits (no compare/select/multiply per element); the 16 MFMAs run as 4
    // independent chains (one per r; one dependent chain exposed the MFMA latency 16 times) started
    // from zero per pair, and the per-sample unscale 2^-s_b is applied once to their sum (exact: a power
    // of two), which is then added to the wave's launch-long accumulator.
    auto c1w_epi = [&](int T0e, int T1e, float us1e, int qe) {
        const int ci = 16 * nt + n16;
        // B operand of the conv1-gradient GEMM: lane col n16 = tap (ky, kx) reads x at pixel offset toff;
        // the bias col 9 reads the ones plane; cols 10-15 read x (their D1 columns are never stored)
        const char* xbb = xbm + (qe & 1) * XB_BYTES;
        const float* xs = n16 == 9 ? ones : reinterpret_cast<const float*>(xbb + ((kc & 1) ? XB_COPY : 0));
        const uint32_t* bs = reinterpret_cast<const uint32_t*>(xbb + XB_BITS);
        const int toff = n16 < 9 ? (n16 / 3) * IN_HW + n16 % 3 : 0;
        const bool t3 = T0e + g + 12 < T1e;  // wave-uniform: tiles 0-2 exist for every wave and part
        uint32_t mw[X3D_MPW];
        float xv[X3D_MPW][4];
        // x index of pixel p = 26 y + x is p + 2 y. The lane's 4-pixel group of tile i starts at
        // p0 = 16 (T0e + g) + 4 kc + 64 i; p0 % 26 (rem) is even, so the group crosses a row end only when
        // rem == 24, between r = 1 and r = 2: two bases per tile, immediate offsets for r, and (y, rem)
        // advanced per tile (+64 = 2 rows + 12) instead of a division per pixel
        const float* xl = xs + toff;
        int p0 = 16 * (T0e + g) + 4 * kc;
        int y0 = p0 / A_HW, rem = p0 - A_HW * y0;
#pragma unroll
        for (int i = 0; i < X3D_MPW; ++i) {
            const int tq = (p0 >> 2);  // conv1_fwd_x3's thread of these 4 pixels (= 4 t + kc)
            // pixels past 675 (tile 42's tail) and a missing tile 3: any valid pixel, mask 0 below
            const bool ok = tq < A_PIX / 4;
            const int base = ok ? p0 + 2 * y0 : 0;
            const int cross = (ok && rem == 24) ? 2 : 0;
            xv[i][0] = xl[base];
            xv[i][1] = xl[base + 1];
            xv[i][2] = xl[base + cross + 2];
            xv[i][3] = xl[base + cross + 3];
            const uint32_t mraw = bs[(ci >> 3) * (A_PIX / 4) + min(tq, A_PIX / 4 - 1)];
            mw[i] = (ok && (i < 3 || t3)) ? mraw >> (4 * (ci & 7)) : 0u;
            p0 += 64;
            rem += 12;
            y0 += 2;
            if (rem >= A_HW) {
                rem -= A_HW;
                ++y0;
            }
        }
#if SLK_X3D_EPI16
        // the same GEMM on the f16 MFMA: g (scaled by 2^-22: |g| < 576 * 2^28 before it, so hi < 36,864)
        // and x split hi/lo, K = the lane group's 8 (tile, r) pixels per instruction, 2 hi*hi + 4 cross
        // products in two chains from zero per pair (the accumulation-bias note above)
        f16x8 gh[2], gl[2], bh[2], bl[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            float gv[8], xw[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i = 2 * s + (j >> 2), r = j & 3;
                gv[j] = __uint_as_float(__float_as_uint(acc[i][r]) & (0u - ((mw[i] >> r) & 1u)));
                xw[j] = xv[i][r];
            }
            x3_split8(gv, 0x1p-22f, gh[s], gl[s]);
            x3_split8(xw, 1.f, bh[s], bl[s]);
        }
        f32x4 dh = f32x4{0.f, 0.f, 0.f, 0.f}, dc = f32x4{0.f, 0.f, 0.f, 0.f};
        slk_keep(dh);
        slk_keep(dc);
        dh = mfma_f16(gh[0], bh[0], dh);
        dc = mfma_f16(gh[0], bl[0], dc);
        dh = mfma_f16(gh[1], bh[1], dh);
        dc = mfma_f16(gl[0], bh[0], dc);
        dc = mfma_f16(gh[1], bl[1], dc);
        dc = mfma_f16(gl[1], bh[1], dc);
        d1s[tid] = d1s[tid] + (dh + dc) * (us1e * 0x1p22f);
        return;
#endif
        f32x4 dr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            dr[r] = f32x4{0.f, 0.f, 0.f, 0.f};
            slk_keep(dr[r]);  // zero chains in VGPRs, not an inline-constant C
        }
#pragma unroll
        for (int i = 0; i < X3D_MPW; ++i) {
            if (i < 3 || t3) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    // g * 2^(s_b + sw) where the client's ReLU passes, +0 elsewhere (AND with 0 / ~0)
                    const uint32_t keep = 0u - ((mw[i] >> r) & 1u);
                    // (by value: __builtin_bit_cast of the vector element acc[i][r] read one element for all r)
                    const float gm = __uint_as_float(__float_as_uint(acc[i][r]) & keep);
#if SLK_X3D_ABL & 4
                    dr[r][0] = fmaf(gm, xv[i][r], dr[r][0]);
#else
                    dr[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(gm, xv[i][r], dr[r], 0, 0, 0);
#endif
                }
            }
        }
        // the weight scale's 2^-sw is applied once to the slab (exact either way)
        d1s[tid] = d1s[tid] + ((dr[0] + dr[1]) + (dr[2] + dr[3])) * us1e;
    };
#pragma unroll 1
    for (; pr < p1; ++pr) {
        const int b = pr / 3, pt = pr - (pr / 3) * 3;
        const int T0 = x3d_t0(pt), T1 = pt == 2 ? X3D_MT : x3d_t0(pt + 1);
        const float amax_b = amax[b];  // for the epilogue, loaded early
        const int cbase = (2 - A_HW * x3d_ybase(pt) - 54) * X3D_REC;
#pragma unroll
        for (int i = 0; i < X3D_MPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int h = 0; h < 2; ++h, ++k) {
            // C1W: this pair's x / bits DMA (issued during the previous pair) retired before the barrier.
            // PACK: the next pair's words (issued at this pair's top) retired at its second unit's top, so
            // the previous epilogue's scattered stores drain during the first unit instead of being waited
            // for here (0.322 -> 0.305 ms at B = 4096, x3_ab dgp; the dense dgrad 0.255)
            X3D_TS(k, 6);
            if ((C1W && h == 0) || (pack && h == 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();  // image k&1 complete; image (k+1)&1 free
            X3D_TS(k, 0);
            // C1W: the next pair's x / bits into the other buffer (last read by the previous epilogue). The
            // staging-first waves issue it after their staging: hipcc cannot see the asm DMA, and its vmcnt(0)
            // for the dY registers would wait for the DMA just issued (a full memory latency per pair)
            const bool sfirst = wave >= 4;
            if (C1W && h == 0) issue_xb(min(pr + 1, p1 - 1), (q + 1) & 1);
            if (pack && h == 0) issue_pk(min(pr + 1, p1 - 1), (q + 1) & 1);
            const char* img = smem + (k & 1) * X3D_IMG;
            char* nimg = smem + ((k & 1) ^ 1) * X3D_IMG;
            const int unx = min(h ? 2 * (pr + 1) : 2 * pr + 1, 2 * p1 - 1);   // the unit after this one
            const int unx2 = min(h ? 2 * (pr + 1) + 1 : 2 * (pr + 1), 2 * p1 - 1);  // and the one after that
            // A fragments of (tile i, tap) through a 4-slot ring, read 3 steps ahead of their MFMAs (one
            // read pair per 3 dependent MFMAs: waiting on each read left the SIMD half idle)
            const char* abw = img + cbase + ((T0 + g) * 16 + n16) * X3D_REC + kc * 16;
            auto rd = [&](int i, int tap, f16x8& fh, f16x8& fl) {
                const char* ab = abw + i * 64 * X3D_REC + (54 - 26 * (tap / 3) - tap % 3) * X3D_REC;
                fh = *reinterpret_cast<const f16x8*>(ab);
                fl = *reinterpret_cast<const f16x8*>(ab + 64);
            };
            // the next unit's dY (always: past the last unit it stages a clamped valid unit, unused).
            // Half the waves stage before their MFMAs, half after, so the two waves of a SIMD overlap
            // one's staging with the other's MFMAs (both staging at once left the SIMD's MFMA idle).
            if (sfirst && !(SLK_X3D_ABL & 1)) {
                store_dy(unx, nimg);
                load_dy(unx2);
            }
            X3D_TS(k, 1);
            f16x8 fh[4], fl[4];
            f32x4 ct;  // cross products of the current tile (see the accumulation note above)
            constexpr int NS = 27;  // tiles 0..2 exist for every wave and part
#pragma unroll
            for (int q = 0; q < 3; ++q) rd(q / 9, q % 9, fh[q], fl[q]);
#pragma unroll
            for (int st = 0; st < NS; ++st) {
                if (st + 3 < NS) rd((st + 3) / 9, (st + 3) % 9, fh[(st + 3) & 3], fl[(st + 3) & 3]);
                const int i = st / 9, tap = st % 9;
                acc[i] = mfma_f16(fh[st & 3], wh[h][tap], acc[i]);
                ct = mfma_f16(fh[st & 3], wl[h][tap], tap == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : ct);
                ct = mfma_f16(fl[st & 3], wh[h][tap], ct);
                if (tap == 8) acc[i] += ct;
            }
            // hold the schedule to that order (hipcc otherwise sinks every read next to its MFMAs)
            __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
            for (int st = 0; st < NS; ++st) {
                __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
                if (st + 3 < NS) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            }
            X3D_TS(k, 2);
            if (!sfirst && !(SLK_X3D_ABL & 1)) {
                store_dy(unx, nimg);
                load_dy(unx2);
            }
            X3D_TS(k, 3);
            if (T0 + g + 12 < T1) {
#pragma unroll
                for (int q = 0; q < 3; ++q) rd(3, q, fh[q], fl[q]);
#pragma unroll
                for (int tap = 0; tap < 9; ++tap) {
                    if (tap + 3 < 9) rd(3, tap + 3, fh[(tap + 3) & 3], fl[(tap + 3) & 3]);
                    acc[3] = mfma_f16(fh[tap & 3], wh[h][tap], acc[3]);
                    ct = mfma_f16(fh[tap & 3], wl[h][tap], tap == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : ct);
                    ct = mfma_f16(fl[tap & 3], wh[h][tap], ct);
                }
                acc[3] += ct;
                __builtin_amdgcn_sched_group_barrier(0x100, 6, 1);
#pragma unroll
                for (int tap = 0; tap < 9; ++tap) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 3, 1);
                    if (tap + 3 < 9) __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
                }
            }
            X3D_TS(k, 4);
        }
        // epilogue: unscale (exact) and store 4 consecutive pixels per lane
        const float us1 = ldexpf(1.f, -x3_exp(amax_b)), us2 = ldexpf(1.f, -sw);
        if constexpr (C1W) {
            if (!(SLK_X3D_ABL & 2)) c1w_epi(T0, T1, us1, q);
            else {
#pragma unroll
                for (int i = 0; i < X3D_MPW; ++i) slk_keep(acc[i]);  // the MFMA stream stays live
            }
            X3D_TS(k - 1, 5);
        } else if (pack) {
            // the lane's 4 pixels are 4 consecutive elements of one mask word (A_PIX and p are multiples of 4);
            // the word and its rank come from this pair's LDS copy (issue_pk, one pair ahead). (Tried: the
            // pair's runs assembled in LDS and written by coalesced stores at the next pair's top, 0.335 vs
            // 0.312 ms: the LDS round trip cost more than the scattered 4-B stores it replaced.)
            const uint32_t* mk;
            const int* rk;
            float* pvals_;
            int lb, nsb;
            pack_ptrs(b, mk, rk, pvals_, lb, nsb);
            const int ci = 16 * nt + n16;
            const uint32_t* smk = reinterpret_cast<const uint32_t*>(xbm + (q & 1) * PK_BYTES) + ci * PKW;
            const int* srk = reinterpret_cast<const int*>(xbm + (q & 1) * PK_BYTES) + C1 * PKW + ci * PKW;
            const int e0 = (lb * C1 + ci) * A_PIX, wst = (e0 + 16 * T0) >> 5;
#pragma unroll
            for (int i = 0; i < X3D_MPW; ++i) {
                const int t = T0 + g + 4 * i, p = 16 * t + 4 * kc;
                if (t < T1 && p < A_PIX) {
                    const int e = e0 + p, jj = (e >> 5) - wst;
                    const int bit = e & 31;
                    const uint32_t m = smk[jj];
                    int r = srk[jj] + __popc(m & ((1u << bit) - 1u));
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr)
                        if ((m >> (bit + rr)) & 1u) pvals_[r++] = x3_unscale(acc[i][rr], us1, us2);
                }
            }
        } else {
            float* gb = cut_grad + (size_t)b * A_SAMPLE + (16 * nt + n16) * A_PIX;
#pragma unroll
            for (int i = 0; i < X3D_MPW; ++i) {
                const int t = T0 + g + 4 * i, p = 16 * t + 4 * kc;
                if (t < T1 && p < A_PIX)
                    *reinterpret_cast<float4*>(gb + p) =
                        make_float4(x3_unscale(acc[i][0], us1, us2), x3_unscale(acc[i][1], us1, us2),
                                    x3_unscale(acc[i][2], us1, us2), x3_unscale(acc[i][3], us1, us2));
            }
        }
        ++q;
    }
    X3D_TS(127, 7);
    if constexpr (C1W) {
        // slab of this workgroup: D1 of the 4 tile-group waves of each ci tile, summed in wave order
        __syncthreads();
        const float* part = reinterpret_cast<const float*>(d1s);  // [wave][lane][4]
        if (tid < C1 * 10) {
            const int ci = tid / 10, j = tid - (tid / 10) * 10;
            const int ntc = ci >> 4, cl = ci & 15;  // D1 row cl = 4 (lane >> 4) + r, col j = lane & 15
            const int src = ((cl >> 2) * 16 + j) * 4 + (cl & 3);
            float sum = 0.f;
            for (int gg = 0; gg < 4; ++gg) sum += part[(ntc + 2 * gg) * 256 + src];
            c1slabs[(size_t)blockIdx.x * (C1 * 10) + (j < 9 ? ci * 9 + j : C1 * 9 + ci)] = sum * ldexpf(1.f, -sw);
        }
    }
}

// ============================================================================ conv2 wgrad (dW2, db2)
// dW2[co][ci][ky][kx] = sum_{b,y,x<24} dY[b][co][y][x] * act[b][ci][y+ky][x+kx], db2[co] = sum dY
// (src/server_part.py:51). GEMM: M = co, N = (tap, ci), K = output pixels of the whole batch. Both
// operands need 8 consecutive PIXELS per lane, so both LDS images store pixels as rows with the
// channels contiguous and are read with ds_read_b64_tr_b16 (one 4-pixel x 16-channel block per 16-lane
// group, delivered column-major): dY image [192 q = 24 y_l + x][32 co], input image [260 px][32 ci], f16
// (h, l) planes. Unit = (sample, third): output rows 8t..8t+7 (K = 192 = 6 K-steps, no padding);
// a K-chunk of 8 pixels = one 8-column segment of one output row (the two 16-lane groups of a half-wave
// on adjacent rows, see abase below), so the input pixel of tap (ky, kx) is a per-(K-step, lane) base +
// an immediate. dY pixel rows keep the two 32-B co tiles swapped on odd 8-pixel groups (the two 16-lane
// groups of a half-wave then hit disjoint banks).
// A workgroup owns one co half (M = 32) and a K share (a contiguous range of units); the two co halves
// of a share run on different workgroups, each splitting the same input rows. A K sum spans samples,
// so every product must carry ONE scale: the input keeps its sample's 2^s_b (the act16 images' scale)
// and the sample's dY takes 2^(sd + sx - s_b) (sx, sd: the launch scales from the maxima of the
// per-sample amax arrays; s_b >= sx, so dY never exceeds its launch range). Staging is register-based and two
// units ahead: unit u+2's input (8 channels of a pixel per item, channel group fastest across lanes so
// the ds_write_b128 of 8 lanes cover 128 distinct bytes) and pooled gradient + codes are loaded at the
// top of unit u and split / routed into the other image at the top of unit u+1.
// 8 waves: wave = (ci half h, K-step parity kp, tap group tg) over BOTH M tiles, so each input fragment
// read feeds 6 MFMAs; parities are summed through LDS at the end. db is summed in f32 from the pooled
// gradients as they are staged (the dY images carry per-sample scales, so a ones-fragment MFMA would
// mix them).
constexpr int X3W_THREADS = 512;
constexpr int X3W_Q = 192;                           // output pixels (K) per unit
constexpr int X3W_DYP = X3W_Q * 64;                  // 12,288 B per dY plane (32 co)
constexpr int X3W_XP = 260 * 64;                     // 16,640 B per input plane (32 ci)
constexpr int X3W_BUF = 2 * X3W_DYP + 2 * X3W_XP;    // 57,856 B per buffer
constexpr int X3W_NKS = 128;                         // K shares (slabs)
constexpr int X3W_XITEMS = 260 * 4;                  // (pixel, 8-channel group) input items per unit
constexpr int X3W_XR = (X3W_XITEMS + X3W_THREADS - 1) / X3W_THREADS;  // 3 (the last partial)
constexpr int X3W_DYITEMS = 48 * 8;                  // (window, 4-co group) dY items per unit
static_assert(X3W_DYITEMS % 64 == 0, "whole waves of dY items");
static_assert(2 * X3W_BUF <= 163840, "LDS");

// X16 = true: the input image of a unit is the f16 image conv2_fwd_pool_x3 / conv1_fwd_x3 wrote (act16,
// per-sample scale 2^s_b, dY compensated by 2^(sd + sx - s_b) as above; chunk slot kc ^ (x & 2), i.e. the 32-B ci-half slot h ^ ((x >> 1) & 1)), moved by LDS-DMA
// one unit ahead straight into the image buffer: no gather loads, no split VALU.
template <bool X16>
__global__ __launch_bounds__(X3W_THREADS, 1) void conv2_wgrad_x3_kernel(
    const float* __restrict__ act, const float* __restrict__ act_amax, const float* __restrict__ dpooled,
    const float* __restrict__ dp_amax, const uint8_t* __restrict__ code, float* __restrict__ slabs, int B,
    const uint16_t* __restrict__ act16 = nullptr) {
    __shared__ __attribute__((aligned(1024))) char smem[2 * X3W_BUF];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = wave & 1, kp = (wave >> 1) & 1, tg = wave >> 2;
    const int nks = (int)gridDim.x / 2;
    // the two co halves of a K share read the same input rows: put them on one XCD (blocks b and b + 8
    // share one, round-robin dispatch) so the second read is an L2 hit
    const int bid = blockIdx.x;
    const bool xcd = (nks & 7) == 0;
    const int cohalf = xcd ? (bid >> 3) & 1 : bid & 1;
    const int ks = xcd ? (bid >> 4) * 8 + (bid & 7) : bid >> 1;
    const int U = 3 * B;
    float* red = reinterpret_cast<float*>(smem);  // prologue scratch (image 0, before any staging)

    // launch scales: max over the batch of the per-sample maxima
    float ma = 0.f, md = 0.f;
    for (int i = tid; i < B; i += X3W_THREADS) {
        ma = fmaxf(ma, act_amax[i]);
        md = fmaxf(md, dp_amax[i]);
    }
    ma = wave_max(ma);
    md = wave_max(md);
    if (lane == 0) {
        red[wave] = ma;
        red[8 + wave] = md;
    }
    __syncthreads();
    ma = red[0];
    md = red[8];
#pragma unroll
    for (int i = 1; i < 8; ++i) {
        ma = fmaxf(ma, red[i]);
        md = fmaxf(md, red[8 + i]);
    }
    __syncthreads();
    // the input operand carries its SAMPLE's scale 2^s_b (as the act16 images do); its dY is scaled by
    // 2^(sd + sx - s_b) (<= 2^sd: s_b >= sx), so every product carries 2^(sx + sd)
    const int sx = x3_exp(ma), sd = x3_exp(md);
    int sb_ld = 0;  // s_b of the unit load_dy last requested (its store_dy / split_x come one unit later)

    // input items: i = tid + 512 r -> channel group cg = i & 3, pixel p = i >> 2 of the unit's 260
    float xv[X3W_XR][8];
    auto load_x = [&](int uu) {
        const int b = uu / 3, t3 = uu - (uu / 3) * 3;
        const float* base = act + (size_t)b * A_SAMPLE + t3 * 8 * A_HW;
#pragma unroll
        for (int r = 0; r < X3W_XR; ++r) {
            // lanes past the last item redo it (same value to the same place): no exec-masked branch
            const int i = min(tid + r * X3W_THREADS, X3W_XITEMS - 1);
            const int cg = i & 3, p = i >> 2;
#pragma unroll
            for (int j = 0; j < 8; ++j) xv[r][j] = base[(8 * cg + j) * A_PIX + p];
        }
    };
    auto split_x = [&](char* img) {
        const float xsc = ldexpf(1.f, sb_ld);
#pragma unroll
        for (int r = 0; r < X3W_XR; ++r) {
            const int i = min(tid + r * X3W_THREADS, X3W_XITEMS - 1);
            const int cg = i & 3, p = i >> 2;
            f16x8 hh, ll;
            x3_split8(xv[r], xsc, hh, ll);
            char* o = img + 2 * X3W_DYP + p * 64 + cg * 16;
            *reinterpret_cast<f16x8*>(o) = hh;
            *reinterpret_cast<f16x8*>(o + X3W_XP) = ll;
        }
    };
    // dY items of a unit: item i < 384 = (4-co group dg = i & 7 of the co half, window dw = i >> 3);
    // threads past 383 redo item 383 (identical stores, no branch)
    const int ditem = min(tid, X3W_DYITEMS - 1);
    const int dg = ditem & 7, dw = ditem >> 3;
    float dv[4];
    uint32_t dcb[4];  // code bytes one per register until store_dy (combining here waits for the loads)
    auto load_dy = [&](int uu) {
        const int b = uu / 3, t3 = uu - (uu / 3) * 3;
        const int w = (4 * t3 + dw / 12) * P_HW + dw % 12;
        const size_t o = (size_t)b * P_SAMPLE + (32 * cohalf + 4 * dg) * P_WIN + w;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            dv[j] = dpooled[o + j * P_WIN];
            dcb[j] = code[o + j * P_WIN];
        }
        sb_ld = max(x3_exp(act_amax[b]), sx);  // = x3_exp(amax_b) unless amax_b is 0 (zero images: any scale)
    };
    // db[co] = sum of the routed dY = the pooled gradients whose code routes them (code != NONE): summed
    // in f32 from the raw values as they are staged (a thread keeps one (4-co group, window) item)
    float dbacc[4] = {0.f, 0.f, 0.f, 0.f};
    auto store_dy = [&](char* img, bool real) {
        const float dsc = ldexpf(1.f, sd + sx - sb_ld);
        const bool mine = real && tid < X3W_DYITEMS;
#pragma unroll
        for (int j = 0; j < 4; ++j) dbacc[j] = (mine && dcb[j] != (uint32_t)CODE_NONE) ? dbacc[j] + dv[j] : dbacc[j];
        uint32_t hv[2], lv[2];
#pragma unroll
        for (int j = 0; j < 4; j += 2) {
            const float a = dv[j] * dsc, c = dv[j + 1] * dsc;
            const _Float16 ha = (_Float16)a, hc = (_Float16)c;
            const _Float16 la = (_Float16)(a - (float)ha), lc = (_Float16)(c - (float)hc);
            hv[j / 2] = __builtin_bit_cast(uint32_t, f16x2{ha, hc});
            lv[j / 2] = __builtin_bit_cast(uint32_t, f16x2{la, lc});
        }
        const uint32_t dc = dcb[0] | (dcb[1] << 8) | (dcb[2] << 16) | (dcb[3] << 24);
        const uint32_t cA = __builtin_amdgcn_perm(0u, dc, 0x01010000u), cB = __builtin_amdgcn_perm(0u, dc, 0x03030202u);
        const int wy = dw / 12, wx = dw % 12;
        // a 16-lane group of ds_write_b64 (banks = dword % 32) holds the 8 co groups of windows dw and dw + 1:
        // the odd window walks the positions in the order pos ^ 1, so the two windows write pixels of
        // opposite parity, 16 banks apart (same order: 2-way on every store, SQ_LDS_BANK_CONFLICT 4.8 M)
        const int pf = dw & 1;
#pragma unroll
        for (int pos0 = 0; pos0 < 4; ++pos0) {
            const int pos = pos0 ^ pf;
            const uint32_t T = 0xFFu << (8 * pos);
            const uint32_t mA = __builtin_amdgcn_perm(0u, T, cA), mB = __builtin_amdgcn_perm(0u, T, cB);
            const int q = (2 * wy + (pos >> 1)) * 24 + 2 * wx + (pos & 1);
            // co tile (dg >> 2) sits in slot (dg >> 2) ^ ((q >> 3) & 1)
            char* o = img + q * 64 + ((((dg >> 2) ^ (q >> 3)) & 1) * 32) + 8 * (dg & 3);
            *reinterpret_cast<uint2*>(o) = make_uint2(hv[0] & mA, hv[1] & mB);
            *reinterpret_cast<uint2*>(o + X3W_DYP) = make_uint2(lv[0] & mA, lv[1] & mB);
        }
    };

    // transposed-read bases: group g4 = lane >> 4 (K-chunk), lane 4qq + pp of the group. K-chunk (K-step
    // s, g4) = 8 output pixels: segment seg of row orow, with the two 16-lane groups of a half-wave on the
    // same segment of two adjacent rows (idx = 2 s + (g4 >> 1): orow = 2 (idx / 3) + (g4 & 1), seg =
    // idx % 3): their input pixels are then 26 apart, 2 mod 4, and the images' (x >> 1) slot swizzle puts
    // them on disjoint banks (chunks 8 pixels apart in one row were 2-way: tools/lds_banks.py)
    const int g4 = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    int abase[3][2];  // dY: pixel q = 24 orow + 8 seg + qq (+4), co tile mi in slot mi ^ ((q >> 3) & 1)
    int xbase[3][3];  // input per (this wave's K-step j, kx); X16 images keep ci half h in slot h ^ ((x >> 1) & 1)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int idx = 2 * (kp + 2 * j) + (g4 >> 1);
        const int orow = 2 * (idx / 3) + (g4 & 1), seg = idx % 3;
        const int q0 = 24 * orow + 8 * seg;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) abase[j][mi] = (q0 + qq) * 64 + ((mi ^ ((q0 >> 3) & 1)) * 32) + pp * 8;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int x = 8 * seg + qq + kx;
            const int slot = X16 ? (h ^ ((x >> 1) & 1)) : h;
            xbase[j][kx] = 2 * X3W_DYP + ((orow * A_HW + x) * 64) + slot * 32 + pp * 8;
        }
    }
    // X16 staging: 2,080 16-B pieces per unit, lane-contiguous (the image is stored as it sits in LDS)
    auto issue_x16 = [&](int uu, char* img) {
        x3_issue_unit_img(act16, uu, __builtin_amdgcn_readfirstlane(tid >> 6), lane, lds_u32(img + 2 * X3W_DYP));
    };
    typedef __fp16 hf4 __attribute__((__vector_size__(8)));
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) hf4* lp4;
    auto trr = [&](const char* p) -> f16x8 {
        const f16x4 lo = __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lp4)p));
        const f16x4 hi = __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lp4)(p + 4 * 64)));
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };

    // wave = (ci half h, K-step parity kp, tap group tg: taps 0-4 or 5-8 + db); waves w and w + 4 share
    // a SIMD, so every SIMD carries one wave of each tap group
    f32x4 acc[2][5];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int t = 0; t < 5; ++t) acc[mi][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // a unit's work for this wave: K-steps kp, kp + 2, kp + 4 x its taps; B fragments (4 transposed reads)
    // run 2 steps ahead through a 3-slot ring, A fragments (8 reads) one K-step ahead; the
    // sched_group_barriers keep that order (hipcc otherwise sinks every read next to its MFMAs)
    auto unit_mfma = [&](const char* img, auto TG) {
        constexpr int T0 = decltype(TG)::value ? 5 : 0, NT = decltype(TG)::value ? 4 : 5;
        constexpr int N = 3 * NT;
        f16x8 Ah[2][2], Al[2][2], Bh[3], Bl[3];
        auto rdA = [&](int j, int slot) {
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) {
                Ah[slot][mi] = trr(img + abase[j][mi]);
                Al[slot][mi] = trr(img + X3W_DYP + abase[j][mi]);
            }
        };
        auto rdB = [&](int n, int slot) {
            const int j = n / NT, tap = T0 + n % NT;
            const int to = (tap / 3) * A_HW * 64;
            Bh[slot] = trr(img + xbase[j][tap % 3] + to);
            Bl[slot] = trr(img + X3W_XP + xbase[j][tap % 3] + to);
        };
        rdA(0, 0);
        rdB(0, 0);
        rdB(1, 1);
#pragma unroll
        for (int n = 0; n < N; ++n) {
            if (n + 2 < N) {
                rdB(n + 2, (n + 2) % 3);
                if ((n + 2) % NT == 0) rdA((n + 2) / NT, ((n + 2) / NT) & 1);
            }
            const int j = n / NT, t = n % NT;
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
                acc[mi][t] = mfma_x3(Ah[j & 1][mi], Al[j & 1][mi], Bh[n % 3], Bl[n % 3], acc[mi][t]);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
#pragma unroll
        for (int n = 0; n < N; ++n) {
            __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
            if (n + 2 < N) {
                if ((n + 2) % NT == 0) __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
                else __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
            }
        }
    };

    // a contiguous range of units per K share: the three thirds of a sample run back to back, so the
    // 2 halo rows each shares with the next come from L2 (both co-half workgroups of the share sit on
    // one XCD and read the same images)
    const int per = (U + nks - 1) / nks;
    const int u0 = min(ks * per, U), u1 = min(u0 + per, U);
    int u = u0;
    if (u < u1) {
        if constexpr (X16) {
            issue_x16(u, smem);
        } else {
            load_x(u);
        }
        load_dy(u);
        if constexpr (!X16) split_x(smem);
        store_dy(smem, true);
        if constexpr (!X16) load_x(min(u + 1, u1 - 1));
        load_dy(min(u + 1, u1 - 1));
    }
    int k = 0;
#pragma unroll 1
    for (; u < u1; ++u, ++k) {
        // X16: this unit's image DMA landed; the 8 dY loads of load_dy, every wave's last memory
        // instructions (issued after its DMA), may stay in flight
        const bool dfirst = !X16 || tg == 1;
        // X16: waves 6-7 hold no dY item (384 items = waves 0-5) and skip the routing (no redundant
        // redo of item 383); their last memory instructions are then the DMA itself
        const bool dstage = !(X16 && wave >= X3W_DYITEMS / 64);
        if constexpr (X16) {
            if (!dstage) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        }
        __syncthreads();  // image k&1 complete; image (k+1)&1 free
        const int nx = u + 1, nx2 = u + 2;
        const char* img = smem + (k & 1) * X3W_BUF;
        char* nimg = smem + ((k & 1) ^ 1) * X3W_BUF;
        // unit u+1's rows and dY were requested a whole unit ago. No branch around the staging (past the
        // last unit it re-stages a clamped valid unit nobody reads), so it shares one basic block with
        // the MFMAs and its VALU can fill their issue gaps
        // X16: the tap-group-1 waves (the lighter MFMA share) route dY before their MFMAs, the tap-group-0
        // waves after theirs, so the two waves of a SIMD overlap routing with MFMAs. store_dy goes before
        // the DMA issue: the compiler does not count the asm DMAs, so its wait for the dY registers
        // would otherwise also wait for the DMA just issued
        if (dfirst && dstage) store_dy(nimg, nx < u1);
        if constexpr (X16) {
            // (spreading these pieces over the MFMA steps, as the forward does, measured 0.2258 -> 0.2388 ms:
            // the pinned read/MFMA order does not absorb them)
            issue_x16(min(nx, u1 - 1), nimg);
        } else {
            split_x(nimg);
        }
        if (dfirst && dstage) {
            if constexpr (!X16) load_x(min(nx2, u1 - 1));
            load_dy(min(nx2, u1 - 1));
        }
        if (tg == 0) unit_mfma(img, std::integral_constant<int, 0>{});
        else unit_mfma(img, std::integral_constant<int, 1>{});
        if (!dfirst && dstage) {
            store_dy(nimg, nx < u1);
            load_dy(min(nx2, u1 - 1));
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (clamped) image DMA lands before LDS reuse
    __syncthreads();
    // K parities: kp = 1 waves hand their sums to kp = 0 through LDS (region per (h, tg))
    constexpr int XN = 2 * 5 * 4;  // floats per lane
    float* xch = reinterpret_cast<float*>(smem) + (h + 2 * tg) * (XN * 64);
    if (kp == 1) {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
            for (int t = 0; t < 5; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) xch[((mi * 5 + t) * 4 + r) * 64 + lane] = acc[mi][t][r];
        }
    }
    // db partials of the staging items -> LDS; co = 32 cohalf + 4 dg + j summed over the 48 windows in order
    float* dbs = reinterpret_cast<float*>(smem) + 4 * XN * 64;
    if (tid < X3W_DYITEMS)
#pragma unroll
        for (int j = 0; j < 4; ++j) dbs[tid * 4 + j] = dbacc[j];
    __syncthreads();
    if (tid < 32) {
        const int g = tid >> 2, j = tid & 3;
        float sum = 0.f;
        for (int w = 0; w < 48; ++w) sum += dbs[(w * 8 + g) * 4 + j];
        slabs[(size_t)ks * (W2_N + C2) + W2_N + 32 * cohalf + tid] = sum;
    }
    if (kp == 0) {
        const float us1 = ldexpf(1.f, -sx), us2 = ldexpf(1.f, -sd);
        float* slab = slabs + (size_t)ks * (W2_N + C2);
        const int ci = 16 * h + (lane & 15);
        const int nt = tg ? 4 : 5;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
            for (int t = 0; t < 5; ++t)
                if (t < nt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int co = 32 * cohalf + 16 * mi + 4 * (lane >> 4) + r;
                        slab[(co * C1 + ci) * 9 + 5 * tg + t] =
                            x3_unscale(acc[mi][t][r] + xch[((mi * 5 + t) * 4 + r) * 64 + lane], us1, us2);
                    }
        }
    }
}

// ============================================================================ conv2 wgrad, both co halves per workgroup
// The act16-image form of the x3 wgrad (round 5) with one workgroup per K share owning ALL of dW2: the
// unit is (sample, sixth) = output rows 4t .. 4t + 3 (K = 96 pixels = 3 K-steps), so both co halves' dY
// planes (4 x 6 KiB) and the unit's input image (rows 4t .. 4t + 5, 2 x 9.75 KiB) fit twice into LDS
// (the 8-row unit with both co halves needed 164,864 B, 1 KiB over): the input image is moved by LDS-DMA
// once for the 64 co instead of once per co half by two workgroups (the DMA of that image was 11 % of the
// round-4 kernel), and no K-parity partial sums are exchanged at the end. 8 waves = (tap group tg, co half
// c, ci half h), wave = 4 tg + 2 c + h: the two waves of a SIMD (w, w + 4) carry one tap group each; per
// unit a wave does all 3 K-steps x its taps x both M tiles of its co half — the same fragment reads and
// MFMAs per unit as the round-4 wave. dY staging as conv2_wgrad_x3_kernel (register loads two units
// ahead, routed one unit ahead), items (4-co group, co half, window) with the co half's planes offset by
// 64 B so a 16-lane store group (8 groups x 2 co halves of one window) covers 32 distinct banks.
constexpr int X3Q_ROWS = 4;                              // output rows per unit (6 units per sample)
constexpr int X3Q_Q = X3Q_ROWS * 24;                     // 96 output pixels = K per unit
constexpr int X3Q_DYP = X3Q_Q * 64;                      // 6,144 B per dY plane (32 co of one co half)
constexpr int X3Q_DYC = 2 * X3Q_DYP + 64;                // co half stride: h | l planes + 64 B
constexpr int X3Q_XPIX = (X3Q_ROWS + 2) * A_HW;          // 156 input pixels per unit
constexpr int X3Q_XP = X3Q_XPIX * 64;                    // 9,984 B per input plane
constexpr int X3Q_DYOFF = 2 * X3Q_XP;                    // dY planes after the input planes (1 KiB aligned start)
constexpr int X3Q_BUF = (X3Q_DYOFF + 2 * X3Q_DYC + 1023) / 1024 * 1024;  // 45,056 B per buffer
constexpr int X3Q_NKS = 256;                             // K shares (slabs): one workgroup per CU
constexpr int X3Q_DYITEMS = 24 * 16;                     // (window, 4-co group, co half) items per unit
constexpr int X3Q_XPIECES = X3Q_XP / 1024 + 1;           // 10 DMA pieces per input plane (the last 768 B)
static_assert(2 * X3Q_BUF <= 163840 && X3Q_XP % 1024 == 768 && (X3Q_DYC / 4) % 32 == 16, "x3q layout");

// (round 5: 12 waves = 3 per SIMD at <= 168 VGPRs, tap groups of 3, measured the same: 0.2369 vs 0.2376 ms)
constexpr int X3Q_THREADS = 512;
constexpr int X3Q_WAVES = X3Q_THREADS / 64;
constexpr int X3Q_NTMAX = 5;                             // taps per wave (max)

// LDS-DMA of unit uu's input image (rows 4t .. 4t + 5 of both planes of the sample's act16 image)
__device__ __forceinline__ void x3q_issue_img(const uint16_t* act16, int uu, int wave, int lane, uint32_t lds) {
    const int b = uu / 6, t = uu - (uu / 6) * 6;
    const char* src = reinterpret_cast<const char*>(act16) + (size_t)b * X3S_SAMPLE + t * (X3Q_ROWS * A_HW * 64);
#pragma unroll
    for (int r = 0; r < (2 * X3Q_XPIECES + X3Q_WAVES - 1) / X3Q_WAVES; ++r) {
        const int k = wave + X3Q_WAVES * r;  // piece k of the 20: plane k / 10, piece k % 10
        if (k < 2 * X3Q_XPIECES) {
            const int pl = k >= X3Q_XPIECES ? 1 : 0, pp = k - X3Q_XPIECES * pl;
            if (pp < X3Q_XPIECES - 1 || lane < (X3Q_XP % 1024) / 16)
                glds16_so(src + pl * X3S_PLANE, (uint32_t)(pp * 1024 + lane * 16), lds + pl * X3Q_XP + pp * 1024);
        }
    }
}

__global__ __launch_bounds__(X3Q_THREADS, 1) void conv2_wgrad_x3q_kernel(
    const uint16_t* __restrict__ act16, const float* __restrict__ act_amax, const float* __restrict__ dpooled,
    const float* __restrict__ dp_amax, const uint8_t* __restrict__ code, float* __restrict__ slabs, int B) {
    __shared__ __attribute__((aligned(1024))) char smem[2 * X3Q_BUF];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = wave & 1, c = (wave >> 1) & 1, tg = wave >> 2;
    const int ks = blockIdx.x, nks = gridDim.x;
    const int U = 6 * B;
    float* red = reinterpret_cast<float*>(smem);  // prologue scratch (buffer 0, before any staging)
    X3Q_TS(0, 7);

    // launch scales: max over the batch of the per-sample maxima (as conv2_wgrad_x3_kernel)
    float ma = 0.f, md = 0.f;
    for (int i = tid; i < B; i += X3Q_THREADS) {
        ma = fmaxf(ma, act_amax[i]);
        md = fmaxf(md, dp_amax[i]);
    }
    ma = wave_max(ma);
    md = wave_max(md);
    if (lane == 0) {
        red[wave] = ma;
        red[16 + wave] = md;
    }
    __syncthreads();
    ma = red[0];
    md = red[16];
#pragma unroll
    for (int i = 1; i < X3Q_WAVES; ++i) {
        ma = fmaxf(ma, red[i]);
        md = fmaxf(md, red[16 + i]);
    }
    __syncthreads();
    const int sx = x3_exp(ma), sd = x3_exp(md);
    int sb_ld = 0;

    // dY items: i = tid < 384 -> 4-co group dg = i & 7 of co half ci2 = (i >> 3) & 1, window dw = i >> 4
    // (24 windows: 2 window rows x 12); waves 6-7 hold none
    const bool dstage = tid < X3Q_DYITEMS;
    const int dg = tid & 7, dc = (tid >> 3) & 1, dw = min(tid >> 4, 23);
    float dv[4];
    uint32_t dcb[4];
    auto load_dy = [&](int uu) {
        const int b = uu / 6, t = uu - (uu / 6) * 6;
        const int w = (2 * t + dw / 12) * P_HW + dw % 12;
        const size_t o = (size_t)b * P_SAMPLE + (32 * dc + 4 * dg) * P_WIN + w;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            dv[j] = dpooled[o + j * P_WIN];
            dcb[j] = code[o + j * P_WIN];
        }
        sb_ld = max(x3_exp(act_amax[b]), sx);
    };
    float dbacc[4] = {0.f, 0.f, 0.f, 0.f};
    auto store_dy = [&](char* img, bool real) {
        const float dsc = ldexpf(1.f, sd + sx - sb_ld);
#pragma unroll
        for (int j = 0; j < 4; ++j) dbacc[j] = (real && dcb[j] != (uint32_t)CODE_NONE) ? dbacc[j] + dv[j] : dbacc[j];
        uint32_t hv[2], lv[2];
#pragma unroll
        for (int j = 0; j < 4; j += 2) {
            const float a = dv[j] * dsc, cc = dv[j + 1] * dsc;
            const _Float16 ha = (_Float16)a, hc = (_Float16)cc;
            const _Float16 la = (_Float16)(a - (float)ha), lc = (_Float16)(cc - (float)hc);
            hv[j / 2] = __builtin_bit_cast(uint32_t, f16x2{ha, hc});
            lv[j / 2] = __builtin_bit_cast(uint32_t, f16x2{la, lc});
        }
        const uint32_t dcw = dcb[0] | (dcb[1] << 8) | (dcb[2] << 16) | (dcb[3] << 24);
        const uint32_t cA = __builtin_amdgcn_perm(0u, dcw, 0x01010000u), cB = __builtin_amdgcn_perm(0u, dcw, 0x03030202u);
        const int wy = dw / 12, wx = dw % 12;
        char* plane = img + X3Q_DYOFF + dc * X3Q_DYC;
#pragma unroll
        for (int pos = 0; pos < 4; ++pos) {
            const uint32_t T = 0xFFu << (8 * pos);
            const uint32_t mA = __builtin_amdgcn_perm(0u, T, cA), mB = __builtin_amdgcn_perm(0u, T, cB);
            const int q = (2 * wy + (pos >> 1)) * 24 + 2 * wx + (pos & 1);
            // co tile (dg >> 2) sits in slot (dg >> 2) ^ ((q >> 3) & 1), as in conv2_wgrad_x3_kernel
            char* o = plane + q * 64 + ((((dg >> 2) ^ (q >> 3)) & 1) * 32) + 8 * (dg & 3);
            *reinterpret_cast<uint2*>(o) = make_uint2(hv[0] & mA, hv[1] & mB);
            *reinterpret_cast<uint2*>(o + X3Q_DYP) = make_uint2(lv[0] & mA, lv[1] & mB);
        }
    };

    // transposed-read bases (conv2_wgrad_x3_kernel's, every K-step j = 0..2 of the 4-row unit)
    const int g4 = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    int abase[3][2], xbase[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int idx = 2 * j + (g4 >> 1);
        const int orow = 2 * (idx / 3) + (g4 & 1), seg = idx % 3;
        const int q0 = 24 * orow + 8 * seg;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
            abase[j][mi] = X3Q_DYOFF + c * X3Q_DYC + (q0 + qq) * 64 + ((mi ^ ((q0 >> 3) & 1)) * 32) + pp * 8;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const int x = 8 * seg + qq + kx;
            xbase[j][kx] = ((orow * A_HW + x) * 64) + (h ^ ((x >> 1) & 1)) * 32 + pp * 8;
        }
    }
    typedef __fp16 hf4 __attribute__((__vector_size__(8)));
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) hf4* lp4;
    auto trr = [&](const char* p) -> f16x8 {
        const f16x4 lo = __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lp4)p));
        const f16x4 hi = __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lp4)(p + 4 * 64)));
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    };

    f32x4 acc[2][X3Q_NTMAX];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int t = 0; t < X3Q_NTMAX; ++t) acc[mi][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto unit_mfma = [&](const char* img, auto TG) {
        constexpr int TGV = decltype(TG)::value;
        constexpr int T0 = TGV ? 5 : 0, NT = TGV ? 4 : 5;
        constexpr int N = 3 * NT;
        f16x8 Ah[2][2], Al[2][2], Bh[3], Bl[3];
        auto rdA = [&](int j, int slot) {
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) {
                Ah[slot][mi] = trr(img + abase[j][mi]);
                Al[slot][mi] = trr(img + X3Q_DYP + abase[j][mi]);
            }
        };
        auto rdB = [&](int n, int slot) {
            const int j = n / NT, tap = T0 + n % NT;
            const int to = (tap / 3) * A_HW * 64;
            Bh[slot] = trr(img + xbase[j][tap % 3] + to);
            Bl[slot] = trr(img + X3Q_XP + xbase[j][tap % 3] + to);
        };
        rdA(0, 0);
        rdB(0, 0);
        rdB(1, 1);
#pragma unroll
        for (int n = 0; n < N; ++n) {
            if (n + 2 < N) {
                rdB(n + 2, (n + 2) % 3);
                if ((n + 2) % NT == 0) rdA((n + 2) / NT, ((n + 2) / NT) & 1);
            }
            const int j = n / NT, t = n % NT;
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
                acc[mi][t] = mfma_x3(Ah[j & 1][mi], Al[j & 1][mi], Bh[n % 3], Bl[n % 3], acc[mi][t]);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
#pragma unroll
        for (int n = 0; n < N; ++n) {
            __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
            if (n + 2 < N) {
                if ((n + 2) % NT == 0) __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
                else __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
            }
        }
    };

    // a contiguous range of units per K share (the six parts of a sample back to back: shared halo rows
    // and dY window rows come from L2)
    const int per = (U + nks - 1) / nks;
    const int u0 = min(ks * per, U), u1 = min(u0 + per, U);
    int u = u0;
    if (u < u1) {
        x3q_issue_img(act16, u, wave, lane, lds_u32(smem));
        if (dstage) {
            load_dy(u);
            store_dy(smem, true);
            load_dy(min(u + 1, u1 - 1));
        }
    }
    int k = 0;
#pragma unroll 1
    for (; u < u1; ++u, ++k) {
        // this unit's image DMA landed; the 8 dY loads (every staging wave's last memory instructions,
        // issued after its DMA) may stay in flight
        X3Q_TS(k, 6);
        if (!dstage) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        __syncthreads();  // buffer k&1 complete; buffer (k+1)&1 free
        X3Q_TS(k, 0);
        const int nx = u + 1, nx2 = u + 2;
        const char* img = smem + (k & 1) * X3Q_BUF;
        char* nimg = smem + ((k & 1) ^ 1) * X3Q_BUF;
        // tap-group-1 waves (the lighter MFMA share) route dY before their MFMAs, tap-group-0 after:
        // the two waves of a SIMD overlap routing with MFMAs; store_dy before the DMA issue (hipcc does
        // not count the asm DMAs: its wait for the dY registers would also wait for them)
        const bool dfirst = tg == 1;
        if (dfirst && dstage) store_dy(nimg, nx < u1);
        x3q_issue_img(act16, min(nx, u1 - 1), wave, lane, lds_u32(nimg));
        if (dfirst && dstage) load_dy(min(nx2, u1 - 1));
        X3Q_TS(k, 1);
        if (tg == 0) unit_mfma(img, std::integral_constant<int, 0>{});
        else unit_mfma(img, std::integral_constant<int, 1>{});
        X3Q_TS(k, 2);
        if (!dfirst && dstage) {
            store_dy(nimg, nx < u1);
            load_dy(min(nx2, u1 - 1));
        }
        X3Q_TS(k, 3);
    }
    X3Q_TS(127, 7);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (clamped) image DMA lands before LDS reuse
    __syncthreads();
    // db partials of the staging items -> LDS; co = 32 dc + 4 dg + j summed over the 24 windows in order
    float* dbs = reinterpret_cast<float*>(smem);
    if (dstage)
#pragma unroll
        for (int j = 0; j < 4; ++j) dbs[tid * 4 + j] = dbacc[j];
    __syncthreads();
    float* slab = slabs + (size_t)ks * (W2_N + C2);
    if (tid < C2) {
        const int cc = tid >> 5, g = (tid >> 2) & 7, j = tid & 3;
        float sum = 0.f;
        for (int w = 0; w < 24; ++w) sum += dbs[(w * 16 + cc * 8 + g) * 4 + j];
        slab[W2_N + tid] = sum;
    }
    const float us1 = ldexpf(1.f, -sx), us2 = ldexpf(1.f, -sd);
    const int ci = 16 * h + (lane & 15);
    const int nt = tg ? 4 : 5, tap0 = 5 * tg;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
        for (int t = 0; t < X3Q_NTMAX; ++t)
            if (t < nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = 32 * c + 16 * mi + 4 * (lane >> 4) + r;
                    slab[(co * C1 + ci) * 9 + tap0 + t] = x3_unscale(acc[mi][t][r], us1, us2);
                }
    }
}

// ============================================================================ conv2 wgrad on the 2:4-sparse f16 MFMA
// Round 6. dY is the max-pool routing of dpooled: in each 2 x 2 pool window at most ONE position carries a
// value. Take the GEMM's K (output pixels) in blocks of 4 consecutive pixels of one output row starting at a
// multiple of 4: such a block holds two positions of each of two windows, so at most 2 of its 4 dY values
// are nonzero for any co — exactly the 2:4 structure of v_smfmac_f32_16x16x64_f16, which multiplies a
// 16 x 64 A given as its nonzeros (2 per group of 4 + a 2-bit position each) by a dense 64 x 16 B at the
// issue cost of one dense v_mfma_f32_16x16x32_f16 (tools/ubench/smfmac_probe.hip: 17.6-18.2 vs 18.1-19.1
// cycles per instruction): half the MFMA instructions of the dense x3 wgrad for the same products.
// Operand layouts of the instruction, measured by that probe (one-hot A against distinct B):
//   B (dense, K x N): lane (gb = lane >> 4, n = lane & 15) holds K slots (gb, j), j = 0..15, of column n;
//   A (compressed, M x K): lane (ga = lane >> 4, m = lane & 15) value i (0..7) is the row-m entry of K slot
//     (gb = 2 (ga & 1) + (i >> 2), j = 8 (ga >> 1) + 4 ((i >> 1) & 1) + idx_i), idx_i = (index >> 2i) & 3;
//   D as the dense 16x16x32 (lane l: D[4 (l >> 4) + r][l & 15]).
// Here M = co (4 tiles), N = (ci half, tap), K = the unit's 192 output pixels (sample, third: output rows
// 8t..8t+7) = 3 K-steps of 64 = 48 blocks: block L = 16 s + 4 gb + jb (jb = j >> 2) is output row L / 6,
// columns 4 (L % 6) .. +3. B = the act16 input image (both planes, LDS-DMA as the forward's) read with
// ds_read_b64_tr_b16, one 4-pixel block per read, 4 per fragment. A = compressed dY records [s][ga][co] of
// 8 halves (h plane, l plane) + a u16 index word each, written by the staging items (co, window row,
// window quad): the 4 windows of a quad are two blocks of each of the two output rows of the window row,
// and those two blocks are one half of one record (8 B) + one byte of its index word. A record is the exact
// register image of a lane's A fragment: one conflict-free ds_read_b128 per (M tile, plane) per K-step.
// Waves: 4 M tiles (all 64 co) per wave, so every B fragment feeds 12 MFMAs; (ci half, tap group) items:
// waves 0/1 taps 0-2, 4/5 taps 3-4, 2/3 taps 5-6, 6/7 taps 7-8 (ci half = wave & 1): SIMD pairs (w, w + 4)
// carry 5, 5, 4, 4 taps. Scales, db and the slab format as conv2_wgrad_x3q_kernel.
#ifndef SLK_X3P_PLAN
#define SLK_X3P_PLAN 0  // 0: staging before (waves 4-7) / after (0-3) the MFMA steps; 1: in pieces between K-steps
#endif
#ifndef SLK_X3P_STG
#define SLK_X3P_STG 0  // 0: items q = wave and 8 + wave (waves 0-3); 1: only the 4-tap SIMDs' waves (2, 3, 6, 7), 3 each
#endif
#ifndef SLK_X3P_ABL
#define SLK_X3P_ABL 0  // profiling only (wrong results): 1 no in-loop dY staging, 2 no MFMA steps, 4 no in-loop DMA
#endif
constexpr int X3P_THREADS = 512;
constexpr int X3P_STEPS = 3;                                   // K64 steps per unit (192 pixels)
constexpr int X3P_REC = X3P_STEPS * 4 * 64 * 16;               // 12,288 B per compressed dY plane
constexpr int X3P_IDXB = X3P_STEPS * 4 * 64 * 2;               // 1,536 B of index words
constexpr int X3P_DYOFF = 2 * X3F_PLANE;                       // after the unit's input image (h | l)
constexpr int X3P_IDXOFF = X3P_DYOFF + 2 * X3P_REC;
constexpr int X3P_BUF = (X3P_IDXOFF + X3P_IDXB + 1023) / 1024 * 1024;  // 59,392 B
constexpr int X3P_ITEMS = C2 * 12;                             // (co, window row of 4, window quad of 3)
constexpr int X3P_SBN = (163840 - 2 * X3P_BUF) / 4;            // per-sample scale table entries (11,264)
static_assert(2 * X3P_BUF <= 163840 && X3P_ITEMS <= 2 * X3P_THREADS && X3P_ITEMS > X3P_THREADS, "x3p layout");

#ifndef SLK_X3P_BAL
#define SLK_X3P_BAL 0  // measured: 0.1677 vs 0.1648 ms unbalanced (profiles/r06_ab_wgrad_balance.txt): not the limiter
#endif
// Work of the four wave types (TGI = 2 ((wave >> 1) & 1) + (wave >> 2); ci half = wave & 1): (tap, M tiles) items,
// 4 M tiles = all 64 co. Waves w and w + 4 share a SIMD, so SIMDs 0-1 carry TGI 0 + 1 and SIMDs 2-3 TGI 2 + 3.
// Taps 0-2 | 3-4 | 5-6 | 7-8 gave them 5 and 4 taps (20 vs 16 (tap, M tile) items: the lighter SIMDs waited
// at every unit barrier); BAL moves tap 2's M tiles 2-3 from TGI 0 to TGI 2: 18 items per SIMD.
template <int TGI>
struct X3pTaps {
    static constexpr bool BAL = SLK_X3P_BAL;
    static constexpr int NT = (TGI == 0 || (TGI == 2 && BAL)) ? 3 : 2;
    static constexpr int tap(int t) {
        return TGI == 0 ? t : (TGI == 1 ? 3 + t : (TGI == 2 ? (t < 2 ? 5 + t : 2) : 7 + t));
    }
    static constexpr int mlo(int t) { return (TGI == 2 && t == 2) ? 2 : 0; }
    static constexpr int mhi(int t) { return (TGI == 0 && t == 2 && BAL) ? 2 : 4; }
};

template <int TGI, class F>
__device__ __forceinline__ void x3p_steps(const char* img, const int (&pb)[X3P_STEPS][4], const int (&sw)[3], int arec,
                                          int aidx, f32x4 (&acc)[3][4], F&& after_step) {
    using TT = X3pTaps<TGI>;
    constexpr int NT = TT::NT;
    typedef __fp16 hf4 __attribute__((__vector_size__(8)));
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    typedef _Float16 f16x16 __attribute__((ext_vector_type(16)));
    typedef __attribute__((address_space(3))) hf4* lp4;
    auto tr = [&](const char* p) -> f16x4 { return __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lp4)p)); };
#pragma unroll
    for (int s = 0; s < X3P_STEPS; ++s) {
        f16x8 ah[4], al[4];
        int ix[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
            ah[mt] = *reinterpret_cast<const f16x8*>(img + X3P_DYOFF + arec + s * 4096 + mt * 256);
            al[mt] = *reinterpret_cast<const f16x8*>(img + X3P_DYOFF + X3P_REC + arec + s * 4096 + mt * 256);
            ix[mt] = *reinterpret_cast<const uint16_t*>(img + X3P_IDXOFF + aidx + s * 512 + mt * 32);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int tap = TT::tap(t), ky = tap / 3, kx = tap % 3;
            f16x4 bh[4], bl[4];
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) {
                const char* p = img + pb[s][jb] + sw[kx] + (ky * A_HW + kx) * 64;
                bh[jb] = tr(p);
                bl[jb] = tr(p + X3F_PLANE);
            }
            const f16x16 Bh = __builtin_shufflevector(__builtin_shufflevector(bh[0], bh[1], 0, 1, 2, 3, 4, 5, 6, 7),
                                                      __builtin_shufflevector(bh[2], bh[3], 0, 1, 2, 3, 4, 5, 6, 7),
                                                      0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
            const f16x16 Bl = __builtin_shufflevector(__builtin_shufflevector(bl[0], bl[1], 0, 1, 2, 3, 4, 5, 6, 7),
                                                      __builtin_shufflevector(bl[2], bl[3], 0, 1, 2, 3, 4, 5, 6, 7),
                                                      0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
#pragma unroll
            for (int mt = TT::mlo(t); mt < TT::mhi(t); ++mt) {
                f32x4 c = acc[t][mt];
                c = __builtin_amdgcn_smfmac_f32_16x16x64_f16(ah[mt], Bh, c, ix[mt], 0, 0);
                c = __builtin_amdgcn_smfmac_f32_16x16x64_f16(ah[mt], Bl, c, ix[mt], 0, 0);
                c = __builtin_amdgcn_smfmac_f32_16x16x64_f16(al[mt], Bh, c, ix[mt], 0, 0);
                acc[t][mt] = c;
            }
        }
        after_step(s);
    }
}

__global__ __launch_bounds__(X3P_THREADS, 1) void conv2_wgrad_x3p_kernel(
    const uint16_t* __restrict__ act16, const float* __restrict__ act_amax, const float* __restrict__ dpooled,
    const float* __restrict__ dp_amax, const uint8_t* __restrict__ code, float* __restrict__ slabs, int B) {
    __shared__ __attribute__((aligned(1024))) char smem[163840];
    // after both buffers: the K share's per-sample dY scale exponents sd + sx - s_b (a scalar load of act_amax per
    // unit in the loop would hold the next LDS waits behind it: lgkmcnt counts both)
    int* sbt = reinterpret_cast<int*>(smem + 2 * X3P_BUF);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = wave & 1, tgi = ((wave >> 1) & 1) * 2 + (wave >> 2);  // 0: taps 0-2, 1: 3-4, 2: 5-6, 3: 7-8
    const int ks = blockIdx.x, nks = gridDim.x;
    const int U = 3 * B;
    float* red = reinterpret_cast<float*>(smem);
    X3Q_TS(0, 7);

    // launch scales: max over the batch of the per-sample maxima (as conv2_wgrad_x3q_kernel)
    float ma = 0.f, md = 0.f;
    for (int i = tid; i < B; i += X3P_THREADS) {
        ma = fmaxf(ma, act_amax[i]);
        md = fmaxf(md, dp_amax[i]);
    }
    ma = wave_max(ma);
    md = wave_max(md);
    if (lane == 0) {
        red[wave] = ma;
        red[16 + wave] = md;
    }
    __syncthreads();
    ma = red[0];
    md = red[16];
#pragma unroll
    for (int i = 1; i < 8; ++i) {
        ma = fmaxf(ma, red[i]);
        md = fmaxf(md, red[16 + i]);
    }
    __syncthreads();
    const int sx = x3_exp(ma), sd = x3_exp(md);

    // staging items (co, q = 3 window row + window quad): co = lane (fastest, so a 16-lane LDS store group
    // writes 16 consecutive 16-B records: 2-way banks instead of the 6-12-way of 12 items of one co), q = wave
    // and, for waves 0-3, 8 + wave. Per item the global offset within the unit and the two LDS destinations
    // (one per output row of the window row) do not depend on the unit: computed once.
#if SLK_X3P_STG == 0
    constexpr int NI = 2;
    const bool two = wave < 4;
    const int nit = two ? 2 : 1;
#else
    constexpr int NI = 3;
    const bool two = false;
    const int sidx = (wave & 1) + 2 * (wave >> 2);           // waves 2, 3, 6, 7 -> 0, 1, 2, 3
    const int nit = (wave & 2) ? 3 : 0;
#endif
    int goff[NI], ldo[NI][2];
#pragma unroll
    for (int r = 0; r < NI; ++r) {
#if SLK_X3P_STG == 0
        const int q = r == 0 ? wave : 8 + (wave & 3);
#else
        const int q = 3 * sidx + r;
#endif
        const int wyl = q / 3, wq = q - (q / 3) * 3;
        goff[r] = lane * P_WIN + wyl * P_HW + 4 * wq;
#pragma unroll
        for (int d = 0; d < 2; ++d) {
            const int L = 6 * (2 * wyl + d) + 2 * wq;  // even: the quad's first block
            const int st = L >> 4, gb = (L >> 2) & 3, jb = L & 3;
            const int rec = (st * 4 + 2 * (jb >> 1) + (gb >> 1)) * 64 + lane;
            ldo[r][d] = rec * 16 + 8 * (gb & 1);  // h plane; the index byte is rec * 2 + (gb & 1)
        }
    }
    float4 dv[NI];
    uint32_t dcw[NI];
    int ld_b = 0, sb0 = 0;
    auto load_dy = [&](int uu) {
        const int b = uu / 3, t3 = uu - (uu / 3) * 3;
        const size_t o = (size_t)b * P_SAMPLE + t3 * 4 * P_HW;
#pragma unroll
        for (int r = 0; r < NI; ++r) {
            if (r < nit) {
                dv[r] = *reinterpret_cast<const float4*>(dpooled + o + goff[r]);
                dcw[r] = *reinterpret_cast<const uint32_t*>(code + o + goff[r]);
            }
        }
        ld_b = b;
    };
    float dbacc[NI] = {};
    int trk = 0;  // (trace builds: the unit index of the stamps inside the staging)
    (void)trk;
    auto store_dy1 = [&](char* img, bool real, int r) {
        const float dsc = ldexpf(1.f, sbt[ld_b - sb0]);
        {
            {
                const float v[4] = {dv[r].x, dv[r].y, dv[r].z, dv[r].w};
#if SLK_X3D_TRACE
                if (r == 0) {
                    asm volatile("" ::"v"(v[0]), "v"(dcw[0]));
                    X3Q_TS(trk, 4);
                }
#endif
                const uint32_t cw = dcw[r];
                // index byte: window j's position in its block = its dx, +2 for the block's second window
                const uint32_t ib = (cw & 1u) | ((cw >> 6) & 4u) | ((cw >> 12) & 16u) | ((cw >> 18) & 64u) | 0x88u;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t c = (cw >> (8 * j)) & 0xFFu;
                    if (real && c < (uint32_t)CODE_NONE) dbacc[r] += v[j];
                }
                // per byte (c >> 1): 0 / 1 = the routed row parity, 2 = ReLU-blocked (CODE_NONE): never a row
                const uint32_t rowp = (cw >> 1) & 0x7F7F7F7Fu;
                uint32_t H[2], Lw[2];
#pragma unroll
                for (int jp = 0; jp < 2; ++jp) {
                    const float a = v[2 * jp] * dsc, bb = v[2 * jp + 1] * dsc;
                    const _Float16 ha = (_Float16)a, hb = (_Float16)bb;
                    const _Float16 la = (_Float16)(a - (float)ha), lb = (_Float16)(bb - (float)hb);
                    H[jp] = __builtin_bit_cast(uint32_t, f16x2{ha, hb});
                    Lw[jp] = __builtin_bit_cast(uint32_t, f16x2{la, lb});
                }
#pragma unroll
                for (int d = 0; d < 2; ++d) {
                    // byte j -> 0xFF where window j routes to row parity d; then halves [b0 b0 b1 b1], [b2 b2 b3 b3]
                    // (bytes are 0..2, so bits 0-1 decide; the shift's carry-in from the next byte is masked)
                    const uint32_t z = (d ? (rowp & ~(rowp >> 1)) : ~(rowp | (rowp >> 1))) & 0x01010101u;
                    const uint32_t m8 = z * 0xFFu;
                    const uint32_t mA = __builtin_amdgcn_perm(0u, m8, 0x01010000u), mB = __builtin_amdgcn_perm(0u, m8, 0x03030202u);
                    char* ph = img + X3P_DYOFF + ldo[r][d];
                    *reinterpret_cast<uint2*>(ph) = make_uint2(H[0] & mA, H[1] & mB);
                    *reinterpret_cast<uint2*>(ph + X3P_REC) = make_uint2(Lw[0] & mA, Lw[1] & mB);
                    img[X3P_IDXOFF + ((ldo[r][d] >> 4) << 1) + ((ldo[r][d] >> 3) & 1)] = (char)ib;
                }
            }
        }
    };
    auto store_dy = [&](char* img, bool real) {
#pragma unroll
        for (int r = 0; r < NI; ++r)
            if (r < nit) store_dy1(img, real, r);
        X3Q_TS(trk, 5);
    };

    // B (tr-read) lane bases: lane (gb, qq, pp) of block (s, jb) -> pixel (y, 4 xb + qq), channels 4 pp.. of
    // its ci half; the chunk-slot swizzle (h ^ (x >> 1) & 1) depends on kx + qq only (4 xb is a multiple of 4)
    const int gbl = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    int pb[X3P_STEPS][4], sw[3];
#pragma unroll
    for (int s = 0; s < X3P_STEPS; ++s)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
            const int L = 16 * s + 4 * gbl + jb, y = L / 6, xb = L - (L / 6) * 6;
            pb[s][jb] = (y * A_HW + 4 * xb + qq) * 64 + pp * 8;
        }
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) sw[kx] = (h ^ (((kx + qq) >> 1) & 1)) * 32;
    const int arec = ((lane >> 4) * 64 + (lane & 15)) * 16, aidx = ((lane >> 4) * 64 + (lane & 15)) * 2;

    f32x4 acc[3][4];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int per = (U + nks - 1) / nks;
    const int u0 = min(ks * per, U), u1 = min(u0 + per, U);
    sb0 = u0 / 3;
    const int nsb = u1 > u0 ? (u1 - 1) / 3 - sb0 + 1 : 0;
    for (int j = tid; j < nsb; j += X3P_THREADS) sbt[j] = sd + sx - max(x3_exp(act_amax[sb0 + j]), sx);
    __syncthreads();
    int u = u0;
    if (u < u1) {
        x3_issue_unit_img(act16, u, wave, lane, lds_u32(smem));
        load_dy(u);
        store_dy(smem, true);
        load_dy(min(u + 1, u1 - 1));
    }
    int k = 0;
#pragma unroll 1
    for (; u < u1; ++u, ++k) {
        // this unit's image DMA landed; the dY loads (every wave's last memory instructions, issued after its
        // DMA pieces) may stay in flight
        X3Q_TS(k, 6);
        if ((SLK_X3P_ABL & 1) || nit == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (nit == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else if (nit == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        __syncthreads();  // buffer k&1 complete; buffer (k+1)&1 free
        X3Q_TS(k, 0);
        trk = k;
        const int nx = u + 1, nx2 = u + 2;
        const char* img = smem + (k & 1) * X3P_BUF;
        char* nimg = smem + ((k & 1) ^ 1) * X3P_BUF;
        // half the waves route dY before their MFMAs, half after (the two waves of a SIMD overlap routing with
        // MFMAs); store_dy before the DMA issue (hipcc does not count the asm DMAs)
#if SLK_X3P_PLAN == 0
        const bool dfirst = wave >= 4 && !(SLK_X3P_ABL & 1);
        if (dfirst) store_dy(nimg, nx < u1);
        if (!(SLK_X3P_ABL & 4)) x3_issue_unit_img(act16, min(nx, u1 - 1), wave, lane, lds_u32(nimg));
        if (dfirst) load_dy(min(nx2, u1 - 1));
        auto hook = [&](int) {};
        X3Q_TS(k, 1);
#else
        // plan 1: the next unit's image pieces and dY routing in pieces between this unit's K-steps; the dY
        // loads last (after every DMA piece: the counted vmcnt at the top)
        const char* srch = x3_unit_img_src(act16, min(nx, u1 - 1));
        const uint32_t nl = lds_u32(nimg);
        auto hook = [&](int st) {
            if (st == 0) {
                if (!(SLK_X3P_ABL & 4)) {
                    x3_issue_img_full(srch, wave, lane, nl, 0);
                    x3_issue_img_full(srch, wave, lane, nl, 1);
                }
                if (!(SLK_X3P_ABL & 1)) store_dy1(nimg, nx < u1, 0);
            } else if (st == 1) {
                if (!(SLK_X3P_ABL & 4)) {
                    x3_issue_img_full(srch, wave, lane, nl, 2);
                    x3_issue_img_full(srch, wave, lane, nl, 3);
                    if (wave < 2) x3_issue_img_quarter(srch, wave, lane, nl);
                }
                if (!(SLK_X3P_ABL & 1) && two) store_dy1(nimg, nx < u1, 1);
            } else {
                if (!(SLK_X3P_ABL & 1)) load_dy(min(nx2, u1 - 1));
            }
        };
#endif
        if (!(SLK_X3P_ABL & 2)) {
            if (tgi == 0) x3p_steps<0>(img, pb, sw, arec, aidx, acc, hook);
            else if (tgi == 1) x3p_steps<1>(img, pb, sw, arec, aidx, acc, hook);
            else if (tgi == 2) x3p_steps<2>(img, pb, sw, arec, aidx, acc, hook);
            else x3p_steps<3>(img, pb, sw, arec, aidx, acc, hook);
        } else {
            hook(0);
            hook(1);
            hook(2);
        }
        X3Q_TS(k, 2);
#if SLK_X3P_PLAN == 0
        if (!dfirst && !(SLK_X3P_ABL & 1)) {
            store_dy(nimg, nx < u1);
            load_dy(min(nx2, u1 - 1));
        }
#endif
        X3Q_TS(k, 3);
    }
    X3Q_TS(127, 7);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (clamped) image DMA lands before LDS reuse
    __syncthreads();
    // db partials per item -> LDS; co's 12 items summed in order
    float* dbs = reinterpret_cast<float*>(smem);  // [item = 64 q + co]
#pragma unroll
    for (int r = 0; r < NI; ++r)
        if (r < nit) dbs[(SLK_X3P_STG == 0 ? (r == 0 ? wave : 8 + (wave & 3)) : 3 * ((wave & 1) + 2 * (wave >> 2)) + r) * 64 + lane] = dbacc[r];
    __syncthreads();
    float* slab = slabs + (size_t)ks * (W2_N + C2);
    if (tid < C2) {
        float sum = 0.f;
        for (int q = 0; q < 12; ++q) sum += dbs[q * 64 + tid];
        slab[W2_N + tid] = sum;
    }
    const float us1 = ldexpf(1.f, -sx), us2 = ldexpf(1.f, -sd);
    const int ci = 16 * h + (lane & 15);
    auto write_slab = [&](auto TG) {
        using TT = X3pTaps<decltype(TG)::value>;
#pragma unroll
        for (int t = 0; t < TT::NT; ++t)
#pragma unroll
            for (int mt = TT::mlo(t); mt < TT::mhi(t); ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = 16 * mt + 4 * (lane >> 4) + r;
                    slab[(co * C1 + ci) * 9 + TT::tap(t)] = x3_unscale(acc[t][mt][r], us1, us2);
                }
    };
    if (tgi == 0) write_slab(std::integral_constant<int, 0>{});
    else if (tgi == 1) write_slab(std::integral_constant<int, 1>{});
    else if (tgi == 2) write_slab(std::integral_constant<int, 2>{});
    else write_slab(std::integral_constant<int, 3>{});
}

// ============================================================================ conv1 -> x3 input images
// The client's conv1 + ReLU (src/model_def.py:8-9, the per-pixel FMA order of slk_client.hip's
// conv1_fwd_kernel: taps from 0, then + bias) writing the server's x3 operand directly: per sample, the
// max act (act_amax), then every unit's f16 image in conv2_fwd_pool_x3's act16 layout (per-sample scale
// 2^s, s = x3_exp(max act): bit-identical to the images that kernel writes from the f32 act), and —
// when act != nullptr — the f32 act too. One workgroup per sample; pass 1 (thread = 4 consecutive
// pixels, float4 act stores) computes the maximum, pass 2 recomputes (9 FMAs a value) per (pixel,
// 8-channel chunk) item and splits into the per-sample image (each pixel stored once).
// BITS: also the ReLU mask act > 0 of every cut element, 1 bit each, for the fused client backward in
// conv2_dgrad_x3_kernel<true> (which then reads 2.7 KB a sample instead of recomputing conv1): per
// sample [4 channel groups cg][169 threads t] u32, bit 4 (c & 7) + u of (cg = c >> 3, t) = (act[c][4t + u]
// > 0) — pass 1's thread t packs its own 4 pixels of 8 channels into one word (act >= 0, so its bit
// pattern is nonzero iff act > 0: min(bits, 1) is the mask bit) and writes 4 coalesced words.
constexpr int C1X_T = 256;
constexpr int C1X_G = A_PIX / 4;  // 169 pixel quads
static_assert(RB_SAMPLE == 4 * C1X_G, "bit map layout");
// Round 5: ONE pass. The per-sample scale comes from conv1_cut_bound (max |x| and the weights: no pass
// over the outputs first; act_amax = that bound), so each (pixel, 8-channel chunk) item is computed once:
// conv1 (taps in order from 0, + bias — the FMA order of slk_client.hip's conv1_fwd_kernel), split, one
// 16-B store per plane (lanes on consecutive items: 1 KiB contiguous per store instruction), the optional
// f32 act (the 8 channel planes' words of the pixel), and the ReLU bit map: lane (pixel 4 t + u, chunk cg)
// spreads its 8 bits to 4 cc + u and the four u lanes of a 16-lane row OR them with two swizzles (items
// start at pixel quads: 256 threads per pass, 16 items per row); 2,704 items over 256 threads.
template <bool BITS, bool ACT>
__global__ __launch_bounds__(C1X_T) void conv1_fwd_x3_kernel(const float* __restrict__ x, const float* __restrict__ W1,
                                                             const float* __restrict__ b1, float* __restrict__ act,
                                                             float* __restrict__ act_amax, uint16_t* __restrict__ act16,
                                                             uint32_t* __restrict__ relu_bits) {
    __shared__ float xs[IN_HW * IN_HW];
    __shared__ float red[8];
    __shared__ float ws[C1 * 10];  // [c][9 taps | bias]
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const float* xb = x + (size_t)b * IN_HW * IN_HW;
    for (int i = tid; i < IN_HW * IN_HW / 4; i += C1X_T)
        reinterpret_cast<float4*>(xs)[i] = reinterpret_cast<const float4*>(xb)[i];
    for (int i = tid; i < C1 * 9; i += C1X_T) ws[(i / 9) * 10 + i % 9] = W1[i];
    if (tid < C1) ws[tid * 10 + 9] = b1[tid];
    __syncthreads();
    const float am = conv1_cut_bound(xs, W1, b1, red);
    if (tid == 0) act_amax[b] = am;
    const float sc = ldexpf(1.f, x3_exp(am));
    // c8 = tid & 3 for every item of a thread (the stride 256 is a multiple of 4): its 8 channels' weights
    // stay in registers
    const int c8 = tid & 3;
    float wr[8][10];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < 10; ++k) wr[j][k] = ws[(8 * c8 + j) * 10 + k];
    char* img = reinterpret_cast<char*>(act16) + (size_t)b * X3S_SAMPLE;
    float* actb = ACT ? act + (size_t)b * A_SAMPLE : nullptr;
#pragma unroll 2
    for (int i = tid; i < A_PIX * 4; i += C1X_T) {
        const int p = i >> 2;
        const int y = p / A_HW, xx = p - (p / A_HW) * A_HW;
        float xw[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) xw[k] = xs[(y + k / 3) * IN_HW + xx + k % 3];
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float sum = 0.f;
#pragma unroll
            for (int k = 0; k < 9; ++k) sum = fmaf(xw[k], wr[j][k], sum);
            sum += wr[j][9];
            v[j] = sum > 0.f ? sum : 0.f;
        }
        if constexpr (ACT) {
#pragma unroll
            for (int j = 0; j < 8; ++j) actb[(8 * c8 + j) * A_PIX + p] = v[j];
        }
        if constexpr (BITS) {
            // bit 4 cc + u of word (cg = c8, t = p >> 2) = v[cc] > 0 (v >= +0: nonzero bits iff > 0)
            const int u = p & 3;
            uint32_t w = 0u;
#pragma unroll
            for (int j = 0; j < 8; ++j) w |= min(__float_as_uint(v[j]), 1u) << (4 * j);
            w <<= u;
            // OR over the row's lanes of the same chunk: lane ^ 4, lane ^ 8 (ds_swizzle bit mode, xor)
            w |= (uint32_t)__builtin_amdgcn_ds_swizzle((int)w, (4 << 10) | 0x1F);
            w |= (uint32_t)__builtin_amdgcn_ds_swizzle((int)w, (8 << 10) | 0x1F);
            if (u == 0) relu_bits[(size_t)b * RB_SAMPLE + c8 * C1X_G + (p >> 2)] = w;
        }
        f16x8 hh, ll;
        x3_split8(v, sc, hh, ll);
        char* o = img + p * 64 + (c8 ^ (xx & 2)) * 16;
        *reinterpret_cast<f16x8*>(o) = hh;
        *reinterpret_cast<f16x8*>(o + X3S_PLANE) = ll;
    }
}

// ============================================================================ codec -> x3 input images
// The server side of the compressed cut exchange (slk_codec.hip) writing conv2's x3 operand directly: a
// micro-batch's received mask + values + word ranks (slk_cut_ranks) and the shipped per-sample scale value
// become the act16 images the client's conv1_fwd_x3 would have written (the same f32 values split at the
// same 2^x3_exp(amax): bit for bit), with no dense f32 cut in HBM. One workgroup per sample: its 676 mask
// words and ranks staged in LDS; item (pixel p, chunk c8) gathers its 8 channels' values (element
// c * 676 + p of the sample; unset elements are +0) and stores 16 B per plane, as conv1_fwd_x3.
// parts (optional): a device table [np][3] of (vals, mask, ranks) pointers, part_b samples each (one launch for
// a dist.Hub chunk: one part per client)
__global__ __launch_bounds__(C1X_T) void cut_unpack_x3_kernel(const float* __restrict__ vals,
                                                              const uint32_t* __restrict__ mask,
                                                              const int* __restrict__ ranks,
                                                              const float* __restrict__ amax,
                                                              uint16_t* __restrict__ act16,
                                                              const uint64_t* __restrict__ parts = nullptr,
                                                              int part_b = 0) {
    constexpr int NW = A_SAMPLE / 32;  // 676 mask words per sample
    __shared__ uint32_t sm[NW];
    __shared__ int sr[NW];
    const int b = blockIdx.x, tid = threadIdx.x;
    int lb = b;
    if (parts != nullptr) {
        const int part = b / part_b;
        lb = b - part * part_b;
        vals = reinterpret_cast<const float*>(parts[3 * part]);
        mask = reinterpret_cast<const uint32_t*>(parts[3 * part + 1]);
        ranks = reinterpret_cast<const int*>(parts[3 * part + 2]);
    }
    for (int i = tid; i < NW; i += C1X_T) {
        sm[i] = mask[(size_t)lb * NW + i];
        sr[i] = ranks[(size_t)lb * NW + i];
    }
    __syncthreads();
    const float sc = ldexpf(1.f, x3_exp(amax[b]));
    const int c8 = tid & 3;
    char* img = reinterpret_cast<char*>(act16) + (size_t)b * X3S_SAMPLE;
    // one item at a time: fewer registers, more resident waves to cover the gathers (unrolled by 2:
    // 0.274 vs 0.241 ms per 7,168 samples; by 4: 0.254, 6: 0.248)
#pragma unroll 1
    for (int i = tid; i < A_PIX * 4; i += C1X_T) {
        const int p = i >> 2, xx = p - (p / A_HW) * A_HW;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int e = (8 * c8 + j) * A_PIX + p, w = e >> 5, bit = e & 31;
            const uint32_t m = sm[w];
            v[j] = 0.f;
            if ((m >> bit) & 1u) v[j] = vals[(size_t)sr[w] + __popc(m & ((1u << bit) - 1u))];
        }
        f16x8 hh, ll;
        x3_split8(v, sc, hh, ll);
        char* o = img + p * 64 + (c8 ^ (xx & 2)) * 16;
        *reinterpret_cast<f16x8*>(o) = hh;
        *reinterpret_cast<f16x8*>(o + X3S_PLANE) = ll;
    }
}

extern "C" int slk_cut_unpack_x3(const float* vals, const uint32_t* mask, const int* ranks, const float* act_amax,
                                 int B, uint16_t* act16, void* stream) {
    SLK_CHECK_ARG(B >= 0 && (int64_t)B * A_SAMPLE <= 2147483647LL);
    if (B == 0) return 0;
    SLK_CHECK_ARG(vals && mask && ranks && act_amax && act16);
    hipLaunchKernelGGL(cut_unpack_x3_kernel, dim3(B), dim3(C1X_T), 0, slk_stream(stream), vals, mask, ranks, act_amax,
                       act16, nullptr, 0);
    return slk_launch_status();
}

// all parts of a chunk in one launch: parts = device table [B / part_b][3] of (vals, mask, ranks) pointers
extern "C" int slk_cut_unpack_x3_parts(const uint64_t* parts, int part_b, const float* act_amax, int B, uint16_t* act16,
                                       void* stream) {
    SLK_CHECK_ARG(B >= 0 && part_b > 0 && B % part_b == 0 && (int64_t)part_b * A_SAMPLE <= 2147483647LL);
    if (B == 0) return 0;
    SLK_CHECK_ARG(parts && act_amax && act16);
    hipLaunchKernelGGL(cut_unpack_x3_kernel, dim3(B), dim3(C1X_T), 0, slk_stream(stream), nullptr, nullptr, nullptr,
                       act_amax, act16, parts, part_b);
    return slk_launch_status();
}

// ============================================================================ C-ABI
// ============================================================================ box probe (measurement only)
// The sustained dense f16 MFMA rate of THIS device (boxes of the pool differ by several per cent in clocks
// under load): every wave issues 6 independent v_mfma_f32_16x16x32_f16 chains on varied nonzero operands
// (the MFMA's power, and so the clock it sustains, depends on the data), 2 waves per SIMD on every CU.
// bench.py reports the kernels' fractions of this next to the nominal 2.5 PF/s. FLOPs per launch:
// blocks x 4 waves x iters x 6 x 16,384.
__global__ __launch_bounds__(256) void mfma_probe_kernel(float* __restrict__ out, int iters) {
    const int tid = threadIdx.x;
    f16x8 a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = (_Float16)((float)((tid * 13 + j * 7 + blockIdx.x) % 97) / 97.f - 0.5f);
        b[j] = (_Float16)((float)((tid * 29 + j * 11) % 89) / 89.f - 0.5f);
    }
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0;
    // the MFMAs as asm on VGPR accumulators: through the builtin, hipcc rotated the chains through
    // AGPR <-> VGPR copies inside the loop (a probe of the copies, not of the MFMA pipe); each chain's next
    // MFMA is 6 instructions later, far past any dependency wait
    for (int i = 0; i < iters; ++i)
        asm volatile(
            "v_mfma_f32_16x16x32_f16 %0, %6, %7, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %1, %6, %7, %1\n\t"
            "v_mfma_f32_16x16x32_f16 %2, %6, %7, %2\n\t"
            "v_mfma_f32_16x16x32_f16 %3, %6, %7, %3\n\t"
            "v_mfma_f32_16x16x32_f16 %4, %6, %7, %4\n\t"
            "v_mfma_f32_16x16x32_f16 %5, %6, %7, %5"
            : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5)
            : "v"(a), "v"(b));
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // the last MFMAs' results settle before VALU reads them
    const f32x4 t4 = ((c0 + c1) + (c2 + c3)) + (c4 + c5);
    out[blockIdx.x * 256 + tid] = (t4[0] + t4[1]) + (t4[2] + t4[3]);
}

extern "C" int slk_mfma_probe_blocks() { return 2 * X3F_GRID; }  // 2 workgroups of 4 waves per CU

extern "C" int slk_mfma_probe(float* out, int iters, void* stream) {
    SLK_CHECK_ARG(out && iters > 0);
    hipLaunchKernelGGL(mfma_probe_kernel, dim3(2 * X3F_GRID), dim3(256), 0, slk_stream(stream), out, iters);
    return slk_launch_status();
}

extern "C" int slk_row_amax(const float* x, int rows, int n, float* amax, void* stream) {
    SLK_CHECK_ARG(rows >= 0 && n > 0 && (rows == 0 || (x && amax)));
    if (rows == 0) return 0;
    hipLaunchKernelGGL(row_amax_kernel, dim3(rows), dim3(256), 0, slk_stream(stream), x, n, amax);
    return slk_launch_status();
}

extern "C" int slk_conv2_fwd_pool_x3s(const float* act, const float* act_amax, const float* W2, const float* b2,
                                      float* pooled, uint8_t* code, uint16_t* act16, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && act && act_amax && W2 && b2 && pooled && code && act16);
    if (B == 0) return 0;
    const int U = 3 * B;
    hipLaunchKernelGGL(conv2_fwd_pool_x3_kernel<false>, dim3(U < X3F_GRID ? U : X3F_GRID), dim3(X3F_THREADS), 0,
                       slk_stream(stream), act, act_amax, W2, b2, pooled, code, B, act16);
    return slk_launch_status();
}
// the same with the per-sample max |act| computed in the kernel (written to act_amax) instead of read
extern "C" int slk_conv2_fwd_pool_x3sa(const float* act, float* act_amax, const float* W2, const float* b2,
                                       float* pooled, uint8_t* code, uint16_t* act16, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && act && act_amax && W2 && b2 && pooled && code && act16);
    if (B == 0) return 0;
    SLK_CHECK_ARG((reinterpret_cast<size_t>(act) & 15) == 0);
    const int G = B < X3F_GRID ? B : X3F_GRID;
    hipLaunchKernelGGL((conv2_fwd_pool_x3_kernel<false, true>), dim3(G), dim3(X3F_THREADS), 0, slk_stream(stream),
                       act, nullptr, W2, b2, pooled, code, B, act16, act_amax);
    return slk_launch_status();
}
extern "C" int64_t slk_conv2_act16_bytes(int B) { return B > 0 ? (int64_t)B * X3S_SAMPLE : 0; }

extern "C" int slk_conv2_fwd_pool_x3(const float* act, const float* act_amax, const float* W2, const float* b2,
                                     float* pooled, uint8_t* code, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && act && act_amax && W2 && b2 && pooled && code);
    if (B == 0) return 0;
    const int U = 3 * B;
    hipLaunchKernelGGL(conv2_fwd_pool_x3_kernel<false>, dim3(U < X3F_GRID ? U : X3F_GRID), dim3(X3F_THREADS), 0,
                       slk_stream(stream), act, act_amax, W2, b2, pooled, code, B, nullptr);
    return slk_launch_status();
}

extern "C" int slk_conv2_fwd_pool_x3i(const uint16_t* act16, const float* act_amax, const float* W2, const float* b2,
                                      float* pooled, uint8_t* code, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && act16 && act_amax && W2 && b2 && pooled && code);
    if (B == 0) return 0;
    const int U = 3 * B;
    hipLaunchKernelGGL(conv2_fwd_pool_x3_kernel<true>, dim3(U < X3F_GRID ? U : X3F_GRID), dim3(X3F_THREADS), 0,
                       slk_stream(stream), nullptr, act_amax, W2, b2, pooled, code, B, const_cast<uint16_t*>(act16));
    return slk_launch_status();
}

extern "C" int slk_conv1_fwd_x3(const float* x, const float* W1, const float* b1, float* act, float* act_amax,
                                uint16_t* act16, uint32_t* relu_bits, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && (B == 0 || (x && W1 && b1 && act_amax && act16)));
    if (B == 0) return 0;
    const dim3 g(B), t(C1X_T);
    if (relu_bits && act)
        hipLaunchKernelGGL((conv1_fwd_x3_kernel<true, true>), g, t, 0, slk_stream(stream), x, W1, b1, act, act_amax, act16, relu_bits);
    else if (relu_bits)
        hipLaunchKernelGGL((conv1_fwd_x3_kernel<true, false>), g, t, 0, slk_stream(stream), x, W1, b1, act, act_amax, act16, relu_bits);
    else if (act)
        hipLaunchKernelGGL((conv1_fwd_x3_kernel<false, true>), g, t, 0, slk_stream(stream), x, W1, b1, act, act_amax, act16, relu_bits);
    else
        hipLaunchKernelGGL((conv1_fwd_x3_kernel<false, false>), g, t, 0, slk_stream(stream), x, W1, b1, act, act_amax, act16, relu_bits);
    return slk_launch_status();
}
extern "C" int64_t slk_relu_bits_bytes(int B) { return B > 0 ? (int64_t)B * RB_SAMPLE * 4 : 0; }

extern "C" int slk_conv2_dgrad_x3(const float* dpooled, const float* dp_amax, const uint8_t* code, const float* W2,
                                  float* cut_grad, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && dpooled && dp_amax && code && W2 && cut_grad);
    if (B == 0) return 0;
    const int P = 3 * B;
    hipLaunchKernelGGL(conv2_dgrad_x3_kernel<false>, dim3(P < X3D_GRID ? P : X3D_GRID), dim3(X3D_THREADS), 0,
                       slk_stream(stream), dpooled, dp_amax, code, W2, cut_grad, B, nullptr, nullptr, nullptr);
    return slk_launch_status();
}

// the cut gradient in the codec's packed form (conv2_dgrad_x3_kernel's PACK note): values of the elements set
// in `mask` (the received cut's, B samples from element 0) at their ranks (slk_cut_ranks)
extern "C" int slk_conv2_dgrad_x3_pack(const float* dpooled, const float* dp_amax, const uint8_t* code, const float* W2,
                                       const uint32_t* mask, const int* ranks, float* vals, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && (int64_t)B * A_SAMPLE <= 2147483647LL);
    if (B == 0) return 0;
    SLK_CHECK_ARG(dpooled && dp_amax && code && W2 && mask && ranks && vals);
    const int P = 3 * B;
    hipLaunchKernelGGL(conv2_dgrad_x3_kernel<false>, dim3(P < X3D_GRID ? P : X3D_GRID), dim3(X3D_THREADS), 0,
                       slk_stream(stream), dpooled, dp_amax, code, W2, nullptr, B, nullptr, nullptr, nullptr, mask, ranks,
                       vals);
    return slk_launch_status();
}

// all parts of a chunk in one launch: parts = device table [B / part_b][3] of (mask, ranks, vals) pointers
extern "C" int slk_conv2_dgrad_x3_pack_parts(const float* dpooled, const float* dp_amax, const uint8_t* code,
                                             const float* W2, const uint64_t* parts, int part_b, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && part_b > 0 && B % part_b == 0 && (int64_t)part_b * A_SAMPLE <= 2147483647LL);
    if (B == 0) return 0;
    SLK_CHECK_ARG(dpooled && dp_amax && code && W2 && parts);
    const int P = 3 * B;
    hipLaunchKernelGGL(conv2_dgrad_x3_kernel<false>, dim3(P < X3D_GRID ? P : X3D_GRID), dim3(X3D_THREADS), 0,
                       slk_stream(stream), dpooled, dp_amax, code, W2, nullptr, B, nullptr, nullptr, nullptr, nullptr,
                       nullptr, nullptr, parts, part_b);
    return slk_launch_status();
}

extern "C" int slk_conv2_dgrad_x3_c1w_nslab(int B) { return B <= 0 ? 0 : (3 * B < X3D_GRID ? 3 * B : X3D_GRID); }

extern "C" int slk_conv2_dgrad_x3_c1w(const float* dpooled, const float* dp_amax, const uint8_t* code, const float* W2,
                                      const float* x, const uint32_t* relu_bits, float* client_slabs, int B,
                                      void* stream) {
    SLK_CHECK_ARG(B >= 0 && (B == 0 || (dpooled && dp_amax && code && W2 && x && relu_bits && client_slabs)));
    if (B == 0) return 0;
    const int P = 3 * B;
    hipLaunchKernelGGL(conv2_dgrad_x3_kernel<true>, dim3(P < X3D_GRID ? P : X3D_GRID), dim3(X3D_THREADS), 0,
                       slk_stream(stream), dpooled, dp_amax, code, W2, nullptr, B, x, relu_bits, client_slabs);
    return slk_launch_status();
}

// round 5: the slab count of both x3 wgrad entries is the images kernel's (conv2_wgrad_x3q/x3p: 6 units a
// sample, up to X3Q_NKS shares). The f32-act kernel (3 units a sample) keeps its own share count min(3B,
// X3W_NKS) x 2 co halves (round 6, ADVICE r5: with the images kernel's count over half its shares were empty
// below B = 86 and it launched 512 one-per-CU workgroups); the slabs past its shares are zeroed.
extern "C" int slk_conv2_wgrad_x3_nslab(int B) { return B <= 0 ? 0 : (6 * B < X3Q_NKS ? 6 * B : X3Q_NKS); }

extern "C" int slk_conv2_wgrad_x3(const float* act, const float* act_amax, const float* dpooled, const float* dp_amax,
                                  const uint8_t* code, float* slabs, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && act && act_amax && dpooled && dp_amax && code && slabs);
    if (B == 0) return 0;
    const int nslab = slk_conv2_wgrad_x3_nslab(B);
#ifndef SLK_X3W_F32NKS
#define SLK_X3W_F32NKS 1  // 0: the round-5 launch (nslab shares), kept for the A/B
#endif
    const int nks = SLK_X3W_F32NKS ? (3 * B < X3W_NKS ? 3 * B : X3W_NKS) : nslab;  // one slab per K share
    if (nks < nslab) {
        const hipError_t e = hipMemsetAsync(slabs + (size_t)nks * (W2_N + C2), 0,
                                            sizeof(float) * (size_t)(nslab - nks) * (W2_N + C2), slk_stream(stream));
        if (e != hipSuccess) return (int)e;
    }
    hipLaunchKernelGGL(conv2_wgrad_x3_kernel<false>, dim3(2 * nks), dim3(X3W_THREADS), 0, slk_stream(stream), act,
                       act_amax, dpooled, dp_amax, code, slabs, B, nullptr);
    return slk_launch_status();
}

extern "C" int slk_conv2_wgrad_x3_form() { return SLK_X3W_ROUND4 ? 0 : (SLK_X3W_SPARSE ? 2 : 1); }

extern "C" int slk_conv2_wgrad_x3s(const uint16_t* act16, const float* act_amax, const float* dpooled,
                                   const float* dp_amax, const uint8_t* code, float* slabs, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && act16 && act_amax && dpooled && dp_amax && code && slabs);
    if (B == 0) return 0;
    const int nks = slk_conv2_wgrad_x3_nslab(B);
#if SLK_X3W_ROUND4  // profiling A/B: the round-4 kernel (one co half per workgroup, 8-row units)
    hipLaunchKernelGGL(conv2_wgrad_x3_kernel<true>, dim3(2 * nks), dim3(X3W_THREADS), 0, slk_stream(stream), nullptr,
                       act_amax, dpooled, dp_amax, code, slabs, B, act16);
#elif SLK_X3W_SPARSE  // round 6: the 2:4-sparse MFMA form (conv2_wgrad_x3p_kernel)
    if (((3 * B + nks - 1) / nks) / 3 + 2 > X3P_SBN) {  // a K share's samples exceed the LDS scale table
        hipLaunchKernelGGL(conv2_wgrad_x3q_kernel, dim3(nks), dim3(X3Q_THREADS), 0, slk_stream(stream), act16, act_amax,
                           dpooled, dp_amax, code, slabs, B);
        return slk_launch_status();
    }
    hipLaunchKernelGGL(conv2_wgrad_x3p_kernel, dim3(nks), dim3(X3P_THREADS), 0, slk_stream(stream), act16, act_amax,
                       dpooled, dp_amax, code, slabs, B);
#else
    hipLaunchKernelGGL(conv2_wgrad_x3q_kernel, dim3(nks), dim3(X3Q_THREADS), 0, slk_stream(stream), act16, act_amax,
                       dpooled, dp_amax, code, slabs, B);
#endif
    return slk_launch_status();
}
