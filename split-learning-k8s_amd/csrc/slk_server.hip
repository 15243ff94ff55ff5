// slk_server.hip — server stage (ModelPartB, src/model_def.py:15-28; step src/server_part.py:25-58)
// for gfx950 / MI355X.
//
// conv2 is 97.95 % of the step's FLOPs, so its three products run on the f32-input MFMA
// (v_mfma_f32_32x32x2_f32 / v_mfma_f32_16x16x4_f32: exact f32, k-ordered fma chains, the same
// 157 TF/s peak as the f32 VALU but one VGPR per operand per lane and a free VALU for epilogues):
//
//   conv2_fwd_pool : implicit GEMM  M = 576 px/sample, N = 64 co, K = 288;  epilogue fuses bias,
//                    ReLU and the 2x2 max-pool (first max wins, as torch CPU) -> pooled + code.
//   conv2_dgrad    : implicit GEMM  M = 32 ci, N = 676 px/sample, K = 576;   the cut gradient.
//   conv2_wgrad    : GEMM           M = 64 co, N = 288, K = 576 px x B;      slab per workgroup.
//
// Operands are staged per sample (or per half / band of a sample) in LDS so that every MFMA operand
// read is a ds_read_b32 with a per-lane base and a compile-time immediate offset. The reduction
// orders (K orders) are chosen so both lane halves of a 32x32x2 MFMA read with one base register.
//
// The fc1 / cross-entropy head is tiny (0.6 % of FLOPs) and HBM/L2-bound: VALU kernels.
#include "slk_common.h"

using namespace slk;

// ============================================================================ conv2 forward + pool
// One workgroup per sample, 6 waves. The sample's K = 288 is processed as two channel halves
// (ci 0-15, 16-31) so LDS = 16x676 image + 72x2x64 weights = 80,128 B -> two workgroups per CU, one
// staging while the other computes.
// K order inside a half: step s = tap*8 + ci_lo (72 steps), lane half h picks ci = 16*hc + ci_lo + 8h.
// Pixel tile = 32 pixels = 8 pooling windows x 4 (window-major), so after the MFMA each lane holds
// the 4 pixels of a pooling window in 4 consecutive accumulator registers: pooling is in-register.
constexpr int C2F_WAVES = 6;
constexpr int C2F_THREADS = C2F_WAVES * 64;
constexpr int C2F_IMG = 16 * A_PIX;        // 10816 floats
constexpr int C2F_W = 72 * 2 * 64;         // 9216 floats
constexpr int C2F_TILES_PER_WAVE = 6;      // 18 pixel tiles x 2 co tiles / 6 waves

__global__ __launch_bounds__(C2F_THREADS, 3) void conv2_fwd_pool_kernel(
    const float* __restrict__ act, const float* __restrict__ W2, const float* __restrict__ b2,
    float* __restrict__ pooled, uint8_t* __restrict__ code) {
    __shared__ __attribute__((aligned(16))) float smem[C2F_IMG + C2F_W];
    float* img = smem;
    float* w2s = smem + C2F_IMG;

    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, j = lane & 31;
    const int ct = wave & 1;                       // co tile (32 channels)
    const int pt0 = (wave >> 1) * C2F_TILES_PER_WAVE;  // first pixel tile of this wave

    int pbase[C2F_TILES_PER_WAVE];
#pragma unroll
    for (int t = 0; t < C2F_TILES_PER_WAVE; ++t) {
        const int win = 8 * (pt0 + t) + (j >> 2);
        const int py = win / P_HW, px = win - (win / P_HW) * P_HW;
        const int q = j & 3;
        const int oy = 2 * py + (q >> 1), ox = 2 * px + (q & 1);
        pbase[t] = h * 8 * A_PIX + oy * A_HW + ox;
    }
    f32x16 acc[C2F_TILES_PER_WAVE];
#pragma unroll
    for (int t = 0; t < C2F_TILES_PER_WAVE; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

    const float* ab = act + (size_t)b * A_SAMPLE;
#pragma unroll 1
    for (int hc = 0; hc < 2; ++hc) {
        if (hc) __syncthreads();
        // image half: contiguous 16 x 676 floats
        const float4* src = reinterpret_cast<const float4*>(ab + hc * C2F_IMG);
        for (int i = tid; i < C2F_IMG / 4; i += C2F_THREADS) reinterpret_cast<float4*>(img)[i] = src[i];
        // weight half, re-laid as [s][h][co]
        for (int e = tid; e < C2 * 144; e += C2F_THREADS) {
            const int co = e / 144, r = e - co * 144;
            const int ci_l = r / 9, tap = r - ci_l * 9;
            const int s = tap * 8 + (ci_l & 7);
            w2s[(s * 2 + (ci_l >> 3)) * 64 + co] = W2[co * K2 + hc * 144 + r];
        }
        __syncthreads();
        const float* wl = w2s + h * 64 + ct * 32 + j;
#pragma unroll 1
        for (int tap = 0; tap < 9; ++tap) {
            const int ky = tap / 3, kx = tap - (tap / 3) * 3;
            const int toff = ky * A_HW + kx;
            int tb[C2F_TILES_PER_WAVE];
#pragma unroll
            for (int t = 0; t < C2F_TILES_PER_WAVE; ++t) tb[t] = pbase[t] + toff;
            const float* wt = wl + tap * 8 * 128;
#pragma unroll
            for (int ci_lo = 0; ci_lo < 8; ++ci_lo) {
                const float bv = wt[ci_lo * 128];
#pragma unroll
                for (int t = 0; t < C2F_TILES_PER_WAVE; ++t)
                    acc[t] = mfma32x32x2(img[tb[t] + ci_lo * A_PIX], bv, acc[t]);
            }
        }
    }

    // epilogue: bias + ReLU + 2x2 max-pool (torch CPU order: scan q = 0..3, strict >, first max
    // wins), staged through LDS for coalesced stores.
    __syncthreads();
    float* pl = smem;                                         // [64][144] f32
    uint8_t* cl = reinterpret_cast<uint8_t*>(smem + P_SAMPLE);  // [64][144] u8
    const int co = ct * 32 + j;
    const float bias = b2[co];
#pragma unroll
    for (int t = 0; t < C2F_TILES_PER_WAVE; ++t) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            float m = -__builtin_inff();
            int idx = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float v = acc[t][4 * g + q] + bias;
                v = v > 0.f ? v : 0.f;
                if (v > m) { m = v; idx = q; }
            }
            const int win = 8 * (pt0 + t) + 2 * g + h;
            pl[co * P_WIN + win] = m;
            cl[co * P_WIN + win] = (uint8_t)(m > 0.f ? idx : CODE_NONE);
        }
    }
    __syncthreads();
    float4* pout = reinterpret_cast<float4*>(pooled + (size_t)b * P_SAMPLE);
    for (int i = tid; i < P_SAMPLE / 4; i += C2F_THREADS) pout[i] = reinterpret_cast<const float4*>(pl)[i];
    uint4* cout = reinterpret_cast<uint4*>(code + (size_t)b * P_SAMPLE);
    for (int i = tid; i < P_SAMPLE / 16; i += C2F_THREADS) cout[i] = reinterpret_cast<const uint4*>(cl)[i];
}

// ============================================================================ conv2 dgrad (cut grad)
// g[ci][y][x] = sum_{co,ky,kx} dc[co][y-ky][x-kx] * W2[co][ci][ky][kx], dc = maxpool/relu-routed
// dpooled. One workgroup per sample, 8 waves, K = 576 in 4 chunks of 16 output channels.
// LDS: dc chunk expanded to a zero-bordered 28x28 plane per channel (16 x 784 floats) + the W2 chunk
// as [s][h][ci] (72 x 2 x 32) = 68,608 B -> two workgroups per CU.
// MFMA roles: A = W2 (rows ci, one 32-row tile), B = dc-im2col (cols = 32 consecutive pixels), so
// each lane's accumulator column is one pixel and the stores are 128-B coalesced rows of cut_grad.
constexpr int C2D_WAVES = 8;
constexpr int C2D_THREADS = C2D_WAVES * 64;
constexpr int C2D_PLANE = 28 * 28;
constexpr int C2D_DC = 16 * C2D_PLANE;     // 12544 floats
constexpr int C2D_W = 72 * 2 * 32;         // 4608 floats
constexpr int C2D_NTILE = 22;              // ceil(676 / 32)

template <int NT>
__device__ __forceinline__ void c2d_chunk(const float* __restrict__ dcp, const float* __restrict__ w2d,
                                          const int (&pbase)[3], f32x16 (&acc)[3], int h, int j) {
    const float* wl = w2d + h * 32 + j;
#pragma unroll 1
    for (int co_lo = 0; co_lo < 8; ++co_lo) {
        int cb[NT];
#pragma unroll
        for (int i = 0; i < NT; ++i) cb[i] = pbase[i] + co_lo * C2D_PLANE;
        const float* wc = wl + co_lo * 9 * 64;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int ky = tap / 3, kx = tap % 3;
            const float av = wc[tap * 64];
            const int imm = (2 - ky) * 28 + (2 - kx);
#pragma unroll
            for (int i = 0; i < NT; ++i) acc[i] = mfma32x32x2(av, dcp[cb[i] + imm], acc[i]);
        }
    }
}

__global__ __launch_bounds__(C2D_THREADS, 4) void conv2_dgrad_kernel(
    const float* __restrict__ dpool, const uint8_t* __restrict__ code, const float* __restrict__ W2,
    float* __restrict__ gcut) {
    __shared__ __attribute__((aligned(16))) float smem[C2D_DC + C2D_W];
    float* dcp = smem;
    float* w2d = smem + C2D_DC;

    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, j = lane & 31;
    const int nt = (wave < C2D_NTILE - 2 * C2D_WAVES) ? 3 : 2;  // waves 0-5: 3 tiles, 6-7: 2

    int pbase[3];
    int pix[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int p = 32 * (wave + C2D_WAVES * i) + j;
        pix[i] = p;
        const int pc = p < A_PIX ? p : A_PIX - 1;
        const int y = pc / A_HW, x = pc - (pc / A_HW) * A_HW;
        pbase[i] = h * 8 * C2D_PLANE + y * 28 + x;
    }
    f32x16 acc[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

    // zero the planes once: the 2-wide border stays zero, the interior is rewritten per chunk
    for (int i = tid; i < C2D_DC / 4; i += C2D_THREADS)
        reinterpret_cast<float4*>(dcp)[i] = make_float4(0.f, 0.f, 0.f, 0.f);

    const float* dpb = dpool + (size_t)b * P_SAMPLE;
    const uint8_t* cb = code + (size_t)b * P_SAMPLE;
#pragma unroll 1
    for (int chunk = 0; chunk < 4; ++chunk) {
        __syncthreads();
        // expand dc for 16 channels: each window writes its 2x2 block (value at the routed position)
        for (int e = tid; e < 16 * P_WIN; e += C2D_THREADS) {
            const int col = e / P_WIN, win = e - col * P_WIN;
            const int gi = (chunk * 16 + col) * P_WIN + win;
            const int cd = cb[gi];
            const float v = dpb[gi];
            const int py = win / P_HW, px = win - (win / P_HW) * P_HW;
            float* d = dcp + col * C2D_PLANE + (2 * py + 2) * 28 + 2 * px + 2;
            *reinterpret_cast<float2*>(d) = make_float2(cd == 0 ? v : 0.f, cd == 1 ? v : 0.f);
            *reinterpret_cast<float2*>(d + 28) = make_float2(cd == 2 ? v : 0.f, cd == 3 ? v : 0.f);
        }
        // W2 chunk as [s = co_lo*9 + tap][h = co_l >> 3][ci]
        for (int e = tid; e < 16 * K2; e += C2D_THREADS) {
            const int col = e / K2, r = e - col * K2;
            const int ci = r / 9, tap = r - ci * 9;
            const int s = (col & 7) * 9 + tap;
            w2d[(s * 2 + (col >> 3)) * 32 + ci] = W2[(chunk * 16 + col) * K2 + r];
        }
        __syncthreads();
        if (nt == 3) c2d_chunk<3>(dcp, w2d, pbase, acc, h, j);
        else c2d_chunk<2>(dcp, w2d, pbase, acc, h, j);
    }

    float* gb = gcut + (size_t)b * A_SAMPLE;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i < nt && pix[i] < A_PIX) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int ci = (r & 3) + 8 * (r >> 2) + 4 * h;
                gb[ci * A_PIX + pix[i]] = acc[i][r];
            }
        }
    }
}

// ============================================================================ conv2 wgrad
// dW2[co][ci][tap] = sum_b sum_{y,x} dc[b][co][y][x] * act[b][ci][y+ky][x+kx];  db2[co] = sum dc.
// Work unit = (sample, band of 6 pooled rows). K runs window by window: one 16x16x4 MFMA consumes
// the 4 pixels of one pooling window, and the A operand (dc) is just `code == q ? dpooled : 0`.
// 6 waves; wave w owns co tiles {2(w&1), 2(w&1)+1} and 6 of the 18 (tap, ci-half) column tiles:
// 12 tiles = 48 accumulator registers that persist over every unit the workgroup processes. The
// workgroup then writes one [dW2 | db2] slab; slabs are summed in fixed order by the SGD kernel.
// LDS: act rows of one band (32 x 14 x 26) + dc band as [win][co] + code band = 70,208 B.
constexpr int C2W_WAVES = 6;
constexpr int C2W_THREADS = C2W_WAVES * 64;
constexpr int C2W_ROWS = 14;
constexpr int C2W_CSTR = C2W_ROWS * A_HW;   // 364
constexpr int C2W_IMG = C1 * C2W_CSTR;      // 11648 floats
constexpr int C2W_DSTR = 65;                // dc row stride (floats), padded
constexpr int C2W_CDSTR = 68;               // code row stride (bytes), padded
constexpr int C2W_MAXSLAB = 512;
constexpr int C2W_SLAB = W2_N + C2;         // 18496

__global__ __launch_bounds__(C2W_THREADS, 3) void conv2_wgrad_kernel(
    const float* __restrict__ act, const float* __restrict__ dpool, const uint8_t* __restrict__ code,
    float* __restrict__ slabs, int B) {
    __shared__ __attribute__((aligned(16))) float img[C2W_IMG];
    __shared__ float dcb[72 * C2W_DSTR];
    __shared__ uint8_t cdb[72 * C2W_CDSTR];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int g4 = lane >> 4, c = lane & 15;
    const int cp = wave & 1;            // co tiles 2cp, 2cp+1
    const int ntb = 6 * (wave >> 1);    // column tiles ntb .. ntb+5

    int base[6];
#pragma unroll
    for (int tt = 0; tt < 6; ++tt) {
        const int ntile = ntb + tt, tap = ntile >> 1, chalf = ntile & 1;
        const int ky = tap / 3, kx = tap % 3;
        base[tt] = (chalf * 16 + c) * C2W_CSTR + ((g4 >> 1) + ky) * A_HW + (g4 & 1) + kx;
    }
    f32x4 acc[2][6];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int tt = 0; tt < 6; ++tt) acc[m][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float db_acc = 0.f;

    const int nunit = 2 * B;
#pragma unroll 1
    for (int u = blockIdx.x; u < nunit; u += gridDim.x) {
        const int b = u >> 1, band = u & 1;
        __syncthreads();
        // act rows 12*band .. 12*band+13 of every channel (364 contiguous floats per channel)
        const float* ab = act + (size_t)b * A_SAMPLE + band * 12 * A_HW;
        for (int i = tid; i < C1 * (C2W_CSTR / 4); i += C2W_THREADS) {
            const int ci = i / (C2W_CSTR / 4), r4 = i - ci * (C2W_CSTR / 4);
            reinterpret_cast<float4*>(img + ci * C2W_CSTR)[r4] =
                reinterpret_cast<const float4*>(ab + ci * A_PIX)[r4];
        }
        const float* dpb = dpool + (size_t)b * P_SAMPLE + band * 72;
        const uint8_t* cbb = code + (size_t)b * P_SAMPLE + band * 72;
        for (int e = tid; e < C2 * 72; e += C2W_THREADS) {
            const int co = e / 72, w = e - co * 72;
            dcb[w * C2W_DSTR + co] = dpb[co * P_WIN + w];
            cdb[w * C2W_CDSTR + co] = cbb[co * P_WIN + w];
        }
        __syncthreads();
        if (tid < C2) {  // db2: fixed-order sum over the band's routed windows
            float s = 0.f;
            for (int w = 0; w < 72; ++w)
                s += (cdb[w * C2W_CDSTR + tid] != CODE_NONE) ? dcb[w * C2W_DSTR + tid] : 0.f;
            db_acc += s;
        }
#pragma unroll 1
        for (int pyl = 0; pyl < 6; ++pyl) {
            const float* dr = dcb + pyl * P_HW * C2W_DSTR + cp * 32 + c;
            const uint8_t* cr = cdb + pyl * P_HW * C2W_CDSTR + cp * 32 + c;
            const float* ir = img + 2 * pyl * A_HW;
#pragma unroll
            for (int px = 0; px < P_HW; ++px) {
                float av[2];
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    const float dv = dr[px * C2W_DSTR + m * 16];
                    const int cd = cr[px * C2W_CDSTR + m * 16];
                    av[m] = (cd == g4) ? dv : 0.f;
                }
#pragma unroll
                for (int tt = 0; tt < 6; ++tt) {
                    const float bv = ir[base[tt] + 2 * px];
                    acc[0][tt] = mfma16x16x4(av[0], bv, acc[0][tt]);
                    acc[1][tt] = mfma16x16x4(av[1], bv, acc[1][tt]);
                }
            }
        }
    }

    float* slab = slabs + (size_t)blockIdx.x * C2W_SLAB;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int tt = 0; tt < 6; ++tt) {
            const int ntile = ntb + tt, tap = ntile >> 1, chalf = ntile & 1;
            const int ci = chalf * 16 + c;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = (2 * cp + m) * 16 + g4 * 4 + r;
                slab[co * K2 + ci * 9 + tap] = acc[m][tt][r];
            }
        }
    if (tid < C2) slab[W2_N + tid] = db_acc;
}

extern "C" int slk_conv2_wgrad_nslab(int B) { return B > 0 ? (2 * B < C2W_MAXSLAB ? 2 * B : C2W_MAXSLAB) : 0; }

// ============================================================================ fc1 + cross-entropy
// 4 samples per 256-thread workgroup. MODE bits: 1 = fc forward (logits), 2 = cross-entropy fwd+bwd,
// 4 = fc input gradient (dpooled = dlogits @ W3). W3 (368 KB) is L2/MALL-resident and is re-read
// once per 4 samples per phase; pooled is streamed from HBM once.
constexpr int FC_S = 4;
constexpr int FC_K4 = P_SAMPLE / 4;  // 2304

template <int MODE>
__global__ __launch_bounds__(256) void fc_head_kernel(
    const float* __restrict__ pooled, const float* __restrict__ W3, const float* __restrict__ b3,
    const int64_t* __restrict__ labels, float* __restrict__ logits, float* __restrict__ loss_i,
    float* __restrict__ dlogits, float* __restrict__ dpooled, float grad_scale, int* err_flag, int B) {
    __shared__ float red[4][FC_S * NCLS];
    __shared__ float zl[FC_S][NCLS];
    __shared__ float dl[FC_S][NCLS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b0 = blockIdx.x * FC_S;
    const int ns = min(FC_S, B - b0);
    const float4* W34 = reinterpret_cast<const float4*>(W3);

    if (MODE & 1) {
        float acc[FC_S][NCLS];
#pragma unroll
        for (int s = 0; s < FC_S; ++s)
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) acc[s][jj] = 0.f;
        const float4* P4 = reinterpret_cast<const float4*>(pooled + (size_t)b0 * P_SAMPLE);
        for (int k4 = tid; k4 < FC_K4; k4 += 256) {
            float4 w[NCLS];
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) w[jj] = W34[jj * FC_K4 + k4];
#pragma unroll
            for (int s = 0; s < FC_S; ++s) {
                if (s < ns) {
                    const float4 p = P4[s * FC_K4 + k4];
#pragma unroll
                    for (int jj = 0; jj < NCLS; ++jj)
                        acc[s][jj] = fmaf(p.w, w[jj].w, fmaf(p.z, w[jj].z, fmaf(p.y, w[jj].y, fmaf(p.x, w[jj].x, acc[s][jj]))));
                }
            }
        }
#pragma unroll
        for (int s = 0; s < FC_S; ++s)
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) {
                const float v = wave_sum(acc[s][jj]);
                if (lane == 0) red[wave][s * NCLS + jj] = v;
            }
        __syncthreads();
        if (tid < FC_S * NCLS) {
            const int s = tid / NCLS, jj = tid - s * NCLS;
            const float v = (((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid]) + b3[jj];
            zl[s][jj] = v;
            if (s < ns) logits[(size_t)(b0 + s) * NCLS + jj] = v;
        }
        __syncthreads();
    } else if (MODE & 2) {
        if (tid < FC_S * NCLS) {
            const int s = tid / NCLS, jj = tid - s * NCLS;
            zl[s][jj] = s < ns ? logits[(size_t)(b0 + s) * NCLS + jj] : 0.f;
        }
        __syncthreads();
    }

    if (MODE & 2) {
        if (tid < ns) {
            const int s = tid;
            float z[NCLS];
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) z[jj] = zl[s][jj];
            float m = z[0];
#pragma unroll
            for (int jj = 1; jj < NCLS; ++jj) m = fmaxf(m, z[jj]);
            float se = 0.f;
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) se += expf(z[jj] - m);
            const float lse = m + logf(se);
            const int64_t y = labels[b0 + s];
            const bool ok = (y >= 0 && y < NCLS);
            if (!ok && err_flag) atomicOr(err_flag, 1);
            float yz = 0.f;
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) yz = (jj == y) ? z[jj] : yz;
            const float nanv = __builtin_nanf("");
            loss_i[b0 + s] = ok ? (lse - yz) : nanv;
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) {
                const float g = ok ? (expf(z[jj] - lse) - (jj == y ? 1.f : 0.f)) * grad_scale : nanv;
                dl[s][jj] = g;
                dlogits[(size_t)(b0 + s) * NCLS + jj] = g;
            }
        }
        __syncthreads();
    } else if (MODE & 4) {
        if (tid < FC_S * NCLS) {
            const int s = tid / NCLS, jj = tid - s * NCLS;
            dl[s][jj] = s < ns ? dlogits[(size_t)(b0 + s) * NCLS + jj] : 0.f;
        }
        __syncthreads();
    }

    if (MODE & 4) {
        float4* D4 = reinterpret_cast<float4*>(dpooled + (size_t)b0 * P_SAMPLE);
        for (int k4 = tid; k4 < FC_K4; k4 += 256) {
            float4 w[NCLS];
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) w[jj] = W34[jj * FC_K4 + k4];
#pragma unroll
            for (int s = 0; s < FC_S; ++s) {
                if (s < ns) {
                    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                    for (int jj = 0; jj < NCLS; ++jj) {
                        const float d = dl[s][jj];
                        o.x = fmaf(d, w[jj].x, o.x); o.y = fmaf(d, w[jj].y, o.y);
                        o.z = fmaf(d, w[jj].z, o.z); o.w = fmaf(d, w[jj].w, o.w);
                    }
                    D4[s * FC_K4 + k4] = o;
                }
            }
        }
    }
}

// fc1 weight gradient partials. Grid (36 column blocks of 256, nsplit batch slices). Thread t owns
// column k and sums its slice of the batch in order; db3 comes from column block 0.
constexpr int FCW_MAXSPLIT = 32;
constexpr int FCW_SLAB = W3_N + NCLS;  // 92170
__global__ __launch_bounds__(256) void fc_wgrad_kernel(const float* __restrict__ dlogits,
                                                       const float* __restrict__ pooled,
                                                       float* __restrict__ slabs, int B, int per) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int sp = blockIdx.y;
    const int bs = sp * per, be = min(B, bs + per);
    float acc[NCLS];
#pragma unroll
    for (int jj = 0; jj < NCLS; ++jj) acc[jj] = 0.f;
    for (int b = bs; b < be; ++b) {
        const float p = pooled[(size_t)b * P_SAMPLE + k];
#pragma unroll
        for (int jj = 0; jj < NCLS; ++jj) acc[jj] = fmaf(dlogits[b * NCLS + jj], p, acc[jj]);
    }
    float* slab = slabs + (size_t)sp * FCW_SLAB;
#pragma unroll
    for (int jj = 0; jj < NCLS; ++jj) slab[jj * P_SAMPLE + k] = acc[jj];
    if (blockIdx.x == 0 && threadIdx.x < NCLS) {
        float s = 0.f;
        for (int b = bs; b < be; ++b) s += dlogits[b * NCLS + threadIdx.x];
        slab[W3_N + threadIdx.x] = s;
    }
}

static inline int fcw_per(int B) {
    int ns = (B + 127) / 128;
    if (ns > FCW_MAXSPLIT) ns = FCW_MAXSPLIT;
    if (ns < 1) ns = 1;
    return (B + ns - 1) / ns;
}
extern "C" int slk_fc_wgrad_nslab(int B) {
    if (B <= 0) return 0;
    const int per = fcw_per(B);
    return (B + per - 1) / per;
}

// ============================================================================ C ABI
extern "C" int slk_conv2_fwd_pool(const float* act, const float* W2, const float* b2, float* pooled,
                                  uint8_t* code, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(act && W2 && b2 && pooled && code);
    conv2_fwd_pool_kernel<<<B, C2F_THREADS, 0, slk_stream(stream)>>>(act, W2, b2, pooled, code);
    return slk_launch_status();
}

extern "C" int slk_conv2_dgrad(const float* dpooled, const uint8_t* code, const float* W2,
                               float* cut_grad, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(dpooled && code && W2 && cut_grad);
    conv2_dgrad_kernel<<<B, C2D_THREADS, 0, slk_stream(stream)>>>(dpooled, code, W2, cut_grad);
    return slk_launch_status();
}

extern "C" int slk_conv2_wgrad(const float* act, const float* dpooled, const uint8_t* code,
                               float* slabs, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(act && dpooled && code && slabs);
    conv2_wgrad_kernel<<<slk_conv2_wgrad_nslab(B), C2W_THREADS, 0, slk_stream(stream)>>>(
        act, dpooled, code, slabs, B);
    return slk_launch_status();
}

extern "C" int slk_fc_fwd(const float* pooled, const float* W3, const float* b3, float* logits,
                          int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(pooled && W3 && b3 && logits);
    fc_head_kernel<1><<<(B + FC_S - 1) / FC_S, 256, 0, slk_stream(stream)>>>(
        pooled, W3, b3, nullptr, logits, nullptr, nullptr, nullptr, 0.f, nullptr, B);
    return slk_launch_status();
}

extern "C" int slk_xent_fwd_bwd(const float* logits, const int64_t* labels, float* loss_i,
                                float* dlogits, float grad_scale, int* err_flag, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(logits && labels && loss_i && dlogits);
    fc_head_kernel<2><<<(B + FC_S - 1) / FC_S, 256, 0, slk_stream(stream)>>>(
        nullptr, nullptr, nullptr, labels, const_cast<float*>(logits), loss_i, dlogits, nullptr,
        grad_scale, err_flag, B);
    return slk_launch_status();
}

extern "C" int slk_fc_dgrad(const float* dlogits, const float* W3, float* dpooled, int B,
                            void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(dlogits && W3 && dpooled);
    fc_head_kernel<4><<<(B + FC_S - 1) / FC_S, 256, 0, slk_stream(stream)>>>(
        nullptr, W3, nullptr, nullptr, nullptr, nullptr, const_cast<float*>(dlogits), dpooled, 0.f,
        nullptr, B);
    return slk_launch_status();
}

extern "C" int slk_fc_xent(const float* pooled, const float* W3, const float* b3,
                           const int64_t* labels, float* logits, float* loss_i, float* dlogits,
                           float* dpooled, float grad_scale, int* err_flag, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(pooled && W3 && b3 && labels && logits && loss_i && dlogits && dpooled);
    fc_head_kernel<7><<<(B + FC_S - 1) / FC_S, 256, 0, slk_stream(stream)>>>(
        pooled, W3, b3, labels, logits, loss_i, dlogits, dpooled, grad_scale, err_flag, B);
    return slk_launch_status();
}

extern "C" int slk_fc_wgrad(const float* dlogits, const float* pooled, float* slabs, int B,
                            void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(dlogits && pooled && slabs);
    const int per = fcw_per(B);
    dim3 grid(P_SAMPLE / 256, (B + per - 1) / per);
    fc_wgrad_kernel<<<grid, 256, 0, slk_stream(stream)>>>(dlogits, pooled, slabs, B, per);
    return slk_launch_status();
}
