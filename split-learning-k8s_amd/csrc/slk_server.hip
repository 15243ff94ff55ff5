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
// Persistent: one 12-wave workgroup per CU walks samples blockIdx.x, +gridDim.x, ...
// LDS (160,256 B of the CU's 163,840): W2 resident for the whole launch as [half][s][h][co]
// (73,728 B, loaded once) + the sample image double-buffered by channel halves (2 x 43,264 B). The
// next half is fetched by LDS-DMA (global_load_lds_dwordx4) while the current half is on the MFMAs;
// the end-of-half barrier retires it.
// K order inside a half: step s = tap*8 + ci_lo (72 steps), MFMA lane half h picks ci = 16*hc +
// ci_lo + 8h, so both halves of a 32x32x2 MFMA read with one base register + immediate offsets.
// Pixel tile = 32 pixels = 8 pooling windows x 4; MFMA row i = q + 8g + 4hq (the C/D layout's row
// order) holds window 4hq + g, position q. After the MFMAs a lane (col = co, half h) therefore owns
// the 4 pixels of windows 8p+4h .. 8p+4h+3 in its 16 accumulators: bias, ReLU and the 2x2 max-pool
// are in-register and pooled/code leave as one float4 / one u32 per lane and tile.
// Work split: 18 pixel tiles x 2 co tiles = 36 tasks per sample; wave w owns co tile (w & 1) and
// pixel tiles 3*(w >> 1) + {0, 1, 2}.
constexpr int C2F_WAVES = 12;
constexpr int C2F_THREADS = C2F_WAVES * 64;
constexpr int C2F_IMG = 16 * A_PIX;        // 10816 floats = 43,264 B per channel half
constexpr int C2F_WH = 72 * 2 * 64;        // 9216 floats per half
constexpr int C2F_TPW = 3;                 // pixel tiles per wave
constexpr int C2F_GRID = 256;              // one workgroup per CU (MI355X)
constexpr int C2F_CHUNKS = (C2F_IMG * 4 + 1023) / 1024;  // 43 x 1 KiB LDS-DMA pieces per half

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void c2f_dma_half(const float* __restrict__ src, float* dst, int wave, int lane) {
    // one wave-instruction moves 1 KiB: lane l copies bytes [16l, 16l+16) of the piece
    const char* s = reinterpret_cast<const char*>(src);
    char* d = reinterpret_cast<char*>(dst);
    for (int c = wave; c < C2F_CHUNKS; c += C2F_WAVES) {
        const int off = c * 1024 + lane * 16;
        if (off < C2F_IMG * 4)
            __builtin_amdgcn_global_load_lds((const void*)(s + off), (lds_ptr_t)(d + c * 1024), 16, 0, 0);
    }
}

__global__ __launch_bounds__(C2F_THREADS, 3) void conv2_fwd_pool_kernel(
    const float* __restrict__ act, const float* __restrict__ W2, const float* __restrict__ b2,
    float* __restrict__ pooled, uint8_t* __restrict__ code, int B) {
    __shared__ __attribute__((aligned(16))) float smem[2 * C2F_WH + 2 * C2F_IMG];
    float* w2s = smem;                    // [hc][s][h][co]
    float* imgb = smem + 2 * C2F_WH;      // [2][16][676]

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, j = lane & 31;
    const int ct = wave & 1;
    const int pt0 = (wave >> 1) * C2F_TPW;

    int pbase[C2F_TPW];
#pragma unroll
    for (int t = 0; t < C2F_TPW; ++t) {
        const int g = j >> 3, hq = (j >> 2) & 1, q = j & 3;
        const int win = 8 * (pt0 + t) + 4 * hq + g;
        const int py = win / P_HW, px = win - (win / P_HW) * P_HW;
        const int oy = 2 * py + (q >> 1), ox = 2 * px + (q & 1);
        pbase[t] = h * 8 * A_PIX + oy * A_HW + ox;
    }
    const int co = ct * 32 + j;
    const float bias = b2[co];

    int b = blockIdx.x;
    if (b < B) c2f_dma_half(act + (size_t)b * A_SAMPLE, imgb, wave, lane);
    // W2, once: natural [co][ci][tap] -> [hc][s = tap*8 + (ci_l & 7)][h = ci_l >> 3][co]
    for (int e = tid; e < W2_N; e += C2F_THREADS) {
        const int c = e / K2, r = e - c * K2;
        const int ci = r / 9, tap = r - ci * 9;
        const int hc = ci >> 4, ci_l = ci & 15;
        w2s[hc * C2F_WH + ((tap * 8 + (ci_l & 7)) * 2 + (ci_l >> 3)) * 64 + c] = W2[e];
    }
    __syncthreads();

    int buf = 0;
#pragma unroll 1
    for (; b < B; b += gridDim.x) {
        f32x16 acc[C2F_TPW];
#pragma unroll
        for (int t = 0; t < C2F_TPW; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
#pragma unroll 1
        for (int hc = 0; hc < 2; ++hc) {
            // prefetch the next half (this sample's second half, or the next sample's first)
            const int nb = hc ? b + gridDim.x : b;
            if (nb < B) c2f_dma_half(act + (size_t)nb * A_SAMPLE + (hc ? 0 : C2F_IMG), imgb + (buf ^ 1) * C2F_IMG,
                                     wave, lane);
            const float* img = imgb + buf * C2F_IMG;
            const float* wl = w2s + hc * C2F_WH + h * 64 + ct * 32 + j;
#pragma unroll 1
            for (int tap = 0; tap < 9; ++tap) {
                const int ky = tap / 3, kx = tap - (tap / 3) * 3;
                const int toff = ky * A_HW + kx;
                int tb[C2F_TPW];
#pragma unroll
                for (int t = 0; t < C2F_TPW; ++t) tb[t] = pbase[t] + toff;
                const float* wt = wl + tap * 8 * 128;
#pragma unroll
                for (int ci_lo = 0; ci_lo < 8; ++ci_lo) {
                    const float bv = wt[ci_lo * 128];
#pragma unroll
                    for (int t = 0; t < C2F_TPW; ++t)
                        acc[t] = mfma32x32x2(img[tb[t] + ci_lo * A_PIX], bv, acc[t]);
                }
            }
            __syncthreads();  // all reads of `buf` done; the prefetch into buf^1 has landed
            buf ^= 1;
        }
        // epilogue: bias + ReLU + 2x2 max-pool (torch CPU: scan q = 0..3, strict >, first max wins)
        float* prow = pooled + (size_t)b * P_SAMPLE + co * P_WIN;
        uint8_t* crow = code + (size_t)b * P_SAMPLE + co * P_WIN;
#pragma unroll
        for (int t = 0; t < C2F_TPW; ++t) {
            float m4[4];
            unsigned int c4 = 0;
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
                m4[g] = m;
                c4 |= (unsigned int)(m > 0.f ? idx : CODE_NONE) << (8 * g);
            }
            const int w0 = 8 * (pt0 + t) + 4 * h;
            *reinterpret_cast<float4*>(prow + w0) = make_float4(m4[0], m4[1], m4[2], m4[3]);
            *reinterpret_cast<unsigned int*>(crow + w0) = c4;
        }
    }
}

// ============================================================================ conv2 dgrad (cut grad)
// g[ci][y][x] = sum_{co,ky,kx} dc[co][y-ky][x-kx] * W2[co][ci][ky][kx], dc = max-pool/ReLU-routed
// dpooled (routing code from the forward). Persistent: one 12-wave workgroup per CU.
// LDS: W2 resident as [chunk(8)][s(36)][h][ci] (73,728 B) + dc for 8 output channels expanded into
// zero-bordered 28x28 planes, double-buffered (2 x 25,088 B). K = 576 runs as 8 chunks of 8 channels;
// the next chunk's dpooled/code are loaded into registers before the current chunk's MFMAs and
// written (expanded) into the other buffer after them: one barrier per chunk.
// MFMA roles: A = W2 (rows ci: one 32-row tile), B = dc-im2col (cols = 32 consecutive output
// pixels), k step s = co_lo*9 + tap with lane half h picking channel co_lo + 4h; every operand read
// is a ds_read_b32 with a per-lane base and an immediate offset. Each lane's accumulator column is
// one pixel, so cut_grad leaves in 128-B coalesced rows. 22 pixel tiles (676 -> 704) per sample.
constexpr int C2D_WAVES = 12;
constexpr int C2D_THREADS = C2D_WAVES * 64;
constexpr int C2D_PLANE = 28 * 28;
constexpr int C2D_CO = 8;                        // output channels per chunk
constexpr int C2D_NCHUNK = C2 / C2D_CO;          // 8
constexpr int C2D_DC = C2D_CO * C2D_PLANE;       // 6272 floats per buffer
constexpr int C2D_WC = 36 * 2 * 32;              // 2304 floats of W2 per chunk
constexpr int C2D_NTILE = 22;                    // ceil(676 / 32)
constexpr int C2D_GRID = 256;
constexpr int C2D_STG = (C2D_CO * P_WIN + C2D_THREADS - 1) / C2D_THREADS;  // 2 windows / thread

template <int NT>
__device__ __forceinline__ void c2d_chunk(const float* __restrict__ dcp, const float* __restrict__ wc,
                                          const int (&pbase)[2], f32x16 (&acc)[2]) {
#pragma unroll
    for (int co_lo = 0; co_lo < 4; ++co_lo) {
        // gather this channel's 9 taps of operands, then 9*NT MFMAs back to back
        float av[9], bv[9][NT];
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int ky = tap / 3, kx = tap % 3;
            av[tap] = wc[(co_lo * 9 + tap) * 64];
            const int imm = co_lo * C2D_PLANE + (2 - ky) * 28 + (2 - kx);
#pragma unroll
            for (int i = 0; i < NT; ++i) bv[tap][i] = dcp[pbase[i] + imm];
        }
#if SLK_PIN_PHASES
        __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int i = 0; i < NT; ++i) acc[i] = mfma32x32x2(av[tap], bv[tap][i], acc[i]);
#if SLK_PIN_PHASES
        __builtin_amdgcn_sched_barrier(0);
#endif
    }
}

__global__ __launch_bounds__(C2D_THREADS, 3) void conv2_dgrad_kernel(
    const float* __restrict__ dpool, const uint8_t* __restrict__ code, const float* __restrict__ W2,
    float* __restrict__ gcut, int B) {
    __shared__ __attribute__((aligned(16))) float smem[C2D_NCHUNK * C2D_WC + 2 * C2D_DC];
    float* w2d = smem;
    float* dcb = smem + C2D_NCHUNK * C2D_WC;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, j = lane & 31;
    // waves 0-9: tiles {w, w+12}; waves 10, 11: tile {w} (22 tiles)
    const int nt = (wave + C2D_WAVES < C2D_NTILE) ? 2 : 1;
    int pbase[2], pix[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int p = 32 * (wave + C2D_WAVES * i) + j;
        pix[i] = p;
        const int pc = p < A_PIX ? p : A_PIX - 1;
        const int y = pc / A_HW, x = pc - (pc / A_HW) * A_HW;
        pbase[i] = h * 4 * C2D_PLANE + y * 28 + x;
    }

    // W2 once: [co][ci][tap] -> [chunk = co/8][s = (co%4)*9 + tap][h = (co%8)/4][ci]
    for (int e = tid; e < W2_N; e += C2D_THREADS) {
        const int c = e / K2, r = e - c * K2;
        const int ci = r / 9, tap = r - ci * 9;
        const int cl = c & 7;
        w2d[(c >> 3) * C2D_WC + (((cl & 3) * 9 + tap) * 2 + (cl >> 2)) * 32 + ci] = W2[e];
    }
    for (int i = tid; i < 2 * C2D_DC / 4; i += C2D_THREADS)
        reinterpret_cast<float4*>(dcb)[i] = make_float4(0.f, 0.f, 0.f, 0.f);

    // staging registers: window e = tid + 768*i of the chunk (e < 1152): channel e / 144
    float sv[C2D_STG];
    int sc[C2D_STG];
    auto load_chunk = [&](int bb, int ch) {
#pragma unroll
        for (int i = 0; i < C2D_STG; ++i) {
            const int e = tid + C2D_THREADS * i;
            if (e < C2D_CO * P_WIN && bb < B) {
                const size_t gi = (size_t)bb * P_SAMPLE + ch * C2D_CO * P_WIN + e;
                sv[i] = dpool[gi];
                sc[i] = code[gi];
            }
        }
    };
    auto write_chunk = [&](float* dst) {
#pragma unroll
        for (int i = 0; i < C2D_STG; ++i) {
            const int e = tid + C2D_THREADS * i;
            if (e < C2D_CO * P_WIN) {
                const int col = e / P_WIN, win = e - col * P_WIN;
                const int py = win / P_HW, px = win - (win / P_HW) * P_HW;
                const float v = sv[i];
                const int cd = sc[i];
                float* d = dst + col * C2D_PLANE + (2 * py + 2) * 28 + 2 * px + 2;
                *reinterpret_cast<float2*>(d) = make_float2(cd == 0 ? v : 0.f, cd == 1 ? v : 0.f);
                *reinterpret_cast<float2*>(d + 28) = make_float2(cd == 2 ? v : 0.f, cd == 3 ? v : 0.f);
            }
        }
    };

    int b = blockIdx.x;
    __syncthreads();  // zeroed planes before the first interior write
    load_chunk(b, 0);
    write_chunk(dcb);
    __syncthreads();

    int buf = 0;
    f32x16 acc[2];
#pragma unroll 1
    for (; b < B; b += gridDim.x) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll 1
        for (int ch = 0; ch < C2D_NCHUNK; ++ch) {
            const int nb = (ch + 1 < C2D_NCHUNK) ? b : b + gridDim.x;
            const int nch = (ch + 1 < C2D_NCHUNK) ? ch + 1 : 0;
            load_chunk(nb, nch);
            const float* dcp = dcb + buf * C2D_DC;
            const float* wc = w2d + ch * C2D_WC + h * 32 + j;
            if (nt == 2) c2d_chunk<2>(dcp, wc, pbase, acc);
            else c2d_chunk<1>(dcp, wc, pbase, acc);
            if (nb < B) write_chunk(dcb + (buf ^ 1) * C2D_DC);
            __syncthreads();
            buf ^= 1;
        }
        float* gb = gcut + (size_t)b * A_SAMPLE;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i < nt && pix[i] < A_PIX) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int ci = (r & 3) + 8 * (r >> 2) + 4 * h;
                    gb[ci * A_PIX + pix[i]] = acc[i][r];
                }
            }
        }
    }
}

// ============================================================================ conv2 wgrad
// dW2[co][ci][tap] = sum_b sum_{y,x} dc[b][co][y][x] * act[b][ci][y+ky][x+kx];  db2[co] = sum dc.
// Persistent: one 12-wave workgroup per CU walks work units (sample, band of 6 pooled rows).
// GEMM view: M = 64 co, N = 288 (tap, ci), K = pixels. 32x32x2 MFMAs: a tile is [32 co][32 ci] of
// one tap; a k step is 2 pixels of one pooling window (lane half h: q = 2t + h, t = 0, 1), so the A
// operand (dc) of a lane is `code == q ? dpooled : 0` — the max-pool/ReLU routing applied in the
// operand — and one dc read serves 2 k steps x 3 taps = 6 MFMAs.
// Waves: w = kh + 2*(ct + 2*tg): co tile ct (32 channels), tap group tg (taps 3tg..3tg+2) and
// K half kh (windows of even / odd px). The two K halves of each tile are summed in LDS at the end
// in a fixed order; 48 accumulator registers per wave live across every unit of the launch.
// LDS, double-buffered per unit: act rows 12*band .. 12*band+13 of all 32 channels at an ODD channel
// stride of 369 floats (conflict-free B reads; filled by 4-byte LDS-DMA with per-lane sources) +
// the dc band as [win][co] + code band; the dc band is register-staged (transposed on the LDS
// write). db2 is summed in registers while staging (thread t owns channel t % 64). The workgroup
// writes one [dW2 | db2] slab; slabs are summed in a fixed order by the SGD kernel.
constexpr int C2W_WAVES = 12;
constexpr int C2W_THREADS = C2W_WAVES * 64;
constexpr int C2W_ROWS = 14;
constexpr int C2W_BAND = C2W_ROWS * A_HW;   // 364 floats of one channel per band
constexpr int C2W_CSTR = 369;               // odd LDS channel stride
constexpr int C2W_IMG = C1 * C2W_CSTR;      // 11808 floats = 47,232 B
constexpr int C2W_DSTR = 65;                // dc row stride (floats), padded
constexpr int C2W_CDSTR = 68;               // code row stride (bytes), padded
constexpr int C2W_DC = 72 * C2W_DSTR;       // 4680 floats
constexpr int C2W_CD = 72 * C2W_CDSTR / 4;  // 1224 floats worth of bytes
constexpr int C2W_BUF = C2W_IMG + C2W_DC + C2W_CD;  // 17712 floats = 70,848 B
constexpr int C2W_MAXSLAB = 256;
constexpr int C2W_SLAB = W2_N + C2;         // 18496
constexpr int C2W_PIECES = (C2W_IMG + 63) / 64;  // 185 four-byte LDS-DMA pieces per band
constexpr int C2W_STG = 72 / (C2W_THREADS / C2);  // 6 windows per thread

__device__ __forceinline__ void c2w_dma_band(const float* __restrict__ ab, float* dst, int wave, int lane) {
    for (int c = wave; c < C2W_PIECES; c += C2W_WAVES) {
        const int o = c * 64 + lane;  // LDS float index
        const int ci = o / C2W_CSTR, r = o - ci * C2W_CSTR;
        if (ci < C1 && r < C2W_BAND)
            __builtin_amdgcn_global_load_lds((const void*)(ab + ci * A_PIX + r), (lds_ptr_t)(dst + c * 64), 4, 0, 0);
    }
}

__global__ __launch_bounds__(C2W_THREADS, 3) void conv2_wgrad_kernel(
    const float* __restrict__ act, const float* __restrict__ dpool, const uint8_t* __restrict__ code,
    float* __restrict__ slabs, int B) {
    __shared__ __attribute__((aligned(16))) float smem[2 * C2W_BUF];

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, j = lane & 31;
    const int kh = wave & 1, ct = (wave >> 1) & 1, tg = wave >> 2;

    // B operand base per tap: channel j, window row offset (t + ky), column (h + kx) + 2px
    int base[3];
#pragma unroll
    for (int tt = 0; tt < 3; ++tt) {
        const int tap = 3 * tg + tt, ky = tap / 3, kx = tap % 3;
        base[tt] = j * C2W_CSTR + ky * A_HW + h + kx;
    }
    f32x16 acc[3];
#pragma unroll
    for (int tt = 0; tt < 3; ++tt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[tt][r] = 0.f;

    // dc staging, coalesced: element e = tid + 768*i of the band's [64 co][72 win] block (consecutive
    // lanes = consecutive windows of one channel row); the transpose to [win][co] happens in the LDS
    // write (stride 65 floats / 68 bytes: conflict-free).
    float sv[C2W_STG];
    int sc[C2W_STG];
    float db_acc = 0.f;  // db2 partial: channel (tid & 63), windows 6*(tid >> 6) .. +5 of every band
    const int nunit = 2 * B;
    auto load_dc = [&](int u) {
        if (u < nunit) {
            const int bb = u >> 1, band = u & 1;
            const float* dp0 = dpool + (size_t)bb * P_SAMPLE + band * 72;
            const uint8_t* cd0 = code + (size_t)bb * P_SAMPLE + band * 72;
#pragma unroll
            for (int i = 0; i < C2W_STG; ++i) {
                const int e = tid + C2W_THREADS * i;
                const int co = e / 72, w = e - co * 72;
                sv[i] = dp0[co * P_WIN + w];
                sc[i] = cd0[co * P_WIN + w];
            }
        }
    };
    auto write_dc = [&](float* bufp) {
        float* dcb = bufp + C2W_IMG;
        uint8_t* cdb = reinterpret_cast<uint8_t*>(bufp + C2W_IMG + C2W_DC);
#pragma unroll
        for (int i = 0; i < C2W_STG; ++i) {
            const int e = tid + C2W_THREADS * i;
            const int co = e / 72, w = e - co * 72;
            dcb[w * C2W_DSTR + co] = sv[i];
            cdb[w * C2W_CDSTR + co] = (uint8_t)sc[i];
        }
    };
    auto db_accum = [&](const float* bufp) {  // fixed (channel, windows) per thread: deterministic
        const float* dcb = bufp + C2W_IMG;
        const uint8_t* cdb = reinterpret_cast<const uint8_t*>(bufp + C2W_IMG + C2W_DC);
        const int co = tid & 63, w0 = 6 * (tid >> 6);
#pragma unroll
        for (int k = 0; k < 6; ++k)
            db_acc += (cdb[(w0 + k) * C2W_CDSTR + co] != CODE_NONE) ? dcb[(w0 + k) * C2W_DSTR + co] : 0.f;
    };

    int u = blockIdx.x;
    if (u < nunit) c2w_dma_band(act + (size_t)(u >> 1) * A_SAMPLE + (u & 1) * 12 * A_HW, smem, wave, lane);
    load_dc(u);
    if (u < nunit) write_dc(smem);
    __syncthreads();

    const int q0 = h, q1 = 2 + h;  // pixel of this lane half in k steps t = 0, 1
    int buf = 0;
#pragma unroll 1
    for (; u < nunit; u += gridDim.x) {
        const int nu = u + gridDim.x;
        float* cur = smem + buf * C2W_BUF;
        float* nxt = smem + (buf ^ 1) * C2W_BUF;
        if (nu < nunit) c2w_dma_band(act + (size_t)(nu >> 1) * A_SAMPLE + (nu & 1) * 12 * A_HW, nxt, wave, lane);
        load_dc(nu);
        db_accum(cur);
        const float* img = cur;
        const float* dcb = cur + C2W_IMG;
        const uint8_t* cdb = reinterpret_cast<const uint8_t*>(cur + C2W_IMG + C2W_DC);
#pragma unroll 1
        for (int pyl = 0; pyl < 6; ++pyl) {
            const float* dr = dcb + pyl * P_HW * C2W_DSTR + ct * 32 + j;
            const uint8_t* cr = cdb + pyl * P_HW * C2W_CDSTR + ct * 32 + j;
            const float* ir = img + 2 * pyl * A_HW;
            // this wave's 6 windows of the row (px = 2i + kh): gather, then 36 MFMAs
            float dv[6], bv[6][2][3];
            int cd[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int px = 2 * i + kh;
                dv[i] = dr[px * C2W_DSTR];
                cd[i] = cr[px * C2W_CDSTR];
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int tt = 0; tt < 3; ++tt) bv[i][t][tt] = ir[base[tt] + t * A_HW + 2 * px];
            }
#if SLK_PIN_PHASES
            __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const float a0 = (cd[i] == q0) ? dv[i] : 0.f;
                const float a1 = (cd[i] == q1) ? dv[i] : 0.f;
#pragma unroll
                for (int tt = 0; tt < 3; ++tt) {
                    acc[tt] = mfma32x32x2(a0, bv[i][0][tt], acc[tt]);
                    acc[tt] = mfma32x32x2(a1, bv[i][1][tt], acc[tt]);
                }
            }
#if SLK_PIN_PHASES
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
        if (nu < nunit) write_dc(nxt);
        __syncthreads();
        buf ^= 1;
    }

    // combine: K-half 1 waves park their tiles in LDS, K-half 0 waves add them (fixed order)
    float* park = smem;  // 6 waves x 3 tiles x 16 regs x 64 lanes = 18432 floats
    float* red = smem + 18432;
    const int pw = wave >> 1;  // (ct, tg) pair index 0..5
    if (kh == 1) {
#pragma unroll
        for (int tt = 0; tt < 3; ++tt)
#pragma unroll
            for (int r = 0; r < 16; ++r) park[((pw * 3 + tt) * 16 + r) * 64 + lane] = acc[tt][r];
    }
    red[tid] = db_acc;
    __syncthreads();
    float* slab = slabs + (size_t)blockIdx.x * C2W_SLAB;
    if (tid < C2) {  // the 12 window groups of channel tid, in order
        float s = 0.f;
        for (int k = 0; k < C2W_THREADS / C2; ++k) s += red[k * C2 + tid];
        slab[W2_N + tid] = s;
    }
    if (kh == 0) {
#pragma unroll
        for (int tt = 0; tt < 3; ++tt) {
            const int tap = 3 * tg + tt;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = ct * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                slab[co * K2 + j * 9 + tap] = acc[tt][r] + park[((pw * 3 + tt) * 16 + r) * 64 + lane];
            }
        }
    }
}

extern "C" int slk_conv2_wgrad_direct_nslab(int B) { return B > 0 ? (2 * B < C2W_MAXSLAB ? 2 * B : C2W_MAXSLAB) : 0; }

// ============================================================================ fc1 + cross-entropy
// FCH_S = 16 samples per 512-thread workgroup (B = 4096: one workgroup per CU, one dispatch round).
// MODE bits: 1 = fc forward (logits), 2 = cross-entropy fwd+bwd, 4 = fc input gradient (dpooled =
// dlogits @ W3, + dp_amax = per-sample max |dpooled| when asked).
// Logits on v_mfma_f32_16x16x4_f32 (A = 16 samples x 4 features, B = 4 features x 16 classes, 10 used):
// wave w owns features [1152 w, 1152 (w + 1)) and streams them in 18 chunks of 64 features — the 16
// sample rows and W3's 10 rows of the chunk — by LDS-DMA into its own two slots (no barrier in the
// loop: each wave waits for its own DMA with a counted vmcnt). Rows sit 288 B apart in LDS, so the
// fragment reads (ds_read_b128, lane = (row, 4-feature group)) are conflict-free. W3 crosses L2 once per
// 16 samples: the VALU head this replaces (4 samples per workgroup) re-read all of W3 per 4 samples
// (377 MB of L2 reads per pass at B = 4096) and its logits pass read pooled at 2.7 TB/s.
// dpooled on the VALU: thread = float4 column k4 with W3's 10 float4 of it in registers, every sample's
// row stored as 1-KiB-contiguous wave stores (the 10-term fmaf chain per output, classes in order).
#ifndef SLK_FCH_CK
#define SLK_FCH_CK 64
#endif
#ifndef SLK_FCH_NS
#define SLK_FCH_NS 2
#endif
#ifndef SLK_FCH_S
#define SLK_FCH_S 16  // samples per workgroup (8: 256-thread workgroups, two per CU at B = 4096)
#endif
constexpr int FCH_S = SLK_FCH_S, FCH_T = 32 * FCH_S, FCH_W = FCH_T / 64;
constexpr int FCH_KW = P_SAMPLE / FCH_W;  // 1152 features per wave
constexpr int FCH_CK = SLK_FCH_CK;        // features per chunk (64)
constexpr int FCH_NS = SLK_FCH_NS;        // LDS slots per wave = chunks in flight + 1 (2)
constexpr int FCH_NCH = FCH_KW / FCH_CK;  // 18
constexpr int FCH_ROW = FCH_CK * 4 + 32;  // 288-B LDS rows: (72 s + 4 kg) dwords are 16 distinct 4-bank slots per lane group
constexpr int FCH_A = FCH_S * FCH_ROW;    // 4,608 B of sample rows (4 full DMA pieces + half of a fifth)
constexpr int FCH_PA = (FCH_A + 1023) / 1024, FCH_ALAST = FCH_A - 1024 * (FCH_PA - 1);
constexpr int FCH_PW = (NCLS * FCH_ROW + 1023) / 1024;  // W3 rows (10 x 288 = 2,880 B in 3 DMA pieces)
constexpr int FCH_NDMA = FCH_PA + FCH_PW;               // DMA instructions per chunk (8)
constexpr int FCH_SLOT = FCH_A + FCH_PW * 1024;
constexpr int FCH_U = 64 / FCH_CK;                      // chunks per 64 features (accumulator rotation)
constexpr int FC_K4 = P_SAMPLE / 4;         // 2304 float4 columns
static_assert(P_SAMPLE % FCH_W == 0 && FCH_KW % 64 == 0 && (FCH_CK == 64 || FCH_CK == 32) && FCH_NS >= 2 &&
                  FCH_NS <= 4 && FCH_NCH >= FCH_NS && FCH_ALAST % 16 == 0 && FCH_NDMA * (FCH_NS - 1) <= 63,
              "fc head tiling");

template <int N>
__device__ __forceinline__ void fch_vmwait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int MODE>
__global__ __launch_bounds__(FCH_T, 1) void fc_head16_kernel(
    const float* __restrict__ pooled, const float* __restrict__ W3, const float* __restrict__ b3,
    const int64_t* __restrict__ labels, float* __restrict__ logits, float* __restrict__ loss_i,
    float* __restrict__ dlogits, float* __restrict__ dpooled, float grad_scale, int* err_flag, int B,
    float* __restrict__ dp_amax) {
    __shared__ __attribute__((aligned(1024))) char smem[(MODE & 1) ? FCH_W * FCH_NS * FCH_SLOT : 16];
    __shared__ __attribute__((aligned(16))) f32x4 red[(MODE & 1) ? FCH_W * 64 : 1];
    __shared__ float zl[FCH_S][NCLS];
    __shared__ float dl[FCH_S][NCLS];
    __shared__ float mx[FCH_W][FCH_S];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int s0 = blockIdx.x * FCH_S;
    const int ns = min(FCH_S, B - s0);

    if constexpr ((MODE & 1) != 0) {
        char* const slots = smem + wave * FCH_NS * FCH_SLOT;
        const int kb = wave * FCH_KW;
        // DMA lane offsets: piece j fills slot bytes [1024 j, 1024 j + 1024), lane l the 16 B at
        // X = 1024 j + 16 l = row X / FCH_ROW, byte X % FCH_ROW (pad bytes and rows past the batch: a valid dummy)
        uint32_t va[FCH_PA], vw[FCH_PW];
#pragma unroll
        for (int j = 0; j < FCH_PA; ++j) {
            const int X = 1024 * j + 16 * lane, r = X / FCH_ROW, off = X - (X / FCH_ROW) * FCH_ROW;
            va[j] = (r < FCH_S && off < FCH_CK * 4) ? (uint32_t)(min(r, ns - 1) * P_SAMPLE * 4 + off) : 0u;
        }
#pragma unroll
        for (int j = 0; j < FCH_PW; ++j) {
            const int X = 1024 * j + 16 * lane, r = X / FCH_ROW, off = X - (X / FCH_ROW) * FCH_ROW;
            vw[j] = (r < NCLS && off < FCH_CK * 4) ? (uint32_t)(r * P_SAMPLE * 4 + off) : 0u;
        }
        auto issue = [&](int c) {  // FCH_NDMA DMA instructions per chunk (the last A piece: lanes < FCH_ALAST / 16)
            const uint32_t la = lds_u32(slots + (c % FCH_NS) * FCH_SLOT);
            const float* pa = pooled + (size_t)s0 * P_SAMPLE + kb + c * FCH_CK;
            const float* pw = W3 + kb + c * FCH_CK;
#pragma unroll
            for (int j = 0; j < FCH_PA - 1; ++j) glds16_so(pa, va[j], la + 1024 * j);
            if (lane < FCH_ALAST / 16) glds16_so(pa, va[FCH_PA - 1], la + 1024 * (FCH_PA - 1));
#pragma unroll
            for (int j = 0; j < FCH_PW; ++j) glds16_so(pw, vw[j], la + FCH_A + 1024 * j);
        };
#pragma unroll
        for (int c = 0; c < FCH_NS; ++c) issue(c);
        // A fragment: lane (sample s16, group kg) holds features 16 blk + 4 kg + i; B: lane (class, kg) the
        // same features of W3 row `nrow` (classes 10-15: duplicates, never stored). Accumulator
        // (feature / 16) % 4 for every chunk size, so the sum order (and the result) does not depend on FCH_CK.
        // classes 10-15 (never stored) read W3 rows 2-7: row 9 for all of them put row 9 (72 dwords x 9 = 8 mod
        // 64) on row 1's banks in every ds_read_b128 lane group (0.59 M conflict cycles per launch); with rows
        // 2-7 each 16-lane group's 16 reads hit 16 distinct 4-bank slots (any valid row gives the same classes 0-9)
        const int s16 = lane & 15, kg = lane >> 4, nrow = s16 < NCLS ? s16 : s16 - 8;
        f32x4 acc[4];
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
            acc[blk] = f32x4{0.f, 0.f, 0.f, 0.f};
            slk_keep(acc[blk]);
        }
#pragma unroll 2
        for (int cc = 0; cc < FCH_NCH; cc += FCH_U) {
#pragma unroll
            for (int u = 0; u < FCH_U; ++u) {
                const int c = cc + u, left = FCH_NCH - 1 - c;  // chunks issued after c
                if (left >= FCH_NS - 1) fch_vmwait<FCH_NDMA * (FCH_NS - 1)>();  // chunk c landed
                else if (FCH_NS > 3 && left == 2) fch_vmwait<FCH_NDMA * 2>();
                else if (FCH_NS > 2 && left == 1) fch_vmwait<FCH_NDMA>();
                else fch_vmwait<0>();
                const char* sl = slots + (c % FCH_NS) * FCH_SLOT;
                f32x4 a[FCH_CK / 16], w[FCH_CK / 16];
#pragma unroll
                for (int blk = 0; blk < FCH_CK / 16; ++blk) {
                    a[blk] = *reinterpret_cast<const f32x4*>(sl + s16 * FCH_ROW + 64 * blk + 16 * kg);
                    w[blk] = *reinterpret_cast<const f32x4*>(sl + FCH_A + nrow * FCH_ROW + 64 * blk + 16 * kg);
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read before chunk c + FCH_NS overwrites it
                if (c + FCH_NS < FCH_NCH) issue(c + FCH_NS);
#pragma unroll
                for (int blk = 0; blk < FCH_CK / 16; ++blk)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        acc[u * (FCH_CK / 16) + blk] =
                            __builtin_amdgcn_mfma_f32_16x16x4f32(a[blk][i], w[blk][i], acc[u * (FCH_CK / 16) + blk], 0, 0, 0);
            }
        }
        // D[4 (lane >> 4) + r][lane & 15] = (sample, class) partial over this wave's features
        red[wave * 64 + lane] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        __syncthreads();
        if (tid < 256) {
            const int l = tid & 63, r = tid >> 6, n = l & 15, s = 4 * (l >> 4) + r;
            float v = 0.f;
#pragma unroll
            for (int w = 0; w < FCH_W; ++w) v += red[w * 64 + l][r];
            if (n < NCLS && s < FCH_S) {  // (FCH_S = 8: MFMA rows 8-15 read stand-in rows, never stored)
                v += b3[n];
                zl[s][n] = v;
                if (s < ns) logits[(size_t)(s0 + s) * NCLS + n] = v;
            }
        }
        __syncthreads();
    } else if constexpr ((MODE & 2) != 0) {
        if (tid < FCH_S * NCLS) {
            const int s = tid / NCLS, jj = tid - s * NCLS;
            zl[s][jj] = s < ns ? logits[(size_t)(s0 + s) * NCLS + jj] : 0.f;
        }
        __syncthreads();
    }

    if constexpr ((MODE & 2) != 0) {
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
            const int64_t y = labels[s0 + s];
            const bool ok = (y >= 0 && y < NCLS);
            if (!ok && err_flag) atomicOr(err_flag, 1);
            float yz = 0.f;
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) yz = (jj == y) ? z[jj] : yz;
            const float nanv = __builtin_nanf("");
            loss_i[s0 + s] = ok ? (lse - yz) : nanv;
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) {
                const float g = ok ? (expf(z[jj] - lse) - (jj == y ? 1.f : 0.f)) * grad_scale : nanv;
                dl[s][jj] = g;
                dlogits[(size_t)(s0 + s) * NCLS + jj] = g;
            }
        }
        __syncthreads();
    } else if constexpr ((MODE & 4) != 0) {
        if (tid < FCH_S * NCLS) {
            const int s = tid / NCLS, jj = tid - s * NCLS;
            dl[s][jj] = s < ns ? dlogits[(size_t)(s0 + s) * NCLS + jj] : 0.f;
        }
        __syncthreads();
    }

    if constexpr ((MODE & 4) != 0) {
        const float4* W34 = reinterpret_cast<const float4*>(W3);
        float4* D4 = reinterpret_cast<float4*>(dpooled + (size_t)s0 * P_SAMPLE);
        float dmx[FCH_S];
#pragma unroll
        for (int s = 0; s < FCH_S; ++s) dmx[s] = 0.f;
        for (int k4 = tid; k4 < FC_K4; k4 += FCH_T) {
            // dl stays in LDS (broadcast reads per use): hoisted out of this loop it took 160 VGPRs and spilled
            asm volatile("" ::: "memory");
            float4 w[NCLS];
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) w[jj] = W34[jj * FC_K4 + k4];
#pragma unroll
            for (int s = 0; s < FCH_S; ++s) {
                if (s < ns) {
                    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                    for (int jj = 0; jj < NCLS; ++jj) {
                        const float d = dl[s][jj];  // LDS broadcast
                        o.x = fmaf(d, w[jj].x, o.x);
                        o.y = fmaf(d, w[jj].y, o.y);
                        o.z = fmaf(d, w[jj].z, o.z);
                        o.w = fmaf(d, w[jj].w, o.w);
                    }
                    D4[s * FC_K4 + k4] = o;
                    dmx[s] = fmaxf(dmx[s], fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
                }
            }
        }
        if (dp_amax) {
#pragma unroll
            for (int s = 0; s < FCH_S; ++s) {
                const float v = wave_max(dmx[s]);
                if (lane == 0) mx[wave][s] = v;
            }
            __syncthreads();
            if (tid < ns) {
                float v = mx[0][tid];
#pragma unroll
                for (int w = 1; w < FCH_W; ++w) v = fmaxf(v, mx[w][tid]);
                dp_amax[s0 + tid] = v;
            }
        }
    }
}

// fc1 weight gradient partials. Grid (9 column blocks of 1024, nsplit batch slices). Thread t owns
// the 4 columns 4*(blockIdx.x*256 + t) .. +3 and sums its slice of the batch in order, 8 samples'
// float4 rows in flight; db3 comes from column block 0. dlogits are wave-uniform scalar loads.
#ifndef SLK_FCW_MAXSPLIT
#define SLK_FCW_MAXSPLIT 64
#endif
constexpr int FCW_MAXSPLIT = SLK_FCW_MAXSPLIT;
constexpr int FCW_SLAB = W3_N + NCLS;  // 92170
__global__ __launch_bounds__(256) void fc_wgrad_kernel(const float* __restrict__ dlogits,
                                                       const float* __restrict__ pooled,
                                                       float* __restrict__ slabs, int B, int per) {
    const int k4 = blockIdx.x * 256 + threadIdx.x;  // float4 column index (< 2304)
    const int sp = blockIdx.y;
    const int bs = sp * per, be = min(B, bs + per);
    float4 acc[NCLS];
#pragma unroll
    for (int jj = 0; jj < NCLS; ++jj) acc[jj] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4* P4 = reinterpret_cast<const float4*>(pooled);
    int b = bs;
    for (; b + 8 <= be; b += 8) {
        float4 p[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) p[u] = P4[(size_t)(b + u) * FC_K4 + k4];
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int jj = 0; jj < NCLS; ++jj) {
                const float d = dlogits[(b + u) * NCLS + jj];
                acc[jj].x = fmaf(d, p[u].x, acc[jj].x); acc[jj].y = fmaf(d, p[u].y, acc[jj].y);
                acc[jj].z = fmaf(d, p[u].z, acc[jj].z); acc[jj].w = fmaf(d, p[u].w, acc[jj].w);
            }
    }
    for (; b < be; ++b) {
        const float4 p = P4[(size_t)b * FC_K4 + k4];
#pragma unroll
        for (int jj = 0; jj < NCLS; ++jj) {
            const float d = dlogits[b * NCLS + jj];
            acc[jj].x = fmaf(d, p.x, acc[jj].x); acc[jj].y = fmaf(d, p.y, acc[jj].y);
            acc[jj].z = fmaf(d, p.z, acc[jj].z); acc[jj].w = fmaf(d, p.w, acc[jj].w);
        }
    }
    float* slab = slabs + (size_t)sp * FCW_SLAB;
#pragma unroll
    for (int jj = 0; jj < NCLS; ++jj) reinterpret_cast<float4*>(slab + jj * P_SAMPLE)[k4] = acc[jj];
    if (blockIdx.x == 0 && threadIdx.x < NCLS) {
        float s = 0.f;
        for (int bb = bs; bb < be; ++bb) s += dlogits[bb * NCLS + threadIdx.x];
        slab[W3_N + threadIdx.x] = s;
    }
}

static inline int fcw_per(int B) {
    int ns = (B + 63) / 64;
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
extern "C" int slk_conv2_fwd_pool_direct(const float* act, const float* W2, const float* b2, float* pooled,
                                  uint8_t* code, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(act && W2 && b2 && pooled && code);
    conv2_fwd_pool_kernel<<<B < C2F_GRID ? B : C2F_GRID, C2F_THREADS, 0, slk_stream(stream)>>>(
        act, W2, b2, pooled, code, B);
    return slk_launch_status();
}

extern "C" int slk_conv2_dgrad_direct(const float* dpooled, const uint8_t* code, const float* W2,
                               float* cut_grad, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(dpooled && code && W2 && cut_grad);
    conv2_dgrad_kernel<<<B < C2D_GRID ? B : C2D_GRID, C2D_THREADS, 0, slk_stream(stream)>>>(
        dpooled, code, W2, cut_grad, B);
    return slk_launch_status();
}

extern "C" int slk_conv2_wgrad_direct(const float* act, const float* dpooled, const uint8_t* code,
                               float* slabs, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(act && dpooled && code && slabs);
    conv2_wgrad_kernel<<<slk_conv2_wgrad_direct_nslab(B), C2W_THREADS, 0, slk_stream(stream)>>>(
        act, dpooled, code, slabs, B);
    return slk_launch_status();
}

extern "C" int slk_fc_fwd(const float* pooled, const float* W3, const float* b3, float* logits,
                          int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(pooled && W3 && b3 && logits);
    fc_head16_kernel<1><<<(B + FCH_S - 1) / FCH_S, FCH_T, 0, slk_stream(stream)>>>(
        pooled, W3, b3, nullptr, logits, nullptr, nullptr, nullptr, 0.f, nullptr, B, nullptr);
    return slk_launch_status();
}

extern "C" int slk_xent_fwd_bwd(const float* logits, const int64_t* labels, float* loss_i,
                                float* dlogits, float grad_scale, int* err_flag, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(logits && labels && loss_i && dlogits);
    fc_head16_kernel<2><<<(B + FCH_S - 1) / FCH_S, FCH_T, 0, slk_stream(stream)>>>(
        nullptr, nullptr, nullptr, labels, const_cast<float*>(logits), loss_i, dlogits, nullptr,
        grad_scale, err_flag, B, nullptr);
    return slk_launch_status();
}

extern "C" int slk_fc_logits_xent(const float* pooled, const float* W3, const float* b3, const int64_t* labels,
                                  float* logits, float* loss_i, float* dlogits, float grad_scale, int* err_flag, int B,
                                  void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(pooled && W3 && b3 && labels && logits && loss_i && dlogits);
    fc_head16_kernel<3><<<(B + FCH_S - 1) / FCH_S, FCH_T, 0, slk_stream(stream)>>>(
        pooled, W3, b3, labels, logits, loss_i, dlogits, nullptr, grad_scale, err_flag, B, nullptr);
    return slk_launch_status();
}

extern "C" int slk_fc_dgrad(const float* dlogits, const float* W3, float* dpooled, int B,
                            void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(dlogits && W3 && dpooled);
    fc_head16_kernel<4><<<(B + FCH_S - 1) / FCH_S, FCH_T, 0, slk_stream(stream)>>>(
        nullptr, W3, nullptr, nullptr, nullptr, nullptr, const_cast<float*>(dlogits), dpooled, 0.f,
        nullptr, B, nullptr);
    return slk_launch_status();
}

// slk_fc_dgrad + the per-sample max |dpooled| the x3 conv2 kernels scale by (fused, as slk_fc_xent_amax)
extern "C" int slk_fc_dgrad_amax(const float* dlogits, const float* W3, float* dpooled, float* dp_amax, int B,
                                 void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(dlogits && W3 && dpooled && dp_amax);
    fc_head16_kernel<4><<<(B + FCH_S - 1) / FCH_S, FCH_T, 0, slk_stream(stream)>>>(
        nullptr, W3, nullptr, nullptr, nullptr, nullptr, const_cast<float*>(dlogits), dpooled, 0.f,
        nullptr, B, dp_amax);
    return slk_launch_status();
}

extern "C" int slk_fc_xent(const float* pooled, const float* W3, const float* b3,
                           const int64_t* labels, float* logits, float* loss_i, float* dlogits,
                           float* dpooled, float grad_scale, int* err_flag, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(pooled && W3 && b3 && labels && logits && loss_i && dlogits && dpooled);
    fc_head16_kernel<7><<<(B + FCH_S - 1) / FCH_S, FCH_T, 0, slk_stream(stream)>>>(
        pooled, W3, b3, labels, logits, loss_i, dlogits, dpooled, grad_scale, err_flag, B, nullptr);
    return slk_launch_status();
}

extern "C" int slk_fc_xent_amax(const float* pooled, const float* W3, const float* b3, const int64_t* labels,
                                float* logits, float* loss_i, float* dlogits, float* dpooled, float* dp_amax,
                                float grad_scale, int* err_flag, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(pooled && W3 && b3 && labels && logits && loss_i && dlogits && dpooled && dp_amax);
    fc_head16_kernel<7><<<(B + FCH_S - 1) / FCH_S, FCH_T, 0, slk_stream(stream)>>>(
        pooled, W3, b3, labels, logits, loss_i, dlogits, dpooled, grad_scale, err_flag, B, dp_amax);
    return slk_launch_status();
}

extern "C" int slk_fc_wgrad(const float* dlogits, const float* pooled, float* slabs, int B,
                            void* stream) {
    SLK_CHECK_ARG(B >= 0);
    if (B == 0) return 0;
    SLK_CHECK_ARG(dlogits && pooled && slabs);
    const int per = fcw_per(B);
    dim3 grid(FC_K4 / 256, (B + per - 1) / per);
    fc_wgrad_kernel<<<grid, 256, 0, slk_stream(stream)>>>(dlogits, pooled, slabs, B, per);
    return slk_launch_status();
}
