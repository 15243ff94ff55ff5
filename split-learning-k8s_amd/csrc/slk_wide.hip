// slk_wide.hip — the WIDENED split CNN (BASELINE.json config 5, "K5") on gfx950 bf16 MFMA.
//
// Model (oracle/wide_step.py restates it): client conv1 3->64 (32x32) + ReLU, conv2 64->128 + ReLU +
// pool, conv3 128->256 + ReLU + pool -> cut [B,256,8,8]; server Dropout(0.25) + Linear(16384,10) +
// cross-entropy; Adam on both sides. The reference has no such model: it keeps
// the reference's step contract (src/client_part.py:110-138 <-> src/server_part.py:25-58) with the
// channel widths at which a 3x3 convolution is a real contraction (K = 9*Cin = 576 .. 2304).
//
// Activation layout in HBM ("C8"): bf16 [B][C/8][H][W][8] — eight channels of one pixel are one
// 16-byte chunk, and a chunk plane [H][W][8] is contiguous, so an image row of one chunk is one
// coalesced run and a 16x16x32 MFMA operand fragment (8 consecutive K = channels) is one 16-byte read.
//
// conv3x3 (pad 1) forward and input-gradient ("dgrad") are one implicit-GEMM kernel:
//   out[m][px] = sum_{tap, c} A[tap][c][m] * In[c][px + off(tap)]
// with A = the bf16 weight shadow (forward: W[co][ci][tap]; dgrad: W[co][ci][8 - tap], m = ci) and In
// the activation (forward) or the layer's output gradient (dgrad). A workgroup (4 waves, 2 per CU)
// owns MT output channels x NPX pixels (TR whole image rows); each wave a 64 x 64 sub-tile as
// 4 x 4 v_mfma_f32_16x16x32_bf16 accumulators. The input tile of one 32-channel group is staged in
// LDS with its 1-pixel halo as [4 chunks][(TR+2)*(W+2) pixels][16 B] by LDS-DMA (halo lanes read a
// static zero block), so all 9 taps read it with a constant offset and every fragment read is a
// conflict-free ds_read_b128 (16 consecutive pixels of one chunk = 256 contiguous bytes). The weight
// slice of each (group, tap) step [4 chunks][MT][16 B] streams through a 3-slot LDS ring two steps
// ahead; the next group's input tile streams into the other input slot during the current group.
// One counted `s_waitcnt vmcnt` + one barrier per step; the stream continues across tiles.
// Epilogues: forward = bias + ReLU + 2x2 max-pool in registers (vertical pairs are sibling
// accumulators, horizontal pairs neighbouring lanes) -> pooled bf16 + routing code; dgrad of conv3 =
// the gradient of p2 as is (16 x 16, bf16); dgrad of conv2 = ReLU mask of a1 -> the gradient conv1's
// wgrad consumes. The dgrads' own input is a max-pool backward (conv3: dcut by code3, conv2: dp2 by
// code2) that is never stored: the kernel expands the pooled gradient while staging it into LDS (EXP).
#include "slk_common.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Build-time knobs (tools/ablate_wide.py builds variants): weight lookahead of the conv stream, and
// XCD grouping of tiles (all row blocks / channel blocks of one image on one XCD at the same time,
// so halo rows and shared input tiles are L2 hits).
#ifndef SLK_WIDE_XCD
#define SLK_WIDE_XCD 1
#endif
// Wave priority: raise it around each step's MFMA block (1: conv kernels, 2: also wgrad), so a wave
// with MFMAs ready issues ahead of a co-resident wave's epilogue VALU / staging work.
#ifndef SLK_WIDE_DMA_LATE
#define SLK_WIDE_DMA_LATE 0
#endif
#ifndef SLK_WIDE_PRIO
#define SLK_WIDE_PRIO 0
#endif
// Stagger: the second half of the grid (the second workgroup of each CU under round-robin dispatch)
// sleeps SLK_WIDE_STAGGER x 127 x 64 cycles before its first tile, so the two co-resident workgroups
// run half a tile apart and one's epilogue (VALU + stores) overlaps the other's MFMA main loop.
#ifndef SLK_WIDE_STAGGER
#define SLK_WIDE_STAGGER 0
#endif
__device__ __forceinline__ void wide_stagger() {
#if SLK_WIDE_STAGGER
    if (blockIdx.x >= gridDim.x / 2)
        for (int i = 0; i < SLK_WIDE_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
#endif
}

namespace wide {
constexpr int IMG = 32;                 // input 3 x 32 x 32
constexpr int C1 = 64, C2 = 128, C3 = 256;
constexpr int CUT = C3 * 8 * 8;         // 16384 features per sample
constexpr int NCLS = 10;
constexpr int MODE_FWD_POOL = 0, MODE_DGRAD_MASK = 2, MODE_DGRAD_PLAIN = 3;
}  // namespace wide

__device__ __attribute__((aligned(64))) uint32_t slk_wide_zero[64];  // zero source for halo lanes

// bf16(a) | bf16(b) << 16, round to nearest even — the instruction the (__bf16) casts compile to, as
// asm: from the casts hipcc pairs accumulator elements across calls and repacks with 4 extra VALU
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    uint32_t r;
    asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }

__device__ __forceinline__ float dpp_xor1(float v) {
    // quad_perm [1,0,3,2]: lane l reads lane l^1
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}

// Epilogue forms (SLK_WIDE_EPI2 = 0: the first forms, for A/B): relu + 2x2 max-pool by v_max3 and
// first-equal argmax, bias folded into the accumulator's initial value; the a1 > 0 mask of conv2's
// dgrad on packed bf16 pairs.
#ifndef SLK_WIDE_EPI2
#define SLK_WIDE_EPI2 1
#endif
__device__ __forceinline__ float max3f(float a, float b, float c) {
    float r;   // asm: hipcc would canonicalize each operand of a plain fmaxf first
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// relu + max-pool of the window (v0, v1 | v2, v3) as torch's CPU kernel (strict > scan, first max
// wins): m = max(v, 0); the code is the first i with v_i == m when m > 0 (then relu(v_i) == m iff
// v_i == m), else CODE_NONE with value +0.
__device__ __forceinline__ float pool4(float v0, float v1, float v2, float v3, uint32_t& code) {
    const float m = max3f(max3f(v0, v1, v2), v3, 0.f);
    uint32_t c = v2 == m ? 2u : 3u;
    c = v1 == m ? 1u : c;
    c = v0 == m ? 0u : c;
    const bool pos = m > 0.f;
    code = pos ? c : (uint32_t)slk::CODE_NONE;
    return pos ? m : 0.f;
}
// keep the bf16 halves of w where the matching bf16 half of a1w is > 0 (as a signed int16: sign clear,
// not +0), zero the others. asm: hipcc turns the packed min/max into per-half compares and selects.
__device__ __forceinline__ uint32_t mask_pos_bf16x2(uint32_t w, uint32_t a1w) {
    uint32_t k;
    asm("v_pk_max_i16 %0, %1, 0\n\tv_pk_min_i16 %0, %0, %2\n\tv_pk_sub_u16 %0, 0, %0"
        : "=&v"(k) : "v"(a1w), "v"(0x00010001u));
    return w & k;
}

// the a1 > 0 bits of 4 consecutive channels (a nibble of a pixel's 64-bit ReLU word, slk_wide_conv1_fwd)
// as bf16-half masks of the packed pairs (channels 0,1 | 2,3): bit b -> 0xFFFF in half b
__device__ __forceinline__ uint2 relu_nibble_masks(uint32_t nib) {
    return make_uint2((nib & 1u) * 0xFFFFu + (nib & 2u) * 0x7FFF8000u,
                      ((nib >> 2) & 1u) * 0xFFFFu + ((nib >> 2) & 2u) * 0x7FFF8000u);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// vmcnt is 6 bits: an allowance above 63 saturates (waiting for more than needed is always safe)
template <int N>
__device__ __forceinline__ void wait_vmcnt_sat() { wait_vmcnt<(N > 63 ? 63 : N)>(); }

// Epilogue-aware waits: the first steps of a tile wait for weight slices that were issued BEFORE the
// previous tile's epilogue, so that epilogue's stores (and this tile's prefetched epilogue loads) are
// younger and may stay in flight. Without the allowance those steps drain every store before the
// next MFMA. 0 = plain counts (profiling only).
#ifndef SLK_WIDE_EPI
#define SLK_WIDE_EPI 1
#endif

// ----------------------------------------------------------------------------- conv geometry
template <int CI_, int CO_, int HW_, int MT_, int MODE_, int FW_, int NWV_, int EXP_ = 0>
struct ConvCfg {
    static constexpr int CI = CI_, CO = CO_, HW = HW_, MT = MT_, MODE = MODE_;
    static constexpr bool K32 = false;                      // 16x16x32 kernel (wide_conv_kernel)
    static constexpr bool ADMA = false;                     // builtin LDS-DMA (conv_dma16)
    static constexpr int FW = FW_;                          // 16-pixel fragments per wave (wave tile 64 x 16*FW)
    static constexpr int NWV = NWV_;                        // waves per workgroup (4: 2 WGs/CU; 8: 1 WG/CU)
    static constexpr int THREADS = NWV * 64;
    static constexpr int WM = MT / 64, WN = NWV / WM;       // WM waves along channels x WN along pixels
    static constexpr int NPX = WN * 16 * FW;                // pixels per tile
    static constexpr int TR = NPX / HW;                     // image rows per tile
    static constexpr int PW = HW + 2;                       // LDS row pitch (pixels, with halo)
    static constexpr int NP = (TR + 2) * PW;
    static constexpr int NPP = (NP + 63) / 64 * 64;         // pixels per chunk plane in LDS
    static constexpr int ND = NPP / 64;                     // LDS-DMA instructions per chunk plane
    static constexpr int G = CI / 32;                       // 32-channel groups (one MFMA K each)
    static constexpr int S = G * 9;                         // steps per tile
    static constexpr int IN_SLOT = NPP * 64;                // bytes: 4 chunks x NPP x 16
    static constexpr int W_SLOT = MT * 64;                  // bytes: 4 chunks x MT x 16
    static constexpr int NW = W_SLOT / 1024 / NWV;          // weight DMA instructions per wave per step
    static constexpr int DSPLIT = NWV / 4;                  // waves sharing one input chunk plane
    static constexpr int NDW = ND / DSPLIT;                 // input DMA instructions per wave per group
    static constexpr int L = 3;                             // weight lookahead (steps)
    static constexpr int RW = L + 1;                        // weight ring slots
    static constexpr int RB = HW / TR;                      // row blocks per image
    static constexpr int NCB = CO / MT;                     // output-channel blocks
    static constexpr int FPR = HW / 16;                     // 16-pixel fragments per image row
    // VMEM instructions per lane in the epilogue: stores (pooled value + code, plain or masked value)
    // and the a1 words loaded at tile start. Must never over-count.
    static constexpr int EPI_ST = 4 * FW;
    static constexpr int EPI_LD = MODE == 2 ? FW : 0;       // dgrad-mask: one 8-B a1 ReLU word per pixel fragment
    // EXP: the input is the max-pool backward of a POOLED gradient (HW/2 x HW/2, bf16 C8) and its
    // routing code: both move by LDS-DMA into a raw staging area (values [XR*THREADS][16 B], code
    // dwords 2 x [XR*THREADS][4 B]) and are expanded from there into the tile (exp_expand), so the
    // unpooled tensor is never written nor read, and no VGPR-destination load enters the main loop.
    static constexpr bool EXP = EXP_;
    static constexpr int XPR = TR / 2 + 2;                  // pooled rows feeding a tile (with halo)
    static constexpr int XITEMS = 4 * XPR * (HW / 2);       // pooled chunks per 32-channel group
    static constexpr int XR = (XITEMS + THREADS - 1) / THREADS;
    static constexpr int XN = XR * THREADS;                 // staged items (the excess reads zeros)
    static constexpr int RAW = EXP ? XN * 24 : 0;
    // input VMEM instructions per wave per group, issued at tap 0
    static constexpr int NIN = EXP ? 3 * XR : NDW;
    static constexpr int LDS = 2 * IN_SLOT + RW * W_SLOT + RAW;
    static_assert(MT == 128 || MT == 64, "MT");
    static_assert(HW % TR == 0 && TR % 2 == 0 && (16 * FW) % (2 * HW) == 0, "tile rows / pool pairs per wave");
    static_assert(NW >= 1 && W_SLOT % (1024 * NWV) == 0, "weight slot must split over the waves");
    static_assert(ND % DSPLIT == 0, "input planes must split over the waves");
    static_assert(NCB == 1 || NCB == 2, "NCB");
};

struct TileState {
    int valid, n, rb, cob;
};

template <class C>
__device__ __forceinline__ TileState tile_state(int t, int B) {
    // Blocks b and b + 8 of a grid that is a multiple of 8 share an XCD under round-robin placement
    // and process tiles t and t + 8 in the same round. XCD grouping sends all RB x NCB tiles of image
    // n to XCD (n % 8) in one round: neighbouring row blocks share halo rows and the channel blocks
    // share the input tile through that XCD's L2. (Speed only; any placement is correct.)
    TileState s;
#if SLK_WIDE_XCD
    const int xcd = t & 7, j = t >> 3;
    s.rb = j % C::RB;
    s.cob = (j / C::RB) % C::NCB;
    s.n = (j / (C::RB * C::NCB)) * 8 + xcd;
    s.valid = s.n < B;
#else
    int pt;
    if (C::NCB == 2) {
        s.cob = (t >> 3) & 1;
        pt = ((t >> 4) << 3) | (t & 7);
    } else {
        s.cob = 0;
        pt = t;
    }
    s.valid = pt < B * C::RB;
    s.n = pt / C::RB;
    s.rb = pt - s.n * C::RB;
#endif
    return s;
}

template <class C>
__device__ __forceinline__ void tile_poff(const TileState& s, int wave, int lane, int (&poff)[C::NDW]) {
    // this wave's DMA pieces of its chunk plane: d = (wave / 4) + k * DSPLIT
#pragma unroll
    for (int k = 0; k < C::NDW; ++k) {
        const int d = (wave >> 2) + k * C::DSPLIT;
        const int P = d * 64 + lane;
        const int ry = P / C::PW, rx = P - (P / C::PW) * C::PW;
        const int y = s.rb * C::TR - 1 + ry, x = rx - 1;
        const bool ok = P < C::NP && y >= 0 && y < C::HW && x >= 0 && x < C::HW;
        poff[k] = ok ? y * C::HW + x : -1;
    }
}

// LDS-DMA of the conv kernels: C::ADMA selects the asm form (glds16: invisible to hipcc's waitcnt
// pass) or the builtin. Measured per kernel (tools/ablate_wide.py): the 32x32 forward is faster with
// asm; wide_conv_kernel with the builtin (the asm statement pins the fragment reads around each DMA),
// whose only hipcc-inserted drains were at the EXP staging reads/writes — those are asm instead.
template <class C>
__device__ __forceinline__ void conv_dma16(const void* src, char* dst) {
    if constexpr (C::ADMA) glds16(src, lds_u32(dst));
    else __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)dst, 16, 0, 0);
}
template <class C>
__device__ __forceinline__ void conv_dma4(const void* src, char* dst) {
    if constexpr (C::ADMA) glds4(src, lds_u32(dst));
    else __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)dst, 4, 0, 0);
}

// input tile of group g (chunks 4g .. 4g+3) -> LDS slot; wave w moves chunk plane w
template <class C>
__device__ __forceinline__ void issue_input(const uint16_t* __restrict__ in, const TileState& s,
                                            const int (&poff)[C::NDW], int g, char* slot, int wave, int lane) {
    const int c = wave & 3;
    const char* plane = reinterpret_cast<const char*>(in) +
                        ((size_t)(s.n * (C::CI / 8) + g * 4 + c) * (C::HW * C::HW)) * 16;
    const char* zero = reinterpret_cast<const char*>(slk_wide_zero);
    char* dst = slot + c * C::NPP * 16;
#pragma unroll
    for (int k = 0; k < C::NDW; ++k) {
        const int d = (wave >> 2) + k * C::DSPLIT;
        const char* src = poff[k] >= 0 ? plane + (size_t)poff[k] * 16 : zero;
        conv_dma16<C>((const void*)src, dst + d * 1024);
    }
}

// EXP staging. Pooled chunk i = (plane c, pooled row pr, pooled col px) of group g: its 8 channels'
// values and routing codes (code 0..3 = window position, 4 = ReLU-blocked). Wave w moves items
// r * THREADS + 64 w + lane of every round r by LDS-DMA (value + two code dwords); items outside the
// image or past XITEMS read the zero block, so each wave issues exactly NIN instructions.
template <class C>
__device__ __forceinline__ void exp_issue(const uint16_t* __restrict__ dp, const uint8_t* __restrict__ code,
                                          const TileState& s, int g, char* raw, int wave, int lane) {
    constexpr int PH = C::HW / 2;
    const char* zero = reinterpret_cast<const char*>(slk_wide_zero);
#pragma unroll
    for (int r = 0; r < C::XR; ++r) {
        const int i0 = r * C::THREADS + wave * 64, i = i0 + lane;
        const int c = i / (C::XPR * PH), rem = i - c * (C::XPR * PH), pr = rem / PH, px = rem - pr * PH;
        const int py = s.rb * (C::TR / 2) - 1 + pr;
        const bool ok = i < C::XITEMS && py >= 0 && py < PH;
        const size_t idx = ((size_t)(s.n * (C::CI / 8) + g * 4 + c) * PH + (ok ? py : 0)) * PH + px;
        const char* sv = ok ? reinterpret_cast<const char*>(dp) + idx * 16 : zero;
        const char* sc = ok ? reinterpret_cast<const char*>(code) + idx * 8 : zero;
        conv_dma16<C>((const void*)sv, raw + i0 * 16);
        conv_dma4<C>((const void*)sc, raw + C::XN * 16 + i0 * 4);
        conv_dma4<C>((const void*)(sc + 4), raw + C::XN * 20 + i0 * 4);
    }
}

// 16-bit lane masks of one window position: v_perm_b32 with the codes as byte selectors into the table
// {0 (bytes 4-7), 0xFF << 8 pos (bytes 0-3)} gives 0xFF exactly where code == pos.
__device__ __forceinline__ uint4 route_chunk(uint4 v, uint32_t cA, uint32_t cB, uint32_t cC, uint32_t cD, int pos) {
    const uint32_t T = 0xFFu << (8 * pos);
    return make_uint4(v.x & __builtin_amdgcn_perm(0u, T, cA), v.y & __builtin_amdgcn_perm(0u, T, cB),
                      v.z & __builtin_amdgcn_perm(0u, T, cC), v.w & __builtin_amdgcn_perm(0u, T, cD));
}

// A 16-byte LDS store hipcc does not see (see exp_expand); published by the caller's own lgkmcnt
// wait + barrier.
__device__ __forceinline__ void lds_store16(char* p, uint4 v) {
    const uint32_t a = (uint32_t)(size_t)(lds_ptr_t)p;
    const u32x4 d = {v.x, v.y, v.z, v.w};
    asm volatile("ds_write_b128 %0, %1\n\ts_nop 1" ::"v"(a), "v"(d) : "memory");
}

// max-pool backward of the loaded pooled chunk i into the tile's LDS image [4][NPP][16 B]: pooled
// (pr, px) feeds unpooled rows 2 pr - 1 + dy (tile-local, halo row 0 included) and columns 2 px + dx.
template <class C>
__device__ __forceinline__ void exp_store(char* slot, int i, uint4 v, uint2 cw) {
    constexpr int PH = C::HW / 2;
    if (i >= C::XITEMS) return;
    const int c = i / (C::XPR * PH), rem = i - c * (C::XPR * PH), pr = rem / PH, px = rem - pr * PH;
    const uint32_t cA = __builtin_amdgcn_perm(0u, cw.x, 0x01010000u), cB = __builtin_amdgcn_perm(0u, cw.x, 0x03030202u);
    const uint32_t cC = __builtin_amdgcn_perm(0u, cw.y, 0x01010000u), cD = __builtin_amdgcn_perm(0u, cw.y, 0x03030202u);
    char* base = slot + (c * C::NPP + 2 * px + 1) * 16;
    // an 8-lane group of ds_write_b128 (banks = dword % 32) holds 8 consecutive px, whose pieces sit 32 B
    // apart: storing the same column everywhere hit only 4 of the 8 16-B slots of 128 B (2-way on every
    // store, 10.5 M conflict cycles per conv2-dgrad launch); lanes with px & 4 store the other column first
    // (measured: conv3 dgrad, HW = 16, 0.5105 -> 0.5032 ms; conv2 dgrad, HW = 32, 0.5828 -> 0.6168: kept for HW = 16)
    const int f = C::HW == 16 ? (px >> 2) & 1 : 0;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
        const int ry = 2 * pr + dy - 1;
        if (ry < 0 || ry > C::TR + 1) continue;
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
            const int ddx = dx ^ f;
            lds_store16(base + (ry * C::PW + ddx) * 16, route_chunk(v, cA, cB, cC, cD, 2 * dy + ddx));
        }
    }
}

// the staged items of this thread (landed and barrier-published) -> the tile in `slot`
template <class C>
__device__ __forceinline__ void exp_expand(char* slot, const char* raw, int tid) {
#pragma unroll
    for (int r = 0; r < C::XR; ++r) {
        const int i = tid + r * C::THREADS;
        if (i >= C::XITEMS) break;
        // one asm statement with its own lgkmcnt wait: beside the builtin LDS-DMA, hipcc drains every
        // DMA in flight (vmcnt(0)) before a plain LDS access it cannot prove disjoint from them
        const uint32_t a = (uint32_t)(size_t)(lds_ptr_t)(raw + i * 16);
        const uint32_t b = (uint32_t)(size_t)(lds_ptr_t)(raw + C::XN * 16 + i * 4);
        const uint32_t c = (uint32_t)(size_t)(lds_ptr_t)(raw + C::XN * 20 + i * 4);
        u32x4 v4;
        uint32_t c0, c1;
        asm volatile("ds_read_b128 %0, %3\n\tds_read_b32 %1, %4\n\tds_read_b32 %2, %5\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(v4), "=&v"(c0), "=&v"(c1)
                     : "v"(a), "v"(b), "v"(c)
                     : "memory");
        exp_store<C>(slot, i, make_uint4(v4[0], v4[1], v4[2], v4[3]), make_uint2(c0, c1));
    }
}

// the halo columns (x = -1, HW) of both input slots, zero for the kernel's lifetime (EXP never writes them)
template <class C>
__device__ __forceinline__ void exp_zero_halo(char* slots, int tid) {
    constexpr int N = 2 * 4 * (C::TR + 2) * 2;
    for (int k = tid; k < N; k += C::THREADS) {
        const int side = k & 1, ry = (k >> 1) % (C::TR + 2), c = ((k >> 1) / (C::TR + 2)) & 3, sl = (k >> 1) / (4 * (C::TR + 2));
        *reinterpret_cast<uint4*>(slots + sl * C::IN_SLOT + (c * C::NPP + ry * C::PW + side * (C::PW - 1)) * 16) =
            make_uint4(0u, 0u, 0u, 0u);
    }
}

// weight slice of step (cob, g, tap) -> LDS slot; wave w moves NW consecutive KiB
template <class C>
__device__ __forceinline__ void issue_weight(const uint16_t* __restrict__ wsh, int cob, int sl, char* slot,
                                             int wave, int lane) {
    const int g = sl / 9, tap = sl - (sl / 9) * 9;
    const char* src = reinterpret_cast<const char*>(wsh) +
                      ((size_t)((cob * 9 + tap) * (C::CI / 8) + g * 4) * C::MT) * 16;
#pragma unroll
    for (int i = 0; i < C::NW; ++i) {
        const int j = wave * C::NW + i;
        conv_dma16<C>((const void*)(src + j * 1024 + lane * 16), slot + j * 1024);
    }
}

// Epilogue operands of a tile (dgrad-mask: a1 words), loaded when the tile
// starts so their latency hides under its main loop instead of draining the DMA queue at the epilogue.
// dgrad-mask: the ReLU word of each of the lane's FW pixels ([B][HW*HW] u64, bit c = a1[c] > 0 for the
// 64 channels: slk_wide_conv1_fwd writes it beside a1), 8 B per pixel instead of the 4 x 8 B of a1 words
// the mask once read (32 VGPRs held across the main loop, and 537 MB of a1 per launch at B = 4096)
template <class C>
__device__ __forceinline__ void epi_prefetch(const void* __restrict__ aux, const TileState& s, int wm, int wn,
                                             int lane, uint2 (&em)[C::FW]) {
    if constexpr (C::MODE == wide::MODE_DGRAD_MASK) {
        static_assert(C::CO == 64 && C::MT == 64, "one 64-bit ReLU word covers the tile's channels");
#pragma unroll
        for (int f = 0; f < C::FW; ++f) {
            const int q = wn * 16 * C::FW + f * 16 + (lane & 15);
            const int y = s.rb * C::TR + q / C::HW, x = q % C::HW;
            em[f] = reinterpret_cast<const uint2*>(aux)[((size_t)s.n * C::HW + y) * C::HW + x];
        }
    }
}

// in: forward = activation, dgrad = the POOLED output gradient (EXP; out2 = its routing code, u8 C8);
// aux: forward = bias (f32 [CO]); dgrad-plain = unused;
//      dgrad-mask = a1 (bf16, C8 [B][CO/8][HW][HW][8]).
// out: forward = pooled bf16 C8 [B][CO/8][HW/2][HW/2][8] (+ code u8 same layout in out2);
//      dgrad-plain / dgrad-mask = bf16 C8 [B][CO/8][HW][HW][8].
template <class C>
__global__ __launch_bounds__(C::THREADS, C::NWV == 4 ? 2 : 1) void wide_conv_kernel(const uint16_t* __restrict__ in,
                                                           const uint16_t* __restrict__ wsh,
                                                           const void* __restrict__ aux,
                                                           uint16_t* __restrict__ out,
                                                           uint8_t* __restrict__ out2, int B) {
    __shared__ __attribute__((aligned(1024))) char smem[C::LDS];
    char* islot0 = smem;
    char* wslot0 = smem + 2 * C::IN_SLOT;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / C::WN, wn = wave - (wave / C::WN) * C::WN;
    const int grid = gridDim.x;

    int t = blockIdx.x;
    TileState cur = tile_state<C>(t, B);
    if (!cur.valid) return;
    wide_stagger();
    int tn = t + grid;
    TileState nxt = tile_state<C>(tn, B);
    int pcur[C::NDW], pnxt[C::NDW];
    tile_poff<C>(cur, wave, lane, pcur);
    tile_poff<C>(nxt, wave, lane, pnxt);

    // per-lane fragment read offsets (bytes, relative to the slot)
    const int a_off = ((lane >> 4) * C::MT + wm * 64 + (lane & 15)) * 16;
    int b_off[C::FW];
#pragma unroll
    for (int f = 0; f < C::FW; ++f) {
        const int q = wn * 16 * C::FW + f * 16 + (lane & 15);
        const int r = q / C::HW, x = q - (q / C::HW) * C::HW;
        b_off[f] = ((lane >> 4) * C::NPP + (r + 1) * C::PW + x + 1) * 16;
    }

    float bias[4][4];
    if constexpr (C::MODE == wide::MODE_FWD_POOL) {
        const float* b = reinterpret_cast<const float*>(aux);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) bias[i][r] = b[cur.cob * C::MT + wm * 64 + i * 16 + 4 * (lane >> 4) + r];
    }

    // Fragment prefetch: during step s the MFMAs consume fragments read in step s-1 while the reads
    // for step s+1 are in flight, so no step opens with an LDS-latency bubble. The wait of step s
    // therefore covers weight step s+1 (issued 2 steps earlier; lookahead L = 3, 4 ring slots) and,
    // at tap 8, the next group's input tile.
    static_assert(C::L == 3, "prefetch schedule assumes a weight lookahead of 3");
    char* raw = smem + 2 * C::IN_SLOT + C::RW * C::W_SLOT;
    if constexpr (C::EXP) {
        exp_zero_halo<C>(islot0, tid);
        exp_issue<C>(in, out2, cur, 0, raw, wave, lane);
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        exp_expand<C>(islot0, raw, tid);
    } else {
        issue_input<C>(in, cur, pcur, 0, islot0, wave, lane);
    }
#pragma unroll
    for (int k = 0; k < C::L; ++k) issue_weight<C>(wsh, cur.cob, k, wslot0 + k * C::W_SLOT, wave, lane);
    if (!nxt.valid && C::S == 1) wait_vmcnt<0>();
    else wait_vmcnt<2 * C::NW>();
    if constexpr (C::EXP) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    bf16x8 av_n[4], bv_n[C::FW];
    {
        const int toff = -(C::PW + 1) * 16;
#pragma unroll
        for (int i = 0; i < 4; ++i) av_n[i] = *reinterpret_cast<const bf16x8*>(wslot0 + a_off + i * 256);
#pragma unroll
        for (int f = 0; f < C::FW; ++f) bv_n[f] = *reinterpret_cast<const bf16x8*>(islot0 + b_off[f] + toff);
    }
    int wslot = 0;   // ring slot of the current step
    int islot = 0;   // input slot of the current group
    bool post = false;   // a previous tile's epilogue stores may be in flight
    uint2 em[C::FW];
#pragma unroll 1
    while (true) {
        const bool tail = !nxt.valid;
        epi_prefetch<C>(aux, cur, wm, wn, lane, em);
        f32x4 acc[4][C::FW];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int f = 0; f < C::FW; ++f) {
                if (C::MODE == wide::MODE_FWD_POOL && SLK_WIDE_EPI2)
                    acc[i][f] = f32x4{bias[i][0], bias[i][1], bias[i][2], bias[i][3]};
                else
                    acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};
            }

#pragma unroll 1
        for (int g = 0; g < C::G; ++g) {
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const bool last = tail && g == C::G - 1 && tap == 8;
                // step s+1's weight slice (and at tap 8 the next group's input tile) has landed
                if (tail) wait_vmcnt<0>();
                else if (SLK_WIDE_EPI && tap < 2 && g == 0) {
                    // weight step +1 predates the previous epilogue and this tile's epilogue loads
                    if (tap == 0) {
                        if (post) wait_vmcnt_sat<C::NW + C::EPI_ST + C::EPI_LD>();
                        else wait_vmcnt_sat<C::NW + C::EPI_LD>();
                    } else {
                        if (post) wait_vmcnt_sat<C::NW + C::NIN + C::EPI_ST + C::EPI_LD>();
                        else wait_vmcnt_sat<C::NW + C::NIN + C::EPI_LD>();
                    }
                }
                else if (tap == 1 || tap == 2) wait_vmcnt<C::NW + C::NIN>();
                else wait_vmcnt<C::NW>();
                // EXP: the next group's staged items landed by tap 3's wait and were expanded after its
                // barrier; this wave's tile writes (and raw reads) complete before tap 4's barrier
                if (C::EXP && tap == 4) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                // weight step +3 into the slot of step -1; at tap 0 the next group's input tile. Both
                // after this step's MFMAs when SLK_WIDE_DMA_LATE (same order of VMEM operations, so
                // the counted waits are unchanged; every target slot is free since the barrier).
                auto issue_dma = [&]() {
                    {
                        const int sl = g * 9 + tap + C::L;
                        int ws = wslot + C::L;
                        ws = ws >= C::RW ? ws - C::RW : ws;
                        if (sl < C::S) issue_weight<C>(wsh, cur.cob, sl, wslot0 + ws * C::W_SLOT, wave, lane);
                        else if (!tail) issue_weight<C>(wsh, nxt.cob, sl - C::S, wslot0 + ws * C::W_SLOT, wave, lane);
                    }
                    if constexpr (C::EXP) {
                        if ((g + 1 < C::G || !tail) && tap == 0) {
                            if (g + 1 < C::G) exp_issue<C>(in, out2, cur, g + 1, raw, wave, lane);
                            else exp_issue<C>(in, out2, nxt, 0, raw, wave, lane);
                        }
                    } else if (tap == 0) {
                        char* nslot = islot0 + (islot ^ 1) * C::IN_SLOT;
                        if (g + 1 < C::G) issue_input<C>(in, cur, pcur, g + 1, nslot, wave, lane);
                        else if (!tail) issue_input<C>(in, nxt, pnxt, 0, nslot, wave, lane);
                    }
                };
                if (!SLK_WIDE_DMA_LATE) issue_dma();
                // EXP: the next group's pooled input, staged by LDS-DMA at tap 0, is expanded into the
                // free slot at tap 3 (read from tap 8 on)
                if constexpr (C::EXP) {
                    if ((g + 1 < C::G || !tail) && tap == 3)
                        exp_expand<C>(islot0 + (islot ^ 1) * C::IN_SLOT, raw, tid);
                }
                bf16x8 av[4], bv[C::FW];
#pragma unroll
                for (int i = 0; i < 4; ++i) av[i] = av_n[i];
#pragma unroll
                for (int f = 0; f < C::FW; ++f) bv[f] = bv_n[f];
                const int wn1 = wslot + 1 == C::RW ? 0 : wslot + 1;
                if (!last) {
                    const char* wb = wslot0 + wn1 * C::W_SLOT;
                    const char* ib = islot0 + (tap == 8 ? (islot ^ 1) : islot) * C::IN_SLOT;
                    const int tn = tap == 8 ? 0 : tap + 1;
                    const int toff = ((tn / 3 - 1) * C::PW + (tn % 3 - 1)) * 16;
#pragma unroll
                    for (int i = 0; i < 4; ++i) av_n[i] = *reinterpret_cast<const bf16x8*>(wb + a_off + i * 256);
#pragma unroll
                    for (int f = 0; f < C::FW; ++f) bv_n[f] = *reinterpret_cast<const bf16x8*>(ib + b_off[f] + toff);
                }
                if (SLK_WIDE_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int f = 0; f < C::FW; ++f)
                        acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[f], acc[i][f], 0, 0, 0);
                if (SLK_WIDE_PRIO) __builtin_amdgcn_s_setprio(0);
                if (SLK_WIDE_DMA_LATE) issue_dma();
                wslot = wn1;
            }
            islot ^= 1;
        }
        // ------------------------------------------------------------------ epilogue
        const int ch_base = cur.cob * C::MT + wm * 64 + 4 * (lane >> 4);
        if constexpr (C::MODE == wide::MODE_FWD_POOL) {
            constexpr int PH = C::HW / 2;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ch0 = ch_base + i * 16;
#pragma unroll
                for (int f = 0; f < C::FW; ++f) {
                    if ((f / C::FPR) & 1) continue;       // bottom row of a window pair
                    const int fb = f + C::FPR;
                    float pv[4];
                    uint32_t cw = 0;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if (SLK_WIDE_EPI2) {   // the bias is already in the accumulators
                            const float v0 = acc[i][f][r], v2 = acc[i][fb][r];
                            uint32_t code;
                            pv[r] = pool4(v0, dpp_xor1(v0), v2, dpp_xor1(v2), code);
                            cw |= code << (8 * r);
                            continue;
                        }
                        const float v0 = acc[i][f][r] + bias[i][r];
                        const float v2 = acc[i][fb][r] + bias[i][r];
                        const float v1 = dpp_xor1(v0), v3 = dpp_xor1(v2);
                        // torch CPU max-pool over relu(c): strict > scan, first max wins
                        float best = v0 > 0.f ? v0 : 0.f;
                        int idx = 0;
                        const float r1 = v1 > 0.f ? v1 : 0.f, r2 = v2 > 0.f ? v2 : 0.f, r3 = v3 > 0.f ? v3 : 0.f;
                        if (r1 > best) { best = r1; idx = 1; }
                        if (r2 > best) { best = r2; idx = 2; }
                        if (r3 > best) { best = r3; idx = 3; }
                        pv[r] = best;
                        cw |= (uint32_t)(best > 0.f ? idx : slk::CODE_NONE) << (8 * r);
                    }
                    if ((lane & 1) == 0) {
                        const int q = wn * 16 * C::FW + f * 16 + (lane & 15);
                        const int y = cur.rb * C::TR + q / C::HW, x = q % C::HW;
                        const size_t o = (((size_t)(cur.n * (C::CO / 8) + (ch0 >> 3)) * PH + (y >> 1)) * PH + (x >> 1)) * 8 + (ch0 & 7);
                        *reinterpret_cast<uint2*>(out + o) = make_uint2(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]));
                        *reinterpret_cast<uint32_t*>(out2 + o) = cw;
                    }
                }
            }
        } else if constexpr (C::MODE == wide::MODE_DGRAD_PLAIN) {
            // the input gradient as is (bf16): conv3's dgrad writes the gradient of p2 at pooled
            // resolution; conv2's consumers route it by code2 while staging (EXP)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ch0 = ch_base + i * 16;
#pragma unroll
                for (int f = 0; f < C::FW; ++f) {
                    const int q = wn * 16 * C::FW + f * 16 + (lane & 15);
                    const int y = cur.rb * C::TR + q / C::HW, x = q % C::HW;
                    const size_t o = (((size_t)(cur.n * (C::CO / 8) + (ch0 >> 3)) * C::HW + y) * C::HW + x) * 8 + (ch0 & 7);
                    *reinterpret_cast<uint2*>(out + o) = make_uint2(pack_bf16x2(acc[i][f][0], acc[i][f][1]),
                                                                    pack_bf16x2(acc[i][f][2], acc[i][f][3]));
                }
            }
        } else {
            // channels ch0 .. ch0 + 3 = bits 16 i + 4 (lane >> 4) .. + 3 of the pixel's ReLU word
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ch0 = ch_base + i * 16;
#pragma unroll
                for (int f = 0; f < C::FW; ++f) {
                    const int q = wn * 16 * C::FW + f * 16 + (lane & 15);
                    const int y = cur.rb * C::TR + q / C::HW, x = q % C::HW;
                    const size_t o = (((size_t)(cur.n * (C::CO / 8) + (ch0 >> 3)) * C::HW + y) * C::HW + x) * 8 + (ch0 & 7);
                    const uint32_t word = (i < 2) ? em[f].x : em[f].y;
                    const uint2 m = relu_nibble_masks(word >> (16 * (i & 1) + 4 * (lane >> 4)));
                    *reinterpret_cast<uint2*>(out + o) = make_uint2(pack_bf16x2(acc[i][f][0], acc[i][f][1]) & m.x,
                                                                    pack_bf16x2(acc[i][f][2], acc[i][f][3]) & m.y);
                }
            }
        }

        if (tail) break;
        cur = nxt;
#pragma unroll
        for (int d = 0; d < C::NDW; ++d) pcur[d] = pnxt[d];
        tn += grid;
        nxt = tile_state<C>(tn, B);
        tile_poff<C>(nxt, wave, lane, pnxt);
    }
}



// ----------------------------------------------------------------------------- 32x32x16 variant
// Same stream and LDS images as wide_conv_kernel, but each wave owns a 64-channel x 128-pixel tile as
// 2 x 4 v_mfma_f32_32x32x16_bf16 accumulators (128 VGPRs): per 32-channel step a wave issues 12
// fragment reads for 16 MFMAs of 32 cycles (vs 8 reads for 16 MFMAs of 16 cycles), and every weight
// slice streamed into LDS now serves 256 pixels — half the LDS-DMA instructions per FLOP of the
// 64 x 64 / 16x16x32 form, at the same 2 workgroups per CU.
// Fragment maps (cdna_hip_programming.md §3): lane l (r = l & 31, h = l >> 5) holds A[row r][k = 8h+j]
// and B[k = 8h+j][col r]; C/D: col = r, row = (reg & 3) + 8 (reg >> 2) + 4h.
typedef float f32x16v __attribute__((ext_vector_type(16)));

template <int CI_, int CO_, int HW_, int MODE_>
struct Conv32Cfg {
    static constexpr int CI = CI_, CO = CO_, HW = HW_, MT = 128, MODE = MODE_;
    static constexpr bool K32 = true;
    static constexpr bool ADMA = true;                      // asm LDS-DMA (conv_dma16)
    static constexpr int NWV = 4, THREADS = 256;
    static constexpr int WM = 2, WN = 2;                    // waves: 2 along channels x 2 along pixels
    static constexpr int NPX = WN * 128;                    // 256 pixels per tile
    static constexpr int TR = NPX / HW;
    static constexpr int PW = HW + 2;
    static constexpr int NP = (TR + 2) * PW;
    static constexpr int NPP = (NP + 63) / 64 * 64;
    static constexpr int ND = NPP / 64;
    static constexpr int DSPLIT = 1, NDW = ND;
    static constexpr int G = CI / 32;
    static constexpr int S = G * 9;
    static constexpr int IN_SLOT = NPP * 64;
    static constexpr int W_SLOT = MT * 64;
    static constexpr int NW = W_SLOT / 1024 / NWV;          // 2
    static constexpr int L = 2, RW = 3;
    static constexpr int LDS = 2 * IN_SLOT + RW * W_SLOT;
    static constexpr int RB = HW / TR;
    static constexpr int NCB = CO / MT;
    static constexpr int EPI_ST = HW == 32 ? 32 : 64;
    static constexpr int EPI_LD = 0;
    static_assert(HW % TR == 0 && TR % 2 == 0 && (HW == 32 || HW == 16), "tile rows");
    static_assert(NCB == 1 || NCB == 2, "NCB");
};

template <class C>
__global__ __launch_bounds__(256, 2) void wide_conv32_kernel(const uint16_t* __restrict__ in,
                                                             const uint16_t* __restrict__ wsh,
                                                             const void* __restrict__ aux,
                                                             uint16_t* __restrict__ out,
                                                             uint8_t* __restrict__ out2, int B) {
    __shared__ __attribute__((aligned(1024))) char smem[C::LDS + C::MT * 4];   // + bias (fwd)
    char* islot0 = smem;
    char* wslot0 = smem + 2 * C::IN_SLOT;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int r = lane & 31, h = lane >> 5;
    const int grid = gridDim.x;

    int t = blockIdx.x;
    TileState cur = tile_state<C>(t, B);
    if (!cur.valid) return;
    wide_stagger();
    int tn = t + grid;
    TileState nxt = tile_state<C>(tn, B);
    int pcur[C::NDW], pnxt[C::NDW];
    tile_poff<C>(cur, wave, lane, pcur);
    tile_poff<C>(nxt, wave, lane, pnxt);

    // A: chunk (2ks + h), channel wm*64 + ct*32 + r;  B: chunk (2ks + h), pixel wn*128 + pt*32 + r
    const int a_off = (h * C::MT + wm * 64 + r) * 16;
    int b_off[4];
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
        const int q = wn * 128 + pt * 32 + r;
        const int y = q / C::HW, x = q - (q / C::HW) * C::HW;
        b_off[pt] = (h * C::NPP + (y + 1) * C::PW + x + 1) * 16;
    }
    float* bias_s = reinterpret_cast<float*>(smem + C::LDS);   // this workgroup's channel block (fixed cob)
    if constexpr (C::MODE == wide::MODE_FWD_POOL) {
        if (tid < C::MT) bias_s[tid] = reinterpret_cast<const float*>(aux)[cur.cob * C::MT + tid];
        __syncthreads();
    }

    issue_input<C>(in, cur, pcur, 0, islot0, wave, lane);
#pragma unroll
    for (int k = 0; k < C::L; ++k) issue_weight<C>(wsh, cur.cob, k, wslot0 + k * C::W_SLOT, wave, lane);

    int wslot = 0, islot = 0;
    bool post = false;
#pragma unroll 1
    while (true) {
        const bool tail = !nxt.valid;
        f32x16v acc[2][4];
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int pt = 0; pt < 4; ++pt)
#pragma unroll
                for (int g = 0; g < 16; ++g) acc[ct][pt][g] = 0.f;
#pragma unroll 1
        for (int g = 0; g < C::G; ++g) {
            const char* ib = islot0 + islot * C::IN_SLOT;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                if (tail) wait_vmcnt<0>();
                else if (SLK_WIDE_EPI && tap < C::L && g == 0) {
                    if (tap == 0) {
                        if (post) wait_vmcnt_sat<(C::L - 1) * C::NW + C::EPI_ST + C::EPI_LD>();
                        else wait_vmcnt_sat<(C::L - 1) * C::NW + C::EPI_LD>();
                    } else {
                        if (post) wait_vmcnt_sat<(C::L - 1) * C::NW + C::NDW + C::EPI_ST + C::EPI_LD>();
                        else wait_vmcnt_sat<(C::L - 1) * C::NW + C::NDW + C::EPI_LD>();
                    }
                }
                else if (tap >= 1 && tap <= C::L) wait_vmcnt<(C::L - 1) * C::NW + C::NDW>();
                else wait_vmcnt<(C::L - 1) * C::NW>();
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                {
                    const int sl = g * 9 + tap + C::L;
                    int ws = wslot + C::L;
                    ws = ws >= C::RW ? ws - C::RW : ws;
                    if (sl < C::S) issue_weight<C>(wsh, cur.cob, sl, wslot0 + ws * C::W_SLOT, wave, lane);
                    else if (!tail) issue_weight<C>(wsh, nxt.cob, sl - C::S, wslot0 + ws * C::W_SLOT, wave, lane);
                }
                if (tap == 0) {
                    char* nslot = islot0 + (islot ^ 1) * C::IN_SLOT;
                    if (g + 1 < C::G) issue_input<C>(in, cur, pcur, g + 1, nslot, wave, lane);
                    else if (!tail) issue_input<C>(in, nxt, pnxt, 0, nslot, wave, lane);
                }
                const char* wb = wslot0 + wslot * C::W_SLOT;
                const int toff = ((tap / 3 - 1) * C::PW + (tap % 3 - 1)) * 16;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    bf16x8 av[2], bv[4];
#pragma unroll
                    for (int ct = 0; ct < 2; ++ct)
                        av[ct] = *reinterpret_cast<const bf16x8*>(wb + a_off + (2 * ks * C::MT + ct * 32) * 16);
#pragma unroll
                    for (int pt = 0; pt < 4; ++pt)
                        bv[pt] = *reinterpret_cast<const bf16x8*>(ib + b_off[pt] + 2 * ks * C::NPP * 16 + toff);
#pragma unroll
                    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                        for (int pt = 0; pt < 4; ++pt)
                            acc[ct][pt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[ct], bv[pt], acc[ct][pt], 0, 0, 0);
                }
                wslot = wslot + 1 == C::RW ? 0 : wslot + 1;
            }
            islot ^= 1;
        }

        // ------------------------------------------------------------------ epilogue
        static_assert(C::MODE == wide::MODE_FWD_POOL, "conv32: forward + pool only");
        {
            constexpr int PH = C::HW / 2;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
#pragma unroll
                for (int pp = 0; pp < (C::HW == 32 ? 2 : 4); ++pp) {
                    // HW 32: windows of tiles (2pp, 2pp+1) [rows], lanes (r, r^1) [cols];
                    // HW 16: tile pp holds rows 2y, 2y+1 in lane halves 0-15 / 16-31
#pragma unroll
                    for (int g4 = 0; g4 < 4; ++g4) {
                        float pv[4];
                        uint32_t cw = 0;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int g = 4 * g4 + e;
                            const float bb = bias_s[wm * 64 + ct * 32 + 8 * g4 + 4 * h + e];
                            float v0, v2;
                            if (C::HW == 32) {
                                v0 = acc[ct][2 * pp][g] + bb;
                                v2 = acc[ct][2 * pp + 1][g] + bb;
                            } else {
                                v0 = acc[ct][pp][g] + bb;
                                v2 = __shfl_xor(v0, 16, 64);
                            }
                            const float v1 = dpp_xor1(v0), v3 = dpp_xor1(v2);
                            if (SLK_WIDE_EPI2) {
                                uint32_t code;
                                pv[e] = pool4(v0, v1, v2, v3, code);
                                cw |= code << (8 * e);
                                continue;
                            }
                            float best = v0 > 0.f ? v0 : 0.f;
                            int idx = 0;
                            const float r1 = v1 > 0.f ? v1 : 0.f, r2 = v2 > 0.f ? v2 : 0.f, r3 = v3 > 0.f ? v3 : 0.f;
                            if (r1 > best) { best = r1; idx = 1; }
                            if (r2 > best) { best = r2; idx = 2; }
                            if (r3 > best) { best = r3; idx = 3; }
                            pv[e] = best;
                            cw |= (uint32_t)(best > 0.f ? idx : slk::CODE_NONE) << (8 * e);
                        }
                        const bool owner = C::HW == 32 ? (r & 1) == 0 : (r & 17) == 0;
                        if (owner) {
                            int y, x;
                            if (C::HW == 32) {
                                const int q = wn * 128 + 2 * pp * 32 + r;
                                y = cur.rb * C::TR + q / 32;
                                x = q % 32;
                            } else {
                                const int q = wn * 128 + pp * 32 + r;
                                y = cur.rb * C::TR + q / 16;
                                x = q % 16;
                            }
                            const int ch0 = cur.cob * C::MT + wm * 64 + ct * 32 + 8 * g4 + 4 * h;
                            const size_t o = (((size_t)(cur.n * (C::CO / 8) + (ch0 >> 3)) * PH + (y >> 1)) * PH + (x >> 1)) * 8 + (ch0 & 7);
                            *reinterpret_cast<uint2*>(out + o) = make_uint2(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]));
                            *reinterpret_cast<uint32_t*>(out2 + o) = cw;
                        }
                    }
                }
            }
        }

        if (tail) break;
        cur = nxt;
#pragma unroll
        for (int d = 0; d < C::NDW; ++d) pcur[d] = pnxt[d];
        tn += grid;
        nxt = tile_state<C>(tn, B);
        tile_poff<C>(nxt, wave, lane, pnxt);
    }
}

#ifndef SLK_WIDE_FW
#define SLK_WIDE_FW 4
#endif
#ifndef SLK_WIDE_NWV
#define SLK_WIDE_NWV 4
#endif
#ifndef SLK_WIDE_K32
#define SLK_WIDE_K32 1
#endif
// Per-layer kernel choice from tools/ablate_wide.py on MI355X (B = 4096): conv2 forward runs faster on
// the 32x32x16 form (0.655 vs 0.693 ms), conv3 forward on the 16x16x32 form (0.585 vs 0.672), conv3
// dgrad ties (0.667 / 0.672). SLK_WIDE_K32 = 0 / 2 forces all-16x16 / all-32x32 for A/B runs.
#if SLK_WIDE_K32 == 2
using CfgConv2Fwd = Conv32Cfg<64, 128, 32, wide::MODE_FWD_POOL>;
using CfgConv3Fwd = Conv32Cfg<128, 256, 16, wide::MODE_FWD_POOL>;
#elif SLK_WIDE_K32 == 1
using CfgConv2Fwd = Conv32Cfg<64, 128, 32, wide::MODE_FWD_POOL>;
using CfgConv3Fwd = ConvCfg<128, 256, 16, 128, wide::MODE_FWD_POOL, SLK_WIDE_FW, SLK_WIDE_NWV>;
#else
using CfgConv2Fwd = ConvCfg<64, 128, 32, 128, wide::MODE_FWD_POOL, SLK_WIDE_FW, SLK_WIDE_NWV>;
using CfgConv3Fwd = ConvCfg<128, 256, 16, 128, wide::MODE_FWD_POOL, SLK_WIDE_FW, SLK_WIDE_NWV>;
#endif
// Backward: no unpooled gradient is ever materialised. conv3's dgrad and wgrad read the pooled cut
// gradient dcut + code3 and route it while staging (EXP); conv3's dgrad writes dp2 (the gradient of
// p2, 16 x 16), which conv2's dgrad and wgrad route by code2 the same way.
// waves per workgroup of the two dgrads (round 6: conv3's at 8 waves, one workgroup per CU, 0.4915 -> 0.4648 ms,
// bitwise equal; conv3's forward stays at 4: 0.517 vs 0.526; profiles/r06_ab_wide_conv_waves.txt)
#ifndef SLK_WIDE_C3D_NWV
#define SLK_WIDE_C3D_NWV 8
#endif
using CfgConv3Dgrad = ConvCfg<256, 128, 16, 128, wide::MODE_DGRAD_PLAIN, SLK_WIDE_FW, SLK_WIDE_C3D_NWV, 1>;
using CfgConv2Dgrad = ConvCfg<128, 64, 32, 64, wide::MODE_DGRAD_MASK, 4, 4, 1>;  // (8 waves: its 4-KB weight slices do not split)

template <class C>
static int launch_conv(const uint16_t* in, const uint16_t* wsh, const void* aux, uint16_t* out, uint8_t* out2,
                       int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && in && wsh && out && (aux || C::MODE == wide::MODE_DGRAD_PLAIN));
    if (C::MODE == wide::MODE_FWD_POOL) SLK_CHECK_ARG(out2 != nullptr);
    if (B == 0) return 0;
    const long ntiles = (long)B * C::RB * C::NCB;
    long grid = C::NWV == 4 ? 512 : 256;               // 2 (4-wave) or 1 (8-wave) workgroups per CU
#if SLK_WIDE_XCD
    const long span = 8L * ((B + 7) / 8) * C::RB * C::NCB;  // tile indices covering every image
    if (span < grid) grid = span;                           // a multiple of 8
#else
    if (ntiles < grid) grid = C::NCB == 2 ? ((ntiles + 15) / 16) * 16 : ntiles;
#endif
    if constexpr (C::K32)
        hipLaunchKernelGGL(wide_conv32_kernel<C>, dim3((unsigned)grid), dim3(256), 0, slk_stream(stream), in, wsh, aux,
                           out, out2, B);
    else
        hipLaunchKernelGGL(wide_conv_kernel<C>, dim3((unsigned)grid), dim3(C::THREADS), 0, slk_stream(stream), in, wsh,
                           aux, out, out2, B);
    return slk_launch_status();
}

extern "C" int slk_wide_conv2_fwd(const uint16_t* a1, const uint16_t* w2f, const float* b2, uint16_t* p2,
                                  uint8_t* code2, int B, void* stream) {
    return launch_conv<CfgConv2Fwd>(a1, w2f, b2, p2, code2, B, stream);
}
extern "C" int slk_wide_conv3_fwd(const uint16_t* p2, const uint16_t* w3f, const float* b3, uint16_t* cut,
                                  uint8_t* code3, int B, void* stream) {
    return launch_conv<CfgConv3Fwd>(p2, w3f, b3, cut, code3, B, stream);
}
extern "C" int slk_wide_conv3_dgrad(const uint16_t* dcut, const uint8_t* code3, const uint16_t* w3d, uint16_t* dp2,
                                    int B, void* stream) {
    SLK_CHECK_ARG(code3 != nullptr);
    return launch_conv<CfgConv3Dgrad>(dcut, w3d, nullptr, dp2, const_cast<uint8_t*>(code3), B, stream);
}
extern "C" int slk_wide_conv2_dgrad(const uint16_t* dp2, const uint8_t* code2, const uint16_t* w2d, const uint64_t* a1bits,
                                    uint16_t* da1m, int B, void* stream) {
    SLK_CHECK_ARG(code2 != nullptr && a1bits != nullptr);
    return launch_conv<CfgConv2Dgrad>(dp2, w2d, a1bits, da1m, const_cast<uint8_t*>(code2), B, stream);
}

// ============================================================================ conv3x3 weight gradient
// dW[co][ci][tap] = sum_{n,y,x} dC[n][co][y][x] * In[n][ci][y+ky-1][x+kx-1];  db[co] = sum dC.
// GEMM M = co, N = (tap, ci), K = pixels. A workgroup (8 waves, 1 per CU) owns a 128-co x 64-ci block
// of dW (all 9 taps) and a K-split share of the batch's (image, row-block) tiles; each wave holds
// 64 co x (9 taps x 16 ci) = 4 x 9 accumulators of v_mfma_f32_16x16x32_bf16 (144 VGPRs). Both operands
// need 8 consecutive PIXELS per lane while the C8 layout stores 8 consecutive CHANNELS per 16 bytes, so
// the fragments come from LDS by ds_read_b64_tr_b16 (the hardware transpose read): dC tile
// [16 chunks][TR*W pixels] and the input halo tile [8 chunks][(TR+2)*(W+2) pixels], chunk planes
// padded to a stride of 64 mod 256 bytes so every 32-lane half of a transposed read hits 64 distinct
// banks. The whole next tile streams in by LDS-DMA while the current one is on the MFMAs (2 buffers,
// one wait + barrier per tile). db rides along as one MFMA per step against a ones fragment. Each
// workgroup writes its partial dW/db into its own slab (torch layout [co][ci][3][3] | db), reduced in
// fixed order by slk_reduce_slabs / slk_adam_from_slabs.
// SP (round 6, the default): dC is the max-pool backward of a pooled gradient, so in every block of 4
// consecutive pixels of one row (x % 4 == 0: two pool windows' columns) at most 2 values per co are nonzero —
// the 2:4 structure of v_smfmac_f32_16x16x64_bf16 (layout measured on the f16 form: slk_x3.hip's x3p notes,
// tools/ubench/smfmac_probe.hip). The staging writes dC as compressed records (the exact register image of a
// lane's A fragment: 8 bf16 + a u16 index word) instead of the dense tile, and each K64 step issues 4 x 9
// sparse instructions instead of 2 x 4 x 9 dense ones on the same B fragments: the same products, summed in
// another order (slabs within ~1e-8 of the dense form's).
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
// the K5 weight gradients on the 2:4-sparse bf16 MFMA (wide_wgrad_kernel<C, true>; 0: the dense form)
#ifndef SLK_WIDE_WG_SPARSE
#define SLK_WIDE_WG_SPARSE 1
#endif
#ifndef SLK_WIDE_WG_SPLIT
#define SLK_WIDE_WG_SPLIT 1
#endif
#ifndef SLK_WIDE_WG_ABL
#define SLK_WIDE_WG_ABL 0  // profiling only (wrong results): 1 no dC staging (sparse records), 2 no MFMA steps
#endif

template <int CI_, int CO_, int HW_, int TR_, int EXP_ = 0>
struct WgCfg {
    static constexpr int CI = CI_, CO = CO_, HW = HW_, TR = TR_;
    // EXP: dC is the max-pool backward of a pooled gradient + routing code (as ConvCfg::EXP), expanded
    // into the dC tile in registers; the input halo tile still moves by LDS-DMA
    static constexpr bool EXP = EXP_;
    static constexpr int XITEMS = 16 * (TR / 2) * (HW / 2);   // pooled dC chunks per tile (16 planes)
    static constexpr int COB = 128, CIB = 64;
    static constexpr int NCOB = CO / COB, NCIB = CI / CIB, NBLK = NCOB * NCIB;
    static constexpr int NPX = TR * HW;                  // pixels per tile (K per tile)
    static constexpr int NPXP = NPX + 4;                 // dC plane stride (pixels): 64 mod 256 bytes
    static constexpr int PW = HW + 2;
    static constexpr int NP = (TR + 2) * PW;
    static constexpr int ND = (NP + 63) / 64;
    static constexpr int NPI = ND * 64 + 4;              // input plane stride (pixels)
    static constexpr int DC_BYTES = (COB / 8) * NPXP * 16;
    static constexpr int IN_BYTES = (CIB / 8) * NPI * 16;
    static constexpr int BUF = DC_BYTES + IN_BYTES;
    static constexpr int RAW = EXP ? XITEMS * 24 : 0;    // EXP staging: values [512][16 B], code dwords 2 x [512][4 B]
    static constexpr int LDS = 2 * BUF + RAW;
    static constexpr int KS = NPX / 32;                  // MFMA k-steps per tile
    static constexpr int RB = HW / TR;
    static constexpr int SLAB = CO * CI * 9 + CO;
    static constexpr int KSPLIT = 256 / NBLK;            // one workgroup per CU
    // SP (the 2:4-sparse form, wide_wgrad_kernel<C, true>): the tile's dC as compressed records
    // [K64 step][ga 4][co 128][8 bf16] + u16 index words [step][ga][co], then the input tile
    static constexpr int KS64 = NPX / 64;
    static constexpr int SREC = KS64 * 4 * COB * 16, SIDX = KS64 * 4 * COB * 2;
    static constexpr int SDC = (SREC + SIDX + 1023) / 1024 * 1024;
    static constexpr int SBUF = SDC + IN_BYTES;
    static_assert(NPX % 32 == 0 && (HW == 32 || HW == 16), "tile");
    static_assert(!EXP || (NPX == 128 && COB == 128 && (HW == 32 ? TR == 4 : TR == 8)), "SP staging geometry");
    static_assert(DC_BYTES % 16 == 0 && ((NPX * 16) % 1024) == 0, "dC rows move in whole KiB");
    static_assert(!EXP || XITEMS == 512, "EXP: one pooled chunk per thread");
};

template <class C, bool SP = false>
__global__ __launch_bounds__(512, 1) void wide_wgrad_kernel(const uint16_t* __restrict__ dc,
                                                            const uint16_t* __restrict__ in,
                                                            float* __restrict__ slabs, int B,
                                                            const uint8_t* __restrict__ dcode = nullptr) {
    static_assert(!SP || C::EXP, "the sparse form stages dC from the pooled gradient");
    constexpr int BUF = SP ? C::SBUF : C::BUF;           // one of the two tile buffers
    constexpr int DCB = SP ? C::SDC : C::DC_BYTES;       // offset of the input tile in a buffer
    // SPLIT: the raw pooled dC double-buffered (DMA two tiles ahead), so half the waves (4-7) can stage the next
    // tile's records before their MFMAs and the other half after (the SIMD pair (w, w + 4) overlaps one's staging
    // with the other's MFMAs); otherwise every wave stages after its MFMAs
    // (conv2's kernel only: conv3's spilled 13 VGPRs with it, 0.369 -> 0.490 ms; conv2 0.373 -> 0.365,
    // profiles/r06_ab_wide_wgrad_split.txt)
    constexpr bool SPLIT = SP && SLK_WIDE_WG_SPLIT && C::HW == 32;
    __shared__ __attribute__((aligned(1024))) char smem[2 * BUF + (SPLIT ? 2 : 1) * C::RAW];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    // XCD-aware block placement: the NBLK blocks of one K-split share sit 8 workgroups apart
    const int w = blockIdx.x;
    int blk, ks;
    if (C::NBLK == 1) { blk = 0; ks = w; }
    else { blk = (w >> 3) % C::NBLK; ks = ((w >> 3) / C::NBLK) * 8 + (w & 7); }
    const int cob = blk / C::NCIB, cib = blk - (blk / C::NCIB) * C::NCIB;

    // per-lane transposed-read bases (bytes within a buffer)
    const int q = lane >> 4, ig = lane & 15, a = ig >> 2, p = ig & 3;
    const int a_base = (((wm * 64 + 4 * p) >> 3) * C::NPXP + 8 * q + a) * 16 + (p & 1) * 8;
    const int pl = 8 * q + a, r0 = pl / C::HW, x0 = pl % C::HW;
    // wave wn owns input channels cib*64 + 16*wn .. +15 (chunks 2wn, 2wn+1) for all 9 taps
    const int b_base = DCB + (((2 * wn + (p >> 1)) * C::NPI) + (r0 + 1) * C::PW + x0 + 1) * 16 + (p & 1) * 8;
    const bool do_db = cib == 0;
    const short one = 0x3F80;  // bf16 1.0
    const bf16x8 ones = __builtin_bit_cast(bf16x8, (__attribute__((ext_vector_type(8))) short){one, one, one, one, one, one, one, one});

    f32x4 acc[4][9];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int u = 0; u < 9; ++u) acc[i][u] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 accb = f32x4{0.f, 0.f, 0.f, 0.f};

    // tile t -> (image, row block). XCD grouping: ks and ks + 8 share an XCD, so tiles t = ks + k*KSPLIT
    // with equal t % 8 run there together; all RB row blocks of image n go to XCD n % 8.
    auto tile_of = [&](int t, int& n, int& rb) {
#if SLK_WIDE_XCD
        const int j = t >> 3;
        rb = j % C::RB;
        n = (j / C::RB) * 8 + (t & 7);
#else
        n = t / C::RB;
        rb = t - n * C::RB;
#endif
    };
    auto valid = [&](int t) {
        int n, rb;
        tile_of(t, n, rb);
        return n < B;
    };
    // EXP: pooled dC chunk tid = (plane c, pooled row pr, pooled col px) of tile t, staged by this
    // thread's own wave (LDS-DMA into `raw`), so its expansion needs only that wave's vmcnt wait
    char* const raw = smem + 2 * BUF;  // SPLIT: raw buffer k & 1 holds the pooled dC of this workgroup's tile k
    auto exp_issue_dc = [&](int t, char* raw) {
        int n, rb;
        tile_of(t, n, rb);
        constexpr int PH = C::HW / 2, PR = C::TR / 2;
        const int c = tid / (PR * PH), rem = tid - c * (PR * PH), pr = rem / PH, px = rem - pr * PH;
        const size_t idx = ((size_t)(n * (C::CO / 8) + cob * 16 + c) * PH + rb * PR + pr) * PH + px;
        const int i0 = wave * 64;
        glds16(reinterpret_cast<const char*>(dc) + idx * 16, lds_u32(raw + i0 * 16));
        glds4(dcode + idx * 8, lds_u32(raw + C::XITEMS * 16 + i0 * 4));
        glds4(dcode + idx * 8 + 4, lds_u32(raw + C::XITEMS * 20 + i0 * 4));
    };
    auto exp_expand_dc = [&](char* buf) {
        constexpr int PH = C::HW / 2, PR = C::TR / 2;
        const int c = tid / (PR * PH), rem = tid - c * (PR * PH), pr = rem / PH, px = rem - pr * PH;
        const uint4 v = *reinterpret_cast<const uint4*>(raw + tid * 16);
        const uint32_t c0 = *reinterpret_cast<const uint32_t*>(raw + C::XITEMS * 16 + tid * 4);
        const uint32_t c1 = *reinterpret_cast<const uint32_t*>(raw + C::XITEMS * 20 + tid * 4);
        const uint32_t cA = __builtin_amdgcn_perm(0u, c0, 0x01010000u), cB = __builtin_amdgcn_perm(0u, c0, 0x03030202u);
        const uint32_t cC = __builtin_amdgcn_perm(0u, c1, 0x01010000u), cD = __builtin_amdgcn_perm(0u, c1, 0x03030202u);
        char* base = buf + (c * C::NPXP + 2 * pr * C::HW + 2 * px) * 16;
        // lanes with px & 4 walk the window's columns in the other order: the 8 lanes of a ds_write_b128
        // group then fill all 8 16-B slots of 128 B (same order: 2-way on every store, 8.4 M cycles a launch)
        const int f = (px >> 2) & 1;
#pragma unroll
        for (int pos0 = 0; pos0 < 4; ++pos0) {
            const int pos = pos0 ^ f;
            *reinterpret_cast<uint4*>(base + ((pos >> 1) * C::HW + (pos & 1)) * 16) = route_chunk(v, cA, cB, cC, cD, pos);
        }
    };
    auto issue_tile = [&](int t, char* buf) {
        int n, rb;
        tile_of(t, n, rb);
        // dC rows: 16 chunk planes x (NPX*16/1024) KiB, 4 pieces per wave
        constexpr int PPC = C::NPX * 16 / 1024;
#pragma unroll
        for (int k = 0; k < (C::EXP ? 0 : (16 * PPC) / 8); ++k) {
            const int piece = wave * ((16 * PPC) / 8) + k;
            const int c = piece / PPC, part = piece - (piece / PPC) * PPC;
            const char* src = reinterpret_cast<const char*>(dc) +
                              (((size_t)(n * (C::CO / 8) + cob * 16 + c) * C::HW + rb * C::TR) * C::HW) * 16 +
                              part * 1024 + lane * 16;
            glds16((const void*)src, lds_u32(buf + c * C::NPXP * 16 + part * 1024));
        }
        // input halo tile: wave w moves chunk plane w (ND pieces), halo lanes read zeros
        const char* plane = reinterpret_cast<const char*>(in) +
                            ((size_t)(n * (C::CI / 8) + cib * 8 + wave) * (C::HW * C::HW)) * 16;
#pragma unroll
        for (int d = 0; d < C::ND; ++d) {
            const int P = d * 64 + lane;
            const int ry = P / C::PW, rx = P - (P / C::PW) * C::PW;
            const int y = rb * C::TR - 1 + ry, x = rx - 1;
            const bool ok = P < C::NP && y >= 0 && y < C::HW && x >= 0 && x < C::HW;
            const char* src = ok ? plane + (size_t)(y * C::HW + x) * 16 : reinterpret_cast<const char*>(slk_wide_zero);
            glds16((const void*)src, lds_u32(buf + DCB + wave * C::NPI * 16 + d * 1024));
        }
    };

    // SP geometry. K64 step s of a tile = 16 blocks of 4 pixels of one row (x % 4 == 0): block L = 16 s + 4 gb + jb
    // is row y, block xb (pixels 4 xb .. +3) with, for HW = 32, y = 2 s + (gb >> 1), xb = 2 (gb & 1) + (jb & 1) +
    // 4 (jb >> 1); for HW = 16, y = 4 s + 2 (gb >> 1) + (jb >> 1), xb = 2 (gb & 1) + (jb & 1). So blocks jb, jb + 1
    // (one record half) are adjacent (a window quad), and the two lane groups gb = 0, 1 of a 32-lane half of a
    // B read are 8 pixels (128 B) apart: their transposed reads hit disjoint banks.
    // B (input tile, ds_read_b64_tr_b16): lane (gb, ig = 4 a + p) reads pixel 4 xb + a of row y, chunk plane
    // 2 wn + (p >> 1), 8-B half p & 1 (as the dense read): one read per block, 4 per fragment.
    // one per-lane base (block L = 4 gb) + a compile-time offset per (s, jb)
    const int spb0 = DCB + (((2 * wn + (p >> 1)) * C::NPI) + ((C::HW == 32 ? (q >> 1) : 2 * (q >> 1)) + 1) * C::PW +
                            8 * (q & 1) + a + 1) * 16 + (p & 1) * 8;
    auto spb_off = [](int st, int jb) {
        return C::HW == 32 ? (2 * st * C::PW + 4 * (jb & 1) + 16 * (jb >> 1)) * 16
                           : ((4 * st + (jb >> 1)) * C::PW + 4 * (jb & 1)) * 16;
    };
    // A: lane (ga = q, m = ig) of M tile i reads record (s, ga, co = 64 wm + 16 i + m) and its index word
    const int sp_arec = ((q * C::COB) + wm * 64 + ig) * 16, sp_aidx = C::SREC + ((q * C::COB) + wm * 64 + ig) * 2;
    // SP staging: thread (wave w, lane l) = items (co = 8 c + (l & 7), c = 2 w + k, k = 0, 1; pooled row pr; window quad
    // P): the quad's 4 windows (pooled px = 4 P .. +3, the raw items this wave's own DMA staged) are the two blocks
    // 2 P, 2 P + 1 of output rows 2 pr + d, i.e. one record half (8 B) + one index byte per d. Lane bits 0-2 = co,
    // bit 3 = the half (P & 1): a 16-lane ds_write_b64 group covers 16 distinct 8-B slots of 128 B.
    const int sco = lane & 7, sP0 = (lane >> 3) & 1, srest = lane >> 4;
    const int spr = C::HW == 32 ? (srest & 1) : srest, sP = C::HW == 32 ? sP0 + 2 * (srest >> 1) : sP0;
    auto sp_expand = [&](char* buf, const char* raw) {
        if (SLK_WIDE_WG_ABL & 1) return;  // profiling only
        constexpr int PH = C::HW / 2, PR = C::TR / 2;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int c = 2 * wave + k, co = 8 * c + sco;
            const int i0 = c * (PR * PH) + spr * PH + 4 * sP;
            const char* rv = raw + i0 * 16 + sco * 2;
            const char* rc = raw + C::XITEMS * 16 + (sco >> 2) * C::XITEMS * 4 + i0 * 4 + (sco & 3);
            uint32_t v[4], cb[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = *reinterpret_cast<const uint16_t*>(rv + j * 16);
                cb[j] = *reinterpret_cast<const uint8_t*>(rc + j * 4);
            }
            const uint32_t cw = cb[0] | (cb[1] << 8) | (cb[2] << 16) | (cb[3] << 24);
            // index byte: window j's position in its block = its dx (code bit 0), + 2 for the block's second window
            // (a window routed elsewhere keeps that position with a zero value)
            const uint32_t ib = (cw & 1u) | ((cw >> 6) & 4u) | ((cw >> 12) & 16u) | ((cw >> 18) & 64u) | 0x88u;
            const uint32_t rowp = (cw >> 1) & 0x7F7F7F7Fu;  // per byte: 0 / 1 = routed row parity, 2 = blocked
            const uint32_t H0 = v[0] | (v[1] << 16), H1 = v[2] | (v[3] << 16);
#pragma unroll
            for (int d = 0; d < 2; ++d) {
                const uint32_t z = (d ? (rowp & ~(rowp >> 1)) : ~(rowp | (rowp >> 1))) & 0x01010101u;
                const uint32_t m8 = z * 0xFFu;
                const uint32_t mA = __builtin_amdgcn_perm(0u, m8, 0x01010000u), mB = __builtin_amdgcn_perm(0u, m8, 0x03030202u);
                const int ga = C::HW == 32 ? 2 * (sP >> 1) + d : 2 * d + (spr & 1);
                const int st = C::HW == 32 ? spr : spr >> 1;
                const int rec = (st * 4 + ga) * C::COB + co;
                *reinterpret_cast<uint2*>(buf + rec * 16 + sP0 * 8) = make_uint2(H0 & mA, H1 & mB);
                buf[C::SREC + rec * 2 + sP0] = (char)ib;
            }
        }
    };

    int t = ks, b = 0;
    if (valid(t)) {
        issue_tile(t, smem);
        if constexpr (C::EXP) {
            exp_issue_dc(t, raw);
            wait_vmcnt<0>();
            if constexpr (SP) sp_expand(smem, raw);
            else exp_expand_dc(smem);
            if (SPLIT && valid(t + C::KSPLIT)) exp_issue_dc(t + C::KSPLIT, raw + C::RAW);
        }
    }
    const bool sfirst = wave >= 4;
#pragma unroll 1
    for (; valid(t); t += C::KSPLIT) {
        wait_vmcnt<0>();
        if constexpr (C::EXP) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // dC tile written
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const bool more = valid(t + C::KSPLIT);
        if (more) {
            issue_tile(t + C::KSPLIT, smem + (b ^ 1) * BUF);
            if constexpr (SPLIT) {
                // tile k + 2's pooled dC into raw buffer k & 1 (tile k's, staged during tile k - 1)
                if (valid(t + 2 * C::KSPLIT)) exp_issue_dc(t + 2 * C::KSPLIT, raw + b * C::RAW);
            } else if constexpr (C::EXP) {
                exp_issue_dc(t + C::KSPLIT, raw);
            }
        }
        // SPLIT: tile k + 1's raw dC landed by the wait above (its DMA was issued a tile ago)
        if (SPLIT && more && sfirst) sp_expand(smem + (b ^ 1) * BUF, raw + (b ^ 1) * C::RAW);
        const char* buf = smem + b * BUF;
        if constexpr (SP && !(SLK_WIDE_WG_ABL & 2)) {
            typedef __attribute__((address_space(3))) bf16x4* lp4;
            typedef __bf16 bf16x16 __attribute__((ext_vector_type(16)));
            const bf16x16 ones16 = __builtin_shufflevector(ones, ones, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
#pragma unroll
            for (int st = 0; st < C::KS64; ++st) {
                bf16x8 av[4];
                int ix[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    av[i] = *reinterpret_cast<const bf16x8*>(buf + sp_arec + st * 4 * C::COB * 16 + i * 256);
                    ix[i] = *reinterpret_cast<const uint16_t*>(buf + sp_aidx + st * 4 * C::COB * 2 + i * 32);
                }
                if (do_db) {  // wave (wm, wn) sums co fragment wn
                    bf16x8 adb = av[0];
                    int idb = ix[0];
#pragma unroll
                    for (int i = 1; i < 4; ++i) {
                        adb = wn == i ? av[i] : adb;
                        idb = wn == i ? ix[i] : idb;
                    }
                    accb = __builtin_amdgcn_smfmac_f32_16x16x64_bf16(adb, ones16, accb, idb, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < 9; ++u) {  // u = tap
                    const int toff = ((u / 3 - 1) * C::PW + (u % 3 - 1)) * 16;
                    bf16x4 r4[4];
#pragma unroll
                    for (int jb = 0; jb < 4; ++jb) r4[jb] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp4)(buf + spb0 + spb_off(st, jb) + toff));
                    const bf16x16 bv = __builtin_shufflevector(__builtin_shufflevector(r4[0], r4[1], 0, 1, 2, 3, 4, 5, 6, 7),
                                                               __builtin_shufflevector(r4[2], r4[3], 0, 1, 2, 3, 4, 5, 6, 7),
                                                               0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[i][u] = __builtin_amdgcn_smfmac_f32_16x16x64_bf16(av[i], bv, acc[i][u], ix[i], 0, 0);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < (SP ? 0 : C::KS); ++j) {
            typedef __attribute__((address_space(3))) bf16x4* lp4;
            bf16x8 av[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const char* pa = buf + a_base + i * 2 * C::NPXP * 16 + j * 32 * 16;
                const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp4)pa);
                const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp4)(pa + 64));
                av[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            }
            if (do_db) {  // wave (wm, wn) sums co fragment wn
                bf16x8 adb = av[0];
#pragma unroll
                for (int i = 1; i < 4; ++i) adb = wn == i ? av[i] : adb;
                accb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(adb, ones, accb, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < 9; ++u) {               // u = tap
                const int toff = ((u / 3 - 1) * C::PW + (u % 3 - 1)) * 16;
                const char* pb = buf + b_base + toff + j * (32 / C::HW) * C::PW * 16;
                const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp4)pb);
                const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp4)(pb + 64));
                const bf16x8 bv = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
                if (SLK_WIDE_PRIO & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv, acc[i][u], 0, 0, 0);
                if (SLK_WIDE_PRIO & 2) __builtin_amdgcn_s_setprio(0);
            }
        }
        // EXP: the next tile's dC, routed into the other buffer (free since this tile's barrier) once
        // this wave's staging DMA has landed
        if constexpr (SPLIT) {
            if (more && !sfirst) sp_expand(smem + (b ^ 1) * BUF, raw + (b ^ 1) * C::RAW);
        } else if constexpr (C::EXP) {
            if (more) {
                wait_vmcnt<0>();
                if constexpr (SP) sp_expand(smem + (b ^ 1) * BUF, raw);
                else exp_expand_dc(smem + (b ^ 1) * BUF);
            }
        }
        b ^= 1;
    }

    // partial dW / db -> slab ks (torch layout)
    float* slab = slabs + (size_t)ks * C::SLAB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int u = 0; u < 9; ++u) {
            const int tap = u;
            const int ci = cib * C::CIB + wn * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = cob * C::COB + wm * 64 + i * 16 + 4 * (lane >> 4) + r;
                slab[((size_t)co * C::CI + ci) * 9 + tap] = acc[i][u][r];
            }
        }
    }
    if (do_db && (lane & 15) == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) slab[C::CO * C::CI * 9 + cob * C::COB + wm * 64 + wn * 16 + 4 * (lane >> 4) + r] = accb[r];
    }
}

using CfgWg2 = WgCfg<64, 128, 32, 4, 1>;   // dC = routed dp2 (EXP)
using CfgWg3 = WgCfg<128, 256, 16, 8, 1>;   // dC = routed dcut (EXP)

template <class C>
static int launch_wgrad(const uint16_t* dc, const uint16_t* in, float* slabs, int B, void* stream,
                        const uint8_t* dcode = nullptr) {
    SLK_CHECK_ARG(B >= 0 && dc && in && slabs && (!C::EXP || dcode));
    hipLaunchKernelGGL((wide_wgrad_kernel<C, SLK_WIDE_WG_SPARSE != 0>), dim3(256), dim3(512), 0, slk_stream(stream), dc, in,
                       slabs, B, dcode);
    return slk_launch_status();
}

extern "C" int slk_wide_conv2_wgrad_nslab(int B) { return B >= 0 ? CfgWg2::KSPLIT : 0; }
extern "C" int slk_wide_wgrad_form() { return SLK_WIDE_WG_SPARSE ? 1 : 0; }
extern "C" int slk_wide_conv3_wgrad_nslab(int B) { return B >= 0 ? CfgWg3::KSPLIT : 0; }
extern "C" int slk_wide_conv2_wgrad(const uint16_t* dp2, const uint8_t* code2, const uint16_t* a1, float* slabs, int B,
                                    void* stream) {
    return launch_wgrad<CfgWg2>(dp2, a1, slabs, B, stream, code2);
}
extern "C" int slk_wide_conv3_wgrad(const uint16_t* dcut, const uint8_t* code3, const uint16_t* p2, float* slabs, int B,
                                    void* stream) {
    return launch_wgrad<CfgWg3>(dcut, p2, slabs, B, stream, code3);
}

// ============================================================================ conv1 (3 -> 64), bf16 MFMA
// conv1 is a 64 x 27 contraction per pixel: one 16x16x32 MFMA K-step with K = (ci, ky, kx) padded to
// 32 (k = 27 is a constant-1 column in the weight gradient: it yields db1 for free). The zero-padded
// image [3][34][34] is staged in LDS as f32 (14 elements per thread: offsets computed once, all loads
// issued back to back); each lane gathers its 8 im2col values of a fragment from it and converts them
// to bf16. HBM-bound: the forward writes a1 (128 KB/sample), the weight gradient reads da1m.
// LDS pitches of the staged image (bank model over both kernels' im2col reads, ds_read_b32 = dword mod 32 over
// 32-lane halves): rows of 35 and planes of 1,233 floats leave the weight gradient's B-fragment gathers 4 and
// the forward's 16 extra cycles per fragment where the dense [3][34][34] image had 46 and 135 (8.6 M and
// 2.9 M conflict cycles per launch)
constexpr int C1P = 35;                               // row pitch (32 + 2 halo + 1 pad)
constexpr int C1PS = 1233;                            // plane pitch (35 x 35 + 8)
constexpr int C1S = (3 * C1P * C1P + 255) / 256;      // 15 staged elements per thread

__device__ __forceinline__ void stage_offsets(int (&off)[C1S]) {
#pragma unroll
    for (int k = 0; k < C1S; ++k) {
        const int e = threadIdx.x + 256 * k;
        const int ci = e / (C1P * C1P), r = e - ci * (C1P * C1P);
        const int yy = r / C1P - 1, xx = r % C1P - 1;
        off[k] = (e < 3 * C1P * C1P && yy >= 0 && yy < 32 && xx >= 0 && xx < 32) ? (ci * 32 + yy) * 32 + xx : -1;
    }
}
__device__ __forceinline__ void stage_load(const float* __restrict__ img, const int (&off)[C1S], float (&v)[C1S]) {
#pragma unroll
    for (int k = 0; k < C1S; ++k) v[k] = off[k] >= 0 ? img[off[k]] : 0.f;
}
__device__ __forceinline__ void stage_store(float* xs, const float (&v)[C1S]) {
#pragma unroll
    for (int k = 0; k < C1S; ++k) {
        const int e = threadIdx.x + 256 * k;
        const int ci = e / (C1P * C1P);
        if (e < 3 * C1P * C1P) xs[e + ci * (C1PS - C1P * C1P)] = v[k];
    }
}
// im2col offset of K index k (ci*C1PS + ky*C1P + kx) inside the padded image, -1 for k >= 27
__device__ __forceinline__ int im2col_off(int k) {
    const int ci = k / 9, t = k - (k / 9) * 9;
    return k < 27 ? ci * C1PS + (t / 3) * C1P + t % 3 : -1;
}

// Forward: a1[co][px] = relu(sum_k W1b[co][k] * bf16(x)[k][px] + b1[co]); A = W1b (4 fragments in
// registers for the whole launch), B = the im2col fragment of 16 pixels. Wave w of a workgroup takes
// pixel fragments w, w+4, ... of its image; grid-strided over images.
// a1bits (optional): the ReLU word of every pixel, [B][1024] u64, bit c = (the stored bf16 a1[c] != 0), i.e.
// a1[c] > 0 (relu output: +0 or positive) — conv2's dgrad masks with it instead of re-reading a1. Lane
// (col, q) holds channels 16 cf + 4 q + r of pixel col; the four q lanes' nibbles are OR-combined by two
// lane swaps and lanes q = 0 store 16 consecutive pixels' words (128 B).
__global__ __launch_bounds__(256) void wide_conv1_fwd_kernel(const float* __restrict__ x, const uint16_t* __restrict__ w1b,
                                                             const float* __restrict__ b1, uint16_t* __restrict__ a1, int B,
                                                             uint2* __restrict__ a1bits = nullptr) {
    __shared__ float xs[3 * C1PS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = lane >> 4, col = lane & 15;
    bf16x8 av[4];
    float bias[4][4];
#pragma unroll
    for (int cf = 0; cf < 4; ++cf) {
        av[cf] = *reinterpret_cast<const bf16x8*>(w1b + (cf * 16 + col) * 32 + 8 * q);
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[cf][r] = b1[cf * 16 + 4 * q + r];
    }
    int koff[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) koff[j] = im2col_off(8 * q + j);
    int off[C1S];
    stage_offsets(off);
#pragma unroll 1
    for (int n = blockIdx.x; n < B; n += gridDim.x) {
        float v[C1S];
        stage_load(x + (size_t)n * 3 * 1024, off, v);
        __syncthreads();
        stage_store(xs, v);
        __syncthreads();
#pragma unroll 2
        for (int f = wave; f < 64; f += 4) {
            const int y = f >> 1, xx = (f & 1) * 16 + col;
            const int base = y * C1P + xx;
            float g[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) g[j] = koff[j] >= 0 ? xs[base + koff[j]] : 0.f;
            bf16x8 bv;
#pragma unroll
            for (int j = 0; j < 8; ++j) bv[j] = (__bf16)g[j];
            uint16_t* dst = a1 + ((size_t)(n * 8) * 1024 + y * 32 + xx) * 8 + 4 * (q & 1);
            uint32_t wlo = 0u, whi = 0u;
#pragma unroll
            for (int cf = 0; cf < 4; ++cf) {
                f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[cf], bv, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                float o[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float t = acc[r] + bias[cf][r];
                    o[r] = t > 0.f ? t : 0.f;
                }
                const uint32_t p0 = pack_bf16x2(o[0], o[1]), p1 = pack_bf16x2(o[2], o[3]);
                // channels cf*16 + 4q .. +3 = chunk 2cf + (q >> 1), offset 4 (q & 1)
                *reinterpret_cast<uint2*>(dst + (size_t)(2 * cf + (q >> 1)) * 1024 * 8) = make_uint2(p0, p1);
                const uint32_t nib = ((p0 & 0xFFFFu) ? 1u : 0u) | ((p0 >> 16) ? 2u : 0u) | ((p1 & 0xFFFFu) ? 4u : 0u) |
                                     ((p1 >> 16) ? 8u : 0u);
                if (cf < 2) wlo |= nib << (16 * cf + 4 * q);
                else whi |= nib << (16 * (cf - 2) + 4 * q);
            }
            if (a1bits) {
                // OR over lanes l, l ^ 32, l ^ 16 (gfx950 lane swaps: a swap of a value with itself
                // returns it with the partner half's copy in the other half)
                auto s32 = __builtin_amdgcn_permlane32_swap(wlo, wlo, false, false);
                wlo = s32[0] | s32[1];
                s32 = __builtin_amdgcn_permlane32_swap(whi, whi, false, false);
                whi = s32[0] | s32[1];
                auto s16 = __builtin_amdgcn_permlane16_swap(wlo, wlo, false, false);
                wlo = s16[0] | s16[1];
                s16 = __builtin_amdgcn_permlane16_swap(whi, whi, false, false);
                whi = s16[0] | s16[1];
                if (q == 0) a1bits[(size_t)n * 1024 + y * 32 + xx] = make_uint2(wlo, whi);
            }
        }
    }
}

// Weight gradient: dW1[co][k] = sum_px da1m[co][px] * bf16(x)[k][px] (k = 27: db1). GEMM M = 64 co,
// N = 32 k, K = pixels. da1m rows of a 4-row block land in LDS by LDS-DMA ([8 chunks][132 px], double
// buffered) and are read transposed (ds_read_b64_tr_b16); wave w takes row w of each block. Each
// workgroup walks images blockIdx.x, +grid, ...; its 4 waves' partial sums are added in fixed order
// into one slab [1792] = [dW1 (torch layout) | db1].
#ifndef SLK_WC1W_GRID
#define SLK_WC1W_GRID 512  // 2 workgroups per CU: twice the LDS-DMA bytes in flight (A/B: 0.182 -> 0.112 ms; 768: 0.112, 1024: 0.132)
#endif
constexpr int C1W_GRID = SLK_WC1W_GRID;
constexpr int C1W_NPXP = 132;                                  // 128 px + 4 pad: plane stride 64 mod 256 B
constexpr int C1W_BUF = 8 * C1W_NPXP * 16;                     // 16,896 B

__global__ __launch_bounds__(256) void wide_conv1_wgrad_kernel(const float* __restrict__ x, const uint16_t* __restrict__ da1m,
                                                               float* __restrict__ slabs, int B) {
    __shared__ __attribute__((aligned(1024))) char smem[2 * C1W_BUF + 3 * C1PS * 4];
    float* xs = reinterpret_cast<float*>(smem + 2 * C1W_BUF);
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, ig = lane & 15, a = ig >> 2, p = ig & 3, col = lane & 15;
    int koff[2];
#pragma unroll
    for (int kf = 0; kf < 2; ++kf) koff[kf] = im2col_off(kf * 16 + col);
    const int a_base = ((p >> 1) * C1W_NPXP + wave * 32 + 8 * q + a) * 16 + (p & 1) * 8;
    int off[C1S];
    stage_offsets(off);

    f32x4 acc[4][2];
#pragma unroll
    for (int cf = 0; cf < 4; ++cf)
#pragma unroll
        for (int kf = 0; kf < 2; ++kf) acc[cf][kf] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto issue = [&](int n, int rb, char* buf) {
        // 8 chunk planes x 2 KiB (4 rows x 32 px x 16 B); wave w moves chunks 2w, 2w+1
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = wave * 2 + (k >> 1), part = k & 1;
            const char* src = reinterpret_cast<const char*>(da1m) + ((size_t)(n * 8 + c) * 1024 + rb * 128) * 16 +
                              part * 1024 + lane * 16;
            glds16((const void*)src, lds_u32(buf + c * C1W_NPXP * 16 + part * 1024));
        }
    };
    const int nimg = B > (int)blockIdx.x ? (B - 1 - (int)blockIdx.x) / C1W_GRID + 1 : 0;
    const int nsteps = nimg * 8;
    float xr[C1S];
    if (nsteps > 0) {
        stage_load(x + (size_t)blockIdx.x * 3 * 1024, off, xr);
        issue(blockIdx.x, 0, smem);
    }
#pragma unroll 1
    for (int s = 0; s < nsteps; ++s) {
        const int n = blockIdx.x + (s >> 3) * C1W_GRID, rb = s & 7;
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (rb == 0) {           // all waves are done with the previous image's xs
            stage_store(xs, xr);
            __syncthreads();
        }
        if (s + 1 < nsteps) {
            const int n1 = blockIdx.x + ((s + 1) >> 3) * C1W_GRID;
            issue(n1, (s + 1) & 7, smem + ((s + 1) & 1) * C1W_BUF);
            if (rb == 7) stage_load(x + (size_t)n1 * 3 * 1024, off, xr);
        }
        const char* buf = smem + (s & 1) * C1W_BUF;
        typedef __attribute__((address_space(3))) bf16x4* lp4;
        bf16x8 av[4];
#pragma unroll
        for (int cf = 0; cf < 4; ++cf) {
            const char* pa = buf + a_base + cf * 2 * C1W_NPXP * 16;
            const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp4)pa);
            const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp4)(pa + 64));
            av[cf] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
        const int y = rb * 4 + wave;
#pragma unroll
        for (int kf = 0; kf < 2; ++kf) {
            // k >= 27 (the bias column and padding; values replaced below) reads k = 18's address: a broadcast
            const int base = y * C1P + 8 * q + (koff[kf] >= 0 ? koff[kf] : im2col_off(18));
            bf16x8 bv;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float g = xs[base + j];
                bv[j] = (__bf16)(koff[kf] >= 0 ? g : (kf * 16 + col == 27 ? 1.f : 0.f));
            }
#pragma unroll
            for (int cf = 0; cf < 4; ++cf) acc[cf][kf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[cf], bv, acc[cf][kf], 0, 0, 0);
        }
        (void)n;
    }
    // fixed-order sum of the 4 waves' partials: red[wave][co][k]
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int cf = 0; cf < 4; ++cf)
#pragma unroll
        for (int kf = 0; kf < 2; ++kf)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[(wave * 64 + cf * 16 + 4 * q + r) * 32 + kf * 16 + col] = acc[cf][kf][r];
    __syncthreads();
    float* slab = slabs + (size_t)blockIdx.x * 1792;
    for (int e = threadIdx.x; e < 64 * 28; e += 256) {
        const int co = e / 28, k = e - co * 28;
        const float v = ((red[co * 32 + k] + red[(64 + co) * 32 + k]) + red[(128 + co) * 32 + k]) + red[(192 + co) * 32 + k];
        if (k < 27) slab[co * 27 + k] = v;
        else slab[1728 + co] = v;
    }
}

extern "C" int slk_wide_conv1_fwd(const float* x, const uint16_t* w1b, const float* b1, uint16_t* a1, uint64_t* a1bits,
                                  int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && x && w1b && b1 && a1);
    if (B == 0) return 0;
    const int grid = B < 2048 ? B : 2048;
    hipLaunchKernelGGL(wide_conv1_fwd_kernel, dim3(grid), dim3(256), 0, slk_stream(stream), x, w1b, b1, a1, B,
                       reinterpret_cast<uint2*>(a1bits));
    return slk_launch_status();
}

// the ReLU words of a1 (as slk_wide_conv1_fwd writes them) from a stored a1: thread = pixel, its 8 chunks
__global__ __launch_bounds__(256) void wide_relu_bits_kernel(const uint4* __restrict__ a1, uint2* __restrict__ bits,
                                                             int npix) {
    const int i = blockIdx.x * 256 + threadIdx.x;  // global pixel (sample * 1024 + p)
    if (i >= npix) return;
    const int n = i >> 10, p = i & 1023;
    uint32_t w[2] = {0u, 0u};
#pragma unroll
    for (int c8 = 0; c8 < 8; ++c8) {
        const uint4 v = a1[((size_t)n * 8 + c8) * 1024 + p];
        const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t h = (d[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
            const int c = 8 * c8 + k;
            w[c >> 5] |= ((int16_t)h > 0 ? 1u : 0u) << (c & 31);   // a1 > 0 (sign clear, not +0)
        }
    }
    bits[i] = make_uint2(w[0], w[1]);
}
extern "C" int slk_wide_relu_bits(const uint16_t* a1, uint64_t* a1bits, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && a1 && a1bits);
    if (B == 0) return 0;
    const int npix = B * 1024;
    hipLaunchKernelGGL(wide_relu_bits_kernel, dim3((npix + 255) / 256), dim3(256), 0, slk_stream(stream),
                       reinterpret_cast<const uint4*>(a1), reinterpret_cast<uint2*>(a1bits), npix);
    return slk_launch_status();
}
extern "C" int slk_wide_conv1_wgrad_nslab(int B) { return B >= 0 ? C1W_GRID : 0; }
extern "C" int slk_wide_conv1_wgrad(const float* x, const uint16_t* da1m, float* slabs, int B, void* stream) {
    SLK_CHECK_ARG(B >= 0 && x && da1m && slabs);
    hipLaunchKernelGGL(wide_conv1_wgrad_kernel, dim3(C1W_GRID), dim3(256), 0, slk_stream(stream), x, da1m, slabs, B);
    return slk_launch_status();
}
