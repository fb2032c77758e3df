// Split-precision direct implicit-GEMM kxk convolution on 16-bit MFMA
// (v_mfma_f32_32x32x16_f16 / _bf16), gfx950.  Same semantics and ABI role as
// conv_mfma.hip / conv_wino.hip (Decoder_model conv + LeakyReLU, optional
// fused 1x1 heads; models/regression_head.py:7-8,31,50,
// models/matching_net.py:63-75).
//
// Precision modes (TMR_PREC_*):
//   F16X3  fp32-grade: x = s_x^-1 (xh + xl), w = s_w^-1 (wh + wl) with fp16
//          hi/lo parts and power-of-two scales s (max |x s| < 2^14), and
//          x.w ~= (wh xh + wl xh + wh xl) / (s_x s_w), fp32 accumulation.
//          The dropped wl xl term and the split residuals are ~2^-22
//          relative: the result keeps the fp32 path's 1e-5 contract at 1/16
//          of the MFMA cost of f32-input MFMA x 3 terms.
//   BF16   one bf16 term (unscaled), fp32 accumulation (config C).
//   F16    one scaled fp16 term.
// Every record is four 16-B pieces (64 B): F16X3 holds 16 channels as
// [hi ch0-7][hi ch8-15][lo ch0-7][lo ch8-15] (3 MFMAs per 32x32 tile per
// chunk), BF16/F16 hold 32 channels [ch0-7]..[ch24-31] (2 MFMAs).
//
// GEMM view: D[n][pixel] = sum_{tap, c} Wt[tap][n][c] X[c][pixel + tap], A =
// weights (rows n), B = activations (columns = 32 consecutive pixels of one
// output row), so a 32x32 accumulator register is one 128-B row segment of
// the NCHW output (coalesced stores / acc_init loads).
//
// Operands live in HBM in MFMA-ready 16-bit layouts written by the pack
// kernels below: per channel chunk a pixel (or output channel) is one
// 64-B record.
// Activations are zero-padded to whole tiles plus the kxk halo, so the
// kernel's loads are never masked.
//
// Block: 512 threads, 128 output channels x 512 pixels (16 rows x 32 cols).
// Waves 2 (64 n) x 4 (4 rows); a wave owns 2x4 32x32 accumulators (128 regs).
// K loop: chunk outer, taps inner, up to 3 taps per barrier step.  The 128
// weight records of step g+D stream into LDS by LDS-DMA (D+1 buffers) while
// step g computes, and the next chunk's (16+k-1)x(32+k-1) activation halo
// (2 buffers) streams in spread over the first steps; each step ends with a
// counted vmcnt (only the DMAs the next step needs) and a raw s_barrier, so
// loads stay in flight across barriers.
// In LDS the records are stored as piece planes (structure of arrays), which
// makes the ds_read_b128 fragment reads bank-conflict free with plain linear
// addresses (immediate offsets).
#include <algorithm>

#include "tmr_common.h"

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void *lds_ptr_t;

constexpr int BM = 128;      // output channels per block
constexpr int TH = 16;       // output rows per block
constexpr int TW = 32;       // output cols per block
constexpr int NTHREADS = 512;
constexpr int NWAVES = 8;
constexpr int NHEAD = 5;

template <int PREC> struct Prec;
template <> struct Prec<TMR_PREC_F16X3> {
    static constexpr int CCH = 16;   // channels per record
    static constexpr int TERMS = 3;  // MFMAs per 32x32 tile per chunk
    static constexpr bool SCALED = true;
    typedef _Float16 E;
    typedef h8 V;
};
template <> struct Prec<TMR_PREC_BF16> {
    static constexpr int CCH = 32;
    static constexpr int TERMS = 2;
    static constexpr bool SCALED = false;
    typedef __bf16 E;
    typedef b8 V;
};
template <> struct Prec<TMR_PREC_F16> {
    static constexpr int CCH = 32;
    static constexpr int TERMS = 2;
    static constexpr bool SCALED = true;
    typedef _Float16 E;
    typedef h8 V;
};
constexpr int P = 4;       // 16-B pieces per record in HBM
constexpr int REC = 64;    // bytes per record in HBM
constexpr int MAXCCH = 32;

// power-of-two scale with max |x| * s < 2^14 (fp16 max 65504)
__device__ __forceinline__ float split_scale(const float *m) {
    if (!m) return 1.0f;
    const float v = *m;
    if (!(v > 0.0f && v <= 3.0e38f)) return 1.0f;
    int e;
    frexpf(v, &e);  // v < 2^e
    return ldexpf(1.0f, 14 - e);
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n
__device__ __forceinline__ void wait_vmcnt(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    }
}

#ifndef TMR_EXP_MFMA16
__device__ __forceinline__ f32x16 mma(h8 a, h8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mma(b8 a, b8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
#else  // timing experiment only (wrong results): the same FLOPs as 2 x 16x16x32
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <typename VT>
__device__ __forceinline__ f32x16 mma(VT a, VT b, f32x16 c) {
    f32x4 c0 = {c[0], c[1], c[2], c[3]}, c1 = {c[4], c[5], c[6], c[7]};
    if constexpr (sizeof(a[0]) == 2 && __is_same(VT, h8)) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c1, 0, 0, 0);
    } else {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c1, 0, 0, 0);
    }
    c[0] = c0[0]; c[1] = c0[1]; c[2] = c0[2]; c[3] = c0[3];
    c[4] = c1[0]; c[5] = c1[1]; c[6] = c1[2]; c[7] = c1[3];
    return c;
}
#endif

// one record: CCH fp32 values -> 4 pieces of 8 x 16-bit
template <int PREC>
__device__ __forceinline__ void split_record(const float (&v)[MAXCCH], float s,
                                             typename Prec<PREC>::V (&out)[P]) {
    typedef typename Prec<PREC>::E E;
    if (Prec<PREC>::TERMS == 3) {
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float xs = v[g * 8 + j] * s;
                const E hi = (E)xs;
                out[g][j] = hi;
                out[2 + g][j] = (E)(xs - (float)hi);
            }
    } else {
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int j = 0; j < 8; ++j) out[g][j] = (E)(v[g * 8 + j] * s);
    }
}

struct SArgs {
    const char *x0;   // packed src0 [img][NC0][Hp][Wp][rec]
    const char *x1;   // packed src1 [u][NC1][Hp][Wp][rec]
    const int32_t *unit_image;
    const char *wp;   // packed weights [tap][NC0+NC1][Npad][rec]
    const float *wmax, *xmax;
    const float *bias, *headw, *acc_init;
    float *out, *partials;
    int NC0, NC1, U, H, W, N, NT, MT, TXN, Hp, Wp, Npad, leaky;
};

template <int KS>
struct Geo {
    static constexpr int HR = TH + KS - 1, HC = TW + KS - 1;
    static constexpr int T = KS * KS;
    // LDS images are piece planes (structure of arrays): plane q holds piece q
    // of every record, 16 B per record, planes 256-B aligned.  A wave's
    // fragment read then touches 16 consecutive records of one plane per
    // 16-lane group: conflict free for ds_read_b128 with linear addresses.
    static constexpr int NPIX = (HR * HC + 15) / 16 * 16;       // halo records per plane
    static constexpr int HPL = NPIX * 16;                        // halo plane bytes
    static constexpr int NIH = (P * HPL + 1023) / 1024;          // halo DMA wave-instructions
    static constexpr int HB = NIH * 1024;                        // bytes per halo buffer
    static constexpr int WPL = BM * 16;                          // weight plane bytes (2 KB)
    static constexpr int WB1 = P * WPL;                          // weight bytes per tap (8 KB)
    static constexpr int NIW1 = WB1 / 1024;                      // weight DMA instructions per tap
    static constexpr bool fits(int tps, int nwb) { return 2 * HB + nwb * tps * WB1 <= 160 * 1024; }
    // taps per barrier step and weight buffers (DMA lookahead NWB-1 steps)
    static constexpr int TPS = T == 1 ? 1 : (fits(3, 2) ? 3 : fits(2, 2) ? 2 : 1);
    static constexpr int NWB = fits(TPS, 3) ? 3 : 2;
    static constexpr int SPC = (T + TPS - 1) / TPS;           // steps per chunk
    static constexpr int WB = TPS * WB1;                      // bytes per weight buffer
    static constexpr int NIWS = TPS * NIW1;                   // weight instructions per full step
    static constexpr int WPW = (NIWS + NWAVES - 1) / NWAVES;  // ... per wave
    static constexpr int MPW = (NIH + NWAVES - 1) / NWAVES;   // halo instructions per wave per chunk
    static constexpr int Q = (MPW + SPC - 1) / SPC;           // ... issued per step
    static constexpr size_t LDS = 2 * (size_t)HB + NWB * (size_t)WB;
    static_assert(fits(TPS, NWB), "LDS");
    static_assert(NIW1 * 1024 == WB1, "whole weight instructions per tap");
};

template <int KS, int PREC, int EPI>
__global__ __launch_bounds__(NTHREADS) void split_conv_kernel(SArgs a) {
    typedef Prec<PREC> PR;
    typedef typename PR::V V;
    typedef Geo<KS> G;
    constexpr int HC = G::HC, T = G::T, MPW = G::MPW, Q = G::Q, NIH = G::NIH, NIW1 = G::NIW1;
    constexpr int HB = G::HB, WB = G::WB, WB1 = G::WB1, NWB = G::NWB, WPW = G::WPW;
    constexpr int TPS = G::TPS, SPC = G::SPC, HPL = G::HPL, WPL = G::WPL, NPIX = G::NPIX;
    constexpr int D = NWB - 1;  // weight DMA lookahead (steps)
    constexpr int TERMS = PR::TERMS;
    extern __shared__ __attribute__((aligned(16))) char lds[];
    char *Hs = lds;           // [2][P planes][NPIX records][16 B]  activation halo
    char *Ws = lds + 2 * HB;  // [NWB][TPS taps][P planes][BM][16 B] weights

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
    const int l32 = lane & 31, h = lane >> 5;
    const int wn = wave & 1, wpix = wave >> 1;

    // XCD-aware bijective remap (the 8 XCDs take blocks round robin): the NT
    // channel tiles of a pixel tile run back to back on one XCD and share its
    // halo through L2.
    const int nblk = gridDim.x, orig = blockIdx.x;
    const int q8 = nblk >> 3, r8 = nblk & 7, xcd = orig & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int nt = L % a.NT;
    const int rest = L / a.NT;
    const int mt = rest % a.MT, u = rest / a.MT;
    const int ty0 = (mt / a.TXN) * TH, tx0 = (mt % a.TXN) * TW;
    const int img = a.unit_image ? a.unit_image[u] : u;
    const int NC = a.NC0 + a.NC1;

    // Per-lane DMA sources (chunk invariant): LDS piece e of the halo image is
    // plane e / NPIX, record e % NPIX; pad records re-read a legal address.
    int hoff[MPW];
#pragma unroll
    for (int m = 0; m < MPW; ++m) {
        const int e = (wave + NWAVES * m) * 64 + lane;
        int q = e / NPIX, p = e % NPIX;
        if (q >= P || p >= G::HR * HC) q = p = 0;
        const int hy = p / HC, hx = p % HC;
        hoff[m] = ((ty0 + hy) * a.Wp + (tx0 + hx)) * REC + q * 16;
    }
    // weight instruction i of a step: tap i / NIW1, plane / channel from i % NIW1
    int woff[WPW];
#pragma unroll
    for (int m = 0; m < WPW; ++m) {
        const int e = ((wave + NWAVES * m) % NIW1) * 64 + lane;
        const int q = e / BM, n = e % BM;
        woff[m] = n * REC + q * 16;
    }
    const size_t cstride = (size_t)a.Hp * a.Wp * REC;
    auto chunk_src = [&](int c) -> const char * {
        return c < a.NC0 ? a.x0 + ((size_t)img * a.NC0 + c) * cstride
                         : a.x1 + ((size_t)u * a.NC1 + (c - a.NC0)) * cstride;
    };
    // issue this wave's halo instructions m0 <= m < m1 of chunk c; returns the count
    auto halo_dma = [&](int c, int m0, int m1) -> int {
        const char *src = chunk_src(c);
        char *dst = Hs + (c & 1) * HB;
        int n = 0;
#pragma unroll
        for (int m = 0; m < MPW; ++m) {
            const int i = wave + NWAVES * m;
            if (m >= m0 && m < m1 && i < NIH) {
                __builtin_amdgcn_global_load_lds((const void *)(src + hoff[m]),
                                                 (lds_ptr_t)(dst + i * 1024), 16, 0, 0);
                ++n;
            }
        }
        return n;
    };
    const char *wsrc0 = a.wp + (size_t)nt * BM * REC;
    const size_t tapstride = (size_t)NC * a.Npad * REC;
    // weights of flat step g (chunk g / SPC, taps TPS*(g % SPC) ...); returns the count
    auto w_dma = [&](int g) -> int {
        const int c = g / SPC, t0 = (g - c * SPC) * TPS;
        const int ni = min(TPS, T - t0) * NIW1;
        const char *src = wsrc0 + (size_t)t0 * tapstride + (size_t)c * a.Npad * REC;
        char *dst = Ws + (g % NWB) * WB;
        int n = 0;
#pragma unroll
        for (int m = 0; m < WPW; ++m) {
            const int i = wave + NWAVES * m;
            if (i < ni) {
                __builtin_amdgcn_global_load_lds(
                    (const void *)(src + (size_t)(i / NIW1) * tapstride + woff[m]),
                    (lds_ptr_t)(dst + i * 1024), 16, 0, 0);
                ++n;
            }
        }
        return n;
    };

    // accumulators start at acc_init (scaled into the accumulator's units by
    // the exact power of two s_x s_w); masked elements read a clamped legal
    // address and are zeroed by a select, never by a branch around the load
    const float sxw = PR::SCALED ? split_scale(a.xmax) * split_scale(a.wmax) : 1.0f;
    const int HW = a.H * a.W;
    const int x = tx0 + l32;
    f32x16 acc[2][4];
    if (a.acc_init) {
        const float *ai = a.acc_init + (size_t)img * a.N * HW;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int y = ty0 + wpix * 4 + j;
                const bool pin = y < a.H && x < a.W;
                const int pix = min(y, a.H - 1) * a.W + min(x, a.W - 1);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int n = nt * BM + wn * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const float v = ai[(size_t)min(n, a.N - 1) * HW + pix];
                    acc[i][j][r] = (pin && n < a.N) ? v * sxw : 0.0f;
                }
            }
    } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    }

    // fragment pieces: lane half h supplies k = 8h..8h+7 of each MFMA
    //   F16X3: v0 = [wh|wl] x [xh|xh] (ch 0-7), v1 = same ch 8-15,
    //          v2 = [wh g0|wh g1] x [xl g0|xl g1]
    //   one term: v0 = ch 0-15, v1 = ch 16-31
    // (piece planes: linear, conflict-free addresses; per-tap offsets fold
    // into the ds_read immediate)
    int aoff[TERMS], boff[TERMS];
#pragma unroll
    for (int v = 0; v < TERMS; ++v) {
        const int aq = TERMS == 3 ? (v == 0 ? 2 * h : v == 1 ? 2 * h + 1 : h) : 2 * v + h;
        const int bqv = TERMS == 3 ? (v == 0 ? 0 : v == 1 ? 1 : 2 + h) : 2 * v + h;
        aoff[v] = aq * WPL + (wn * 64 + l32) * 16;
        boff[v] = bqv * HPL + (wpix * 4 * HC + l32) * 16;
    }

    const int S = NC * SPC;  // barrier steps
    halo_dma(0, 0, MPW);
    for (int g0 = 0; g0 < D && g0 < S; ++g0) w_dma(g0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int c = 0; c < NC; ++c) {
        const char *hl = Hs + (c & 1) * HB;
#pragma unroll
        for (int sg = 0; sg < SPC; ++sg) {
            const int g = c * SPC + sg;
            // DMAs for later steps: halo of chunk c+1 (buffer last read in
            // chunk c-1), then the weights of step g+D (buffer last read in g-1)
            const int nh = (c + 1 < NC && sg * Q < MPW) ? halo_dma(c + 1, sg * Q, sg * Q + Q) : 0;
            const int nw = g + D < S ? w_dma(g + D) : 0;
            const char *wl = Ws + (g % NWB) * WB;
#pragma unroll
            for (int tl = 0; tl < TPS; ++tl) {
                const int tap = sg * TPS + tl;
                if (tap >= T) break;
                const int ky = tap / KS, kx = tap % KS;
                V af[2][TERMS];
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int v = 0; v < TERMS; ++v)
                        af[i][v] = *reinterpret_cast<const V *>(wl + tl * WB1 + aoff[v] + i * 32 * 16);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    V bf[TERMS];
#pragma unroll
                    for (int v = 0; v < TERMS; ++v)
                        bf[v] = *reinterpret_cast<const V *>(hl + boff[v] + ((j + ky) * HC + kx) * 16);
#pragma unroll
                    for (int v = 0; v < TERMS; ++v)
#pragma unroll
                        for (int i = 0; i < 2; ++i) acc[i][j] = mma(af[i][v], bf[v], acc[i][j]);
                }
            }
            // the next step needs W(g+1) and, after a chunk's last step, the
            // whole halo of chunk c+1: leave only younger DMAs in flight
            // (in-order completion; this step issued halo before weights)
            if (D == 1)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else
                wait_vmcnt(sg == SPC - 1 ? nw : nw + nh);
            __builtin_amdgcn_s_barrier();
        }
    }

    // ---------------- epilogue ----------------
    const float inv = 1.0f / sxw;  // 2^-k: exact
    // the block's bias and head weights through LDS (the main loop's last
    // barrier freed it): global loads here would be hoisted into registers
    float *sb = reinterpret_cast<float *>(lds) + NHEAD * 16 * 32;  // past the head scratch
    float *shw = sb + BM;                                           // [BM][NHEAD]
    if (tid < BM) {
        const int n = nt * BM + tid;
        sb[tid] = n < a.N ? a.bias[n] : 0.0f;
    }
    if (EPI == 1)
        for (int e = tid; e < BM * NHEAD; e += NTHREADS) shw[e] = a.headw[(size_t)nt * BM * NHEAD + e];
    __syncthreads();
    float hs[4][NHEAD];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < NHEAD; ++k) hs[j][k] = 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int nl = wn * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            const int n = nt * BM + nl;
            const bool nin = n < a.N;
            const float bn = sb[nl];
            float hw[NHEAD];
            if (EPI == 1) {
#pragma unroll
                for (int k = 0; k < NHEAD; ++k) hw[k] = shw[nl * NHEAD + k];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int y = ty0 + wpix * 4 + j;
                const bool pin = nin && y < a.H && x < a.W;
                const size_t pix = (size_t)y * a.W + x;
                float v = acc[i][j][r] * inv;
                v += bn;
                if (a.leaky) v = v >= 0.0f ? v : v * 0.01f;
                if (EPI == 0) {
                    if (pin) a.out[((size_t)u * a.N + n) * HW + pix] = v;
                } else {
#pragma unroll
                    for (int k = 0; k < NHEAD; ++k) hs[j][k] = fmaf(v, hw[k], hs[j][k]);
                }
            }
        }
    if (EPI == 1) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < NHEAD; ++k) hs[j][k] += __shfl_xor(hs[j][k], 32);
        float *red = reinterpret_cast<float *>(lds);  // [4 wpix][4 j][NHEAD][32]
        if (wn == 1 && h == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int k = 0; k < NHEAD; ++k) red[((wpix * 4 + j) * NHEAD + k) * 32 + l32] = hs[j][k];
        }
        __syncthreads();
        if (wn == 0 && h == 0 && x < a.W) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int y = ty0 + wpix * 4 + j;
                if (y >= a.H) continue;
#pragma unroll
                for (int k = 0; k < NHEAD; ++k) {
                    const float v = hs[j][k] + red[((wpix * 4 + j) * NHEAD + k) * 32 + l32];
                    a.partials[(((size_t)nt * NHEAD + k) * a.U + u) * HW + (size_t)y * a.W + x] = v;
                }
            }
        }
    }
}

template <int KS, int PREC, int EPI>
int launch_split(SArgs a, hipStream_t s) {
    constexpr size_t lds = Geo<KS>::LDS;
    static_assert(lds <= 160 * 1024, "LDS");
    static_assert((NHEAD * 16 * 32 + BM * (NHEAD + 1)) * 4 <= lds, "epilogue scratch");
    auto kern = split_conv_kernel<KS, PREC, EPI>;
    if (hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
        return TMR_E_HIP;
    const int64_t blocks = (int64_t)a.NT * a.MT * a.U;
    if (blocks <= 0) return TMR_OK;
    TMR_REQUIRE(blocks < (1ll << 31));
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NTHREADS), lds, s, a);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

template <int KS, int EPI>
int dispatch_prec(int prec, const SArgs &a, hipStream_t s) {
    switch (prec) {
        case TMR_PREC_F16X3: return launch_split<KS, TMR_PREC_F16X3, EPI>(a, s);
        case TMR_PREC_BF16: return launch_split<KS, TMR_PREC_BF16, EPI>(a, s);
        case TMR_PREC_F16: return launch_split<KS, TMR_PREC_F16, EPI>(a, s);
        default: return TMR_E_INVALID;
    }
}

template <int EPI>
int dispatch_ks(int ks, int prec, const SArgs &a, hipStream_t s) {
    switch (ks) {
        case 1: return dispatch_prec<1, EPI>(prec, a, s);
        case 3: return dispatch_prec<3, EPI>(prec, a, s);
        case 5: return dispatch_prec<5, EPI>(prec, a, s);
        case 7: return dispatch_prec<7, EPI>(prec, a, s);
        default: return TMR_E_INVALID;
    }
}

inline int prec_cch(int prec) { return prec == TMR_PREC_F16X3 ? Prec<TMR_PREC_F16X3>::CCH : Prec<TMR_PREC_BF16>::CCH; }
inline bool prec_ok(int prec) {
    return prec == TMR_PREC_F16X3 || prec == TMR_PREC_BF16 || prec == TMR_PREC_F16;
}
inline bool ks_ok(int ks) { return ks == 1 || ks == 3 || ks == 5 || ks == 7; }
inline int pad_h(int H, int ks) { return (int)tmr_cdiv(H, TH) * TH + ks - 1; }
inline int pad_w(int W, int ks) { return (int)tmr_cdiv(W, TW) * TW + ks - 1; }

// ---------------------------------------------------------------- packing
__global__ void absmax_kernel(const float *__restrict__ x, int64_t n, unsigned *__restrict__ out) {
    float m = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        m = fmaxf(m, fabsf(x[i]));
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));  // m >= 0: uint order
}

__global__ void absmax_vec_kernel(const float4 *__restrict__ x, int64_t n4, unsigned *__restrict__ out) {
    float m = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = x[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

// x [S][C][H][W] fp32 -> [S][ceil(C/CCH)][Hp][Wp][64 B], zero padded:
// padded (yp, xp) holds x[yp - ks/2][xp - ks/2].  One thread per record.
template <int PREC>
__global__ void xpack_kernel(const float *__restrict__ x, int S, int C, int H, int W, int NCc,
                             int Hp, int Wp, int pad, const float *__restrict__ xmax,
                             typename Prec<PREC>::V *__restrict__ out) {
    constexpr int CCH = Prec<PREC>::CCH;
    const int64_t total = (int64_t)S * NCc * Hp * Wp;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int xp = (int)(i % Wp);
    int64_t r = i / Wp;
    const int yp = (int)(r % Hp);
    r /= Hp;
    const int c = (int)(r % NCc);
    const int s = (int)(r / NCc);
    const int y = yp - pad, xx = xp - pad;
    const bool in = y >= 0 && y < H && xx >= 0 && xx < W;
    const float sc = Prec<PREC>::SCALED ? split_scale(xmax) : 1.0f;
    float v[MAXCCH];
#pragma unroll
    for (int k = 0; k < MAXCCH; ++k) {
        const int ch = c * CCH + k;
        v[k] = (k < CCH && in && ch < C) ? x[(((size_t)s * C + ch) * H + y) * W + xx] : 0.0f;
    }
    typename Prec<PREC>::V rec[P];
    split_record<PREC>(v, sc, rec);
#pragma unroll
    for (int q = 0; q < P; ++q) out[i * P + q] = rec[q];
}

// Records of x' = [up2x(f) (or f); 1] straight from the SAM features
// f [S][Cin][Hin][Win]: the input of the decoder's fp half folded through
// input_proj (tmr_split_fold_proj).  The bilinear value is the same fma form
// as tmr_upsample_proj (ATen's CPU kernel); the constant-1 channel carries the
// projection bias and is zero in the padding, like the conv's zero padding.
template <int PREC>
__global__ void xpack_up_kernel(const float *__restrict__ f, int S, int Cin, int Hin, int Win,
                                int ups, int ones, int H, int W, int NCc, int Hp, int Wp, int pad,
                                const float *__restrict__ xmax,
                                typename Prec<PREC>::V *__restrict__ out) {
    constexpr int CCH = Prec<PREC>::CCH;
    const int64_t total = (int64_t)S * NCc * Hp * Wp;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int xp = (int)(i % Wp);
    int64_t r = i / Wp;
    const int yp = (int)(r % Hp);
    r /= Hp;
    const int c = (int)(r % NCc);
    const int s = (int)(r / NCc);
    const int y = yp - pad, xx = xp - pad;
    const bool in = y >= 0 && y < H && xx >= 0 && xx < W;
    const float sc = Prec<PREC>::SCALED ? split_scale(xmax) : 1.0f;
    float v[MAXCCH];
#pragma unroll
    for (int k = 0; k < MAXCCH; ++k) {
        const int ch = c * CCH + k;
        float val = 0.0f;
        if (k < CCH && in) {
            if (ch < Cin) {
                const float *pl = f + ((size_t)s * Cin + ch) * Hin * Win;
                val = ups ? up_value(pl, Hin, Win, y, xx) : pl[(size_t)y * Win + xx];
            } else if (ones && ch == Cin) {
                val = 1.0f;
            }
        }
        v[k] = val;
    }
    typename Prec<PREC>::V rec[P];
    split_record<PREC>(v, sc, rec);
#pragma unroll
    for (int q = 0; q < P; ++q) out[i * P + q] = rec[q];
}

// Fold the decoder's fp half through input_proj (matching_net.py:27-30,56):
// conv(proj(x)) = conv'([x; 1]) with W'[n][c][t] = sum_k Wd[n][k][t] P[k][c]
// (c < Cin) and W'[n][Cin][t] = sum_k Wd[n][k][t] b[k]; fp64 accumulation.
// wd: [N][Cw][T] (its first Cp input channels are the fp half), P: [Cp][Cin].
__global__ void fold_proj_kernel(const float *__restrict__ wd, int N, int Cw, int Cp, int T,
                                 const float *__restrict__ pw, const float *__restrict__ pb,
                                 int Cin, float *__restrict__ out) {
    const int64_t total = (int64_t)N * (Cin + 1) * T;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int t = (int)(i % T);
    const int64_t r = i / T;
    const int c = (int)(r % (Cin + 1));
    const int n = (int)(r / (Cin + 1));
    const float *w = wd + (size_t)n * Cw * T + t;
    double acc = 0.0;
    if (c < Cin) {
        for (int k = 0; k < Cp; ++k) acc += (double)w[(size_t)k * T] * (double)pw[(size_t)k * Cin + c];
    } else {
        for (int k = 0; k < Cp; ++k) acc += (double)w[(size_t)k * T] * (double)pb[k];
    }
    out[i] = (float)acc;
}

// w [N][C0+C1][ks][ks] fp32 -> [ks*ks][NC0+NC1][Npad][64 B]; the src0
// and src1 channel ranges are padded to whole chunks separately.
template <int PREC>
__global__ void wpack_kernel(const float *__restrict__ w, int N, int C0, int C1, int ks, int NC0,
                             int NC, int Npad, const float *__restrict__ wmax,
                             typename Prec<PREC>::V *__restrict__ out) {
    constexpr int CCH = Prec<PREC>::CCH;
    const int T = ks * ks;
    const int64_t total = (int64_t)T * NC * Npad;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int n = (int)(i % Npad);
    int64_t r = i / Npad;
    const int c = (int)(r % NC);
    const int tap = (int)(r / NC);
    const int C = C0 + C1;
    const float sc = Prec<PREC>::SCALED ? split_scale(wmax) : 1.0f;
    float v[MAXCCH];
#pragma unroll
    for (int k = 0; k < MAXCCH; ++k) {
        int ch;
        bool ok;
        if (k >= CCH) {
            ch = 0;
            ok = false;
        } else if (c < NC0) {
            ch = c * CCH + k;
            ok = ch < C0;
        } else {
            const int c1 = (c - NC0) * CCH + k;
            ch = C0 + c1;
            ok = c1 < C1;
        }
        v[k] = (ok && n < N) ? w[((size_t)n * C + ch) * T + tap] : 0.0f;
    }
    typename Prec<PREC>::V rec[P];
    split_record<PREC>(v, sc, rec);
#pragma unroll
    for (int q = 0; q < P; ++q) out[i * P + q] = rec[q];
}

int split_common(const void *xp0, int C0, const int32_t *unit_image, const void *xp1, int C1, int U,
                 int H, int W, int ks, int prec, const void *wpack, const float *wmax,
                 const float *xmax, const float *bias, int N, int leaky, const float *acc_init,
                 float *out, const float *headw, float *partials, int epi, void *stream) {
    TMR_REQUIRE(prec_ok(prec) && ks_ok(ks));
    TMR_REQUIRE(wpack && bias && U > 0 && H > 0 && W > 0 && N > 0 && C0 >= 0 && C1 >= 0);
    TMR_REQUIRE(C0 + C1 > 0 && (C0 == 0 || xp0) && (C1 == 0 || xp1));
    TMR_REQUIRE(prec == TMR_PREC_BF16 || (wmax && xmax));
    SArgs a = {};
    a.x0 = static_cast<const char *>(xp0);
    a.x1 = static_cast<const char *>(xp1);
    a.unit_image = unit_image;
    a.wp = static_cast<const char *>(wpack);
    a.wmax = prec == TMR_PREC_BF16 ? nullptr : wmax;
    a.xmax = prec == TMR_PREC_BF16 ? nullptr : xmax;
    a.bias = bias;
    a.headw = headw;
    a.acc_init = acc_init;
    a.out = out;
    a.partials = partials;
    a.NC0 = (int)tmr_cdiv(C0, prec_cch(prec));
    a.NC1 = (int)tmr_cdiv(C1, prec_cch(prec));
    a.U = U;
    a.H = H;
    a.W = W;
    a.N = N;
    a.NT = (int)tmr_cdiv(N, BM);
    a.Npad = a.NT * BM;
    a.TXN = (int)tmr_cdiv(W, TW);
    a.MT = a.TXN * (int)tmr_cdiv(H, TH);
    a.Hp = pad_h(H, ks);
    a.Wp = pad_w(W, ks);
    a.leaky = leaky;
    hipStream_t s = tmr_stream(stream);
    return epi ? dispatch_ks<1>(ks, prec, a, s) : dispatch_ks<0>(ks, prec, a, s);
}

}  // namespace

extern "C" int tmr_absmax(const float *x, int64_t n, int accumulate, float *out, void *stream) {
    TMR_REQUIRE(out && n >= 0 && (n == 0 || x));
    hipStream_t s = tmr_stream(stream);
    if (!accumulate && hipMemsetAsync(out, 0, sizeof(float), s) != hipSuccess) return TMR_E_HIP;
    if (n == 0) return TMR_OK;
    unsigned *o = reinterpret_cast<unsigned *>(out);
    if ((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (n & 3) == 0) {
        const int64_t n4 = n / 4;
        const int blocks = (int)std::min<int64_t>(tmr_cdiv(n4, 256), 4096);
        hipLaunchKernelGGL(absmax_vec_kernel, dim3(blocks), dim3(256), 0, s,
                           reinterpret_cast<const float4 *>(x), n4, o);
    } else {
        const int blocks = (int)std::min<int64_t>(tmr_cdiv(n, 256), 4096);
        hipLaunchKernelGGL(absmax_kernel, dim3(blocks), dim3(256), 0, s, x, n, o);
    }
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int64_t tmr_split_xpack_size(int S, int C, int H, int W, int ks, int prec) {
    if (S <= 0 || C <= 0 || H <= 0 || W <= 0 || !ks_ok(ks) || !prec_ok(prec)) return -1;
    return (int64_t)S * tmr_cdiv(C, prec_cch(prec)) * pad_h(H, ks) * pad_w(W, ks) * REC;
}

extern "C" int tmr_split_xpack(const float *x, int S, int C, int H, int W, int ks, int prec,
                               const float *xmax, void *out, void *stream) {
    TMR_REQUIRE(x && out && S > 0 && C > 0 && H > 0 && W > 0 && ks_ok(ks) && prec_ok(prec));
    TMR_REQUIRE(prec == TMR_PREC_BF16 || xmax);
    const int NCc = (int)tmr_cdiv(C, prec_cch(prec)), Hp = pad_h(H, ks), Wp = pad_w(W, ks);
    const int64_t total = (int64_t)S * NCc * Hp * Wp;
    const dim3 grid((unsigned)tmr_cdiv(total, 256)), blk(256);
    hipStream_t s = tmr_stream(stream);
    switch (prec) {
        case TMR_PREC_F16X3:
            hipLaunchKernelGGL(xpack_kernel<TMR_PREC_F16X3>, grid, blk, 0, s, x, S, C, H, W, NCc, Hp,
                               Wp, ks / 2, xmax, static_cast<h8 *>(out));
            break;
        case TMR_PREC_BF16:
            hipLaunchKernelGGL(xpack_kernel<TMR_PREC_BF16>, grid, blk, 0, s, x, S, C, H, W, NCc, Hp,
                               Wp, ks / 2, nullptr, static_cast<b8 *>(out));
            break;
        default:
            hipLaunchKernelGGL(xpack_kernel<TMR_PREC_F16>, grid, blk, 0, s, x, S, C, H, W, NCc, Hp,
                               Wp, ks / 2, xmax, static_cast<h8 *>(out));
            break;
    }
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int tmr_split_xpack_up(const float *f, int S, int Cin, int Hin, int Win, int upsample,
                                  int ones, int ks, int prec, const float *xmax, void *out,
                                  void *stream) {
    TMR_REQUIRE(f && out && S > 0 && Cin > 0 && Hin > 0 && Win > 0 && ks_ok(ks) && prec_ok(prec));
    TMR_REQUIRE(prec == TMR_PREC_BF16 || xmax);
    const int H = upsample ? 2 * Hin : Hin, W = upsample ? 2 * Win : Win;
    const int C = Cin + (ones ? 1 : 0);
    const int NCc = (int)tmr_cdiv(C, prec_cch(prec)), Hp = pad_h(H, ks), Wp = pad_w(W, ks);
    const int64_t total = (int64_t)S * NCc * Hp * Wp;
    const dim3 grid((unsigned)tmr_cdiv(total, 256)), blk(256);
    hipStream_t s = tmr_stream(stream);
    const int u = upsample ? 1 : 0, o = ones ? 1 : 0;
    switch (prec) {
        case TMR_PREC_F16X3:
            hipLaunchKernelGGL(xpack_up_kernel<TMR_PREC_F16X3>, grid, blk, 0, s, f, S, Cin, Hin, Win, u,
                               o, H, W, NCc, Hp, Wp, ks / 2, xmax, static_cast<h8 *>(out));
            break;
        case TMR_PREC_BF16:
            hipLaunchKernelGGL(xpack_up_kernel<TMR_PREC_BF16>, grid, blk, 0, s, f, S, Cin, Hin, Win, u,
                               o, H, W, NCc, Hp, Wp, ks / 2, nullptr, static_cast<b8 *>(out));
            break;
        default:
            hipLaunchKernelGGL(xpack_up_kernel<TMR_PREC_F16>, grid, blk, 0, s, f, S, Cin, Hin, Win, u,
                               o, H, W, NCc, Hp, Wp, ks / 2, xmax, static_cast<h8 *>(out));
            break;
    }
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int tmr_split_fold_proj(const float *wd, int N, int Cw, int Cp, int ks, const float *proj_w,
                                   const float *proj_b, int Cin, float *out, void *stream) {
    TMR_REQUIRE(wd && proj_w && proj_b && out && N > 0 && Cp > 0 && Cw >= Cp && Cin > 0 && ks > 0);
    const int64_t total = (int64_t)N * (Cin + 1) * ks * ks;
    hipLaunchKernelGGL(fold_proj_kernel, dim3((unsigned)tmr_cdiv(total, 256)), dim3(256), 0,
                       tmr_stream(stream), wd, N, Cw, Cp, ks * ks, proj_w, proj_b, Cin, out);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int64_t tmr_split_wpack_size(int N, int C0, int C1, int ks, int prec) {
    if (N <= 0 || C0 < 0 || C1 < 0 || C0 + C1 <= 0 || !ks_ok(ks) || !prec_ok(prec)) return -1;
    const int cc = prec_cch(prec);
    return (int64_t)ks * ks * (tmr_cdiv(C0, cc) + tmr_cdiv(C1, cc)) * tmr_cdiv(N, BM) * BM * REC;
}

extern "C" int tmr_split_wpack(const float *w, int N, int C0, int C1, int ks, int prec,
                               const float *wmax, void *out, void *stream) {
    TMR_REQUIRE(w && out && N > 0 && C0 >= 0 && C1 >= 0 && C0 + C1 > 0 && ks_ok(ks) && prec_ok(prec));
    TMR_REQUIRE(prec == TMR_PREC_BF16 || wmax);
    const int cc = prec_cch(prec);
    const int NC0 = (int)tmr_cdiv(C0, cc), NC = NC0 + (int)tmr_cdiv(C1, cc);
    const int Npad = (int)tmr_cdiv(N, BM) * BM;
    const int64_t total = (int64_t)ks * ks * NC * Npad;
    const dim3 grid((unsigned)tmr_cdiv(total, 256)), blk(256);
    hipStream_t s = tmr_stream(stream);
    switch (prec) {
        case TMR_PREC_F16X3:
            hipLaunchKernelGGL(wpack_kernel<TMR_PREC_F16X3>, grid, blk, 0, s, w, N, C0, C1, ks, NC0,
                               NC, Npad, wmax, static_cast<h8 *>(out));
            break;
        case TMR_PREC_BF16:
            hipLaunchKernelGGL(wpack_kernel<TMR_PREC_BF16>, grid, blk, 0, s, w, N, C0, C1, ks, NC0,
                               NC, Npad, nullptr, static_cast<b8 *>(out));
            break;
        default:
            hipLaunchKernelGGL(wpack_kernel<TMR_PREC_F16>, grid, blk, 0, s, w, N, C0, C1, ks, NC0,
                               NC, Npad, wmax, static_cast<h8 *>(out));
            break;
    }
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int tmr_split_conv_store(const void *xp0, int C0, const int32_t *unit_image,
                                    const void *xp1, int C1, int U, int H, int W, int ks, int prec,
                                    const void *wpack, const float *wmax, const float *xmax,
                                    const float *bias, int N, int leaky, const float *acc_init,
                                    float *out, void *stream) {
    TMR_REQUIRE(out);
    return split_common(xp0, C0, unit_image, xp1, C1, U, H, W, ks, prec, wpack, wmax, xmax, bias, N,
                        leaky, acc_init, out, nullptr, nullptr, 0, stream);
}

extern "C" int tmr_split_conv_heads(const void *xp0, int C0, const int32_t *unit_image,
                                    const void *xp1, int C1, int U, int H, int W, int ks, int prec,
                                    const void *wpack, const float *wmax, const float *xmax,
                                    const float *bias, int N, int leaky, const float *headw,
                                    const float *acc_init, float *partials, void *stream) {
    TMR_REQUIRE(headw && partials);
    return split_common(xp0, C0, unit_image, xp1, C1, U, H, W, ks, prec, wpack, wmax, xmax, bias, N,
                        leaky, acc_init, nullptr, headw, partials, 1, stream);
}
