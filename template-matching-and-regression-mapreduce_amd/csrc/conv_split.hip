// Split-precision direct implicit-GEMM kxk convolution on 16-bit MFMA
// (v_mfma_f32_16x16x32_f16 / _bf16), gfx950: the decoder conv stack
// (Decoder_model conv + LeakyReLU, optional fused 1x1 heads;
// models/regression_head.py:7-8,31,50, models/matching_net.py:63-75) and
// the standalone convolutions of the module API.
//
// Precision modes (TMR_PREC_*):
//   F16X3  fp32-grade: x = s_x^-1 (xh + xl), w = s_w^-1 (wh + wl) with fp16
//          hi/lo parts and power-of-two scales s (max |x s| < 2^14), and
//          x.w ~= (wh xh + wl xh + wh xl) / (s_x s_w), fp32 accumulation;
//          wh carries WH_BITS = 8 significant bits (below).  The dropped
//          wl xl term is ~2^-21 and the weights keep 19 bits: inside the
//          fp32 path's 1e-5 contract on every tested shape (below).
//   BF16   one bf16 term (unscaled), fp32 accumulation (config C).
//   F16    one scaled fp16 term.
//
// GEMM view: D[n][pixel] = sum_{tap, c} Wt[tap][n][c] X[c][pixel + tap], A =
// weights (rows n), B = activations (columns = 16 consecutive pixels of one
// output row).  K is walked in 32-channel chunks; one 16x16x32 MFMA consumes
// a whole chunk (lane group g = lane / 16 supplies channels 8g..8g+7).
//
// Operands live in HBM in MFMA-ready 16-bit layouts written by the pack
// kernels below.  Activations: per 32-channel chunk and "half" (F16X3: hi,
// lo; one-term modes: one half) a 64-B record per pixel (4 16-B pieces of 8
// channels), zero-padded to whole tiles plus the kxk halo, so the kernel
// never masks a load.  Weights: per tap and chunk a record per output
// channel, [wh ch0-31][wl ch0-31] (128 B, F16X3) or [w ch0-31] (64 B).  Both
// are stored PLANAR (piece q of every record contiguous), which is also the
// LDS image layout: each 1-KB LDS-DMA wave instruction reads 1 KB of
// contiguous HBM (a record-major layout reads 16 B of every 64-128 B line
// per instruction: 4-8x the L2/TA line traffic, measured ~6% of the kernel).
//
// The F16X3 K loop alternates two half-chunk kinds over the same 32
// channels: "hi" (halo xh; 2 MFMAs per tile: wh.xh + wl.xh) and "lo" (halo
// xl; 1 MFMA: wh.xl).  So every MFMA has a full K = 32, no padding, and the
// hi and lo halos never need LDS at the same time.
//
// Block: 512 threads, 128 output channels x 512 pixels (16 rows x 32 cols).
// Waves 2 (64 n) x 4 (4 rows); a wave owns 4 x 8 16x16 accumulators (128
// regs).  Per barrier step the weight records of step g+D stream into LDS by
// LDS-DMA while step g computes, and the next half-chunk's (16+k-1)x(32+k-1)
// halo (2 buffers) streams in spread over the first steps; each step ends
// with a counted vmcnt (only the DMAs the next step needs) and a raw
// s_barrier, so loads stay in flight across barriers.  LDS images are piece
// planes (structure of arrays, 16 B per record per plane): each 16-lane
// group of a fragment read touches 16 consecutive records of one plane, so
// the ds_read_b128 reads are bank-conflict free with linear addresses and
// every per-tap offset folds into the instruction's immediate.
#include <algorithm>
#include <type_traits>

#include "tmr_common.h"

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 b4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void *lds_ptr_t;

// Measured and dropped (code in git history): register-staged operand loads
// (buffer_load + ds_write instead of LDS-DMA; 3.7% slower, profiles/archive/r02p_*),
// initial values read inside the main loop (slower: a load issued in a step
// is forced by that step's in-order vmcnt wait; profiles/archive/r02ai, r02aj), the
// next step's first B fragments read before the step barrier (4% slower,
// r02an), wave priority over the MFMA stream (no change, r02av).

constexpr int BM = 128;      // output channels per block
constexpr int TH = 16;       // output rows per block
constexpr int TW = 32;       // output cols per block
// LDS budget per block: the whole CU (one block per CU).  TH = 8 with 4 waves
// and 80 KB, two co-resident blocks per CU, was 14-17% slower
constexpr int LDS_KB = 160;
// XCD block groups: PXG pixel tiles x NG channel tiles per XCD wave of 32
// co-resident blocks (8 x 4 minimises the wave's distinct operands, r03ab)
constexpr int PXG = 8, NG = 4;
// waves per block: 8 (2 along n x 4 along rows, 128 accumulator VGPRs, two
// waves per SIMD); the code also holds the 4-wave form (1 x 4, 256
// accumulators, one wave per SIMD), measured 17% slower (r02ah)
constexpr int NWAVES = 8;
constexpr int NTHREADS = NWAVES * 64;
constexpr int WNS = (NWAVES == 8 || TH == 8) ? 2 : 1;  // waves along n
static_assert(TH == 4 * NWAVES / WNS, "a wave owns 4 output rows");
constexpr int NIN = 8 / WNS;              // 16-channel n fragments per wave
constexpr int ACCW = NIN * 8 * 64 * 4;    // accumulator floats per wave
constexpr int NHEAD = 5;
constexpr int CCH = 32;      // channels per chunk (one MFMA K)
constexpr int P = 4;         // 16-B pieces per activation record
constexpr int XREC = 64;     // bytes per activation record
constexpr int WPL = BM * 16; // bytes per LDS weight plane

template <int PREC> struct Prec;
template <> struct Prec<TMR_PREC_F16X3> {
    static constexpr int HALVES = 2;   // hi, lo half-chunks per chunk
    static constexpr int WREC = 128;   // [wh][wl] per output channel
    static constexpr bool SCALED = true;
    typedef _Float16 E;
    typedef h8 V;
};
template <> struct Prec<TMR_PREC_BF16> {
    static constexpr int HALVES = 1;
    static constexpr int WREC = 64;
    static constexpr bool SCALED = false;
    typedef __bf16 E;
    typedef b8 V;
};
template <> struct Prec<TMR_PREC_F16> {
    static constexpr int HALVES = 1;
    static constexpr int WREC = 64;
    static constexpr bool SCALED = true;
    typedef _Float16 E;
    typedef h8 V;
};

// power-of-two scale with max |x| * s < 2^14 (fp16 max 65504), clamped to
// [2^-63, 2^63] so that the product of an activation and a weight scale
// stays a normal fp32 number (sources below 2^-49 or above 2^77 are then
// scaled less than their range would allow)
__device__ __forceinline__ float split_scale(const float *m) {
    if (!m) return 1.0f;
    const float v = *m;
    if (!(v > 0.0f && v <= 3.0e38f)) return 1.0f;
    int e;
    frexpf(v, &e);  // v < 2^e
    return ldexpf(1.0f, min(max(14 - e, -63), 63));
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
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    }
}

// 16-B LDS-DMA through a buffer descriptor.  Kept in a __device__ function:
// the builtin inside the kernel's (host-device) lambdas makes the host pass
// silently drop the kernel stubs.
__device__ __forceinline__ void buffer_lds16(__amdgpu_buffer_rsrc_t r, lds_ptr_t dst, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, soff, 0, 0);
}

__device__ __forceinline__ f32x4 mma(h8 a, h8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma(b8 a, b8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// one 32-channel record: fp32 values -> hi pieces (and lo pieces for F16X3)
template <int PREC>
__device__ __forceinline__ void split_record(const float (&v)[CCH], float s,
                                             typename Prec<PREC>::V (&hi)[P],
                                             typename Prec<PREC>::V (&lo)[P]) {
    typedef typename Prec<PREC>::E E;
#pragma unroll
    for (int g = 0; g < P; ++g)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float xs = v[g * 8 + j] * s;
            const E h = (E)xs;
            hi[g][j] = h;
            if (Prec<PREC>::HALVES == 2) lo[g][j] = (E)(xs - (float)h);
        }
}

// Weight split of the F16X3 records: w s = wh + wl with wh = w s rounded to
// WH_BITS significant bits (fp32 round-to-nearest-even on the bit pattern,
// then exact in fp16) and wl = fp16(w s - wh); WH_BITS = 11 would be the
// plain fp16 hi/lo split (wh = fp16(w s)).  The decoder is power-bound and
// its MFMA rate rises as the operands' bit density falls:
// wh feeds two of the three MFMAs per product.  8 bits: the weights keep
// 8 + 11 = 19 bits, the dropped wl xl term is ~2^-21 of a product.
// Measured (profiles/r04j): heads launch 111.6 / 111.7 -> 109.9 / 109.9 ms
// (config B +1.3%); 6 bits was faster (108.3 ms, +2.6%) but left one random
// module variant (k = 1 over 16 channels, heavy cancellation) at 1.33e-5
// normwise against the 1e-5 contract; 8 bits: 1.5e-6 there and all 1200
// cases of the deep random sweep green (profiles/r04wb).
constexpr int WH_BITS = 8;

template <int PREC>
__device__ __forceinline__ void split_record_w(const float (&v)[CCH], float s,
                                               typename Prec<PREC>::V (&hi)[P],
                                               typename Prec<PREC>::V (&lo)[P]) {
    typedef typename Prec<PREC>::E E;
    if constexpr (Prec<PREC>::HALVES != 2 || WH_BITS >= 11) {
        split_record<PREC>(v, s, hi, lo);
    } else {
#pragma unroll
        for (int g = 0; g < P; ++g)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float xs = v[g * 8 + j] * s;
                const E h = (E)tmr_round_sig_bits(xs, WH_BITS);
                hi[g][j] = h;
                lo[g][j] = (E)(xs - (float)h);
            }
    }
}

struct SArgs {
    const char *x0;   // packed src0 [img][NC0*HALVES][Hp][Wp][64 B]
    const char *x1;   // packed src1 [u][NC1*HALVES][Hp][Wp][64 B]
    const int32_t *unit_image;
    const char *wp;   // packed weights [tap][NC0+NC1][Npad][WREC]
    const float *wmax, *xmax;
    const float *bias, *headw, *acc_init;
    float *out, *partials;
    int NC0, NC1, U, H, W, N, NT, MT, TXN, Hp, Wp, Npad, leaky;
    int flags;  // TMR_SPLIT_TILED_OUT / TMR_SPLIT_TILED_INIT
    int EI;     // units per image of the image-major block order (1: unit-major)
};

template <int KS, int PREC>
struct Geo {
    static constexpr int HR = TH + KS - 1, HC = TW + KS - 1;
    static constexpr int T = KS * KS;
    static constexpr int NPIX = (HR * HC + 15) / 16 * 16;     // halo records per plane
    static constexpr int HPL = NPIX * 16;                      // halo plane bytes (256-B multiple)
    static constexpr int NIH = (P * HPL + 1023) / 1024;        // halo DMA wave-instructions
    static constexpr int MPW = (NIH + NWAVES - 1) / NWAVES;    // halo DMAs per wave per half-chunk
    // bytes per halo buffer, padded to MPW instructions for every wave (the
    // pad KB receives re-read records and is never read)
    static constexpr int HB = MPW * NWAVES * 1024;
    static constexpr int NPLW = Prec<PREC>::WREC / 16;         // weight planes per tap (8 or 4)
    static constexpr int WB1 = NPLW * WPL;                     // weight bytes per tap
    static constexpr bool fits(int tps, int nwb) {
        return 2 * HB + nwb * tps * WB1 <= LDS_KB * 1024;
    }
    // taps per barrier step and weight buffers (DMA lookahead NWB-1 steps)
    static constexpr int TPS = T == 1 ? 1 : fits(3, 2) ? 3 : fits(2, 2) ? 2 : 1;
    static constexpr int NWB = fits(TPS, 3) ? 3 : 2;
    static constexpr int SPC = (T + TPS - 1) / TPS;            // steps per half-chunk
    static constexpr int WB = TPS * WB1;                       // bytes per weight buffer
    static constexpr int Q = (MPW + SPC - 1) / SPC;            // halo DMAs per wave issued per step
    static constexpr size_t LDS = 2 * (size_t)HB + NWB * (size_t)WB;
    // LO3: F16X3 lo half-chunks (one weight term: half a hi tap's bytes) in
    // steps of up to 2 TPS taps, balanced (3 x 3 at k = 3): fewer barrier
    // steps per chunk (10 -> 8).  One weight lookahead step (NWB == 2) only.
    // Measured (r02bm, A/B in one call): fp32 heads 28.02/28.17 -> 27.89/27.97
    // ms per 48 units, config B 451.3/451.5 -> 454.4/454.1 images/s.
    static constexpr bool LO3 = PREC == TMR_PREC_F16X3 && NWB == 2 && T > 1;
    static constexpr int SPCL = LO3 ? (T + 2 * TPS - 1) / (2 * TPS) : SPC;
    static constexpr int TPSL = LO3 ? (T + SPCL - 1) / SPCL : TPS;
    static constexpr int SPCC = Prec<PREC>::HALVES == 2 ? SPC + SPCL : SPC;  // steps per chunk
    static constexpr int tps(int part) { return part ? TPSL : TPS; }
    static constexpr int spc(int part) { return part ? SPCL : SPC; }
    static constexpr int wb1(int part) { return (LO3 && part) ? WB1 / 2 : WB1; }
    static constexpr int qh(int part) { return (MPW + spc(part) - 1) / spc(part); }
    static constexpr int nhp(int part, int sg) {
        return MPW - sg * qh(part) < qh(part) ? (MPW - sg * qh(part) > 0 ? MPW - sg * qh(part) : 0) : qh(part);
    }
    static constexpr int ntapp(int part, int sg) { return T - sg * tps(part) < tps(part) ? T - sg * tps(part) : tps(part); }
    // per-wave DMA counts of step sg of a half-chunk of kind `part` (the
    // kernel issues, in this order, the step's share of the next halo, then
    // the weights of step g + NWB - 1)
    static constexpr int ipt(bool lo) { return lo ? 8 : NPLW * 2; }
    static constexpr int nh(int sg) { return MPW - sg * Q < Q ? (MPW - sg * Q > 0 ? MPW - sg * Q : 0) : Q; }
    static constexpr bool lo_of(int sgx, int part, int halves) { return halves == 2 && ((sgx / SPC + part) & 1); }
    static constexpr int nw(int sg, int part, int halves) {
        return (T - ((sg + NWB - 1) % SPC) * TPS < TPS ? T - ((sg + NWB - 1) % SPC) * TPS : TPS) *
               ipt(lo_of(sg + NWB - 1, part, halves)) / NWAVES;
    }
    // DMAs allowed in flight at the end of step sg: those issued after the
    // weights of step g+1 (issued NWB-2 steps earlier), and at a half-chunk's
    // last step none of the next halo (steps of the previous half-chunk are
    // counted with the other part; before the first steps the prologue has
    // already completed everything they need)
    static constexpr int allowed(int sg, int part, int halves) {
        int n = 0;
        for (int j = 0; j <= NWB - 3; ++j) {
            int s = sg - j, p = part;
            if (s < 0) { s += SPC; p = halves == 2 ? part ^ 1 : part; }
            n += nh(s) + nw(s, p, halves);
        }
        if (sg == SPC - 1) {
            int last = 0;  // last step of this half-chunk that issues halo DMAs
            for (int s = 0; s < SPC; ++s)
                if (nh(s) > 0) last = s;
            int after = 0;
            for (int s = last; s < SPC; ++s) after += nw(s, part, halves);
            n = n < after ? n : after;
        }
        return n;
    }
    static_assert(fits(TPS, NWB), "LDS");
};

template <int KS, int PREC, int EPI>
__global__ __launch_bounds__(NTHREADS) void split_conv_kernel(SArgs a) {
    typedef Prec<PREC> PR;
    typedef typename PR::V V;
    typedef Geo<KS, PREC> G;
    constexpr int HC = G::HC, T = G::T, MPW = G::MPW, Q = G::Q;
    constexpr int HB = G::HB, WB = G::WB, WB1 = G::WB1, NWB = G::NWB;
    constexpr int TPS = G::TPS, SPC = G::SPC, HPL = G::HPL, NPIX = G::NPIX;
    constexpr int HALVES = PR::HALVES, WREC = PR::WREC;
    constexpr int D = NWB - 1;  // weight DMA lookahead (steps)
    extern __shared__ __attribute__((aligned(16))) char lds[];
    char *Hs = lds;           // [2][4 planes][NPIX records][16 B]  activation halo
    char *Ws = lds + 2 * HB;  // [NWB][TPS taps][NPLW planes][BM][16 B] weights

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
    const int l16 = lane & 15, kg = lane >> 4;
    const int wn = wave % WNS, wpix = wave / WNS;

    // XCD-aware bijective remap (the 8 XCDs take blocks round robin): L is
    // contiguous per XCD, so consecutive L run concurrently on one XCD.
    const int nblk = gridDim.x, orig = blockIdx.x;
    const int q8 = nblk >> 3, r8 = nblk & 7, xcd = orig & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    int nt, mt, u;
    {
        // one XCD wave of 32 blocks = PXG pixel tiles x NG channel tiles
        // image-major (TMR_SPLIT_UNITS_PER_IMAGE): an image's EI units innermost,
        // so its units' blocks at one tile run back to back on one XCD
        // (measured, profiles/r05c: config-B heads launch 106.55 -> 105.96 ms)
        const int per_unit = a.NT * a.MT;
        const int ub = L / (a.EI * per_unit), rr = L - ub * a.EI * per_unit;
        u = ub * a.EI + rr % a.EI;
        const int r = rr / a.EI;
        if (a.MT % PXG == 0 && a.NT % NG == 0) {
            // pixel tiles in groups of 8; for each group the channel tiles in
            // groups of 4: the 32 co-resident blocks of an XCD share 4 weight
            // slabs and 8 halos through its L2, and a group's halos stay
            // there while its 4 channel groups pass
            const int gsz = PXG * a.NT;
            const int pg = r / gsz, r2 = r - pg * gsz;
            const int ng = r2 / (PXG * NG), r3 = r2 - ng * (PXG * NG);
            mt = pg * PXG + r3 / NG;
            nt = ng * NG + r3 % NG;
        } else {
            nt = r % a.NT;
            mt = r / a.NT;
        }
    }
    const int ty0 = (mt / a.TXN) * TH, tx0 = (mt % a.TXN) * TW;
    const int img = a.unit_image ? a.unit_image[u] : u;
    const int NC = a.NC0 + a.NC1;


    // Per-lane halo DMA source of wave-instruction m (half-chunk invariant):
    // LDS piece e of the halo image is plane e / NPIX, record e % NPIX; pad
    // records re-read a legal address.  The compiler hoists the MPW offsets
    // out of the main loop into VGPRs (r02ao: a per-DMA dependent VALU chain
    // had sat in the waves' in-order MFMA issue stream).
    auto hoff = [&](int m) -> int {
        const int e = (wave + NWAVES * m) * 64 + lane;
        int q = e / NPIX, p = e % NPIX;
        if (q >= P || p >= G::HR * HC) q = p = 0;
        const int hy = p / HC, hx = p % HC;
        return ((q * a.Hp + ty0 + hy) * a.Wp + (tx0 + hx)) * 16;  // planar records: piece q plane
    };
    // Buffer descriptors (SGPRs) over this block's source slabs and weights:
    // every DMA is base + uniform soffset + a 32-bit per-lane voffset, so the
    // loop holds no 64-bit per-lane addresses (and the range check turns any
    // stray read into zeros instead of a fault).
    const uint32_t cstride = (uint32_t)a.Hp * a.Wp * XREC;
    const int h0 = a.NC0 * HALVES, h1 = a.NC1 * HALVES;
    const __amdgpu_buffer_rsrc_t xr0 = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(h0 ? a.x0 + (size_t)img * h0 * cstride : a.x1), (short)0, h0 * cstride, 0x00020000);
    const __amdgpu_buffer_rsrc_t xr1 = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(h1 ? a.x1 + (size_t)u * h1 * cstride : a.x0), (short)0, h1 * cstride, 0x00020000);
    // this wave's halo instruction m of half-chunk hc (every wave issues
    // MPW per half-chunk; hc == NHC, past the end, reads zeros via the
    // descriptor range check into the free buffer)
    auto halo_dma1 = [&](int hc, int m) {
        const bool s0 = hc < h0;
        const uint32_t soff = (uint32_t)(s0 ? hc : hc - h0) * cstride;
        char *dst = Hs + (hc & 1) * HB;
        buffer_lds16(s0 ? xr0 : xr1, (lds_ptr_t)(dst + (wave + NWAVES * m) * 1024), hoff(m), soff);
    };
    // weights of flat step g: half-chunk g / SPC (hi: wh and wl planes, lo:
    // wh only), taps TPS*(g % SPC)...; instruction i of the step = tap i/IPT,
    // plane (i%IPT)/2, channels 64*((i%IPT)&1) + lane: 1 KB contiguous in the
    // planar HBM layout [tap][chunk][plane][Npad][16 B].
    const uint32_t tapstride = (uint32_t)NC * a.Npad * WREC;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.wp, (short)0, T * tapstride, 0x00020000);
    const int wlane = lane * 16;
    const uint32_t wnt = (uint32_t)nt * BM * 16;
    // this wave's weight instruction m of flat step g, whose shape (lo, taps)
    // the caller knows at compile time: ipt instructions per tap, every wave
    // issuing the same count (ipt is a multiple of NWAVES).  g == S (past the
    // end) loads harmless in-range bytes into the free buffer.
    auto w_src = [&](int g, int ipt, int m) -> uint32_t {
        const int hc = g / SPC, t0 = (g - hc * SPC) * TPS;
        const int c = hc / HALVES;
        const uint32_t src = (uint32_t)t0 * tapstride + (uint32_t)c * a.Npad * WREC + wnt;
        const int i = wave + NWAVES * m;
        const int tl = i / ipt, wi = i - tl * ipt;
        return src + (uint32_t)tl * tapstride + (uint32_t)(wi >> 1) * a.Npad * 16 + (wi & 1) * 64 * 16;
    };
    auto w_dst = [&](int g, int ipt, int m) -> char * {
        const int i = wave + NWAVES * m;
        const int tl = i / ipt, wi = i - tl * ipt;
        return Ws + (g % NWB) * WB + tl * WB1 + wi * 1024;
    };
    auto w_dma1 = [&](int g, int ipt, int m) {
        buffer_lds16(wr, (lds_ptr_t)w_dst(g, ipt, m), wlane, w_src(g, ipt, m));
    };
    // LO3: weights of step sgx of half-chunk (cx, px) (the flat step index no
    // longer determines the shape)
    auto w_dma3 = [&](int cx, int px, int sgx, int ipt, int m) {
        const int i = wave + NWAVES * m;
        const int tl = i / ipt, wi = i - tl * ipt;
        const uint32_t src = (uint32_t)(sgx * G::tps(px) + tl) * tapstride + (uint32_t)cx * a.Npad * WREC + wnt +
                             (uint32_t)(wi >> 1) * a.Npad * 16 + (wi & 1) * 64 * 16;
        const int gbx = cx * G::SPCC + (px ? SPC : 0) + sgx;
        char *dst = Ws + (gbx % NWB) * WB + tl * G::wb1(px) + wi * 1024;
        buffer_lds16(wr, (lds_ptr_t)dst, wlane, src);
    };

    // accumulators start at acc_init (scaled into the accumulator's units by
    // the exact power of two s_x s_w); masked elements read a clamped legal
    // address and are zeroed by a select, never by a branch around the load.
    // 16x16 accumulator: column = pixel l16, row = n 4*kg + r.
    // activation scale: one per launch, or per unit / output slab u
    // (TMR_SPLIT_XMAX_PER_UNIT: a unit's precision then does not depend on
    // the magnitudes of the other units in the batch)
    // (TMR_SPLIT_XMAX_PER_PIXEL: the epilogue undoes a scale per output pixel)
    const float *xm = (a.xmax && !(a.flags & TMR_SPLIT_XMAX_PER_PIXEL))
                          ? a.xmax + ((a.flags & TMR_SPLIT_XMAX_PER_UNIT) ? u : 0) : nullptr;
    const float sxw = PR::SCALED ? split_scale(xm) * split_scale(a.wmax) : 1.0f;
    const int HW = a.H * a.W;
    f32x4 acc[NIN][8];
    // tiled acc layout: [slab][nt][mt][wave][in*8+jp][lane][4] fp32 (bf16
    // slabs: 8 B per 16-B group index), i.e. each accumulator register set is
    // one contiguous KB per wave (no masking).  Read before the main loop: the
    // blocks run in lockstep, so this is a chip-wide burst while no MFMA runs
    // (12% of the one-term kernel with fp32 slabs, profiles/archive/r02ah_*; halved
    // by the bf16 slab of the bf16 contract)
    const int islab = (a.flags & TMR_SPLIT_INIT_BCAST) ? 0 : img;  // acc_init slab
    const size_t tile_off = ((((size_t)islab * a.NT + nt) * a.MT + mt) * NWAVES + wave) * ACCW;
    if (a.acc_init && (a.flags & TMR_SPLIT_TILED_INIT) && (a.flags & TMR_SPLIT_INIT_BF16)) {
        // bf16 slab: the same 16-B-group index, 8 B per group
        const b4 *ai = reinterpret_cast<const b4 *>(a.acc_init) + tile_off / 4 + lane;
#pragma unroll
        for (int in = 0; in < NIN; ++in)
#pragma unroll
            for (int jp = 0; jp < 8; ++jp)
                acc[in][jp] = __builtin_convertvector(ai[(in * 8 + jp) * 64], f32x4) * sxw;
    } else if (a.acc_init && (a.flags & TMR_SPLIT_TILED_INIT)) {
        const f32x4 *ai = reinterpret_cast<const f32x4 *>(a.acc_init + tile_off) + lane;
#pragma unroll
        for (int in = 0; in < NIN; ++in)
#pragma unroll
            for (int jp = 0; jp < 8; ++jp) acc[in][jp] = ai[(in * 8 + jp) * 64] * sxw;
    } else if (a.acc_init) {
        const float *ai = a.acc_init + (size_t)islab * a.N * HW;
#pragma unroll
        for (int jp = 0; jp < 8; ++jp) {
            const int y = ty0 + wpix * 4 + (jp >> 1), x = tx0 + (jp & 1) * 16 + l16;
            const bool pin = y < a.H && x < a.W;
            const int pix = min(y, a.H - 1) * a.W + min(x, a.W - 1);
#pragma unroll
            for (int in = 0; in < NIN; ++in)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int n = nt * BM + wn * 64 + in * 16 + 4 * kg + r;
                    const float v = ai[(size_t)min(n, a.N - 1) * HW + pix];
                    acc[in][jp][r] = (pin && n < a.N) ? v * sxw : 0.0f;
                }
        }
    } else {
#pragma unroll
        for (int in = 0; in < NIN; ++in)
#pragma unroll
            for (int jp = 0; jp < 8; ++jp)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[in][jp][r] = 0.0f;
    }

    // fragment bases: lane group kg supplies K = 8kg..8kg+7 (plane kg; the wl
    // planes follow the wh planes); per-tap offsets are immediates
    const int aoff = kg * WPL + (wn * 64 + l16) * 16;
    const int boff = kg * HPL + (wpix * 4 * HC + l16) * 16;

    // compile-time shape of step sg of a half-chunk of kind lo
    auto ipt_of = [](bool lo_) { return lo_ ? 8 : G::NPLW * 2; };  // weight DMAs per tap
#pragma unroll
    for (int m = 0; m < MPW; ++m) halo_dma1(0, m);
    // prologue weights: steps 0..D-1 of half-chunk 0 (a hi one)
#pragma unroll
    for (int g0 = 0; g0 < D; ++g0) {
        const bool lo0 = HALVES == 2 && ((g0 / SPC) & 1);
        const int nt0 = min(TPS, T - (g0 % SPC) * TPS) * ipt_of(lo0) / NWAVES;
#pragma unroll
        for (int m = 0; m < nt0; ++m) w_dma1(g0, ipt_of(lo0), m);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int c = 0; c < NC; ++c) {
        // one half-chunk; PART is a compile-time constant (F16X3: 0 = hi, 1 = lo)
        auto half_chunk = [&](auto part_c) {
            constexpr int part = decltype(part_c)::value;
            constexpr bool lo = part == 1;  // F16X3 lo half-chunk: wh . xl only
            const int hc = c * HALVES + part;
            const char *hl = Hs + (hc & 1) * HB;
            // the half-chunk's steps as compile-time indices (DMA counts and
            // waits are constants): step(integral_constant<int, sg>)
            auto step = [&](auto sg_c) {
                constexpr int sg = decltype(sg_c)::value;
                constexpr bool L3 = G::LO3;
                constexpr int TPSx = L3 ? G::tps(part) : TPS;
                const int g = L3 ? c * G::SPCC + (part ? SPC : 0) + sg : hc * SPC + sg;
                // DMAs for later steps, issued one per pixel-tile MFMA group
                // from the step's second group on (not in the post-barrier
                // bubble): first this step's share of the halo of half-chunk
                // hc+1 (buffer last read in hc-1), then the weights of step
                // g+D (buffer last read in g-1).  Counts are compile-time and
                // the same in every wave.
                // LO3: the next step is (part, sg+1), the lo half-chunk's step 0
                // or the next chunk's hi step 0
                constexpr bool lastx = sg + 1 >= G::spc(part);
                constexpr int pn = lastx ? 1 - part : part, sgn = lastx ? 0 : sg + 1;
                constexpr int nh = L3 ? G::nhp(part, sg) : G::nh(sg);
                constexpr bool loD = L3 ? pn == 1 : G::lo_of(sg + D, part, HALVES);
                constexpr int nw = L3 ? G::ntapp(pn, sgn) * G::ipt(pn == 1) / NWAVES : G::nw(sg, part, HALVES);
                constexpr int NSLOT = nh + nw;
                auto dma_slot = [&](int k) {  // slot k of this step (k < NSLOT)
                    if constexpr (L3) {
                        if (k < nh)
                            halo_dma1(hc + 1, sg * G::qh(part) + k);
                        else
                            w_dma3(lastx && part == 1 ? c + 1 : c, pn, sgn, ipt_of(loD), k - nh);
                    } else {
                        if (k < nh)
                            halo_dma1(hc + 1, sg * Q + k);
                        else
                            w_dma1(g + D, ipt_of(loD), k - nh);
                    }
                };
                const char *wl = Ws + (g % NWB) * WB;
                // Register pipeline: the A (weight) fragments of a tap are
                // read during the previous tap of the step, the B (halo)
                // fragments DB pixel tiles ahead, so an MFMA group never
                // waits on LDS except at the step's first tap.  F16X3 hi
                // half-chunks run wh.xh and wl.xh off one B read (NA = 8
                // A fragments), the others one term (NA = 4).
                constexpr int NA = (HALVES == 2 && !lo) ? 2 * NIN : NIN;
                constexpr int DB = NA >= 8 ? 1 : 2;
                constexpr int APG = NA >= 8 ? NA / 8 : 1;  // next-tap A reads per pixel tile
                constexpr int NB = DB + 1;
                constexpr int ntap = L3 ? G::ntapp(part, sg) : (T - sg * TPS < TPS ? T - sg * TPS : TPS);
                constexpr int WB1x = L3 ? G::wb1(part) : WB1;
                auto afrag = [&](int tl, int i) -> V {  // term i / NIN, n fragment i % NIN
                    return *reinterpret_cast<const V *>(wl + tl * WB1x + (i / NIN) * 4 * WPL + aoff +
                                                        (i % NIN) * 256);
                };
                auto bfrag = [&](int tap, int jp) -> V {
                    const int ky = tap / KS, kx = tap % KS;
                    return *reinterpret_cast<const V *>(
                        hl + boff + (((jp >> 1) + ky) * HC + kx + (jp & 1) * 16) * 16);
                };
                V aw[2][NA];
                V bx[NB];
#pragma unroll
                for (int i = 0; i < NA; ++i) aw[0][i] = afrag(0, i);
#pragma unroll
                for (int d = 0; d < DB; ++d) bx[d] = bfrag(sg * TPSx, d);
                __builtin_amdgcn_sched_group_barrier(0x100, NA + DB, 0);
#pragma unroll
                for (int tl = 0; tl < TPSx; ++tl) {
                    if (tl >= ntap) break;
                    const int tap = sg * TPSx + tl;
                    const bool more = tl + 1 < ntap;
#pragma unroll
                    for (int jp = 0; jp < 8; ++jp) {
                        const int q = tl * 8 + jp, qn = q + DB;
                        const bool rb = jp + DB < 8 || more;
                        if (rb) bx[qn % NB] = jp + DB < 8 ? bfrag(tap, jp + DB) : bfrag(tap + 1, jp + DB - 8);
                        // next tap's A: one fragment per pixel tile (hi), the
                        // first four tiles (one-term)
                        const int na = (more && jp * APG < NA) ? APG : 0;
#pragma unroll
                        for (int j = 0; j < APG; ++j)
                            if (j < na) aw[(tl + 1) & 1][jp * APG + j] = afrag(tl + 1, jp * APG + j);
                        // DMA slot k = q - 1 (groups 1.. of the step)
                        const int k = q - 1;
                        const bool dm = k >= 0 && k < NSLOT;
                        if (dm) dma_slot(k);
                        const V b = bx[q % NB];
#pragma unroll
                        for (int i = 0; i < NA; ++i)
                            acc[i % NIN][jp] = mma(aw[tl & 1][i], b, acc[i % NIN][jp]);
                        const int nr = (rb ? 1 : 0) + na;
                        if (nr == 3)
                            __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
                        else if (nr == 2)
                            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                        else if (nr == 1)
                            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        if (dm) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x008, NA, 0);
                    }
                }
                // slots beyond the step's groups (not reached by the shapes
                // built here, kept for safety)
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    if (k >= ntap * 8 - 1 && k < NSLOT) dma_slot(k);
                __builtin_amdgcn_sched_barrier(0);
                // the next step needs W(g+1) and, after a half-chunk's last
                // step, the whole halo of hc+1: leave only younger DMAs in
                // flight (in-order completion; halo issued before weights)
                if constexpr (D == 1)
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                else
                    wait_vmcnt(G::allowed(sg, part, HALVES));
                __builtin_amdgcn_s_barrier();
            };
            [&]<int... SG>(std::integer_sequence<int, SG...>) {
                (step(std::integral_constant<int, SG>{}), ...);
            }(std::make_integer_sequence<int, G::LO3 ? G::spc(part) : SPC>{});
        };
        half_chunk(std::integral_constant<int, 0>{});
        if constexpr (HALVES == 2) half_chunk(std::integral_constant<int, 1>{});
    }
    // the last steps issued dummy DMAs (past the end) into LDS the epilogue reuses
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---------------- epilogue ----------------
    const float inv = 1.0f / sxw;  // 2^-k: exact
    if (EPI == 0 && (a.flags & TMR_SPLIT_TILED_OUT) && (a.flags & TMR_SPLIT_OUT_BF16)) {
        b4 *o = reinterpret_cast<b4 *>(a.out) + ((((size_t)u * a.NT + nt) * a.MT + mt) * NWAVES + wave) * ACCW / 4 +
                lane;
#pragma unroll
        for (int in = 0; in < NIN; ++in)
#pragma unroll
            for (int jp = 0; jp < 8; ++jp)
                __builtin_nontemporal_store(__builtin_convertvector(acc[in][jp] * inv, b4), o + (in * 8 + jp) * 64);
        return;
    }
    if (EPI == 0 && (a.flags & TMR_SPLIT_TILED_OUT)) {
        // raw conv result (scaled back) in the tiled acc layout of slab u: the
        // acc_init of a later launch; bias / activation are not applied here
        f32x4 *o = reinterpret_cast<f32x4 *>(
                       a.out + ((((size_t)u * a.NT + nt) * a.MT + mt) * NWAVES + wave) * ACCW) +
                   lane;
#pragma unroll
        for (int in = 0; in < NIN; ++in)
#pragma unroll
            for (int jp = 0; jp < 8; ++jp) {
                // non-temporal: read back by a later launch (+0.4% config B)
                __builtin_nontemporal_store(acc[in][jp] * inv, o + (in * 8 + jp) * 64);
            }
        return;
    }
    // the block's bias and head weights through LDS (the main loop's last
    // barrier freed it): global loads here would be hoisted into registers
    float *red = reinterpret_cast<float *>(lds);   // [4 wpix][8 jp][NHEAD][16]
    float *sb = red + 4 * 8 * NHEAD * 16;
    float *shw = sb + BM;                          // [BM][NHEAD]
    if (tid < BM) {
        const int n = nt * BM + tid;
        sb[tid] = n < a.N ? a.bias[n] : 0.0f;
    }
    if (EPI == 1)
        for (int e = tid; e < BM * NHEAD; e += NTHREADS) shw[e] = a.headw[(size_t)nt * BM * NHEAD + e];
    __syncthreads();
    if constexpr (EPI == 0) {
        // TMR_SPLIT_XMAX_PER_PIXEL (1x1 convs): each accumulator column is one
        // pixel, packed with its own scale (the max over its channels), so
        // every output pixel is fp32-grade relative to its own magnitude
        float invp[8];
#pragma unroll
        for (int jp = 0; jp < 8; ++jp) {
            invp[jp] = inv;
            const int y = ty0 + wpix * 4 + (jp >> 1), x = tx0 + (jp & 1) * 16 + l16;
            if (PR::SCALED && (a.flags & TMR_SPLIT_XMAX_PER_PIXEL) && y < a.H && x < a.W)
                invp[jp] = 1.0f / (split_scale(a.xmax + ((size_t)u * a.H + y) * a.W + x) * split_scale(a.wmax));
        }
#pragma unroll
        for (int in = 0; in < NIN; ++in)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int nl = wn * 64 + in * 16 + 4 * kg + r;
                const int n = nt * BM + nl;
                const bool nin = n < a.N;
                const float bn = sb[nl];
#pragma unroll
                for (int jp = 0; jp < 8; ++jp) {
                    const int y = ty0 + wpix * 4 + (jp >> 1), x = tx0 + (jp & 1) * 16 + l16;
                    float v = acc[in][jp][r] * invp[jp] + bn;
                    if (a.leaky) v = v >= 0.0f ? v : v * 0.01f;
                    if (nin && y < a.H && x < a.W) a.out[((size_t)u * a.N + n) * HW + (size_t)y * a.W + x] = v;
                }
            }
        return;
    }
    // Heads: per pixel pair (jp = 2q, 2q+1) on v_pk_fma_f32.  acc * inv is
    // exact (a power of two), so fma(acc, inv, bias) rounds once, like the
    // separate multiply and add; LeakyReLU as max(v, 0.01 v) (= the select
    // form for every v, incl. -0, inf and NaN).
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 hs2[4][NHEAD];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < NHEAD; ++k) hs2[q][k] = (f2){0.0f, 0.0f};
    const f2 inv2 = {inv, inv};
#pragma unroll
    for (int in = 0; in < NIN; ++in)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int nl = wn * 64 + in * 16 + 4 * kg + r;
            const f2 bn2 = {sb[nl], sb[nl]};
            f2 hw2[NHEAD];
#pragma unroll
            for (int k = 0; k < NHEAD; ++k) hw2[k] = (f2){shw[nl * NHEAD + k], shw[nl * NHEAD + k]};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f2 v = {acc[in][2 * q][r], acc[in][2 * q + 1][r]};
                v = __builtin_elementwise_fma(v, inv2, bn2);
                if (a.leaky) {
                    const f2 m = v * (f2){0.01f, 0.01f};
                    v = (f2){fmaxf(v.x, m.x), fmaxf(v.y, m.y)};
                }
#pragma unroll
                for (int k = 0; k < NHEAD; ++k) hs2[q][k] = __builtin_elementwise_fma(v, hw2[k], hs2[q][k]);
            }
            // keep the LDS reads of bias / head weights per row (hoisted, they
            // would overlap the 128 live accumulators)
            __builtin_amdgcn_sched_barrier(0);
        }
    // Sum over the 4 lane groups (rows of 16 lanes = n rows) by transpose-
    // reduce: the 40 values X[j] (j = 2(5q + k) + (jp & 1)) pairwise through
    // v_permlane16_swap (rows 0+1, 2+3), then v_permlane32_swap (halves):
    // lane group kg ends with X[4p + kg], p = 0..9, summed as
    // (x0 + x1) + (x2 + x3) -- the order of the xor-16 / xor-32 shuffles.
    float X[40];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < NHEAD; ++k) {
            X[2 * (5 * q + k)] = hs2[q][k].x;
            X[2 * (5 * q + k) + 1] = hs2[q][k].y;
        }
    float Y[20], Z[10];
#pragma unroll
    for (int m = 0; m < 20; ++m) {
        const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(X[2 * m]), __float_as_uint(X[2 * m + 1]),
                                                         false, false);
        Y[m] = __uint_as_float(s[0]) + __uint_as_float(s[1]);
    }
#pragma unroll
    for (int p = 0; p < 10; ++p) {
        const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(Y[2 * p]), __float_as_uint(Y[2 * p + 1]),
                                                         false, false);
        Z[p] = __uint_as_float(s[0]) + __uint_as_float(s[1]);
    }
    // then over the two n-waves (wn = 1 through LDS), every lane storing its 10
    __syncthreads();  // sb / shw reads are done before red is written
    if (WNS == 2 && wn == 1) {
#pragma unroll
        for (int p = 0; p < 10; ++p) red[((wpix * 10 + p) * 4 + kg) * 16 + l16] = Z[p];
    }
    __syncthreads();
    if (wn == 0) {
#pragma unroll
        for (int p = 0; p < 10; ++p) {
            const int j = 4 * p + kg, m = j >> 1, q = m / NHEAD, k = m - q * NHEAD;
            const int jp = 2 * q + (j & 1);
            const int y = ty0 + wpix * 4 + (jp >> 1), x = tx0 + (jp & 1) * 16 + l16;
            const float v = Z[p] + (WNS == 2 ? red[((wpix * 10 + p) * 4 + kg) * 16 + l16] : 0.0f);
            if (y < a.H && x < a.W) a.partials[(((size_t)nt * NHEAD + k) * a.U + u) * HW + (size_t)y * a.W + x] = v;
        }
    }
}

template <int KS, int PREC, int EPI>
int launch_split(SArgs a, hipStream_t s) {
    constexpr size_t lds = Geo<KS, PREC>::LDS;
    static_assert(lds <= 160 * 1024, "LDS");
    static_assert((4 * 8 * NHEAD * 16 + BM * (NHEAD + 1)) * 4 <= lds, "epilogue scratch");
    auto kern = split_conv_kernel<KS, PREC, EPI>;
    if (tmr_set_max_lds((const void *)kern, lds) !=
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

inline int prec_halves(int prec) { return prec == TMR_PREC_F16X3 ? 2 : 1; }
inline int prec_wrec(int prec) { return prec == TMR_PREC_F16X3 ? 128 : 64; }
inline bool prec_ok(int prec) {
    return prec == TMR_PREC_F16X3 || prec == TMR_PREC_BF16 || prec == TMR_PREC_F16;
}
inline bool ks_ok(int ks) { return ks == 1 || ks == 3 || ks == 5 || ks == 7; }
inline int pad_h(int H, int ks) { return (int)tmr_cdiv(H, TH) * TH + ks - 1; }
inline int pad_w(int W, int ks) { return (int)tmr_cdiv(W, TW) * TW + ks - 1; }

// ---------------------------------------------------------------- packing
// max |x| into *out (as uint: m >= 0 orders like its bits).  One atomic per
// BLOCK after an LDS reduction, and at most 512 blocks with >= 8 elements
// per thread: per-wave atomics on the one address serialised in L2 (4096 of
// them for a 1-M-float input: 33 us, profiles/r04b/prof_A_kernel_stats.md)
__device__ __forceinline__ void absmax_commit(float m, unsigned *out) {
    __shared__ float red[4];
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(out, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

__global__ __launch_bounds__(256) void absmax_rows_kernel(const float *__restrict__ x, int64_t n, int vec,
                                                          unsigned *__restrict__ out) {
    const float *xr = x + (size_t)blockIdx.y * n;
    float m = 0.0f;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    if (vec) {
        const float4 *x4 = reinterpret_cast<const float4 *>(xr);
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += step) {
            const float4 v = x4[i];
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step)
            m = fmaxf(m, fabsf(xr[i]));
    }
    absmax_commit(m, out + blockIdx.y);
}

// tmr_pixel_absmax: out[s][p] = max_c |x[s][c][p]|.  A block is 64
// consecutive pixels x 8 channel groups (coalesced 256-B rows per wave, each
// thread C/8 planes with its loads in flight together), folded through LDS.
// (One thread per pixel walking all C planes had 16 blocks and a 256-load
// chain at config A: 77 us per image.)
constexpr int PA_PIX = 64, PA_GRP = 8;
__global__ __launch_bounds__(PA_PIX * PA_GRP) void pixel_absmax_kernel(const float *__restrict__ x, int S, int C,
                                                                       int64_t HW, float *__restrict__ out) {
    __shared__ float part[PA_GRP][PA_PIX];
    const int lane = threadIdx.x & (PA_PIX - 1), grp = threadIdx.x / PA_PIX;
    const int64_t i = (int64_t)blockIdx.x * PA_PIX + lane;
    float m = 0.0f;
    if (i < (int64_t)S * HW) {
        const int64_t s = i / HW, p = i - s * HW;
        const float *xp = x + (size_t)s * C * HW + p;
#pragma unroll 8
        for (int c = grp; c < C; c += PA_GRP) m = fmaxf(m, fabsf(xp[(size_t)c * HW]));
    }
    part[grp][lane] = m;
    __syncthreads();
    if (grp == 0 && i < (int64_t)S * HW) {
#pragma unroll
        for (int g = 1; g < PA_GRP; ++g) m = fmaxf(m, part[g][lane]);
        out[i] = m;
    }
}

// tmr_scale_merge: block b finds its image's units (unit_image[u] == b),
// out_img[b] = max(img_max[b], their unit_max), then writes that to each
// of them in out_unit (the shared scale of a launch whose tiles read the
// image's records and the unit's records together)
__global__ __launch_bounds__(256) void scale_merge_kernel(const float *__restrict__ img_max,
                                                          const float *__restrict__ unit_max,
                                                          const int32_t *__restrict__ unit_image, int U,
                                                          float *__restrict__ out_img,
                                                          float *__restrict__ out_unit) {
    __shared__ float red[4];
    const int b = blockIdx.x;
    float m = 0.0f;
    for (int u = threadIdx.x; u < U; u += blockDim.x)
        if (unit_image[u] == b) m = fmaxf(m, unit_max[u]);
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (img_max) m = fmaxf(m, img_max[b]);
    if (threadIdx.x == 0 && out_img) out_img[b] = m;
    for (int u = threadIdx.x; u < U; u += blockDim.x)
        if (unit_image[u] == b) out_unit[u] = m;
}

// Activation records: value v(s, ch, y, x) -> [S][NCc*HALVES][4 pieces][Hp][Wp][16 B],
// padded (yp, xp) holding v at (yp - ks/2, xp - ks/2), zero outside.  One
// thread per (s, chunk, yp, xp) writes the chunk's hi (and lo) record.
// MODE 0: v = x[s][ch][y][x]; MODE 1: v = [up2x(f) or f; 1] from the SAM
// features (the fp-half fold, tmr_split_fold_proj / the input_proj input):
// the same fma form as tmr_upsample_proj (ATen's CPU kernel); the constant-1
// channel carries the projection bias and is zero in the padding.
template <int PREC, int MODE>
__global__ void xpack_kernel(const float *__restrict__ x, int S, int Cin, int Hin, int Win, int ups,
                             int ones, int H, int W, int NCc, int Hp, int Wp, int pad,
                             const float *__restrict__ xmax, int xms,
                             typename Prec<PREC>::V *__restrict__ out) {
    constexpr int HALVES = Prec<PREC>::HALVES;
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
    // scale source: one (xms 0), per sample (1) or per output pixel (2: [S][H][W])
    const float *xm = !xmax ? nullptr
                      : xms == 2 ? (in ? xmax + ((size_t)s * H + y) * W + xx : nullptr)
                                 : xmax + (size_t)s * xms;
    const float sc = Prec<PREC>::SCALED ? split_scale(xm) : 1.0f;
    float v[CCH];
#pragma unroll
    for (int k = 0; k < CCH; ++k) {
        const int ch = c * CCH + k;
        float val = 0.0f;
        if (in) {
            if (MODE == 0) {
                if (ch < Cin) val = x[(((size_t)s * Cin + ch) * H + y) * W + xx];
            } else if (ch < Cin) {
                const float *pl = x + ((size_t)s * Cin + ch) * Hin * Win;
                val = ups ? up_value(pl, Hin, Win, y, xx) : pl[(size_t)y * Win + xx];
            } else if (ones && ch == Cin) {
                val = 1.0f;
            }
        }
        v[k] = val;
    }
    typename Prec<PREC>::V hi[P], lo[P];
    split_record<PREC>(v, sc, hi, lo);
    // planar: [s][chunk][half][piece q][Hp][Wp] 16-B pieces (the conv's
    // LDS-DMA reads 64 consecutive pieces of one plane per instruction)
    const size_t plane = (size_t)Hp * Wp;
    typename Prec<PREC>::V *o = out + ((size_t)s * NCc + c) * HALVES * P * plane + (size_t)yp * Wp + xp;
#pragma unroll
    for (int q = 0; q < P; ++q) o[q * plane] = hi[q];
    if (HALVES == 2) {
#pragma unroll
        for (int q = 0; q < P; ++q) o[(P + q) * plane] = lo[q];
    }
}

// MODE 0 with W % 4 == 0: one 256-thread block per (image, chunk, row, 128-px
// segment) stages the segment's 32 channel rows in LDS from 16-B loads, then
// every thread forms (pixel, 8-channel piece) records and stores them
// pixel-contiguous (1 KB per wave store).  Blocks past `nseg` write the
// padding ring (zero records: the split of 0 is 0 in every term).  Records
// are bit-identical to xpack_kernel<PREC, 0>'s.
constexpr int XSEG = 128;
constexpr int XPACK16_RPB = 4;  // rows per block of the bf16-input record pack (1/4/8: r03s)
// IN: the activation's element type, float or __bf16 (a bf16 f_TM plane from
// tmr_xcorr with out_bf16: bf16 records of it are its own elements, tmr_split_xpack16);
// RPB rows of the segment per block (the bf16 form moves half the bytes per
// row: 4 rows keep as many loads in flight per block).
template <int PREC, typename IN = float, int RPB = 1>
__global__ __launch_bounds__(256) void xpack4_kernel(const IN *__restrict__ x, int S, int Cin, int H, int W,
                                                     int NCc, int Hp, int Wp, int pad, int64_t nseg,
                                                     int64_t nbord, const float *__restrict__ xmax, int xms,
                                                     typename Prec<PREC>::V *__restrict__ out) {
    constexpr int HALVES = Prec<PREC>::HALVES;
    typedef typename Prec<PREC>::V V;
    typedef typename Prec<PREC>::E E;
    constexpr int VE = 16 / sizeof(IN);  // elements per 16-B load
    constexpr int LPR = CCH * XSEG / VE;  // 16-B loads per row
    typedef IN INV __attribute__((ext_vector_type(VE)));
    static_assert(RPB * LPR % 256 == 0 && RPB * XSEG * P % 256 == 0 && XSEG % VE == 0, "xpack4 tiling");
    __shared__ __attribute__((aligned(16))) IN tile[RPB][CCH][XSEG];
    const size_t plane = (size_t)Hp * Wp;
    const int t = threadIdx.x;
    if ((int64_t)blockIdx.x < nseg) {
        const int nsx = (W + XSEG - 1) / XSEG, nyg = (H + RPB - 1) / RPB;
        int64_t r = blockIdx.x;
        const int sx = (int)(r % nsx);
        r /= nsx;
        const int y0 = (int)(r % nyg) * RPB;
        r /= nyg;
        const int c = (int)(r % NCc);
        const int s = (int)(r / NCc);
        const int x0 = sx * XSEG, nx = min(XSEG, W - x0);  // nx % VE == 0
        const IN *src = x + ((size_t)s * Cin + (size_t)c * CCH) * H * W + (size_t)y0 * W + x0;
#pragma unroll
        for (int k = 0; k < RPB * LPR / 256; ++k) {
            const int e = t + 256 * k, rr = e / LPR, ch = (e % LPR) / (XSEG / VE), xv = e % (XSEG / VE);
            INV v = {};
            if (VE * xv < nx && c * CCH + ch < Cin && y0 + rr < H)
                v = *reinterpret_cast<const INV *>(src + (size_t)ch * H * W + (size_t)rr * W + VE * xv);
            *reinterpret_cast<INV *>(&tile[rr][ch][VE * xv]) = v;
        }
        __syncthreads();
        const float sc = Prec<PREC>::SCALED ? split_scale(xmax ? xmax + (size_t)s * xms : nullptr) : 1.0f;
        V *o = out + ((size_t)s * NCc + c) * HALVES * P * plane + (size_t)(y0 + pad) * Wp + x0 + pad;
#pragma unroll
        for (int k = 0; k < RPB * XSEG * P / 256; ++k) {
            const int e = t + 256 * k, rr = e / (XSEG * P), q = (e % (XSEG * P)) / XSEG, px = e % XSEG;
            if (px < nx && y0 + rr < H) {
                V hi, lo;
#pragma unroll
                for (int m = 0; m < 8; ++m) {  // split_record's arithmetic
                    const float xs = (float)tile[rr][q * 8 + m][px] * sc;
                    const E h = (E)xs;
                    hi[m] = h;
                    if (HALVES == 2) lo[m] = (E)(xs - (float)h);
                }
                o[q * plane + (size_t)rr * Wp + px] = hi;
                if (HALVES == 2) o[(P + q) * plane + (size_t)rr * Wp + px] = lo;
            }
        }
        return;
    }
    // padding ring of plane set (s, c): top rows, bottom rows, then the
    // left/right columns of the interior rows
    const int64_t b0 = ((int64_t)blockIdx.x - nseg) * 256 + t;
    if (b0 >= nbord * S * NCc) return;
    const int64_t sc_i = b0 / nbord;
    int64_t b = b0 - sc_i * nbord;
    const int64_t top = (int64_t)pad * Wp, bot = (int64_t)(Hp - H - pad) * Wp;
    int yp, xp;
    if (b < top) {
        yp = (int)(b / Wp), xp = (int)(b % Wp);
    } else if ((b -= top) < bot) {
        yp = H + pad + (int)(b / Wp), xp = (int)(b % Wp);
    } else {
        b -= bot;
        const int side = Wp - W, k = (int)(b % side);
        yp = pad + (int)(b / side), xp = k < pad ? k : W + k;
    }
    V *o = out + (size_t)sc_i * HALVES * P * plane + (size_t)yp * Wp + xp;
    const V z = {};
#pragma unroll
    for (int q = 0; q < HALVES * P; ++q) o[q * plane] = z;
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

// w [N][C0+C1][ks][ks] fp32 -> [ks*ks][NC0+NC1][WREC/16 planes][Npad][16 B]; the src0
// and src1 channel ranges are padded to whole 32-channel chunks separately.
template <int PREC>
__global__ void wpack_kernel(const float *__restrict__ w, int N, int C0, int C1, int ks, int NC0,
                             int NC, int Npad, const float *__restrict__ wmax,
                             typename Prec<PREC>::V *__restrict__ out) {
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
    float v[CCH];
#pragma unroll
    for (int k = 0; k < CCH; ++k) {
        int ch;
        bool ok;
        if (c < NC0) {
            ch = c * CCH + k;
            ok = ch < C0;
        } else {
            const int c1 = (c - NC0) * CCH + k;
            ch = C0 + c1;
            ok = c1 < C1;
        }
        v[k] = (ok && n < N) ? w[((size_t)n * C + ch) * T + tap] : 0.0f;
    }
    typename Prec<PREC>::V hi[P], lo[P];
    split_record_w<PREC>(v, sc, hi, lo);
    // planar: [tap][chunk][plane (wh pieces, then wl pieces)][Npad] 16-B pieces
    constexpr int NP = Prec<PREC>::WREC / 16;
    typename Prec<PREC>::V *o = out + ((size_t)tap * NC + c) * NP * Npad + n;
#pragma unroll
    for (int q = 0; q < P; ++q) o[(size_t)q * Npad] = hi[q];
    if (NP == 8) {
#pragma unroll
        for (int q = 0; q < P; ++q) o[(size_t)(P + q) * Npad] = lo[q];
    }
}

int split_common(const void *xp0, int C0, const int32_t *unit_image, const void *xp1, int C1, int U,
                 int H, int W, int ks, int prec, const void *wpack, const float *wmax,
                 const float *xmax, const float *bias, int N, int leaky, const float *acc_init,
                 float *out, const float *headw, float *partials, int epi, int flags, void *stream) {
    TMR_REQUIRE(prec_ok(prec) && ks_ok(ks));
    TMR_REQUIRE(wpack && bias && U > 0 && H > 0 && W > 0 && N > 0 && C0 >= 0 && C1 >= 0);
    TMR_REQUIRE(C0 + C1 > 0 && (C0 == 0 || xp0) && (C1 == 0 || xp1));
    TMR_REQUIRE(prec == TMR_PREC_BF16 || (wmax && xmax));
    // bf16 slabs: one-term precisions, and only on a tiled out / tiled init
    TMR_REQUIRE(!(flags & (TMR_SPLIT_OUT_BF16 | TMR_SPLIT_INIT_BF16)) || prec != TMR_PREC_F16X3);
    TMR_REQUIRE(!(flags & TMR_SPLIT_OUT_BF16) || (flags & TMR_SPLIT_TILED_OUT));
    TMR_REQUIRE(!(flags & TMR_SPLIT_INIT_BF16) || (flags & TMR_SPLIT_TILED_INIT));
    // per-pixel activation scales: 1x1 plain stores only (the K dimension of a
    // kxk conv mixes neighbouring pixels; the scale is undone in that epilogue)
    TMR_REQUIRE(!(flags & TMR_SPLIT_XMAX_PER_PIXEL) ||
                (ks == 1 && !epi && !acc_init && !(flags & (TMR_SPLIT_TILED_OUT | TMR_SPLIT_XMAX_PER_UNIT))));
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
    a.NC0 = (int)tmr_cdiv(C0, CCH);
    a.NC1 = (int)tmr_cdiv(C1, CCH);
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
    a.flags = flags & 0xff;
    a.EI = std::max(1, (flags >> TMR_SPLIT_UNITS_PER_IMAGE_SHIFT) & 0xff);
    TMR_REQUIRE(U % a.EI == 0);
    hipStream_t s = tmr_stream(stream);
    return epi ? dispatch_ks<1>(ks, prec, a, s) : dispatch_ks<0>(ks, prec, a, s);
}

template <int MODE>
int xpack_launch(const float *x, int S, int Cin, int Hin, int Win, int ups, int ones, int H, int W,
                 int ks, int prec, const float *xmax, int xms, void *out, void *stream) {
    const int C = Cin + (MODE == 1 && ones ? 1 : 0);
    const int NCc = (int)tmr_cdiv(C, CCH), Hp = pad_h(H, ks), Wp = pad_w(W, ks);
    const int64_t total = (int64_t)S * NCc * Hp * Wp;
    const dim3 grid((unsigned)tmr_cdiv(total, 256)), blk(256);
    hipStream_t s = tmr_stream(stream);
    // one-term records from LDS-transposed row segments (bf16 0.61 -> 0.50 ms
    // per 48 units at 128^2, r02bo3); the 3-term records stay on the
    // one-pixel kernel (0.61 vs 0.73 ms: twice the stores per staged byte)
    if (MODE == 0 && W % 4 == 0 && prec != TMR_PREC_F16X3 && xms != 2) {
        const int64_t nseg = (int64_t)S * NCc * H * tmr_cdiv(W, XSEG), nbord = (int64_t)Hp * Wp - (int64_t)H * W;
        const dim3 g4((unsigned)(nseg + tmr_cdiv(nbord * S * NCc, 256)));
        switch (prec) {
            case TMR_PREC_BF16:
                hipLaunchKernelGGL(xpack4_kernel<TMR_PREC_BF16>, g4, blk, 0, s, x, S, Cin, H, W, NCc, Hp, Wp,
                                   ks / 2, nseg, nbord, nullptr, 0, static_cast<b8 *>(out));
                break;
            default:
                hipLaunchKernelGGL(xpack4_kernel<TMR_PREC_F16>, g4, blk, 0, s, x, S, Cin, H, W, NCc, Hp, Wp,
                                   ks / 2, nseg, nbord, xmax, xms, static_cast<h8 *>(out));
                break;
        }
        TMR_CHECK_LAUNCH();
        return TMR_OK;
    }
    switch (prec) {
        case TMR_PREC_F16X3:
            hipLaunchKernelGGL((xpack_kernel<TMR_PREC_F16X3, MODE>), grid, blk, 0, s, x, S, Cin, Hin, Win,
                               ups, ones, H, W, NCc, Hp, Wp, ks / 2, xmax, xms, static_cast<h8 *>(out));
            break;
        case TMR_PREC_BF16:
            hipLaunchKernelGGL((xpack_kernel<TMR_PREC_BF16, MODE>), grid, blk, 0, s, x, S, Cin, Hin, Win,
                               ups, ones, H, W, NCc, Hp, Wp, ks / 2, nullptr, 0, static_cast<b8 *>(out));
            break;
        default:
            hipLaunchKernelGGL((xpack_kernel<TMR_PREC_F16, MODE>), grid, blk, 0, s, x, S, Cin, Hin, Win,
                               ups, ones, H, W, NCc, Hp, Wp, ks / 2, xmax, xms, static_cast<h8 *>(out));
            break;
    }
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

}  // namespace

extern "C" int tmr_absmax_rows(const float *x, int S, int64_t n, int accumulate, float *out, void *stream) {
    TMR_REQUIRE(out && S > 0 && S < 65536 && n >= 0 && (n == 0 || x));
    hipStream_t s = tmr_stream(stream);
    if (!accumulate && hipMemsetAsync(out, 0, sizeof(float) * (size_t)S, s) != hipSuccess) return TMR_E_HIP;
    if (n == 0) return TMR_OK;
    const int vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (n & 3) == 0;
    const int64_t per = vec ? n / 4 : n;
    // about 2048 blocks in all, >= 8 elements per thread
    const int bpr = (int)std::max<int64_t>(1, std::min<int64_t>(tmr_cdiv(per, 256 * 8), std::max(1, 2048 / S)));
    hipLaunchKernelGGL(absmax_rows_kernel, dim3(bpr, S), dim3(256), 0, s, x, n, vec,
                       reinterpret_cast<unsigned *>(out));
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int tmr_pixel_absmax(const float *x, int S, int C, int64_t HW, float *out, void *stream) {
    TMR_REQUIRE(x && out && S > 0 && C > 0 && HW > 0);
    const int64_t n = (int64_t)S * HW;
    TMR_REQUIRE(tmr_cdiv(n, PA_PIX) < (1LL << 31));
    hipLaunchKernelGGL(pixel_absmax_kernel, dim3((unsigned)tmr_cdiv(n, PA_PIX)), dim3(PA_PIX * PA_GRP), 0,
                       tmr_stream(stream), x, S, C, HW, out);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int tmr_scale_merge(const float *img_max, const float *unit_max, const int32_t *unit_image, int B,
                               int U, float *out_img, float *out_unit, void *stream) {
    TMR_REQUIRE(unit_max && unit_image && out_unit && B > 0 && U > 0 && B < (1 << 24));
    hipLaunchKernelGGL(scale_merge_kernel, dim3(B), dim3(256), 0, tmr_stream(stream), img_max, unit_max,
                       unit_image, U, out_img, out_unit);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

int64_t tmr_xpack_bytes(int S, int C, int H, int W, int ks, int prec) {
    if (S <= 0 || C <= 0 || H <= 0 || W <= 0 || !ks_ok(ks) || !prec_ok(prec)) return -1;
    return (int64_t)S * tmr_cdiv(C, CCH) * prec_halves(prec) * pad_h(H, ks) * pad_w(W, ks) * XREC;
}

// up = 0: records of x itself (the 4-wide plain pack); TMR_XPACK_UPSAMPLE /
// TMR_XPACK_ONES: of [up2x(x) or x; 1] straight from the SAM features
extern "C" int tmr_split_xpack(const float *x, int S, int C, int H, int W, int up, int ks, int prec,
                               const float *xmax, int xmax_per_sample, void *out, void *stream) {
    TMR_REQUIRE(x && out && S > 0 && C > 0 && H > 0 && W > 0 && ks_ok(ks) && prec_ok(prec));
    TMR_REQUIRE((up & ~(TMR_XPACK_UPSAMPLE | TMR_XPACK_ONES)) == 0);
    TMR_REQUIRE(prec == TMR_PREC_BF16 || xmax);
    TMR_REQUIRE(xmax_per_sample >= 0 && xmax_per_sample <= 2);
    if (up == 0) return xpack_launch<0>(x, S, C, H, W, 0, 0, H, W, ks, prec, xmax, xmax_per_sample, out, stream);
    const int ups = (up & TMR_XPACK_UPSAMPLE) ? 1 : 0, ones = (up & TMR_XPACK_ONES) ? 1 : 0;
    return xpack_launch<1>(x, S, C, H, W, ups, ones, ups ? 2 * H : H, ups ? 2 * W : W, ks, prec, xmax,
                           xmax_per_sample, out, stream);
}

extern "C" int tmr_split_xpack16(const void *x, int S, int C, int H, int W, int ks, int prec, void *out,
                                 void *stream) {
    TMR_REQUIRE(x && out && S > 0 && C > 0 && H > 0 && W > 0 && ks_ok(ks) && prec == TMR_PREC_BF16);
    TMR_REQUIRE(W % 8 == 0);
    constexpr int RPB = XPACK16_RPB;
    const int NCc = (int)tmr_cdiv(C, CCH), Hp = pad_h(H, ks), Wp = pad_w(W, ks);
    const int64_t nseg = (int64_t)S * NCc * tmr_cdiv(H, RPB) * tmr_cdiv(W, XSEG);
    const int64_t nbord = (int64_t)Hp * Wp - (int64_t)H * W;
    const dim3 g4((unsigned)(nseg + tmr_cdiv(nbord * S * NCc, 256)));
    hipLaunchKernelGGL((xpack4_kernel<TMR_PREC_BF16, __bf16, RPB>), g4, dim3(256), 0, tmr_stream(stream),
                       static_cast<const __bf16 *>(x), S, C, H, W, NCc, Hp, Wp, ks / 2, nseg, nbord, nullptr, 0,
                       static_cast<b8 *>(out));
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

int64_t tmr_acc_floats(int U, int N, int H, int W) {
    if (U <= 0 || N <= 0 || H <= 0 || W <= 0) return -1;
    return (int64_t)U * tmr_cdiv(N, BM) * BM * tmr_cdiv(H, TH) * TH * tmr_cdiv(W, TW) * TW;
}

int64_t tmr_wpack_bytes(int N, int C0, int C1, int ks, int prec) {
    if (N <= 0 || C0 < 0 || C1 < 0 || C0 + C1 <= 0 || !ks_ok(ks) || !prec_ok(prec)) return -1;
    return (int64_t)ks * ks * (tmr_cdiv(C0, CCH) + tmr_cdiv(C1, CCH)) * tmr_cdiv(N, BM) * BM *
           prec_wrec(prec);
}

extern "C" int tmr_split_wpack(const float *w, int N, int C0, int C1, int ks, int prec,
                               const float *wmax, void *out, void *stream) {
    TMR_REQUIRE(w && out && N > 0 && C0 >= 0 && C1 >= 0 && C0 + C1 > 0 && ks_ok(ks) && prec_ok(prec));
    TMR_REQUIRE(prec == TMR_PREC_BF16 || wmax);
    const int NC0 = (int)tmr_cdiv(C0, CCH), NC = NC0 + (int)tmr_cdiv(C1, CCH);
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

extern "C" int tmr_split_conv(const void *xp0, int C0, const int32_t *unit_image, const void *xp1, int C1, int U,
                              int H, int W, int ks, int prec, const void *wpack, const float *wmax, const float *xmax,
                              const float *bias, int N, int leaky, const float *headw, const float *acc_init,
                              float *out, int flags, void *stream) {
    TMR_REQUIRE(out);
    if (!headw)  // activations (or the raw tiled accumulator) to out
        return split_common(xp0, C0, unit_image, xp1, C1, U, H, W, ks, prec, wpack, wmax, xmax, bias, N, leaky,
                            acc_init, out, nullptr, nullptr, 0, flags, stream);
    TMR_REQUIRE(!(flags & TMR_SPLIT_TILED_OUT));  // the head partials of the fused epilogue to out
    return split_common(xp0, C0, unit_image, xp1, C1, U, H, W, ks, prec, wpack, wmax, xmax, bias, N, leaky, acc_init,
                        nullptr, headw, out, 1, flags, stream);
}
