// Winograd F(2x2,3x3) implicit-GEMM 3x3 convolution on fp32 MFMA
// (v_mfma_f32_32x32x2_f32), gfx950.  Same semantics and ABI role as the
// direct kernel in conv_mfma.hip (Decoder_model conv + LeakyReLU, optional
// fused 1x1 heads; models/regression_head.py:7-8,31,50,
// models/matching_net.py:63-75) with 16 multiplies per 2x2 output tile
// instead of 36.
//
//   V = B^T d B   (4x4 input tile, stride 2, pad 1)          per (c, tile)
//   U = G g G^T   (packed once by tmr_wino_pack)              per (n, c)
//   M_xi[n][tile] = sum_c U_xi[n][c] V_xi[c][tile]            16 GEMMs (xi = 4x4)
//   Y = A^T M A   (2x2 outputs)
//
// Block: 512 threads, 64 output channels x 64 tiles (8x32 output pixels).
// Waves: 2 (xi halves) x 2 (32 channels) x 2 (32 tiles); a wave owns 8 xi x
// 32x32 accumulators (128 VGPRs).  In the epilogue each wave applies its half
// of A^T M A, the halves meet in LDS, and bias, LeakyReLU and the head
// reduction run in registers.  Pipeline per 8-channel chunk k (one barrier):
// the U slab of chunk k+1 streams into LDS by LDS-DMA (the pack is the LDS
// image), the zero-padded raw input halo of chunk k+2 is loaded coalesced
// into registers, chunk k is computed, then each thread transforms one
// (c, tile) 4x4 window of raw(k+1) from LDS into its 16 V values and stores
// raw(k+2).  LDS images are [xi][k-half][row][4 k-steps] so a lane's A (or B)
// operands for the chunk's 4 MFMA k-steps are one ds_read_b128.  LDS: V, U
// and raw double buffered, 149 KB.
#include "tmr_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BN = 64;       // output channels per block
constexpr int CC = 8;        // input channels per chunk (4 k-steps of 2)
constexpr int TR = 4;        // tile rows per block
constexpr int TCOL = 16;     // tile cols per block
constexpr int NTILE = TR * TCOL;
constexpr int NTHREADS = 512;
constexpr int NHEAD = 5;
constexpr int VS = 16 * CC * NTILE;  // floats, one V buffer  [16][2][64][4]
constexpr int US = 16 * CC * BN;     // floats, one U buffer  [16][2][64][4]
constexpr int US4 = US / 4;
constexpr int UGLDS = US4 / NTHREADS;  // 4 LDS-DMA pieces (16 B/lane) per thread
constexpr int HR = 2 * TR + 2, HC = 2 * TCOL + 2;  // raw input halo rows / cols
constexpr int RS = CC * HR * HC;                   // floats, one raw buffer (2720)
constexpr int RREG = (RS + NTHREADS - 1) / NTHREADS;
constexpr int LDS_FLOATS = 2 * (VS + US + RS);
static_assert(CC * NTILE == NTHREADS, "one (c, tile) window per thread");
static_assert(US4 % NTHREADS == 0, "");
static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS");

typedef __attribute__((address_space(3))) void *lds_ptr_t;

struct WArgs {
    const float *src0;
    const float *src1;
    const int32_t *unit_image;
    const float *upack;
    const float *bias;
    const float *headw;
    const float *acc_init;
    float *out;
    float *partials;
    int C0, C1, U, H, W, N, NT, nchunks, TX, MT;
    int leaky;
};

// Row base of channel gc (clamped into range so the load is always legal);
// out-of-range channels / pixels are zeroed by the caller's mask, never by a
// branch around the load (a branch makes hipcc wait vmcnt(0) per element).
__device__ __forceinline__ const float *chan_base(const WArgs &a, int img, int u, int gc) {
    const int g = min(gc, a.C0 + a.C1 - 1);
    return g < a.C0 ? a.src0 + ((size_t)img * a.C0 + g) * (size_t)a.H * a.W
                    : a.src1 + ((size_t)u * a.C1 + (g - a.C0)) * (size_t)a.H * a.W;
}

template <int EPI>
__global__ __launch_bounds__(NTHREADS, 2) void conv_wino_kernel(WArgs a) {
    extern __shared__ float lds[];
    float *Vs = lds;                 // [2][16 xi][2 kh][64 tiles][4 ks]
    float *Us = lds + 2 * VS;        // [2][16 xi][2 kh][64 n][4 ks]
    float *Rs = lds + 2 * (VS + US);  // [2][CC][HR][HC] raw input halo (zero padded)

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wh = wave & 1, wn = (wave >> 1) & 1, wtl = wave >> 2;
    const int l32 = lane & 31, kh = lane >> 5;

    const int bid = blockIdx.x;
    int nt, pos;
    if (((a.MT * a.U) & 7) == 0) {  // XCD-aware: a pixel tile's channel tiles share one L2
        const int j = bid >> 3;
        nt = j % a.NT;
        pos = (j / a.NT) * 8 + (bid & 7);
    } else {
        nt = bid % a.NT;
        pos = bid / a.NT;
    }
    const int mt = pos % a.MT, u = pos / a.MT;
    const int ty0 = (mt / a.TX) * TR, tx0 = (mt % a.TX) * TCOL;
    const int img = a.unit_image ? a.unit_image[u] : u;

    // this thread's (c, tile) input window; c = 2*ks + kh inside the chunk.
    // The map makes each half-wave's 32 V stores ((tile*4 + ks) dwords into
    // the [kh][tile][ks] image) cover 8 tile residues x 4 ks = 32 banks.
    const int wks = (lane >> 3) & 3, wkh = wave >> 2;
    const int wt = (lane & 7) + 8 * ((wave & 3) * 2 + (lane >> 5));
    const int wc = 2 * wks + wkh;
    const int ctot = a.C0 + a.C1;
    const f32x4 *usrc = reinterpret_cast<const f32x4 *>(a.upack) + (size_t)nt * a.nchunks * US4;

    // raw halo elements this thread loads: chunk-invariant clamped offsets,
    // channel-in-chunk and in-image bits (loads are unconditional; the value
    // is zeroed on the way into LDS, never by a branch around the load)
    int roff[RREG], rch[RREG];
    uint32_t rok = 0;
#pragma unroll
    for (int k = 0; k < RREG; ++k) {
        const int e = tid + k * NTHREADS;
        const int c = e / (HR * HC), rr = (e / HC) % HR, col = e % HC;
        const int y = 2 * ty0 - 1 + rr, x = 2 * tx0 - 1 + col;
        const bool ok = e < RS && y >= 0 && y < a.H && x >= 0 && x < a.W;
        roff[k] = min(max(y, 0), a.H - 1) * a.W + min(max(x, 0), a.W - 1);
        rch[k] = e < RS ? c : 0;
        rok |= (ok ? 1u : 0u) << k;
    }
    float xreg[RREG];
    auto rload = [&](int ch) {
#pragma unroll
        for (int k = 0; k < RREG; ++k) xreg[k] = chan_base(a, img, u, ch * CC + rch[k])[roff[k]];
    };
    auto rstore = [&](int ch, int buf) {
        float *rd = Rs + buf * RS;
#pragma unroll
        for (int k = 0; k < RREG; ++k) {
            const int e = tid + k * NTHREADS;
            if (RS % NTHREADS == 0 || e < RS)
                rd[e] = (((rok >> k) & 1u) && ch * CC + rch[k] < ctot) ? xreg[k] : 0.0f;
        }
    };
    auto uload = [&](int ch, int buf) {  // LDS-DMA: the pack is the LDS image
        const f32x4 *us = usrc + (size_t)ch * US4;
        float *ud = Us + buf * US;
#pragma unroll
        for (int i = 0; i < UGLDS; ++i) {
            const int piece = wave + i * (NTHREADS / 64);  // 1 KB pieces, wave-uniform base
            __builtin_amdgcn_global_load_lds((const void *)(us + piece * 64 + lane),
                                             (lds_ptr_t)(ud + piece * 256), 16, 0, 0);
        }
    };
    // V = B^T d B of this thread's (c, tile) window, read from the raw image
    const int wrow = 2 * (wt >> 4), wcol = 2 * (wt & 15);
    auto transform = [&](int buf) {
        const float *rs = Rs + buf * RS + wc * (HR * HC) + wrow * HC + wcol;
        float d[16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float2 p0 = *reinterpret_cast<const float2 *>(rs + r * HC);
            const float2 p1 = *reinterpret_cast<const float2 *>(rs + r * HC + 2);
            d[r * 4 + 0] = p0.x; d[r * 4 + 1] = p0.y; d[r * 4 + 2] = p1.x; d[r * 4 + 3] = p1.y;
        }
        float t[16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            t[r * 4 + 0] = d[r * 4 + 0] - d[r * 4 + 2];
            t[r * 4 + 1] = d[r * 4 + 1] + d[r * 4 + 2];
            t[r * 4 + 2] = d[r * 4 + 2] - d[r * 4 + 1];
            t[r * 4 + 3] = d[r * 4 + 1] - d[r * 4 + 3];
        }
        float *vd = Vs + buf * VS + (wkh * NTILE + wt) * 4 + wks;
        constexpr int XS = 2 * NTILE * 4;  // floats per xi
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            vd[(0 * 4 + b) * XS] = t[0 * 4 + b] - t[2 * 4 + b];
            vd[(1 * 4 + b) * XS] = t[1 * 4 + b] + t[2 * 4 + b];
            vd[(2 * 4 + b) * XS] = t[2 * 4 + b] - t[1 * 4 + b];
            vd[(3 * 4 + b) * XS] = t[1 * 4 + b] - t[3 * 4 + b];
        }
    };

    f32x16 acc[8];
#pragma unroll
    for (int x = 0; x < 8; ++x)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[x][r] = 0.0f;

    const int nch = a.nchunks;
    // prologue: raw(0) + U(0) -> LDS; V(0) from raw(0), raw(1) -> LDS
    rload(0);
    uload(0, 0);
    rstore(0, 0);
    __syncthreads();
    transform(0);
    if (nch > 1) {
        rload(1);
        rstore(1, 1);
    }
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
        const int cb = ch & 1, nb = cb ^ 1;
        // ordinary loads first: hipcc drains vmcnt(0) before an ordinary load
        // issued while an LDS-DMA is in flight
        if (ch + 2 < nch) rload(ch + 2);
        if (ch + 1 < nch) uload(ch + 1, nb);   // Us[nb] was last read by compute(ch-1)
        const f32x4 *ub = reinterpret_cast<const f32x4 *>(Us + cb * US) + kh * 64 + wn * 32 + l32;
        const f32x4 *vb = reinterpret_cast<const f32x4 *>(Vs + cb * VS) + kh * 64 + wtl * 32 + l32;
#pragma unroll
        for (int x = 0; x < 8; ++x) {
            const int xi = wh * 8 + x;
            const f32x4 a4 = ub[xi * 128];
            const f32x4 b4 = vb[xi * 128];
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
                acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[ks], b4[ks], acc[x], 0, 0, 0);
        }
        if (ch + 1 < nch) transform(nb);       // raw(ch+1) landed before the last barrier
        if (ch + 2 < nch) rstore(ch + 2, cb);  // raw(ch) was consumed by the last transform
        __syncthreads();                       // also drains the U LDS-DMA (vmcnt(0))
    }

    // ---------------- epilogue ----------------
    // this wave's half of Y = A^T M A (rows alpha = 2wh, 2wh+1 of M)
    float y[16][4];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float s0[4], s1[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const float m0 = acc[b][r], m1 = acc[4 + b][r];  // alpha = 2wh, 2wh+1
            if (wh == 0) { s0[b] = m0 + m1; s1[b] = m1; }
            else { s0[b] = m0; s1[b] = -m0 - m1; }
        }
        y[r][0] = s0[0] + s0[1] + s0[2];
        y[r][1] = s0[1] - s0[2] - s0[3];
        y[r][2] = s1[0] + s1[1] + s1[2];
        y[r][3] = s1[1] - s1[2] - s1[3];
    }
    // wh = 1 hands its half to wh = 0 through LDS ([wn][wtl][r][p][lane])
    float *xch = lds;
    const int xbase = ((wn * 2 + wtl) * 64) * 64;
    if (wh == 1) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
#pragma unroll
            for (int p = 0; p < 4; ++p) xch[xbase + (r * 4 + p) * 64 + lane] = y[r][p];
    }
    __syncthreads();
    const int HW = a.H * a.W;
    const int tile = wtl * 32 + l32;
    const int py0 = 2 * (ty0 + (tile >> 4)), px0 = 2 * (tx0 + (tile & 15));
    const float *ai = a.acc_init ? a.acc_init + (size_t)img * a.N * HW : nullptr;
    float hs[4][NHEAD];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int j = 0; j < NHEAD; ++j) hs[p][j] = 0.0f;
    if (wh == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n = nt * BN + wn * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
            const bool nin = n < a.N;
            const float bn = nin ? a.bias[n] : 0.0f;
            float hw[NHEAD];
            if (EPI == 1) {
#pragma unroll
                for (int j = 0; j < NHEAD; ++j) hw[j] = a.headw[(size_t)n * NHEAD + j];
            }
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int py = py0 + (p >> 1), px = px0 + (p & 1);
                const bool pin = nin && py < a.H && px < a.W;
                float v = y[r][p] + xch[xbase + (r * 4 + p) * 64 + lane];
                if (ai && pin) v += ai[(size_t)n * HW + (size_t)py * a.W + px];
                v += bn;
                if (a.leaky) v = v >= 0.0f ? v : v * 0.01f;
                if (EPI == 0) {
                    if (pin) a.out[((size_t)u * a.N + n) * HW + (size_t)py * a.W + px] = v;
                } else {
#pragma unroll
                    for (int j = 0; j < NHEAD; ++j) hs[p][j] = fmaf(v, hw[j], hs[p][j]);
                }
            }
        }
    }
    if (EPI == 1) {
        // sum over the two k-halves of the lanes, then over the two n-waves
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int j = 0; j < NHEAD; ++j) hs[p][j] += __shfl_xor(hs[p][j], 32);
        __syncthreads();  // xch reads are done; reuse LDS
        float *red = lds;  // [2 wtl][4 p][NHEAD][32]
        if (wh == 0 && wn == 1 && kh == 0) {
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int j = 0; j < NHEAD; ++j) red[((wtl * 4 + p) * NHEAD + j) * 32 + l32] = hs[p][j];
        }
        __syncthreads();
        if (wh == 0 && wn == 0 && kh == 0) {
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int py = py0 + (p >> 1), px = px0 + (p & 1);
                if (py >= a.H || px >= a.W) continue;
#pragma unroll
                for (int j = 0; j < NHEAD; ++j) {
                    const float v = hs[p][j] + red[((wtl * 4 + p) * NHEAD + j) * 32 + l32];
                    a.partials[(((size_t)nt * NHEAD + j) * a.U + u) * HW + (size_t)py * a.W + px] = v;
                }
            }
        }
    }
}

// U = G g G^T for g = w[n][c] (3x3), packed [nt][chunk][xi][kh][n][ks] with
// chunk channel c = 2*ks + kh (the LDS image of conv_wino_kernel)
__global__ void wino_pack_kernel(const float *__restrict__ w, int N, int C, int nchunks,
                                 int64_t total, float *__restrict__ up) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one (n, c) per thread
    if (i >= total) return;
    const int n = (int)(i % BN);
    int64_t r = i / BN;
    const int c = (int)(r % CC);
    r /= CC;
    const int ch = (int)(r % nchunks);
    const int nt = (int)(r / nchunks);
    const int gn = nt * BN + n, gc = ch * CC + c;
    float g[9];
    for (int q = 0; q < 9; ++q) g[q] = (gn < N && gc < C) ? w[((size_t)gn * C + gc) * 9 + q] : 0.0f;
    float tg[4][3];  // G g
    for (int q = 0; q < 3; ++q) {
        tg[0][q] = g[0 * 3 + q];
        tg[1][q] = 0.5f * ((g[0 * 3 + q] + g[1 * 3 + q]) + g[2 * 3 + q]);
        tg[2][q] = 0.5f * ((g[0 * 3 + q] - g[1 * 3 + q]) + g[2 * 3 + q]);
        tg[3][q] = g[2 * 3 + q];
    }
    float *dst = up + (((int64_t)nt * nchunks + ch) * 16) * CC * BN;
    const int kh = c & 1, ks = c >> 1;
    for (int al = 0; al < 4; ++al) {
        const float uv[4] = {tg[al][0], 0.5f * ((tg[al][0] + tg[al][1]) + tg[al][2]),
                             0.5f * ((tg[al][0] - tg[al][1]) + tg[al][2]), tg[al][2]};
        for (int be = 0; be < 4; ++be)
            dst[(((al * 4 + be) * 2 + kh) * BN + n) * 4 + ks] = uv[be];
    }
}

template <int EPI>
int launch_wino(WArgs a, hipStream_t s) {
    const size_t lds = (size_t)LDS_FLOATS * sizeof(float);
    auto kern = conv_wino_kernel<EPI>;
    if (hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
        return TMR_E_HIP;
    a.NT = (int)tmr_cdiv(a.N, BN);
    a.nchunks = (int)tmr_cdiv(a.C0 + a.C1, CC);
    a.TX = (int)tmr_cdiv(tmr_cdiv(a.W, 2), TCOL);
    a.MT = a.TX * (int)tmr_cdiv(tmr_cdiv(a.H, 2), TR);
    const int64_t blocks = (int64_t)a.NT * a.MT * a.U;
    if (blocks <= 0) return TMR_OK;
    TMR_REQUIRE(blocks < (1ll << 31));
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NTHREADS), lds, s, a);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

int wino_common(const float *src0, int C0, const int32_t *unit_image, const float *src1, int C1,
                int U, int H, int W, const float *upack, const float *bias, int N, int leaky,
                float *out, const float *headw, const float *acc_init, float *partials, int epi,
                void *stream) {
    TMR_REQUIRE(upack && bias && U > 0 && H > 0 && W > 0 && N > 0 && C0 >= 0 && C1 >= 0);
    TMR_REQUIRE(C0 + C1 > 0 && (C0 == 0 || src0) && (C1 == 0 || src1));
    WArgs a = {};
    a.src0 = src0;
    a.src1 = src1;
    a.unit_image = unit_image;
    a.upack = upack;
    a.bias = bias;
    a.headw = headw;
    a.acc_init = acc_init;
    a.out = out;
    a.partials = partials;
    a.C0 = C0;
    a.C1 = C1;
    a.U = U;
    a.H = H;
    a.W = W;
    a.N = N;
    a.leaky = leaky;
    hipStream_t s = tmr_stream(stream);
    return epi ? launch_wino<1>(a, s) : launch_wino<0>(a, s);
}

}  // namespace

extern "C" int64_t tmr_wino_pack_size(int N, int C) {
    if (N <= 0 || C <= 0) return -1;
    return tmr_cdiv(N, BN) * tmr_cdiv(C, CC) * 16 * CC * BN;
}

extern "C" int tmr_wino_pack(const float *w, int N, int C, float *upack, void *stream) {
    TMR_REQUIRE(w && upack && N > 0 && C > 0);
    const int nchunks = (int)tmr_cdiv(C, CC);
    const int64_t total = tmr_cdiv(N, BN) * nchunks * CC * BN;
    hipLaunchKernelGGL(wino_pack_kernel, dim3((unsigned)tmr_cdiv(total, 256)), dim3(256), 0,
                       tmr_stream(stream), w, N, C, nchunks, total, upack);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int tmr_wino_conv_store(const float *src0, int C0, const int32_t *unit_image,
                                   const float *src1, int C1, int U, int H, int W,
                                   const float *upack, const float *bias, int N, int leaky,
                                   const float *acc_init, float *out, void *stream) {
    TMR_REQUIRE(out);
    return wino_common(src0, C0, unit_image, src1, C1, U, H, W, upack, bias, N, leaky, out, nullptr,
                       acc_init, nullptr, 0, stream);
}

extern "C" int tmr_wino_conv_heads(const float *src0, int C0, const int32_t *unit_image,
                                   const float *src1, int C1, int U, int H, int W,
                                   const float *upack, const float *bias, int N, int leaky,
                                   const float *headw, const float *acc_init, float *partials,
                                   void *stream) {
    TMR_REQUIRE(headw && partials);
    return wino_common(src0, C0, unit_image, src1, C1, U, H, W, upack, bias, N, leaky, nullptr, headw,
                       acc_init, partials, 1, stream);
}
