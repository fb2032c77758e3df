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
// reduction run in registers.  Per 8-channel chunk each thread gathers one
// (c, tile) 4x4 input window (unconditional loads from clamped addresses,
// masked after), transforms it and writes its 16 V values to LDS; the U slab
// is one contiguous float4 copy.  LDS images are [xi][k-half][row][4 k-steps]
// so a lane's A (or B) operands for the chunk's 4 MFMA k-steps are one
// ds_read_b128.  Double-buffered LDS (128 KB), one barrier per chunk.
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
constexpr int UREG = US4 / NTHREADS;  // 4
static_assert(CC * NTILE == NTHREADS, "one (c, tile) window per thread");
static_assert(US4 % NTHREADS == 0, "");

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
    float *Vs = lds;            // [2][16 xi][2 kh][64 tiles][4 ks]
    float *Us = lds + 2 * VS;   // [2][16 xi][2 kh][64 n][4 ks]

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

    // this thread's (c, tile) input window; c = 2*ks + kh inside the chunk
    const int wc = tid >> 6, wt = tid & 63;
    const int wy = 2 * (ty0 + (wt >> 4)) - 1, wx = 2 * (tx0 + (wt & 15)) - 1;
    uint32_t vmask = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int y = wy + r, x = wx + s;
            vmask |= (y >= 0 && y < a.H && x >= 0 && x < a.W ? 1u : 0u) << (r * 4 + s);
        }
    const int yc0 = wy < 0 ? 0 : wy, xc0 = wx < 0 ? 0 : wx;

    const f32x4 *usrc = reinterpret_cast<const f32x4 *>(a.upack) + (size_t)nt * a.nchunks * US4;
    f32x4 ureg[UREG];
    float d[16];
    int chv = 0;

    auto gload = [&](int ch) {
        const f32x4 *us = usrc + (size_t)ch * US4;
#pragma unroll
        for (int i = 0; i < UREG; ++i) ureg[i] = us[tid + i * NTHREADS];
        chv = ch * CC + wc;
        const float *base = chan_base(a, img, u, chv);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int y = min(yc0 + (wy < 0 ? r - 1 : r), a.H - 1);
            const float *row = base + (size_t)(y < 0 ? 0 : y) * a.W;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int x = min(xc0 + (wx < 0 ? s - 1 : s), a.W - 1);
                d[r * 4 + s] = row[x < 0 ? 0 : x];
            }
        }
    };
    auto lstore = [&](int buf) {
        f32x4 *ud = reinterpret_cast<f32x4 *>(Us + buf * US);
#pragma unroll
        for (int i = 0; i < UREG; ++i) ud[tid + i * NTHREADS] = ureg[i];  // pack == LDS image
        // zero the padding / out-of-range channel, then V = B^T d B
        const uint32_t m = chv < a.C0 + a.C1 ? vmask : 0u;
#pragma unroll
        for (int q = 0; q < 16; ++q) d[q] = ((m >> q) & 1u) ? d[q] : 0.0f;
        float t[16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            t[r * 4 + 0] = d[r * 4 + 0] - d[r * 4 + 2];
            t[r * 4 + 1] = d[r * 4 + 1] + d[r * 4 + 2];
            t[r * 4 + 2] = d[r * 4 + 2] - d[r * 4 + 1];
            t[r * 4 + 3] = d[r * 4 + 1] - d[r * 4 + 3];
        }
        float *vd = Vs + buf * VS + ((wc & 1) * NTILE + wt) * 4 + (wc >> 1);
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

    gload(0);
    lstore(0);
    __syncthreads();
    for (int ch = 0; ch < a.nchunks; ++ch) {
        const int buf = ch & 1;
        if (ch + 1 < a.nchunks) gload(ch + 1);
        const f32x4 *ub = reinterpret_cast<const f32x4 *>(Us + buf * US) + kh * 64 + wn * 32 + l32;
        const f32x4 *vb = reinterpret_cast<const f32x4 *>(Vs + buf * VS) + kh * 64 + wtl * 32 + l32;
#pragma unroll
        for (int x = 0; x < 8; ++x) {
            const int xi = wh * 8 + x;
            const f32x4 a4 = ub[xi * 128];
            const f32x4 b4 = vb[xi * 128];
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
                acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4[ks], b4[ks], acc[x], 0, 0, 0);
        }
        if (ch + 1 < a.nchunks) lstore(buf ^ 1);
        __syncthreads();
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
    const size_t lds = (size_t)2 * (VS + US) * sizeof(float);
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
