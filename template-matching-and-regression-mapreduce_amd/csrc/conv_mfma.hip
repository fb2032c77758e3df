// Implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32), gfx950.
//
// Serves every conv on the path:
//   * the 1x1 input projection with the bilinear x2 upsample fused into the
//     operand load   (models/matching_net.py:50-51,56)
//   * Decoder_model 3x3 conv + LeakyReLU over the virtual concat [fp, f_TM]
//     (models/regression_head.py:7-8, matching_net.py:64,69,74), with the
//     1x1 ObjectnessHead / BboxesHead folded into the epilogue
//     (regression_head.py:31,50, matching_net.py:70,75)
//   * plain kxk / 1x1 convs for the module-level forwards.
//
// GEMM view (transposed so the 1x1 heads reduce in registers):
//   out^T[n][m] = sum_{tap,c} Wp[tap][c][n] * X[c][m + off(tap)]
//   n = output channel (A operand rows), m = pixel (B operand columns).
// Block tile: 128 channels x (8 rows x 32 cols) pixels, 8 waves (2n x 4m),
// each wave 64n x 64m = 2x2 MFMA tiles.  Per channel chunk the block stages
// the (8+ks-1)x(32+ks-1) input halo once in LDS and reuses it for all ks^2
// taps; the packed weight slab [tap][cc][128] is one contiguous read.
// LDS is double buffered with register staging (one barrier per chunk).
#include <algorithm>

#include "tmr_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BN = 128;
constexpr int TH = 8;
constexpr int TW = 32;
constexpr int NTHREADS = 512;
constexpr int NHEAD = 5;  // 4 ltrbs outputs + 1 objectness

__host__ __device__ constexpr int conv_cc(int ks) { return ks == 1 ? 32 : (ks == 3 ? 8 : 2); }

template <int KS>
struct Cfg {
    static constexpr int CC = conv_cc(KS);
    static constexpr int P = KS / 2;
    static constexpr int HR = TH + KS - 1;
    static constexpr int HC = TW + KS - 1;
    static constexpr int XS = CC * HR * HC;       // floats, one X buffer
    static constexpr int WS = KS * KS * CC * BN;  // floats, one W buffer
    static constexpr int WS4 = WS / 4;
    static constexpr int WREG = (WS4 + NTHREADS - 1) / NTHREADS;
    static constexpr int XREG = (XS + NTHREADS - 1) / NTHREADS;
    static constexpr int LDS_FLOATS = 2 * (XS + WS);
};

struct ConvArgs {
    const float *src0;
    const float *src1;
    const int32_t *unit_image;
    const float *wpack;
    const float *bias;
    const float *headw;
    const float *acc_init;  // [img][N][H][W] added to the accumulators (nullable)
    float *out;
    float *partials;
    int C0, C1, U, H, W, N, NT, nchunks, MTX, MT;
    int Hin, Win;  // src0 geometry when UPS
    int leaky;
};

template <int KS, bool UPS>
__device__ __forceinline__ float load_x(const ConvArgs &a, int img, int u, int gc, int y, int x) {
    if (gc >= a.C0 + a.C1 || y < 0 || y >= a.H || x < 0 || x >= a.W) return 0.0f;
    if (gc < a.C0) {
        if (UPS) {
            const float *pl = a.src0 + ((size_t)img * a.C0 + gc) * (size_t)a.Hin * a.Win;
            return up_value(pl, a.Hin, a.Win, y, x);
        }
        return a.src0[((size_t)img * a.C0 + gc) * (size_t)a.H * a.W + (size_t)y * a.W + x];
    }
    return a.src1[((size_t)u * a.C1 + (gc - a.C0)) * (size_t)a.H * a.W + (size_t)y * a.W + x];
}

// EPI: 0 = store act(out) to a.out [U,N,H,W]; 1 = fused heads -> a.partials
template <int KS, bool UPS, int EPI>
__global__ __launch_bounds__(NTHREADS, 2) void conv_mfma_kernel(ConvArgs a) {
    using C = Cfg<KS>;
    extern __shared__ float lds[];
    float *Xs = lds;                 // [2][XS]
    float *Ws = lds + 2 * C::XS;     // [2][WS]

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wn = wave & 1, wm = wave >> 1;
    const int l32 = lane & 31, kh = lane >> 5;

    // XCD-aware mapping: blocks b and b+8 share an XCD (round-robin dispatch),
    // so the NT channel tiles of one (unit, pixel tile) are placed on the same
    // XCD, back to back, and its input halo is fetched into that L2 once.
    const int bid = blockIdx.x;
    int nt, pos;
    if (((a.MT * a.U) & 7) == 0) {
        const int j = bid >> 3;
        nt = j % a.NT;
        pos = (j / a.NT) * 8 + (bid & 7);
    } else {
        nt = bid % a.NT;
        pos = bid / a.NT;
    }
    const int mt = pos % a.MT;
    const int u = pos / a.MT;
    const int y0 = (mt / a.MTX) * TH, x0 = (mt % a.MTX) * TW;
    const int img = a.unit_image ? a.unit_image[u] : u;

    const f32x4 *wsrc = reinterpret_cast<const f32x4 *>(a.wpack) + (size_t)nt * a.nchunks * C::WS4;

    f32x4 wreg[C::WREG];
    float xreg[C::XREG];

    auto gload = [&](int ch) {
        const f32x4 *ws = wsrc + (size_t)ch * C::WS4;
#pragma unroll
        for (int i = 0; i < C::WREG; ++i) {
            int e = tid + i * NTHREADS;
            if (C::WS4 % NTHREADS == 0 || e < C::WS4) wreg[i] = ws[e];
        }
#pragma unroll
        for (int i = 0; i < C::XREG; ++i) {
            int e = tid + i * NTHREADS;
            float v = 0.0f;
            if (C::XS % NTHREADS == 0 || e < C::XS) {
                int c = e / (C::HR * C::HC);
                int r = (e / C::HC) % C::HR;
                int col = e % C::HC;
                v = load_x<KS, UPS>(a, img, u, ch * C::CC + c, y0 - C::P + r, x0 - C::P + col);
            }
            xreg[i] = v;
        }
    };
    auto lstore = [&](int buf) {
        f32x4 *wd = reinterpret_cast<f32x4 *>(Ws + buf * C::WS);
#pragma unroll
        for (int i = 0; i < C::WREG; ++i) {
            int e = tid + i * NTHREADS;
            if (C::WS4 % NTHREADS == 0 || e < C::WS4) wd[e] = wreg[i];
        }
        float *xd = Xs + buf * C::XS;
#pragma unroll
        for (int i = 0; i < C::XREG; ++i) {
            int e = tid + i * NTHREADS;
            if (C::XS % NTHREADS == 0 || e < C::XS) xd[e] = xreg[i];
        }
    };

    f32x16 acc00 = {0}, acc01 = {0}, acc10 = {0}, acc11 = {0};
    if (a.acc_init) {
        const int HWp = a.H * a.W;
        const float *ai = a.acc_init + (size_t)img * a.N * HWp;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n0 = nt * BN + wn * 64 + (r & 3) + 8 * (r >> 2) + 4 * kh;
            const int ya = y0 + wm * 2, xa = x0 + l32;
            const bool xin = xa < a.W;
            auto ld = [&](int n, int y) -> float {
                return (n < a.N && y < a.H && xin) ? ai[(size_t)n * HWp + (size_t)y * a.W + xa] : 0.0f;
            };
            acc00[r] = ld(n0, ya);
            acc01[r] = ld(n0, ya + 1);
            acc10[r] = ld(n0 + 32, ya);
            acc11[r] = ld(n0 + 32, ya + 1);
        }
    }

    gload(0);
    lstore(0);
    __syncthreads();
    for (int ch = 0; ch < a.nchunks; ++ch) {
        const int buf = ch & 1;
        if (ch + 1 < a.nchunks) gload(ch + 1);
        const float *wb = Ws + buf * C::WS + wn * 64 + l32;
        const float *xb = Xs + buf * C::XS + (wm * 2) * C::HC + l32;
#pragma unroll
        for (int tap = 0; tap < KS * KS; ++tap) {
            const int dy = tap / KS, dx = tap % KS;
#pragma unroll
            for (int cp = 0; cp < C::CC / 2; ++cp) {
                const int c = 2 * cp + kh;
                const float *wr = wb + (tap * C::CC + c) * BN;
                const float *xr = xb + (c * C::HR + dy) * C::HC + dx;
                const float a0 = wr[0], a1 = wr[32];
                const float b0 = xr[0], b1 = xr[C::HC];
                acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc00, 0, 0, 0);
                acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc01, 0, 0, 0);
                acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc10, 0, 0, 0);
                acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc11, 0, 0, 0);
            }
        }
        if (ch + 1 < a.nchunks) lstore(buf ^ 1);
        __syncthreads();
    }

    // ---------------- epilogue ----------------
    const int HW = a.H * a.W;
    const int nbase = nt * BN + wn * 64;
    f32x16 accs[2][2] = {{acc00, acc01}, {acc10, acc11}};

    if (EPI == 0) {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
            const int y = y0 + wm * 2 + mi, x = x0 + l32;
            if (y >= a.H || x >= a.W) continue;
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int n = nbase + ni * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                    if (n >= a.N) continue;
                    float v = accs[ni][mi][r] + a.bias[n];
                    if (a.leaky) v = v >= 0.0f ? v : v * 0.01f;
                    a.out[((size_t)u * a.N + n) * HW + (size_t)y * a.W + x] = v;
                }
            }
        }
    } else {
        // stage this tile's head weights + bias (128 x 6 floats) in LDS so the
        // unrolled reduction does not hoist 192 global loads into registers
        float *hs = lds + 2048;  // [BN][8]: hw0..4, bias
        for (int e = tid; e < BN * 6; e += NTHREADS) {
            const int n = e / 6, q = e % 6, gn = nt * BN + n;
            hs[n * 8 + q] = q < NHEAD ? a.headw[(size_t)gn * NHEAD + q] : (gn < a.N ? a.bias[gn] : 0.0f);
        }
        __syncthreads();
        float s[2][NHEAD];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int j = 0; j < NHEAD; ++j) s[mi][j] = 0.0f;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int nl = wn * 64 + ni * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
                const f32x4 h4 = *reinterpret_cast<const f32x4 *>(hs + nl * 8);
                const float h5 = hs[nl * 8 + 4], bn = hs[nl * 8 + 5];
                const float hw[NHEAD] = {h4[0], h4[1], h4[2], h4[3], h5};
#pragma unroll
                for (int mi = 0; mi < 2; ++mi) {
                    float v = accs[ni][mi][r] + bn;
                    if (a.leaky) v = v >= 0.0f ? v : v * 0.01f;
#pragma unroll
                    for (int j = 0; j < NHEAD; ++j) s[mi][j] = fmaf(v, hw[j], s[mi][j]);
                }
            }
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int j = 0; j < NHEAD; ++j) s[mi][j] += __shfl_xor(s[mi][j], 32);
        // combine the two n-waves through LDS (main loop is done: reuse it)
        float *red = lds;  // [4 wm][2 mi][NHEAD][32]
        if (wn == 1 && kh == 0) {
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int j = 0; j < NHEAD; ++j) red[((wm * 2 + mi) * NHEAD + j) * 32 + l32] = s[mi][j];
        }
        __syncthreads();
        if (wn == 0 && kh == 0) {
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) {
                const int y = y0 + wm * 2 + mi, x = x0 + l32;
                if (y >= a.H || x >= a.W) continue;
#pragma unroll
                for (int j = 0; j < NHEAD; ++j) {
                    float v = s[mi][j] + red[((wm * 2 + mi) * NHEAD + j) * 32 + l32];
                    a.partials[(((size_t)nt * NHEAD + j) * a.U + u) * HW + (size_t)y * a.W + x] = v;
                }
            }
        }
    }
}

__global__ void conv_pack_kernel(const float *__restrict__ w, int N, int C, int ks, int cc,
                                 int nchunks, int64_t total, float *__restrict__ wp) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int n = (int)(i % BN);
    int64_t r = i / BN;
    int c = (int)(r % cc);
    r /= cc;
    int tap = (int)(r % (ks * ks));
    r /= (ks * ks);
    int ch = (int)(r % nchunks);
    int nt = (int)(r / nchunks);
    int gn = nt * BN + n, gc = ch * cc + c;
    float v = 0.0f;
    if (gn < N && gc < C) v = w[((size_t)gn * C + gc) * ks * ks + tap];
    wp[i] = v;
}

__global__ void heads_reduce_kernel(const float *__restrict__ part, int NT, int U, int HW,
                                    const float *__restrict__ hb, float *__restrict__ o,
                                    float *__restrict__ b) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)U * HW) return;
    int u = (int)(i / HW), p = (int)(i % HW);
    float s[NHEAD];
#pragma unroll
    for (int j = 0; j < NHEAD; ++j) s[j] = 0.0f;
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < NHEAD; ++j) s[j] += part[(((size_t)t * NHEAD + j) * U + u) * HW + p];
    o[i] = s[4] + hb[4];
    if (b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) b[((size_t)u * 4 + j) * HW + p] = s[j] + hb[j];
    }
}

// bilinear x2 (F.interpolate, align_corners=False), per element exactly
// up_value's fma form.  One block per 32 x 128 output tile of a plane: the
// tile's input window (18 rows x 66 columns, clamped like up_coord) is staged
// in LDS by coalesced loads, then every thread forms 4 consecutive outputs of
// one row from LDS and writes them as one float4 (W % 4 == 0) -- a flat
// one-thread-per-output kernel issued 16 gathered global loads per 4 outputs
// and ran at ~1.5 TB/s.  Grid: x = column tiles, y = row tiles, z = planes.
constexpr int UPT_R = 32, UPT_C = 128;                       // output tile (4 rows per thread)
constexpr int UPI_R = UPT_R / 2 + 2, UPI_C = UPT_C / 2 + 2;  // staged input window
__global__ __launch_bounds__(256) void upsample2x_kernel(const float *__restrict__ in, int Hin, int Win,
                                                         float *__restrict__ out) {
    __shared__ float win[UPI_R][UPI_C + 1];
    const int H = 2 * Hin, W = 2 * Win;
    const int X0 = blockIdx.x * UPT_C, Y0 = blockIdx.y * UPT_R;
    const size_t pc = blockIdx.z;
    const float *pl = in + pc * Hin * Win;
    const int rb = Y0 / 2 - 1, cb = X0 / 2 - 1;  // window origin (global input coords, may be -1)
    for (int e = threadIdx.x; e < UPI_R * UPI_C; e += 256) {
        const int rr = e / UPI_C, cc = e - rr * UPI_C;
        const int gy = min(max(rb + rr, 0), Hin - 1), gx = min(max(cb + cc, 0), Win - 1);
        win[rr][cc] = pl[(size_t)gy * Win + gx];
    }
    __syncthreads();
    const int x0 = X0 + 4 * ((int)threadIdx.x % (UPT_C / 4));
    if (x0 >= W) return;
    int xa[4], xb[4];
    float lx0[4], lx1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) up_coord(x0 + k, Win, xa[k], xb[k], lx0[k], lx1[k]);
#pragma unroll
    for (int rs = 0; rs < UPT_R; rs += 256 / (UPT_C / 4)) {
        const int y = Y0 + rs + (int)threadIdx.x / (UPT_C / 4);
        if (y >= H) break;
        int y0, y1;
        float ly0, ly1;
        up_coord(y, Hin, y0, y1, ly0, ly1);
        const float *r0 = win[y0 - rb], *r1 = win[y1 - rb];
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float a = r0[xa[k] - cb], b = r0[xb[k] - cb], c = r1[xa[k] - cb], d = r1[xb[k] - cb];
            const float top = fmaf(lx0[k], a, lx1[k] * b);
            const float bot = fmaf(lx0[k], c, lx1[k] * d);
            v[k] = fmaf(ly0, top, ly1 * bot);
        }
        float *op = out + pc * H * W + (size_t)y * W + x0;
        if ((W & 3) == 0) {
            *reinterpret_cast<float4 *>(op) = float4{v[0], v[1], v[2], v[3]};
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (x0 + k < W) op[k] = v[k];
        }
    }
}

static int launch_upsample2x(const float *in, int64_t BC, int Hin, int Win, float *out, hipStream_t s) {
    TMR_REQUIRE(4ll * Hin * Win < (1ll << 31));
    for (int64_t p0 = 0; p0 < BC; p0 += 65535) {  // grid z <= 65535 planes per launch
        const int64_t np = std::min<int64_t>(65535, BC - p0);
        const dim3 grid((unsigned)tmr_cdiv(2 * Win, UPT_C), (unsigned)tmr_cdiv(2 * Hin, UPT_R), (unsigned)np);
        hipLaunchKernelGGL(upsample2x_kernel, grid, dim3(256), 0, s, in + p0 * Hin * Win, Hin, Win,
                           out + p0 * 4 * Hin * Win);
        TMR_CHECK_LAUNCH();
    }
    return TMR_OK;
}

template <int KS, bool UPS, int EPI>
int launch_conv(const ConvArgs &a, hipStream_t s) {
    using C = Cfg<KS>;
    const size_t lds = (size_t)C::LDS_FLOATS * sizeof(float);
    static_assert(Cfg<KS>::LDS_FLOATS * 4 <= 160 * 1024, "LDS");
    auto kern = conv_mfma_kernel<KS, UPS, EPI>;
    if (lds > 64 * 1024) {
        if (hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds) != hipSuccess)
            return TMR_E_HIP;
    }
    int64_t blocks = (int64_t)a.NT * a.MT * a.U;
    if (blocks <= 0) return TMR_OK;
    TMR_REQUIRE(blocks < (1ll << 31));
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NTHREADS), lds, s, a);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

int conv_dispatch(ConvArgs a, int ks, bool ups, int epi, hipStream_t s) {
    a.NT = (int)tmr_cdiv(a.N, BN);
    a.nchunks = (int)tmr_cdiv(a.C0 + a.C1, conv_cc(ks));
    a.MTX = (int)tmr_cdiv(a.W, TW);
    a.MT = a.MTX * (int)tmr_cdiv(a.H, TH);
    if (ups) {
        if (ks != 1 || epi != 0) return TMR_E_UNSUPPORTED;
        return launch_conv<1, true, 0>(a, s);
    }
    switch (ks * 2 + epi) {
        case 2: return launch_conv<1, false, 0>(a, s);
        case 3: return launch_conv<1, false, 1>(a, s);
        case 6: return launch_conv<3, false, 0>(a, s);
        case 7: return launch_conv<3, false, 1>(a, s);
        case 10: return launch_conv<5, false, 0>(a, s);
        case 11: return launch_conv<5, false, 1>(a, s);
        case 14: return launch_conv<7, false, 0>(a, s);
        case 15: return launch_conv<7, false, 1>(a, s);
        default: return TMR_E_UNSUPPORTED;
    }
}

bool ks_ok(int ks) { return ks == 1 || ks == 3 || ks == 5 || ks == 7; }

}  // namespace

extern "C" int64_t tmr_conv_pack_size(int N, int C, int ks) {
    if (N <= 0 || C <= 0 || !ks_ok(ks)) return -1;
    int cc = conv_cc(ks);
    return tmr_cdiv(N, BN) * tmr_cdiv(C, cc) * ks * ks * cc * BN;
}

extern "C" int tmr_conv_pack(const float *w, int N, int C, int ks, float *wpack, void *stream) {
    TMR_REQUIRE(w && wpack && N > 0 && C > 0 && ks_ok(ks));
    int cc = conv_cc(ks);
    int nchunks = (int)tmr_cdiv(C, cc);
    int64_t total = tmr_conv_pack_size(N, C, ks);
    hipLaunchKernelGGL(conv_pack_kernel, dim3((unsigned)tmr_cdiv(total, 256)), dim3(256), 0,
                       tmr_stream(stream), w, N, C, ks, cc, nchunks, total, wpack);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int tmr_upsample2x(const float *feat, int BC, int Hin, int Win, float *out, void *stream) {
    TMR_REQUIRE(feat && out && BC > 0 && Hin > 0 && Win > 0);
    return launch_upsample2x(feat, BC, Hin, Win, out, tmr_stream(stream));
}

extern "C" int tmr_upsample_proj(const float *feat, int B, int Cin, int Hin, int Win, int upsample,
                                 const float *wpack, const float *bias, int N, float *fp,
                                 float *f0, void *stream) {
    TMR_REQUIRE(feat && wpack && bias && fp && B > 0 && Cin > 0 && Hin > 0 && Win > 0 && N > 0);
    hipStream_t s = tmr_stream(stream);
    ConvArgs a = {};
    a.src0 = feat;
    a.C0 = Cin;
    a.C1 = 0;
    a.U = B;
    a.H = upsample ? 2 * Hin : Hin;
    a.W = upsample ? 2 * Win : Win;
    a.Hin = Hin;
    a.Win = Win;
    a.wpack = wpack;
    a.bias = bias;
    a.N = N;
    a.out = fp;
    a.leaky = 0;
    int rc = conv_dispatch(a, 1, upsample != 0, 0, s);
    if (rc) return rc;
    if (f0) {
        if (upsample) {
            rc = launch_upsample2x(feat, (int64_t)B * Cin, Hin, Win, f0, s);
            if (rc) return rc;
        } else if (f0 != feat) {
            if (hipMemcpyAsync(f0, feat, sizeof(float) * (size_t)B * Cin * Hin * Win,
                               hipMemcpyDeviceToDevice, s) != hipSuccess)
                return TMR_E_HIP;
        }
    }
    return TMR_OK;
}

static int conv_common(const float *src0, int C0, const int32_t *unit_image, const float *src1,
                       int C1, int U, int H, int W, const float *wpack, const float *bias, int N,
                       int ks, int leaky, float *out, const float *headw, const float *acc_init,
                       float *partials, int epi, void *stream) {
    TMR_REQUIRE(wpack && bias && U > 0 && H > 0 && W > 0 && N > 0 && C0 >= 0 && C1 >= 0);
    TMR_REQUIRE(C0 + C1 > 0 && (C0 == 0 || src0) && (C1 == 0 || src1) && ks_ok(ks));
    ConvArgs a = {};
    a.src0 = src0;
    a.src1 = src1;
    a.unit_image = unit_image;
    a.C0 = C0;
    a.C1 = C1;
    a.U = U;
    a.H = H;
    a.W = W;
    a.wpack = wpack;
    a.bias = bias;
    a.N = N;
    a.out = out;
    a.headw = headw;
    a.acc_init = acc_init;
    a.partials = partials;
    a.leaky = leaky;
    return conv_dispatch(a, ks, false, epi, tmr_stream(stream));
}

extern "C" int tmr_conv_store(const float *src0, int C0, const int32_t *unit_image,
                              const float *src1, int C1, int U, int H, int W, const float *wpack,
                              const float *bias, int N, int ks, int leaky, float *out,
                              void *stream) {
    TMR_REQUIRE(out);
    return conv_common(src0, C0, unit_image, src1, C1, U, H, W, wpack, bias, N, ks, leaky, out,
                       nullptr, nullptr, nullptr, 0, stream);
}

extern "C" int tmr_conv_heads(const float *src0, int C0, const int32_t *unit_image,
                              const float *src1, int C1, int U, int H, int W, const float *wpack,
                              const float *bias, int N, int ks, int leaky, const float *headw,
                              const float *acc_init, float *partials, void *stream) {
    TMR_REQUIRE(headw && partials);
    return conv_common(src0, C0, unit_image, src1, C1, U, H, W, wpack, bias, N, ks, leaky,
                       nullptr, headw, acc_init, partials, 1, stream);
}

extern "C" int64_t tmr_heads_partials_size(int N, int U, int H, int W) {
    if (N <= 0 || U <= 0 || H <= 0 || W <= 0) return -1;
    return tmr_cdiv(N, 64) * NHEAD * (int64_t)U * H * W;  // enough for 64- and 128-wide tiles
}

extern "C" int tmr_heads_reduce(const float *partials, int N, int tile_n, int U, int H, int W,
                                const float *head_bias, float *o, float *b, void *stream) {
    TMR_REQUIRE(partials && head_bias && o && N > 0 && U > 0 && H > 0 && W > 0);
    TMR_REQUIRE(tile_n == 64 || tile_n == 128);
    int NT = (int)tmr_cdiv(N, tile_n);
    int64_t tot = (int64_t)U * H * W;
    hipLaunchKernelGGL(heads_reduce_kernel, dim3((unsigned)tmr_cdiv(tot, 256)), dim3(256), 0,
                       tmr_stream(stream), partials, NT, U, H * W, head_bias, o, b);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}
