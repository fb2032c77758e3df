// Depthwise cross-correlation of each unit's exemplar template with its
// image's projected features (gfx950, fp32 VALU), then the divide by the
// template area, the zero pad back to HxW and the learned scale:
//   models/template_matching.py:23-41 (cross_correlation), :97 (f * scale).
//
// Two kernels, same results: xcorr_rows_kernel (rows 16-B aligned, templates
// <= 31 wide: the engine's shapes) and xcorr_kernel (any shape).
//
// One workgroup per (band of RB output rows, channel, image): the band's
// input rows of the image's fp plane are staged once in LDS and reused by
// every exemplar unit of that image (the reference's per-exemplar forwards
// re-read it E times).  Each lane owns a 2x8 block of outputs and slides the
// template over register windows (compile-time template width, wave-uniform
// taps from SGPRs, v_pk_fma_f32 on output pairs).  Measured at config B
// (kbench_xcorr): 4x4 scalar 7.31 ms, 4x4 packed 7.47, 2x8 packed 7.37; at
// config E (k <= 31) 12.9 / 10.5 / 10.4 ms.  Not VALU-bound: without stores
// and border zeroing it is 5.4 ms (1.6 ms of packed FMA issue); taps staged
// in LDS instead of SGPRs: 9.1 ms.  xcorr_rows_kernel (aligned 16-B row
// stores, border in the tiles) then takes config B to 6.66 ms and k = 3 from
// 5.44 to 3.66 ms (k = 15: 10.7 -> 11.3, config E 10.4 -> 11.7: the border
// tiles' compute); staging loads batched 8 per thread before the LDS writes:
// k = 3 2.98 ms, k = 5 5.59 -> 3.58 ms, config B 6.53 ms.  (Whole-template
// taps preloaded for 3x3: no change; for 5x5 the 25 taps spill SGPRs.)  The
// divide by fl32(h*w) is correctly
// rounded (div_cr), bit-identical to the reference's `/ (h*w + 1e-14)`.
#include <algorithm>

#include "tmr_common.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256;
constexpr int RY = 2;  // output rows per lane
constexpr int RX = 8;  // output cols per lane
constexpr int XSLACK = 16;  // zeroed floats past the last LDS row (16-B row reads over-read)

struct XArgs {
    const float *f;
    const float *tmpl;
    const tmr_unit_t *units;
    const int32_t *img_units;  // [B+1] unit ranges per image (units sorted by image)
    const float *scale;
    float *out;
    float *relu_out;
    float *work;
    unsigned *out_absmax;  // nullable [U]: per-unit atomicMax of |out| (unit_max_*)
    int C, H, W, RB, squeeze, LR;  // LR = LDS rows allocated
    int HG;                          // rows kernel: max template height / 2
};

// Per-unit max |out| (the decoder's per-unit activation scale source,
// tmr_xcorr out_absmax[u]): after each unit a wave reduces its lanes' max
// and raises an LDS slot of the unit (UMAX slots, the image's first units;
// later ones go straight to the global max); the block then raises each
// used slot's global max once.  Slots are zeroed before the staging barrier.
constexpr int UMAX = 64;
__device__ __forceinline__ void unit_max_wave(float v, int ul, unsigned *slots, unsigned *gout) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) {
        if (ul < UMAX)
            atomicMax(slots + ul, __float_as_uint(v));
        else
            atomicMax(gout, __float_as_uint(v));
    }
}
__device__ __forceinline__ void unit_max_flush(const unsigned *slots, const tmr_unit_t *units, int u_beg, int nu,
                                               unsigned *gout) {
    __syncthreads();
    for (int i = threadIdx.x; i < min(nu, UMAX); i += blockDim.x) {
        const unsigned m = slots[i];
        if (m) atomicMax(gout + u_beg + i, m);
    }
}

// x / d correctly rounded (= the reference's IEEE `/ (h*w + 1e-14)` in fp32)
// from rd = RN(1/d): q = RN(x rd), then one fma residual step (Markstein).
// Checked bit-exact against true division on 4.2e8 normal-range x for every
// odd h, w <= 31 (oracle-free host check); 3 VALU ops instead of the ~10 of
// the v_div_scale/fmas/fixup sequence.
__device__ __forceinline__ float div_cr(float x, float d, float rd) {
    const float q = x * rd;
    const float r = fmaf(-q, d, x);
    return fmaf(r, rd, q);
}

// acc[r][q] += sum_{i<h, j<KW} X[r0 + r + i][x0 + q + j] * T[i][j] as
// v_pk_fma_f32 on output pairs (q, q+1) with the
// wave-uniform tap broadcast from an SGPR (op_sel), two outputs per VALU
// issue.  A tap at even j reads the row's even-aligned register pairs
// (x[j], x[j+1]); at odd j the odd pairs (x[j], x[j+1]) built once per row
// (one v_pk_mov_b32 each).
template <int KW>
__device__ __forceinline__ void corr_block_pk(const float *xs, int W, int x0, int r0,
                                              const float *__restrict__ tc, int h,
                                              float (&acc)[RY][RX]) {
    constexpr int NV = (KW + RX - 1 + 3) / 4;
    constexpr int NO = (KW >= 2 ? (KW - 2) / 2 : 0) + RX / 2;  // odd pairs (x[2m+1], x[2m+2]) used
    f32x2 pa[RY][RX / 2];
#pragma unroll
    for (int r = 0; r < RY; ++r)
#pragma unroll
        for (int q = 0; q < RX / 2; ++q) pa[r][q] = f32x2{acc[r][2 * q], acc[r][2 * q + 1]};
    for (int ii = 0; ii < RY + h - 1; ++ii) {
        const float4 *xr = reinterpret_cast<const float4 *>(xs + (r0 + ii) * W + x0);
        f32x2 xe[2 * NV], xo[NO];
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const float4 v4 = xr[j];
            xe[2 * j] = f32x2{v4.x, v4.y};
            xe[2 * j + 1] = f32x2{v4.z, v4.w};
        }
#pragma unroll
        for (int m = 0; m < NO; ++m) xo[m] = f32x2{xe[m].y, xe[m + 1].x};
#pragma unroll
        for (int r = 0; r < RY; ++r) {
            const int i = ii - r;
            if (i < 0 || i >= h) continue;  // wave-uniform
            const float *tr = tc + i * KW;
#pragma unroll
            for (int j = 0; j < KW; ++j) {
                const float t = tr[j];
                const f32x2 tt = {t, t};
#pragma unroll
                for (int q = 0; q < RX / 2; ++q) {
                    const f32x2 xv2 = (j & 1) ? xo[(j >> 1) + q] : xe[(j >> 1) + q];
                    pa[r][q] = __builtin_elementwise_fma(xv2, tt, pa[r][q]);
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RY; ++r)
#pragma unroll
        for (int q = 0; q < RX / 2; ++q) {
            acc[r][2 * q] = pa[r][q].x;
            acc[r][2 * q + 1] = pa[r][q].y;
        }
}

// generic width (templates wider than 31)
__device__ __forceinline__ void corr_block_any(const float *xs, int W, int x0, int r0,
                                               const float *__restrict__ tc, int h, int w,
                                               float (&acc)[RY][RX]) {
    for (int ii = 0; ii < RY + h - 1; ++ii) {
        const float *xr = xs + (r0 + ii) * W + x0;
        for (int r = 0; r < RY; ++r) {
            const int i = ii - r;
            if (i < 0 || i >= h) continue;
            for (int j = 0; j < w; ++j) {
                const float t = tc[i * w + j];
#pragma unroll
                for (int q = 0; q < RX; ++q) acc[r][q] = fmaf(xr[q + j], t, acc[r][q]);
            }
        }
    }
}

__device__ void corr_dispatch(int w, const float *xs, int W, int x0, int r0, const float *tc, int h,
                              float (&acc)[RY][RX]) {
    if (W & 3) {  // rows not 16-B aligned: scalar reads
        corr_block_any(xs, W, x0, r0, tc, h, w, acc);
        return;
    }
    switch (w) {
#define TMR_W(K) case K: corr_block_pk<K>(xs, W, x0, r0, tc, h, acc); break;
        TMR_W(1) TMR_W(3) TMR_W(5) TMR_W(7) TMR_W(9) TMR_W(11) TMR_W(13) TMR_W(15)
        TMR_W(17) TMR_W(19) TMR_W(21) TMR_W(23) TMR_W(25) TMR_W(27) TMR_W(29) TMR_W(31)
#undef TMR_W
        default: corr_block_any(xs, W, x0, r0, tc, h, w, acc); break;
    }
}

// tmpl / outp are passed as __restrict__ kernel arguments (not only in XArgs)
// so the compiler can prove the template reads unclobbered and use scalar
// loads (s_load_dwordx16 rows) for the wave-uniform taps.
__global__ __launch_bounds__(NT) void xcorr_kernel(XArgs a, const float *__restrict__ tmpl,
                                                  float *__restrict__ outp) {
    extern __shared__ __attribute__((aligned(16))) float xs[];
    const int band = blockIdx.x, c = blockIdx.y, img = blockIdx.z;
    const int H = a.H, W = a.W;
    // wave-uniform unit range and descriptors (SGPRs): the template taps then
    // come in by scalar loads and feed the FMAs as scalar operands
    const int u_beg = __builtin_amdgcn_readfirstlane(a.img_units[img]);
    const int u_end = __builtin_amdgcn_readfirstlane(a.img_units[img + 1]);
    if (u_beg >= u_end) return;
    const int yb0 = band * a.RB, yb1 = min(yb0 + a.RB, H);
    // input rows needed by any unit of this image: [yb0 - hmax/2, yb1 + hmax/2)
    int hmax = 1;
    for (int u = u_beg; u < u_end; ++u) hmax = max(hmax, __builtin_amdgcn_readfirstlane(a.units[u].ht));
    const int rlo = max(yb0 - hmax / 2, 0), rhi = min(yb1 + hmax / 2, H);
    const float *__restrict__ fc = a.f + ((size_t)img * a.C + c) * H * W;
    const int nld = (rhi - rlo) * W;
    if ((W & 3) == 0) {  // 16-B staging loads (rows are 16-B aligned)
        const float4 *src4 = reinterpret_cast<const float4 *>(fc + (size_t)rlo * W);
        float4 *dst4 = reinterpret_cast<float4 *>(xs);
        for (int e = threadIdx.x; e < nld / 4; e += NT) dst4[e] = src4[e];
    } else
        for (int e = threadIdx.x; e < nld; e += NT) xs[e] = fc[(size_t)rlo * W + e];
    // zero the slack rows/cols the 4x4 register blocks may over-read
    for (int e = nld + threadIdx.x; e < a.LR * W + XSLACK; e += NT) xs[e] = 0.0f;
    unsigned *slots = reinterpret_cast<unsigned *>(xs + a.LR * W + XSLACK);
    const bool umax = a.out_absmax && !a.squeeze;
    if (threadIdx.x < UMAX) slots[threadIdx.x] = 0u;
    __syncthreads();

    const size_t plane = (size_t)H * W;
    for (int u = u_beg; u < u_end; ++u) {
        float vmax = 0.0f;
        const tmr_unit_t &un = a.units[u];
        const int h = __builtin_amdgcn_readfirstlane(un.ht), w = __builtin_amdgcn_readfirstlane(un.wt);
        const int uo = u;  // output plane
        const int64_t toff = ((int64_t)__builtin_amdgcn_readfirstlane((int)(un.tmpl_offset >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)un.tmpl_offset);
        const int ph = h / 2, pw = w / 2;
        const int Ho = H - h + 1, Wo = W - w + 1;
        const int ya = max(yb0, ph), yz = min(yb1, ph + Ho);  // valid output rows in band
        const int nv = max(yz - ya, 0);
        const float sc = a.squeeze ? 1.0f : *a.scale;
        const float denom = (float)(h * w);
        const float rden = 1.0f / denom;  // correctly rounded reciprocal
        float *op = a.squeeze ? a.work + ((size_t)uo * a.C + c) * plane
                              : outp + ((size_t)uo * a.C + c) * plane;
        float *rp = (a.relu_out && !a.squeeze) ? a.relu_out + ((size_t)uo * a.C + c) * plane : nullptr;
        if (!a.squeeze) {  // zero border of this band ((yo, xo) stepped, no per-element division)
            int yo = yb0 + (int)threadIdx.x / W, xo = (int)threadIdx.x % W;
            const int sy = NT / W, sx = NT % W;
            for (; yo < yb1;) {
                if (!(yo >= ya && yo < yz && xo >= pw && xo < pw + Wo)) {
                    op[(size_t)yo * W + xo] = 0.0f;
                    if (rp) rp[(size_t)yo * W + xo] = 0.0f;
                }
                yo += sy;
                xo += sx;
                if (xo >= W) { xo -= W; ++yo; }
            }
        }
        const float *__restrict__ tc = tmpl + toff + (size_t)c * h * w;
        // x blocks per row group padded to a multiple of 16: a 16-lane group of
        // a ds_read_b128 never straddles two row groups (bank conflicts)
        const int nbx = ((Wo + RX - 1) / RX + 15) / 16 * 16, nby = (nv + RY - 1) / RY;
        const int nbx_v = (Wo + RX - 1) / RX;
        // LDS row of conv row (ya - ph): ya - ph - rlo
        const int rbase = ya - ph - rlo;
        for (int task = threadIdx.x; task < nbx * nby; task += NT) {
            const int x0 = (task % nbx) * RX, r0 = (task / nbx) * RY;
            if (task % nbx >= nbx_v) continue;
            float acc[RY][RX];
#pragma unroll
            for (int r = 0; r < RY; ++r)
#pragma unroll
                for (int q = 0; q < RX; ++q) acc[r][q] = 0.0f;
            corr_dispatch(w, xs, W, x0, rbase + r0, tc, h, acc);
#pragma unroll
            for (int r = 0; r < RY; ++r) {
                if (r0 + r >= nv) break;
#pragma unroll
                for (int q = 0; q < RX; ++q) {
                    if (x0 + q >= Wo) break;
                    const size_t o = (size_t)(ya + r0 + r) * W + x0 + q + pw;
                    const float v = div_cr(acc[r][q], denom, rden) * sc;
                    op[o] = v;
                    vmax = fmaxf(vmax, fabsf(v));
                    if (rp) rp[o] = v > 0.0f ? v : 0.0f;
                }
            }
        }
        if (umax) unit_max_wave(vmax, u - u_beg, slots, a.out_absmax + uo);
    }
    if (umax) unit_max_flush(slots, a.units, u_beg, u_end - u_beg, a.out_absmax);
}

// ---------------------------------------------------------------------------
// Row-tiled variant (W % 4 == 0, templates up to 31 wide): lane tiles cover
// the WHOLE output band, zero border included, in 4x4 tiles aligned to the
// output columns, so every output row leaves as one 16-B store per lane (a
// wave writes 1 KB contiguous) and no separate border pass exists.  The band
// is staged with zero pads (PADL columns left, PADR right, zero rows above
// and below the image), so a tile's input window is always in range; border
// outputs are computed from the pads and masked to 0.  The window of output
// columns c0..c0+3 starts at input column c0 - KW/2, whose misalignment
// OFF = (-(KW/2)) mod 4 is a compile-time constant of the width
// specialisation: reads are aligned b128, pairs are picked at compile time.
constexpr int PADL = 20;  // >= 15 + 3 (max half-width + OFF), multiple of 4
constexpr int PADR = 24;  // covers the window over-read past column W
constexpr int TRY = 4;  // max tile rows (the LDS slack rows cover it)
// rows kernel FMA form per template width: scalar v_fma_f32 up to this width
// (no odd pairs to build; measured k = 3 1.79 vs 2.02 ms, k = 5 2.58 vs 2.65),
// v_pk_fma_f32 on column pairs above it (k = 15 7.97 vs 10.81 ms; profiles/archive/r02s_*)
constexpr int XCORR_SCALAR_MAXW = 5;

// (a.y, b.x) as ONE v_pk_mov_b32 (left to itself the compiler often builds
// the odd pair with two v_mov_b32)
__device__ __forceinline__ f32x2 odd_pair(f32x2 a, f32x2 b) {
    f32x2 r;
    asm("v_pk_mov_b32 %0, %1, %2 op_sel:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int KW, int TRY, int TRX>
__device__ __forceinline__ void corr_tile(const float *xs, int WS, int lrow0, int lcol0,
                                          const float *__restrict__ tc, int h,
                                          f32x2 (&pa)[TRY][TRX / 2]) {
    constexpr int OFF = (4 - ((KW / 2) & 3)) & 3;
    constexpr int NV = (OFF + KW + TRX + 3) / 4;   // b128 reads per row (+1 float for odd pairs)
    constexpr int NO = (OFF + KW + TRX - 2) / 2;   // odd pairs (x[2m+1], x[2m+2])
    for (int ii = 0; ii < TRY + h - 1; ++ii) {
        const f32x4 *xr = reinterpret_cast<const f32x4 *>(xs + (lrow0 + ii) * WS + lcol0);
        f32x2 xe[2 * NV];
        f32x4 v4[NV];
#pragma unroll
        for (int j = 0; j < NV; ++j) v4[j] = xr[j];
        // Pin every window vector whole in 4 consecutive VGPRs: left alone,
        // the compiler narrows the partly used vectors into ds_read2_b32 /
        // ds_read2_b64 of the odd-aligned pairs (4- / 2-way bank conflicts
        // at a 16-B lane stride, and ~1 v_mov per FMA to rebuild the even
        // pairs) -- the xcorr kernel's SQ_LDS_BANK_CONFLICT of round 1.
#pragma unroll
        for (int j = 0; j < NV; ++j) asm volatile("" : "+v"(v4[j]));
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            xe[2 * j] = f32x2{v4[j].x, v4[j].y};
            xe[2 * j + 1] = f32x2{v4[j].z, v4[j].w};
        }
        if constexpr (KW <= XCORR_SCALAR_MAXW) {
        // scalar v_fma_f32 on the even-pair registers' halves: no odd pairs
#pragma unroll
        for (int r = 0; r < TRY; ++r) {
            const int i = ii - r;
            if (i < 0 || i >= h) continue;  // wave-uniform
            const float *tr = tc + i * KW;
#pragma unroll
            for (int j = 0; j < KW; ++j) {
                const float t = tr[j];
#pragma unroll
                for (int q = 0; q < TRX; ++q) {
                    const int s0 = q + j + OFF;
                    const float xv = (s0 & 1) ? xe[s0 >> 1].y : xe[s0 >> 1].x;
                    if (q & 1)
                        pa[r][q >> 1].y = fmaf(xv, t, pa[r][q >> 1].y);
                    else
                        pa[r][q >> 1].x = fmaf(xv, t, pa[r][q >> 1].x);
                }
            }
        }
        } else {
        f32x2 xo[NO];
#pragma unroll
        for (int m = 0; m < NO; ++m) xo[m] = odd_pair(xe[m], xe[m + 1]);
#pragma unroll
        for (int r = 0; r < TRY; ++r) {
            const int i = ii - r;
            if (i < 0 || i >= h) continue;  // wave-uniform
            const float *tr = tc + i * KW;
#pragma unroll
            for (int j = 0; j < KW; ++j) {
                const float t = tr[j];
                const f32x2 tt = {t, t};
#pragma unroll
                for (int q = 0; q < TRX / 2; ++q) {
                    const int s0 = 2 * q + j + OFF;  // compile-time after unrolling
                    const f32x2 xv2 = (s0 & 1) ? xo[s0 >> 1] : xe[s0 >> 1];
                    pa[r][q] = __builtin_elementwise_fma(xv2, tt, pa[r][q]);
                }
            }
        }
        }
    }
}

// One unit's band for the rows kernel in TY x TX lane tiles; width
// specialisations up to MAXW (the launch's widest template: a kernel without
// the 17..31 cases holds fewer scalar registers live and spills fewer).
template <int TY, int TX, int MAXW>
__device__ __forceinline__ void rows_unit(const float *xs, int WS, int W, int yb0, int yb1, int hg, int h,
                                          int w, int ph, int pw, int Ho, int Wo,
                                          const float *__restrict__ tc, float denom, float rden, float sc,
                                          float *op, float *rp, float &vmax) {
    const int nbx = W / TX, nby = (yb1 - yb0 + TY - 1) / TY;
    for (int task = threadIdx.x; task < nbx * nby; task += NT) {
        const int c0 = (task % nbx) * TX, y0 = yb0 + (task / nbx) * TY;
        f32x2 pa[TY][TX / 2];
#pragma unroll
        for (int r = 0; r < TY; ++r)
#pragma unroll
            for (int q = 0; q < TX / 2; ++q) pa[r][q] = f32x2{0.0f, 0.0f};
        const int lrow0 = y0 - yb0 + hg - ph;
        const int lcol0 = PADL + c0 - pw - ((4 - (pw & 3)) & 3);
        // tiles wholly in the border rows or columns only store zeros
        const bool live = y0 + TY > ph && y0 < ph + Ho && c0 + TX > pw && c0 < pw + Wo;
        if (live) switch (w) {
#define TMR_W(K) case K: if constexpr (K <= MAXW) corr_tile<K, TY, TX>(xs, WS, lrow0, lcol0, tc, h, pa); break;
            TMR_W(1) TMR_W(3) TMR_W(5) TMR_W(7) TMR_W(9) TMR_W(11) TMR_W(13) TMR_W(15)
            TMR_W(17) TMR_W(19) TMR_W(21) TMR_W(23) TMR_W(25) TMR_W(27) TMR_W(29) TMR_W(31)
#undef TMR_W
            default: break;  // even widths never reach this kernel (template sizes are odd)
        }
#pragma unroll
        for (int r = 0; r < TY; ++r) {
            const int y = y0 + r;
            if (y >= yb1) break;
            const bool vy = y >= ph && y < ph + Ho;
            float v[TX];
#pragma unroll
            for (int q = 0; q < TX; ++q) {
                const int cx = c0 + q;
                const float acc = (q & 1) ? pa[r][q >> 1].y : pa[r][q >> 1].x;
                v[q] = (vy && cx >= pw && cx < pw + Wo) ? div_cr(acc, denom, rden) * sc : 0.0f;
                vmax = fmaxf(vmax, fabsf(v[q]));
            }
            const size_t o = (size_t)y * W + c0;
#pragma unroll
            for (int q = 0; q < TX; q += 4) {
                *reinterpret_cast<float4 *>(op + o + q) = float4{v[q], v[q + 1], v[q + 2], v[q + 3]};
                if (rp)
                    *reinterpret_cast<float4 *>(rp + o + q) =
                        float4{fmaxf(v[q], 0.0f), fmaxf(v[q + 1], 0.0f), fmaxf(v[q + 2], 0.0f),
                               fmaxf(v[q + 3], 0.0f)};
            }
        }
    }
}

template <int MAXW>
__global__ __launch_bounds__(NT) void xcorr_rows_kernel(XArgs a, const float *__restrict__ tmpl,
                                                       float *__restrict__ outp,
                                                       const tmr_unit_t *__restrict__ units) {
    extern __shared__ __attribute__((aligned(16))) float xs[];
    const int band = blockIdx.x, c = blockIdx.y, img = blockIdx.z;
    const int H = a.H, W = a.W, WS = W + PADL + PADR;
    const int u_beg = __builtin_amdgcn_readfirstlane(a.img_units[img]);
    const int u_end = __builtin_amdgcn_readfirstlane(a.img_units[img + 1]);
    if (u_beg >= u_end) return;
    const int yb0 = band * a.RB, yb1 = min(yb0 + a.RB, H);
    const int hg = a.HG;  // half of the largest template height: LDS row 0 = image row yb0 - hg
    const float *__restrict__ fc = a.f + ((size_t)img * a.C + c) * H * W;
    const float sc = a.squeeze ? 1.0f : *a.scale;  // read once, before any store
    // stage rows [yb0 - hg, yb0 - hg + LR) with zero pads (rows outside the image: zeros)
    // SU loads per thread in flight before any LDS write (a load -> ds_write
    // loop waits out one global-load latency per element)
    constexpr int SU = 8;
    const int W4 = W / 4, WS4 = WS / 4, n4 = a.LR * WS4;
    float4 *xs4 = reinterpret_cast<float4 *>(xs);
    // e / WS4 as one fp32 multiply: exact for e < 2^16 (the quotient's
    // rounding error is < 2^-8 of the 0.5 / WS4 margin); the integer
    // division by a runtime divisor cost ~30 VALU per staged float4, which
    // dominated the instruction count at small templates (PMC: 7x the FMAs)
    const float rws4 = 1.0f / (float)WS4;
    for (int e0 = threadIdx.x; e0 < n4; e0 += NT * SU) {
        float4 v[SU];
#pragma unroll
        for (int k = 0; k < SU; ++k) {
            const int e = e0 + k * NT;
            const int lr = (int)(((float)e + 0.5f) * rws4), cc = e - lr * WS4 - PADL / 4;
            const int yy = yb0 - hg + lr;
            v[k] = float4{0.0f, 0.0f, 0.0f, 0.0f};
            if (e < n4 && yy >= 0 && yy < H && cc >= 0 && cc < W4)
                v[k] = reinterpret_cast<const float4 *>(fc + (size_t)yy * W)[cc];
        }
#pragma unroll
        for (int k = 0; k < SU; ++k)
            if (e0 + k * NT < n4) xs4[e0 + k * NT] = v[k];
    }
    unsigned *slots = reinterpret_cast<unsigned *>(xs + (size_t)a.LR * WS);
    const bool umax = a.out_absmax && !a.squeeze;
    if (threadIdx.x < UMAX) slots[threadIdx.x] = 0u;
    __syncthreads();

    const size_t plane = (size_t)H * W;
    for (int u = u_beg; u < u_end; ++u) {
        float vmax = 0.0f;
        const tmr_unit_t &un = units[u];  // restrict: scalar loads, no wait behind the stores
        const int h = __builtin_amdgcn_readfirstlane(un.ht), w = __builtin_amdgcn_readfirstlane(un.wt);
        const int uo = u;  // output plane
        const int64_t toff = ((int64_t)__builtin_amdgcn_readfirstlane((int)(un.tmpl_offset >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)un.tmpl_offset);
        const int ph = h / 2, pw = w / 2;
        const int Ho = H - h + 1, Wo = W - w + 1;
        const float denom = (float)(h * w);
        const float rden = 1.0f / denom;  // correctly rounded reciprocal
        float *op = a.squeeze ? a.work + ((size_t)uo * a.C + c) * plane
                              : outp + ((size_t)uo * a.C + c) * plane;
        float *rp = (a.relu_out && !a.squeeze) ? a.relu_out + ((size_t)uo * a.C + c) * plane : nullptr;
        const float *__restrict__ tc = tmpl + toff + (size_t)c * h * w;
        // 4x4 tiles: one 16-B store per lane row (1 KB per wave row).  2x8
        // tiles (twice the FMAs per scalar tap-row load) measured 5.1 vs 5.5
        // ms at k = 9 but 10.4 vs 7.4 at k = 11 and 16.4 vs 11.4 at k = 15.
        rows_unit<4, 4, MAXW>(xs, WS, W, yb0, yb1, hg, h, w, ph, pw, Ho, Wo, tc, denom, rden, sc, op, rp, vmax);
        if (umax) unit_max_wave(vmax, u - u_beg, slots, a.out_absmax + uo);
    }
    if (umax) unit_max_flush(slots, units, u_beg, u_end - u_beg, a.out_absmax);
}


// ---------------------------------------------------------------------------
// MFMA variant (kernel (2) of BASELINE north_star): the depthwise correlation
// as a 2-D Toeplitz GEMM on v_mfma_f32_16x16x32_{f16,bf16} with an fp32-grade
// 3-term split (the decoder's F16X3 scheme, conv_split.hip).
//
// Geometry (round 6).  M = 16 outputs of one PATCH, 2 output rows x 8 output
// columns (r, c); K = 32 inputs of one WINDOW, 4 input rows x 8 input columns
// (iy, ix); N = 16 patches.  For a patch at (y0, x0) and window (a, b):
//   A_ab[(r,c)][(iy,ix)] = T[4a + iy - r][8b + ix - c - s],  zero outside the template,
//   B_ab[(iy,ix)][n]     = F[y0(n) - ph + 4a + iy][x0(n) - pw - s + 8b + ix],
// summed over the windows a < ceil((h+1)/4), b < ceil((w+7+s)/8), where
// s = (-pw) mod 8 aligns every window's first column to 8 fp16 (16 bytes:
// each B chunk is one ds_read_b128).  A depends on the template and (a, b)
// only -- one pre-expanded 1-KB fragment per window and term
// (tmr_template_split), shared by every patch.  The K window is dense in the
// template's interior, so the useful share of each MFMA is
// h*w / (32 * windows): at k = 9 / 15 / 19 / 31, 0.28 / 0.59 / 0.45 / 0.75,
// against 0.28 / 0.47 / 0.30 / 0.48 of the round-5 row Toeplitz (one template
// row x 32 input columns per MFMA, 16 outputs of one row): the config-B mix
// (k 3..15) runs 10% fewer MFMAs, the config-E mix (k 3..31) 29% fewer.  The
// MFMA shape study (profiles/mfma_shapes, round 6: random operands, every
// 16-bit gfx950 form) found no shape with a better useful rate -- 16x16x16 /
// 32x32x8 run at 0.65 of 16x16x32's FLOP rate, the 4x4x4 and 16x16x4
// multi-block forms at 0.31 / 0.36; useful rate = useful share x rate per w in
// profiles/mfma_shapes/toeplitz_table.md) -- so the geometry, not the
// instruction, changed.  The one exception is the 4x4x4 16-block row form at
// w <= 5 (192 / 319 useful TFLOP/s vs 154 / 214), where this kernel is bound
// by its staging, epilogue and stores, not by MFMA issue (k = 3: the MFMA
// loop is ~1.1 of 2.9 ms, profiles/archive/r06/ablation).
//
// The 16 patches of one accumulator tile 4 output rows x 64 columns: patch n
// at (R + 2 (n >> 3), C0 + 8 (n & 7)).  Lane (n, g) of D holds output row
// R + 2 (n >> 3) + (g >> 1), columns C0 + 8 (n & 7) + 4 (g & 1) + 0..3: one
// 16-B store, 256 contiguous bytes per row per wave instruction.
//
// Both operands are split x*s_x = xh + xl (fp16, power-of-two scales: the
// staged band's max for F, the template's max for T) and every product is
// th*fh + th*fl + tl*fh with fp32 accumulation (dropped tl*fl and the split
// residuals ~2^-22 relative), then exactly unscaled, divided by fl32(h*w)
// correctly rounded and scaled like the VALU kernels.
//
// Measured (kbench_xcorr incl. tmr_template_split, one box): config-B mix
// 4.42 ms (round-5 row Toeplitz, 64-row bands) -> 4.19 (windows) -> 3.76
// (rolling band rows, mfma_unit); config E mix 15.0 -> 11.4 -> 9.66 ms; C
// 2.78 -> 2.72 -> 2.43 ms (profiles/r06_xcorr_window, r06_xcorr_rolling).
//
// Block = (band of BR output rows, channel, image), 4 waves; the band's input
// rows (+- the image's largest template half height, zero rows outside the
// image, zero columns left/right) are staged ONCE as fp16 hi/lo planes and
// reused by every exemplar unit of the image.  Wave w owns BR/16 row quads of
// the band, every 64-column group of them.  LDS rows: see band_stride (B
// reads conflict free).  The 1-D grid is remapped so each XCD runs a
// contiguous range of (band, channel, image) blocks: neighbouring bands' halo
// rows meet in that XCD's L2.
constexpr int MPADL = 16;   // zero fp16 columns left of the image (>= pw + s = 16 at most)
constexpr int MPADR = 24;   // zero fp16 columns right of the image (>= pw + 7)
constexpr int MAXV4 = 16;   // staged float4 per thread (LR * W <= 16384)
// The last window row block of a template reaches up to 3 rows past the
// h + 1 input rows of a 2-row patch (4 ceil((h + 1) / 4) >= h + 1); its A
// taps there are zero, but zero x (stale LDS bits) can be NaN, so the band
// stages WIN_OVER more (zero) rows below the halo.
constexpr int WIN_OVER = 3;

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef __bf16 b4 __attribute__((ext_vector_type(4)));

// Operand precision of the MFMA kernel (PM, the TMR_PREC_* codes):
// TMR_PREC_F16X3 the fp32-grade 3-term fp16 split (1e-5 contract);
// TMR_PREC_BF16 / TMR_PREC_F16 ONE 16-bit term, fp32 accumulation (the bf16
// path of config C, 1e-2 contract): the lo plane, the lo fragments and two
// of the three MFMAs drop out.
template <int PM> struct XOp {
    typedef _Float16 E;
    typedef h8 V8;
    typedef h4 V4;
    static constexpr bool SPLIT = PM == TMR_PREC_F16X3;
};
template <> struct XOp<TMR_PREC_BF16> {
    typedef __bf16 E;
    typedef b8 V8;
    typedef b4 V4;
    static constexpr bool SPLIT = false;
};
__device__ __forceinline__ f32x4 xmma(h8 a, h8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 xmma(b8 a, b8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

struct MArgs {
    int SB;     // LDS plane row stride in bytes (128 mod 256)
    int LR;     // staged rows: band rows + 2 * HG + WIN_OVER
    int HG;     // max template height / 2
    int BR;     // output rows per block (64 or 32)
    int nband;  // bands per channel plane
    int nlog;   // logical blocks = nband * C * B
};

__device__ __forceinline__ float pow2_scale(float m, int &e) {
    // s = 2^(14 - e') with m < 2^e' (max |x s| < 2^14); e = -log2(s); s is
    // clamped to [2^-63, 2^63] (a finite scale, whatever m is)
    if (!(m > 0.0f && m <= 3.0e38f)) { e = 0; return 1.0f; }
    int ex;
    frexpf(m, &ex);
    const int se = min(max(14 - ex, -63), 63);
    e = -se;
    return ldexpf(1.0f, se);
}

__device__ __forceinline__ float block_max(float v, float *red) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// Per (unit, channel) split of the exemplar templates for the MFMA kernel
// (tmr_template_split): t * 2^-et = th + tl (fp16) with 2^-et the power-of-two
// scale of the template's own max |t| (max |t| 2^-et < 2^14), written as the
// kernel's A fragments themselves: for window (a, b) and term (hi, lo), 64
// lanes x 16 B in lane order, lane (m, g) holding T[4a + g - (m >> 3)]
// [8b + q - (m & 7) - s], q = 0..7 (zero outside the template).  The
// kernel's A load is one aligned, contiguous 1-KB wave read per window and
// term.  One wave per (unit, channel).
constexpr int AFRAG = 64 * 16;  // bytes per (window, term) fragment

// Template split of the 3-term fragments: t 2^-e = th + tl with th rounded to
// TH_BITS significant bits (exact in fp16) and tl = fp16(t 2^-e - th), the
// correlation's counterpart of conv_split.hip's WH_BITS.  11 = the plain fp16
// hi/lo split (profiles/r04k: fewer hi bits measured no faster here).
constexpr int TH_BITS = 11;

__host__ __device__ inline int win_s(int w) { return (8 - ((w / 2) & 7)) & 7; }  // (-pw) mod 8
__host__ __device__ inline int win_na(int h) { return (h + 4) / 4; }                  // ceil((h + 1) / 4)
__host__ __device__ inline int win_nb(int w) { return (w + win_s(w) + 14) / 8; }     // ceil((w + 7 + s) / 8)
__host__ __device__ inline int win_count(int h, int w) { return win_na(h) * win_nb(w); }

__global__ __launch_bounds__(256) void template_split_kernel(const float *__restrict__ tmpl,
                                                             const tmr_unit_t *__restrict__ units, int U,
                                                             int C, int64_t total_rows, int bf, int lo_too,
                                                             char *__restrict__ frags,
                                                             int32_t *__restrict__ exps) {
    // the wave's template through LDS (coalesced global reads once; the
    // fragments' lane-shifted taps are then LDS reads)
    __shared__ float tsh[4][31 * 31];
    const int64_t wid = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (wid >= (int64_t)U * C) return;  // wave-uniform
    const int u = (int)(wid / C), c = (int)(wid % C);
    const tmr_unit_t un = units[u];
    const int h = un.ht, w = un.wt, hw = h * w;
    const float *tg = tmpl + un.tmpl_offset + (int64_t)c * hw;
    const bool staged = hw <= 31 * 31;  // larger templates (not MFMA shapes) read global memory
    float *ts = tsh[threadIdx.x >> 6];
    float m = 0.0f;
    for (int e = lane; e < hw; e += 64) {
        const float v = tg[e];
        if (staged) ts[e] = v;
        m = fmaxf(m, fabsf(v));
    }
    const float *t = staged ? ts : tg;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    int et;
    const float st = pow2_scale(m, et);
    const int na = win_na(h), nb = win_nb(w), s = win_s(w);
    const int mm = lane & 15, g = lane >> 4, r = mm >> 3, cc = mm & 7;
    char *dst = frags + ((int64_t)C * un.row_offset + (int64_t)c * na * nb) * 2 * AFRAG + lane * 16;
    for (int a = 0; a < na; ++a) {
        const int i = 4 * a + g - r;
        for (int b = 0; b < nb; ++b) {
            float x[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int j = 8 * b + q - cc - s;
                x[q] = (i >= 0 && i < h && j >= 0 && j < w) ? t[i * w + j] * st : 0.0f;
            }
            char *f = dst + (size_t)((b * na + a) * 2) * AFRAG;  // column-major: mfma_unit's order
            if (bf) {  // wave-uniform: bf16 hi (the one-term bf16 MFMA reads hi only)
                b8 hi;
#pragma unroll
                for (int q = 0; q < 8; ++q) hi[q] = (__bf16)x[q];
                *reinterpret_cast<b8 *>(f) = hi;
            } else {
                h8 hi, lo;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    // 3-term: sparse hi (TH_BITS); one-term f16 reads the plain fp16 hi
                    hi[q] = (lo_too && TH_BITS < 11) ? (_Float16)tmr_round_sig_bits(x[q], TH_BITS) : (_Float16)x[q];
                    lo[q] = (_Float16)(x[q] - (float)hi[q]);
                }
                *reinterpret_cast<h8 *>(f) = hi;
                if (lo_too) *reinterpret_cast<h8 *>(f + AFRAG) = lo;  // the 3-term kernel's tl
            }
        }
    }
    if (lane == 0) exps[(int64_t)u * C + c] = et;
}

// LDS row stride of a band W = 64 NCG columns wide (MPADL + W + MPADR fp16
// per row): the smallest stride >= the row that is 128 or 0 mod 256 bytes.
// The 16 lanes of a ds_read_b128 group read 16 B each from 4 rows (2 patch
// rows x 2 window rows), 4 lanes per row over 64 contiguous bytes; the rows
// fall on disjoint banks when odd rows sit 128 mod 256 bytes from even ones:
// by the stride itself (128 mod 256), or (0 mod 256) by XOR-ing bit 7 of the
// byte column of odd rows.  W 64 / 128 / 192 / 256: 256 (XOR) / 384 / 512
// (XOR) / 640 B.
__host__ __device__ constexpr int band_stride(int ncg) {
    const int bytes = 2 * (64 * ncg + MPADL + MPADR);
    const int a = (bytes + 127) / 256 * 256 + 128, b = (bytes + 255) / 256 * 256;
    return a < b ? a : b;
}
// XOR applied to the byte column of staged row lr: bit 7 of odd rows under a
// 0 mod 256 stride (the same for rows 4 apart: windows and row quads)
template <int SB>
__device__ __forceinline__ int band_swz(int lr) {
    if constexpr (SB % 256 == 0) return (lr & 1) ? 128 : 0;
    else return 0;
}
template <int SB>
__device__ __forceinline__ int lds_off(int lr, int col) {  // col % 4 == 0 (elements)
    return lr * SB + ((2 * col) ^ band_swz<SB>(lr));
}

// One unit over the wave's accumulators: acc[t] += sum over windows of
// A_ab B_ab(t).  Accumulator t = (row quad tq, 64-column group tc).  `rh` /
// `rl`: the hi / lo plane's staged row of this lane's B chunk at window row
// block a = 0, accumulator row quad 0; `cb`: the chunk's logical byte column
// at b = 0, accumulator column group 0 (16-B aligned); `swz`: the row's
// swizzle (rows move by 4 per window row block and row quad, so it is the
// same for all).  Each window's B chunks of every accumulator are loaded
// first (one ds_read_b128 per plane and accumulator, logical column
// cb + 16 b + 128 tc), then its MFMAs; the A fragments (hi and lo) are
// aligned 16-B lane loads of the pre-expanded fragments, issued PF windows
// ahead.
template <int NRQ, int NCG, int PM, int UA>
__device__ __forceinline__ void mfma_unit(f32x4 (&acc)[NRQ * NCG], const char *rh, const char *rl, int cb, int swz,
                                          int na, int nb, const char *arow) {
    // Windows are walked column by column (b outer, a inner).  Accumulator
    // row-quad tq at window row a reads band row-quad a + tq, so within a
    // column each staged chunk serves NRQ accumulators at NRQ consecutive
    // windows: the chunks live in a rolling set of NRQ row slots and a window
    // step reads ONE new row-quad per column group from LDS (NCG chunks per
    // plane instead of NRQ * NCG).  The a loop is unrolled by UA (a multiple
    // of NRQ, prefetch_windows) so every slot index is static; the A fragment
    // of slot j is prefetched UA windows ahead along the column, wrapping to
    // row j of the next column.
    typedef typename XOp<PM>::V8 V;
    constexpr bool SPLIT = XOp<PM>::SPLIT;
    constexpr int SB = band_stride(NCG);
    auto afrag = [&](int wi, int term) -> V {
        return *reinterpret_cast<const V *>(arow + (size_t)(wi * 2 + term) * AFRAG);
    };
    V ah[UA], al[UA];
    // (every prefetch loads SOME fragment of the unit -- a clamped index, not a
    // branch -- so the loads stay in flight across the window steps instead of
    // being waited for at a branch join)
    const int wlast = na * nb - 1;
#pragma unroll
    for (int j = 0; j < UA; ++j) {
        ah[j] = afrag(min(j, wlast), 0);
        if (SPLIT) al[j] = afrag(min(j, wlast), 1);
    }
    V xb[NRQ][NCG], xl[NRQ][NCG];
    auto load_row = [&](V (&hb)[NCG], V (&lb)[NCG], int row, int cw) {
#pragma unroll
        for (int tc = 0; tc < NCG; ++tc) {
            const int o = row * 4 * SB + ((cw + 128 * tc) ^ swz);
            hb[tc] = *reinterpret_cast<const V *>(rh + o);
            if (SPLIT) lb[tc] = *reinterpret_cast<const V *>(rl + o);
        }
    };
    for (int b = 0; b < nb; ++b) {
        const int cw = cb + 16 * b;
#pragma unroll
        for (int j = 0; j < NRQ - 1; ++j) load_row(xb[j], xl[j], j, cw);
        for (int a0 = 0; a0 < na; a0 += UA) {
#pragma unroll
            for (int j = 0; j < UA; ++j) {
                const int a = a0 + j;
                if (a >= na) break;
                load_row(xb[(j + NRQ - 1) % NRQ], xl[(j + NRQ - 1) % NRQ], a + NRQ - 1, cw);
#pragma unroll
                for (int tq = 0; tq < NRQ; ++tq)
#pragma unroll
                    for (int tc = 0; tc < NCG; ++tc) {
                        const int t = tq * NCG + tc;
                        const V &bh = xb[(j + tq) % NRQ][tc];
                        acc[t] = xmma(ah[j], bh, acc[t]);
                        if (SPLIT) {
                            acc[t] = xmma(ah[j], xl[(j + tq) % NRQ][tc], acc[t]);
                            acc[t] = xmma(al[j], bh, acc[t]);
                        }
                    }
                // the slot's next fragment (UA rows down, else row j of the next
                // column) lands in the registers just consumed: no copy at the
                // loop back edge, so nothing waits for it before its use
                const int wn = min(a + UA < na ? b * na + a + UA : (b + 1) * na + j, wlast);
                ah[j] = afrag(wn, 0);
                if (SPLIT) al[j] = afrag(wn, 1);
            }
        }
    }
}

// OB: f_TM leaves as bf16 (the bf16 contract's detect path: the decoder's
// bf16 records are bf16(f_TM) either way, so the fp32 plane is never needed;
// half the bytes written here and read by the record pack)
template <int NRQ, int NCG, int NV4, int PM, bool OB = false, int UA = 4>
__global__ __launch_bounds__(NT) void xcorr_mfma_kernel(XArgs a, MArgs m, const _Float16 *__restrict__ trows,
                                                       const int32_t *__restrict__ texp,
                                                       float *__restrict__ outp,
                                                       const tmr_unit_t *__restrict__ units) {
    typedef typename XOp<PM>::E E;
    typedef typename XOp<PM>::V4 V4;
    constexpr bool SPLIT = XOp<PM>::SPLIT;
    constexpr int NPL = SPLIT ? 2 : 1;  // staged planes (hi, lo)
    constexpr int NACC = NRQ * NCG;
    constexpr int SB = band_stride(NCG);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // XCD-aware map: hardware block L runs on XCD L % 8; give each XCD a
    // contiguous range of logical blocks (band fastest)
    const int L = blockIdx.x, per = gridDim.x >> 3;
    const int q = (L & 7) * per + (L >> 3);
    if (q >= m.nlog) return;
    const int band = q % m.nband, c = (q / m.nband) % a.C, img = q / (m.nband * a.C);
    const int H = a.H, W = a.W, LR = m.LR, hg = m.HG, BR = m.BR;
    const int u_beg = __builtin_amdgcn_readfirstlane(a.img_units[img]);
    const int u_end = __builtin_amdgcn_readfirstlane(a.img_units[img + 1]);
    if (u_beg >= u_end) return;
    char *Fh = smem, *Fl = smem + (size_t)LR * SB;  // Fl: F16X3 only
    float *red = reinterpret_cast<float *>(smem + NPL * (size_t)LR * SB);
    unsigned *slots = reinterpret_cast<unsigned *>(red + 16);  // [UMAX] per-unit max |out|
    const int tid = threadIdx.x;
    const bool umax = a.out_absmax && !a.squeeze;
    if (tid < UMAX) slots[tid] = 0u;  // (ordered before the uses by block_max's barriers)
    const int yb0 = band * BR, yb1 = min(yb0 + BR, H);
    const float *__restrict__ fc = a.f + ((size_t)img * a.C + c) * H * W;
    const float sc = a.squeeze ? 1.0f : *a.scale;

    // ---- stage the band: fp32 -> registers -> block max -> fp16 hi/lo planes.
    // Only the rows THIS image's units read (its own largest template's
    // halo, not the launch's) are staged and enter the scale, so a unit's
    // f_TM depends on its image and exemplars alone, never on the other
    // images of the batch (tests/test_gpu_precision.py: batch invariance)
    int hmax_img = 1;
    for (int u = u_beg; u < u_end; ++u) hmax_img = max(hmax_img, __builtin_amdgcn_readfirstlane(units[u].ht));
    const int ylo = yb0 - hmax_img / 2, yhi = yb1 + hmax_img / 2;
    const int W4 = W >> 2, n4 = LR * W4;
    const float rw4 = 1.0f / (float)W4;  // e / W4 by one multiply (exact for e < 2^16)
    float4 v[NV4];
    float vm = 0.0f;
#pragma unroll
    for (int k = 0; k < NV4; ++k) {
        const int e = tid + k * NT;
        v[k] = float4{0.0f, 0.0f, 0.0f, 0.0f};
        const int lr = (int)(((float)e + 0.5f) * rw4), cc = e - lr * W4;
        const int yy = yb0 - hg + lr;
        if (e < n4 && yy >= 0 && yy < H && yy >= ylo && yy < yhi)
            v[k] = reinterpret_cast<const float4 *>(fc + (size_t)yy * W)[cc];
        vm = fmaxf(vm, fmaxf(fmaxf(fabsf(v[k].x), fabsf(v[k].y)), fmaxf(fabsf(v[k].z), fabsf(v[k].w))));
    }
    // zero pad columns: [0, MPADL) and [MPADL + W, SB / 2) of every row, both
    // planes, in 16-B pieces
    {
        const int pr = SB / 16 - W / 8;   // 16-B pieces of pad per row (MPADL / 8 left, the rest right)
        const float rpr = 1.0f / (float)pr;
        for (int e = tid; e < NPL * LR * pr; e += NT) {
            const int pl = SPLIT ? e & 1 : 0, rr = SPLIT ? e >> 1 : e;
            const int r = (int)(((float)rr + 0.5f) * rpr), j = rr - r * pr;
            const int col = j < MPADL / 8 ? 8 * j : W + 8 * j;
            *reinterpret_cast<h8 *>((pl ? Fl : Fh) + lds_off<SB>(r, col)) = h8{};
        }
    }
    int ef;
    const float sf = pow2_scale(block_max(vm, red), ef);
#pragma unroll
    for (int k = 0; k < NV4; ++k) {
        const int e = tid + k * NT;
        if (e >= n4) break;
        const int lr = (int)(((float)e + 0.5f) * rw4), cc = e - lr * W4;
        const float x0 = v[k].x * sf, x1 = v[k].y * sf, x2 = v[k].z * sf, x3 = v[k].w * sf;
        const V4 hv = {(E)x0, (E)x1, (E)x2, (E)x3};
        const int off = lds_off<SB>(lr, MPADL + 4 * cc);
        *reinterpret_cast<V4 *>(Fh + off) = hv;
        if (SPLIT) {
            const V4 lv = {(E)(x0 - (float)hv[0]), (E)(x1 - (float)hv[1]), (E)(x2 - (float)hv[2]),
                           (E)(x3 - (float)hv[3])};
            *reinterpret_cast<V4 *>(Fl + off) = lv;
        }
    }
    __syncthreads();

    const int lane = tid & 63, wave = tid >> 6, n = lane & 15, g = lane >> 4;
    const int pr = n >> 3, pc = n & 7;
    const int rq0 = wave * 4 * NRQ;  // the wave's first output row in the band (NRQ quads of 4 rows)
    const size_t plane = (size_t)H * W;
    for (int u = u_beg; u < u_end; ++u) {
        float vmax = 0.0f;
        const tmr_unit_t &un = units[u];
        const int h = __builtin_amdgcn_readfirstlane(un.ht), w = __builtin_amdgcn_readfirstlane(un.wt);
        const int uo = u;  // output plane (texp row)
        const int roff = __builtin_amdgcn_readfirstlane(un.row_offset);
        const int et = __builtin_amdgcn_readfirstlane(texp[(size_t)uo * a.C + c]);
        const int ph = h / 2, pw = w / 2, Ho = H - h + 1, Wo = W - w + 1;
        const int na = win_na(h), nb = win_nb(w), s = win_s(w);
        f32x4 acc[NACC];
#pragma unroll
        for (int t = 0; t < NACC; ++t) acc[t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        if (yb0 + rq0 < yb1) {
            // staged row / column of this lane's B chunk at window (0, 0), accumulator 0
            const int rbase = rq0 + 2 * pr + g + hg - ph;
            const int cbase = 8 * pc + MPADL - pw - s;
            const char *arow = reinterpret_cast<const char *>(trows) +
                               ((int64_t)a.C * roff + (int64_t)c * na * nb) * 2 * AFRAG + lane * 16;
            mfma_unit<NRQ, NCG, PM, UA>(acc, Fh + rbase * SB, Fl + rbase * SB, 2 * cbase, band_swz<SB>(rbase), na, nb,
                                    arow);
        }
        // ---- epilogue: exact unscale, correctly rounded /(h*w), scale, pad mask
        const float inv = ldexpf(1.0f, ef + et);  // 1 / (sf * st)
        const float denom = (float)(h * w);
        const float rden = 1.0f / denom;
        float *op = a.squeeze ? a.work + ((size_t)uo * a.C + c) * plane
                    : OB ? reinterpret_cast<float *>(reinterpret_cast<__bf16 *>(outp) + ((size_t)uo * a.C + c) * plane)
                         : outp + ((size_t)uo * a.C + c) * plane;
        float *rp = (a.relu_out && !a.squeeze) ? a.relu_out + ((size_t)uo * a.C + c) * plane : nullptr;
        // the pad mask without exec-mask blocks: a lane's column validity per
        // (column group, element) once per unit, its row validity once per row
        // quad; every element is computed and a pad element selected to 0
        bool cv[NCG][4];
#pragma unroll
        for (int tc = 0; tc < NCG; ++tc)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int xx = 64 * tc + 8 * pc + 4 * (g & 1) + j;
                cv[tc][j] = xx >= pw && xx < pw + Wo;
            }
#pragma unroll
        for (int tq = 0; tq < NRQ; ++tq) {
            const int y = yb0 + rq0 + 4 * tq + 2 * pr + (g >> 1);
            if (y >= yb1) continue;
            const bool vy = y >= ph && y < ph + Ho;
#pragma unroll
            for (int tc = 0; tc < NCG; ++tc) {
                const int t = tq * NCG + tc;
                const int x = 64 * tc + 8 * pc + 4 * (g & 1);
                float r4[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float v = div_cr(acc[t][j] * inv, denom, rden) * sc;
                    r4[j] = (vy && cv[tc][j]) ? v : 0.0f;
                    vmax = fmaxf(vmax, fabsf(r4[j]));
                }
                if (OB) {
                    *reinterpret_cast<b4 *>(reinterpret_cast<__bf16 *>(op) + (size_t)y * W + x) =
                        b4{(__bf16)r4[0], (__bf16)r4[1], (__bf16)r4[2], (__bf16)r4[3]};
                    continue;
                }
                *reinterpret_cast<float4 *>(op + (size_t)y * W + x) = float4{r4[0], r4[1], r4[2], r4[3]};
                if (rp)
                    *reinterpret_cast<float4 *>(rp + (size_t)y * W + x) =
                        float4{fmaxf(r4[0], 0.0f), fmaxf(r4[1], 0.0f), fmaxf(r4[2], 0.0f), fmaxf(r4[3], 0.0f)};
            }
        }
        if (umax) unit_max_wave(vmax, u - u_beg, slots, a.out_absmax + uo);
    }
    if (umax) unit_max_flush(slots, units, u_beg, u_end - u_beg, a.out_absmax);
}

// squeeze (template_matching.py:34-35): sum over channels, pad, scale
__global__ void xcorr_squeeze_kernel(const float *__restrict__ work, const tmr_unit_t *__restrict__ units,
                                     int U, int C, int H, int W, const float *__restrict__ scale,
                                     float *__restrict__ out, float *__restrict__ relu_out,
                                     unsigned *__restrict__ out_absmax) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float v = 0.0f;
    if (i < (int64_t)U * H * W) {  // no early return: whole waves reach the max reduction
        const int u = (int)(i / ((int64_t)H * W));
        const int p = (int)(i % ((int64_t)H * W));
        const int y = p / W, x = p % W;
        const tmr_unit_t un = units[u];
        const int ph = un.ht / 2, pw = un.wt / 2, Ho = H - un.ht + 1, Wo = W - un.wt + 1;
        if (y >= ph && y < ph + Ho && x >= pw && x < pw + Wo) {
            const float *wp = work + (size_t)u * C * H * W + p;
            float s = 0.0f;
            for (int c = 0; c < C; ++c) s += wp[(size_t)c * H * W];
            v = s * *scale;
        }
        out[i] = v;
        if (relu_out) relu_out[i] = v > 0.0f ? v : 0.0f;
    }
    if (out_absmax) {  // per unit: a wave covers at most two units when H*W >= 64
        const int64_t tot = (int64_t)U * H * W;
        const int u = i < tot ? (int)(i / ((int64_t)H * W)) : -1;
        const int u0 = __builtin_amdgcn_readfirstlane(u);
        float m0 = u == u0 ? fabsf(v) : 0.0f, m1 = u != u0 ? fabsf(v) : 0.0f;
        for (int o = 32; o > 0; o >>= 1) {
            m0 = fmaxf(m0, __shfl_xor(m0, o));
            m1 = fmaxf(m1, __shfl_xor(m1, o));
        }
        const int u1 = __shfl(u, 63);
        if ((threadIdx.x & 63) == 0 && u0 >= 0) atomicMax(out_absmax + u0, __float_as_uint(m0));
        if ((int64_t)H * W >= 64) {
            if ((threadIdx.x & 63) == 0 && u1 >= 0 && u1 != u0) atomicMax(out_absmax + u1, __float_as_uint(m1));
        } else if (u >= 0 && u != u0) {
            atomicMax(out_absmax + u, __float_as_uint(fabsf(v)));
        }
    }
}

}  // namespace

// Crossover between the VALU kernels and the MFMA kernel (TMR_XCORR_AUTO):
// the MFMA kernel runs a launch when every unit's template is at least
// kMfmaMinK wide or tall (set from the rocprof counters) and
// the shape fits it (W % 32 == 0, W <= 256, templates <= 31).
static constexpr int kMfmaMinK = 1;

static bool mfma_fits(int H, int W, int max_ht, int max_wt) {
    if (W % 64 != 0 || W > 256 || max_ht > 31 || max_wt > 31 || H < 1) return false;
    const int LR = 32 + 2 * (max_ht / 2) + WIN_OVER;
    return (int64_t)LR * W <= (int64_t)MAXV4 * NT * 4;
}

// A-fragment prefetch distance (windows): 8 where the extra 16 (3-term) VGPRs
// keep the occupancy -- the 2-row-quad, 3-group 3-term kernel (config E's
// 32-row bands at 192 columns: 168 + 24 registers, 2 waves per SIMD either way
// once the LDS is counted): E mix 9.12 -> 8.73 ms, k = 31 13.72 -> 13.33
// (kbench_xcorr, one box, profiles/archive/r06/ua); elsewhere 4 (8 measured
// equal at B and C and 1.4x slower at E k = 7, whose kernel drops to one wave
// per SIMD).
template <int NRQ, int NCG, int PM>
constexpr int prefetch_windows() { return NRQ == 2 && NCG == 3 && PM == TMR_PREC_F16X3 ? 8 : 4; }

template <int NRQ, int NCG, int PM, bool OB>
static int launch_mfma_t(const XArgs &a, const MArgs &m, size_t lds, unsigned nblk, hipStream_t s,
                         const _Float16 *trows, const int32_t *texp) {
    constexpr int UA = prefetch_windows<NRQ, NCG, PM>();
    const void *kfn = (const void *)xcorr_mfma_kernel<NRQ, NCG, MAXV4, PM, OB, UA>;
    if (lds > 64 * 1024 && tmr_set_max_lds(kfn, lds) != hipSuccess) return TMR_E_HIP;
    hipLaunchKernelGGL((xcorr_mfma_kernel<NRQ, NCG, MAXV4, PM, OB, UA>), dim3(nblk), dim3(NT), lds, s, a, m, trows,
                       texp, a.out, a.units);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

template <int NRQ, int PM, bool OB = false>
static int launch_mfma_w(const XArgs &a, const MArgs &m, size_t lds, unsigned nblk, hipStream_t s,
                         const _Float16 *trows, const int32_t *texp) {
    switch (a.W / 64) {  // 64-column accumulator groups per row quad
        case 1: return launch_mfma_t<NRQ, 1, PM, OB>(a, m, lds, nblk, s, trows, texp);
        case 2: return launch_mfma_t<NRQ, 2, PM, OB>(a, m, lds, nblk, s, trows, texp);
        case 3: return launch_mfma_t<NRQ, 3, PM, OB>(a, m, lds, nblk, s, trows, texp);
        case 4: return launch_mfma_t<NRQ, 4, PM, OB>(a, m, lds, nblk, s, trows, texp);
        default: return TMR_E_UNSUPPORTED;
    }
}

template <int NRQ>
static int launch_mfma_p(const XArgs &a, const MArgs &m, size_t lds, unsigned nblk, hipStream_t s,
                         const _Float16 *trows, const int32_t *texp, int prec, bool out16) {
    if (out16)
        return prec == TMR_PREC_BF16 ? launch_mfma_w<NRQ, TMR_PREC_BF16, true>(a, m, lds, nblk, s, trows, texp)
                                     : TMR_E_UNSUPPORTED;
    switch (prec) {
        case TMR_PREC_F16X3: return launch_mfma_w<NRQ, TMR_PREC_F16X3>(a, m, lds, nblk, s, trows, texp);
        case TMR_PREC_BF16: return launch_mfma_w<NRQ, TMR_PREC_BF16>(a, m, lds, nblk, s, trows, texp);
        case TMR_PREC_F16: return launch_mfma_w<NRQ, TMR_PREC_F16>(a, m, lds, nblk, s, trows, texp);
        default: return TMR_E_INVALID;
    }
}

// Band height: 64 output rows (each wave 4 row quads) when the band and its
// halo fit the staging registers, else 32 (2 row quads per wave).  Round 6,
// row-Toeplitz kernel (kbench_xcorr, one box, two reps): 64-row bands took
// the config-B mix 4.77 / 4.75 -> 4.42 / 4.45 ms and config C 3.22 / 3.20 ->
// 2.80 / 2.77 ms -- half the bands, so half the A-fragment fetches and halo
// re-stages per output.  The window kernel adds the LDS rule: a 64-row band
// whose two planes exceed 78 KB leaves one block per CU -- config E at k = 15
// (192 columns) 6.77 ms at 64 rows vs 5.40 at 32; where two blocks fit, 64
// rows (E k = 3: 2.83 vs 3.13 ms; config C 2.49 vs 2.86; config B equal,
// profiles/archive/r06/brexp).
static int band_rows(int W, int max_ht, int prec) {
    const int64_t lr64 = 64 + 2 * (max_ht / 2) + WIN_OVER;
    const int64_t lds64 = (prec == TMR_PREC_F16X3 ? 2 : 1) * lr64 * band_stride(W / 64);
    // 64 rows where the band fits the staging registers and two blocks still fit a CU's LDS
    return lr64 * W <= (int64_t)MAXV4 * NT * 4 && lds64 <= 78 * 1024 ? 64 : 32;
}

static int launch_mfma(const XArgs &a, hipStream_t s, int B, int max_ht, const void *tmpl_split,
                       int64_t total_rows, int prec, bool out16) {
    MArgs m;
    m.BR = band_rows(a.W, max_ht, prec);
    m.HG = max_ht / 2;
    m.LR = m.BR + 2 * m.HG + WIN_OVER;
    m.SB = band_stride(a.W / 64);
    m.nband = (int)tmr_cdiv(a.H, m.BR);
    const int64_t nlog = (int64_t)m.nband * a.C * B;
    TMR_REQUIRE(nlog < (1LL << 31) - 8);
    m.nlog = (int)nlog;
    const size_t lds = (prec == TMR_PREC_F16X3 ? 2 : 1) * (size_t)m.LR * m.SB + 64 + 4 * UMAX;
    const unsigned nblk = (unsigned)((nlog + 7) / 8 * 8);
    const _Float16 *trows = reinterpret_cast<const _Float16 *>(tmpl_split);
    const int32_t *texp = reinterpret_cast<const int32_t *>(reinterpret_cast<const char *>(tmpl_split) +
                                                            (int64_t)a.C * total_rows * 2 * AFRAG);
    return m.BR == 64 ? launch_mfma_p<4>(a, m, lds, nblk, s, trows, texp, prec, out16)
                      : launch_mfma_p<2>(a, m, lds, nblk, s, trows, texp, prec, out16);
}

int64_t tmr_template_split_bytes(int U, int C, int64_t total_rows) {
    if (U <= 0 || C <= 0 || total_rows <= 0) return -1;
    return (int64_t)C * total_rows * 2 * AFRAG + 4 * (int64_t)U * C;
}

extern "C" int tmr_template_split(const float *templates, const tmr_unit_t *units, int U, int C,
                                  int64_t total_rows, int prec, void *out, void *stream) {
    TMR_REQUIRE(templates && units && out && U > 0 && C > 0 && total_rows > 0);
    TMR_REQUIRE(prec == TMR_PREC_F16X3 || prec == TMR_PREC_BF16 || prec == TMR_PREC_F16);
    char *frags = reinterpret_cast<char *>(out);
    int32_t *ex = reinterpret_cast<int32_t *>(frags + (int64_t)C * total_rows * 2 * AFRAG);
    const int64_t waves = (int64_t)U * C;
    hipLaunchKernelGGL(template_split_kernel, dim3((unsigned)tmr_cdiv(waves, 4)), dim3(256), 0,
                       tmr_stream(stream), templates, units, U, C, total_rows, (int)(prec == TMR_PREC_BF16),
                       (int)(prec == TMR_PREC_F16X3), frags, ex);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int tmr_xcorr(const tmr_xcorr_args_t *x, void *stream) {
    TMR_REQUIRE(x);
    const int B = x->B, C = x->C, H = x->H, W = x->W, U = x->U, max_ht = x->max_ht, max_wt = x->max_wt;
    TMR_REQUIRE(x->f && x->templates && x->units && x->img_units && x->scale && x->out && B > 0 && C > 0 &&
                U > 0 && H > 0 && W > 0);
    TMR_REQUIRE(x->out_bf16 == 0 || x->out_bf16 == 1);
    // a bf16 f_TM plane: the one-term bf16 MFMA kernel only, no relu / squeeze outputs
    TMR_REQUIRE(!x->out_bf16 ||
                (x->algo == TMR_XCORR_MFMA && x->prec == TMR_PREC_BF16 && !x->squeeze && !x->relu_out));
    TMR_REQUIRE(max_ht >= 1 && max_wt >= 1 && max_ht <= H && max_wt <= W);
    TMR_REQUIRE(!x->squeeze || x->work);
    TMR_REQUIRE(x->algo >= TMR_XCORR_AUTO && x->algo <= TMR_XCORR_MFMA);
    TMR_REQUIRE(x->prec == TMR_PREC_F16X3 || x->prec == TMR_PREC_BF16 || x->prec == TMR_PREC_F16);
    TMR_REQUIRE(C < 65536 && B < 65536);
    XArgs a;
    a.f = x->f;
    a.tmpl = x->templates;
    a.units = x->units;
    a.img_units = x->img_units;
    a.scale = x->scale;
    a.out = static_cast<float *>(x->out);  // bf16 elements when out_bf16
    a.relu_out = x->relu_out;
    a.work = x->work;
    a.out_absmax = reinterpret_cast<unsigned *>(x->out_absmax);
    a.C = C;
    a.H = H;
    a.W = W;
    a.squeeze = x->squeeze;
    hipStream_t s = tmr_stream(stream);
    // the MFMA kernel reads its A fragments from tmpl_split (tmr_template_split)
    const bool fits = mfma_fits(H, W, max_ht, max_wt) && x->tmpl_split && x->total_rows > 0;
    if (x->algo == TMR_XCORR_MFMA && !fits) return TMR_E_UNSUPPORTED;
    const bool use_mfma = x->algo == TMR_XCORR_MFMA || (x->algo == TMR_XCORR_AUTO && fits && x->min_k >= kMfmaMinK);
    if (use_mfma) {
        const int rc = launch_mfma(a, s, B, max_ht, x->tmpl_split, x->total_rows, x->prec, x->out_bf16 != 0);
        if (rc != TMR_OK) return rc;
    } else {
        TMR_REQUIRE(!x->out_bf16);
        // row-tiled kernel when rows are 16-B aligned and templates fit its
        // width specialisations (template sizes are odd, template_matching.py:66-73)
        const bool rows = (W % 4) == 0 && max_wt <= 31;
        const int WS = rows ? W + PADL + PADR : W;
        // LDS rows: band + template halo + slack rows for partial 4-row tiles
        const int max_rows = (150 * 1024) / (4 * WS) - 1;
        const int RB = min(32, max_rows - (max_ht - 1) - (rows ? TRY + 3 : RY));
        if (RB < 1) return TMR_E_UNSUPPORTED;
        a.RB = RB;
        a.LR = rows ? RB + max_ht + 3 : RB + max_ht - 1 + RY;
        a.HG = max_ht / 2;
        const size_t lds = (rows ? (size_t)a.LR * WS * sizeof(float)
                                 : ((size_t)a.LR * W + XSLACK) * sizeof(float)) + 4 * UMAX;
        const bool narrow = max_wt <= 15;
        const void *kfn = !rows ? (const void *)xcorr_kernel
                          : narrow ? (const void *)xcorr_rows_kernel<15> : (const void *)xcorr_rows_kernel<31>;
        if (lds > 64 * 1024 && tmr_set_max_lds(kfn, lds) != hipSuccess) return TMR_E_HIP;
        dim3 grid((unsigned)tmr_cdiv(H, RB), (unsigned)C, (unsigned)B);
        if (rows && narrow)
            hipLaunchKernelGGL(xcorr_rows_kernel<15>, grid, dim3(NT), lds, s, a, a.tmpl, a.out, a.units);
        else if (rows)
            hipLaunchKernelGGL(xcorr_rows_kernel<31>, grid, dim3(NT), lds, s, a, a.tmpl, a.out, a.units);
        else
            hipLaunchKernelGGL(xcorr_kernel, grid, dim3(NT), lds, s, a, a.tmpl, a.out);
        TMR_CHECK_LAUNCH();
    }
    if (x->squeeze) {
        int64_t tot = (int64_t)U * H * W;
        hipLaunchKernelGGL(xcorr_squeeze_kernel, dim3((unsigned)tmr_cdiv(tot, 256)), dim3(256), 0, s, x->work,
                           x->units, U, C, H, W, x->scale, a.out, x->relu_out,
                           reinterpret_cast<unsigned *>(x->out_absmax));
        TMR_CHECK_LAUNCH();
    }
    return TMR_OK;
}
