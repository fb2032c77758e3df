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
#include "tmr_common.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

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
    unsigned *out_absmax;  // nullable [TMR_ABSMAX_SLOTS]: slot-wise atomicMax of |out|
    int C, H, W, RB, squeeze, LR;  // LR = LDS rows allocated
    int HG;                          // rows kernel: max template height / 2
};

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
    __syncthreads();

    const size_t plane = (size_t)H * W;
    float vmax = 0.0f;
    for (int u = u_beg; u < u_end; ++u) {
        const tmr_unit_t &un = a.units[u];
        const int h = __builtin_amdgcn_readfirstlane(un.ht), w = __builtin_amdgcn_readfirstlane(un.wt);
        const int64_t toff = ((int64_t)__builtin_amdgcn_readfirstlane((int)(un.tmpl_offset >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)un.tmpl_offset);
        const int ph = h / 2, pw = w / 2;
        const int Ho = H - h + 1, Wo = W - w + 1;
        const int ya = max(yb0, ph), yz = min(yb1, ph + Ho);  // valid output rows in band
        const int nv = max(yz - ya, 0);
        const float sc = a.squeeze ? 1.0f : *a.scale;
        const float denom = (float)(h * w);
        const float rden = 1.0f / denom;  // correctly rounded reciprocal
        float *op = a.squeeze ? a.work + ((size_t)u * a.C + c) * plane
                              : outp + ((size_t)u * a.C + c) * plane;
        float *rp = (a.relu_out && !a.squeeze) ? a.relu_out + ((size_t)u * a.C + c) * plane : nullptr;
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
    }
    if (a.out_absmax && !a.squeeze) {  // one atomic per workgroup, spread over the slots
        for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
        __syncthreads();  // xs is free: every unit's reads are done
        if ((threadIdx.x & 63) == 0) xs[threadIdx.x >> 6] = vmax;
        __syncthreads();
        if (threadIdx.x == 0) {
            float m = xs[0];
            for (int w = 1; w < NT / 64; ++w) m = fmaxf(m, xs[w]);
            const unsigned slot = (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) %
                                  TMR_ABSMAX_SLOTS;
            atomicMax(a.out_absmax + slot, __float_as_uint(m));
        }
    }
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

template <int KW, int TRY, int TRX>
__device__ __forceinline__ void corr_tile(const float *xs, int WS, int lrow0, int lcol0,
                                          const float *__restrict__ tc, int h,
                                          f32x2 (&pa)[TRY][TRX / 2]) {
    constexpr int OFF = (4 - ((KW / 2) & 3)) & 3;
    constexpr int NV = (OFF + KW + TRX + 3) / 4;   // b128 reads per row (+1 float for odd pairs)
    constexpr int NO = (OFF + KW + TRX - 2) / 2;   // odd pairs (x[2m+1], x[2m+2])
    for (int ii = 0; ii < TRY + h - 1; ++ii) {
        const float4 *xr = reinterpret_cast<const float4 *>(xs + (lrow0 + ii) * WS + lcol0);
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

// One unit's band for the rows kernel in TY x TX lane tiles.
template <int TY, int TX>
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
#define TMR_W(K) case K: corr_tile<K, TY, TX>(xs, WS, lrow0, lcol0, tc, h, pa); break;
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
    __syncthreads();

    const size_t plane = (size_t)H * W;
    float vmax = 0.0f;
    for (int u = u_beg; u < u_end; ++u) {
        const tmr_unit_t &un = units[u];  // restrict: scalar loads, no wait behind the stores
        const int h = __builtin_amdgcn_readfirstlane(un.ht), w = __builtin_amdgcn_readfirstlane(un.wt);
        const int64_t toff = ((int64_t)__builtin_amdgcn_readfirstlane((int)(un.tmpl_offset >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)un.tmpl_offset);
        const int ph = h / 2, pw = w / 2;
        const int Ho = H - h + 1, Wo = W - w + 1;
        const float denom = (float)(h * w);
        const float rden = 1.0f / denom;  // correctly rounded reciprocal
        float *op = a.squeeze ? a.work + ((size_t)u * a.C + c) * plane
                              : outp + ((size_t)u * a.C + c) * plane;
        float *rp = (a.relu_out && !a.squeeze) ? a.relu_out + ((size_t)u * a.C + c) * plane : nullptr;
        const float *__restrict__ tc = tmpl + toff + (size_t)c * h * w;
        // 4x4 tiles: one 16-B store per lane row (1 KB per wave row).  2x8
        // tiles (twice the FMAs per scalar tap-row load) measured 5.1 vs 5.5
        // ms at k = 9 but 10.4 vs 7.4 at k = 11 and 16.4 vs 11.4 at k = 15.
        rows_unit<4, 4>(xs, WS, W, yb0, yb1, hg, h, w, ph, pw, Ho, Wo, tc, denom, rden, sc, op, rp, vmax);
    }
    if (a.out_absmax && !a.squeeze) {  // one atomic per workgroup, spread over the slots
        for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
        __syncthreads();  // xs is free: every unit's reads are done
        if ((threadIdx.x & 63) == 0) xs[threadIdx.x >> 6] = vmax;
        __syncthreads();
        if (threadIdx.x == 0) {
            float m = xs[0];
            for (int w = 1; w < NT / 64; ++w) m = fmaxf(m, xs[w]);
            const unsigned slot = (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) %
                                  TMR_ABSMAX_SLOTS;
            atomicMax(a.out_absmax + slot, __float_as_uint(m));
        }
    }
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
    if (out_absmax) {
        float m = fabsf(v);
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
        if ((threadIdx.x & 63) == 0)
            atomicMax(out_absmax + (blockIdx.x * 4 + (threadIdx.x >> 6)) % TMR_ABSMAX_SLOTS,
                      __float_as_uint(m));
    }
}

}  // namespace

extern "C" int tmr_xcorr(const float *f, int B, int C, int H, int W, const float *templates,
                         const tmr_unit_t *units, const int32_t *img_units, int U, int max_ht,
                         int max_wt, const float *scale, int squeeze, float *out, float *relu_out,
                         float *work, float *out_absmax, void *stream) {
    TMR_REQUIRE(f && templates && units && img_units && scale && out && B > 0 && C > 0 && U > 0);
    TMR_REQUIRE(max_ht >= 1 && max_wt >= 1 && max_ht <= H && max_wt <= W);
    TMR_REQUIRE(!squeeze || work);
    // row-tiled kernel when rows are 16-B aligned and templates fit its
    // width specialisations (template sizes are odd, template_matching.py:66-73)
    const bool rows = (W % 4) == 0 && max_wt <= 31;
    const int WS = rows ? W + PADL + PADR : W;
    // LDS rows: band + template halo + slack rows for partial 4-row tiles
    const int max_rows = (150 * 1024) / (4 * WS) - 1;
    const int RB = min(32, max_rows - (max_ht - 1) - (rows ? TRY + 3 : RY));
    if (RB < 1) return TMR_E_UNSUPPORTED;
    XArgs a;
    a.f = f;
    a.tmpl = templates;
    a.units = units;
    a.img_units = img_units;
    a.scale = scale;
    a.out = out;
    a.relu_out = relu_out;
    a.work = work;
    a.out_absmax = reinterpret_cast<unsigned *>(out_absmax);
    a.C = C;
    a.H = H;
    a.W = W;
    a.RB = RB;
    a.squeeze = squeeze;
    a.LR = rows ? RB + max_ht + 3 : RB + max_ht - 1 + RY;
    a.HG = max_ht / 2;
    const size_t lds = rows ? (size_t)a.LR * WS * sizeof(float)
                            : ((size_t)a.LR * W + XSLACK) * sizeof(float);
    const void *kfn = rows ? (const void *)xcorr_rows_kernel : (const void *)xcorr_kernel;
    hipStream_t s = tmr_stream(stream);
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return TMR_E_HIP;
    TMR_REQUIRE(C < 65536 && B < 65536);
    dim3 grid((unsigned)tmr_cdiv(H, RB), (unsigned)C, (unsigned)B);
    if (rows)
        hipLaunchKernelGGL(xcorr_rows_kernel, grid, dim3(NT), lds, s, a, a.tmpl, a.out, a.units);
    else
        hipLaunchKernelGGL(xcorr_kernel, grid, dim3(NT), lds, s, a, a.tmpl, a.out);
    TMR_CHECK_LAUNCH();
    if (squeeze) {
        int64_t tot = (int64_t)U * H * W;
        hipLaunchKernelGGL(xcorr_squeeze_kernel, dim3((unsigned)tmr_cdiv(tot, 256)), dim3(256), 0, s,
                           work, units, U, C, H, W, scale, out, relu_out,
                           reinterpret_cast<unsigned *>(out_absmax));
        TMR_CHECK_LAUNCH();
    }
    return TMR_OK;
}
