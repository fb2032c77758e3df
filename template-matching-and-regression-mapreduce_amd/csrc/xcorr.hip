// Depthwise cross-correlation of each unit's exemplar template with its
// image's projected features (gfx950, fp32 VALU), then the divide by the
// template area, the zero pad back to HxW and the learned scale:
//   models/template_matching.py:23-41 (cross_correlation), :97 (f * scale).
//
// One workgroup per (band of 32 output rows, channel, unit).  The band's
// input rows are staged once in LDS; each lane owns one output column and
// RY=8 consecutive output rows and streams the input rows past them (register
// sliding window), so each LDS read feeds RY*h/(RY+h-1) FMAs.  Template taps
// are wave-uniform (scalar loads).  The divide is an IEEE fp32 division by
// fl32(h*w) exactly like the reference's `/ (h*w + 1e-14)`.
#include "tmr_common.h"

namespace {

constexpr int NT = 256;
constexpr int RY = 8;
constexpr int JC = 8;

struct XArgs {
    const float *f;
    const float *tmpl;
    const tmr_unit_t *units;
    const float *scale;
    float *out;
    float *relu_out;
    float *work;
    int C, H, W, RB, squeeze;
};

__global__ __launch_bounds__(NT) void xcorr_kernel(XArgs a) {
    extern __shared__ float xs[];
    const int band = blockIdx.x, c = blockIdx.y, u = blockIdx.z;
    const tmr_unit_t un = a.units[u];
    const int h = un.ht, w = un.wt;
    const int H = a.H, W = a.W;
    const int ph = h / 2, pw = w / 2;
    const int Ho = H - h + 1, Wo = W - w + 1;
    const int yb0 = band * a.RB, yb1 = min(yb0 + a.RB, H);
    const int ya = max(yb0, ph), yz = min(yb1, ph + Ho);
    const int nv = max(yz - ya, 0);
    const float *__restrict__ fc = a.f + ((size_t)un.image * a.C + c) * H * W;
    const float *__restrict__ tc = a.tmpl + un.tmpl_offset + (size_t)c * h * w;
    const int nrows = nv ? nv + h - 1 : 0;
    const int r_base = ya - ph;
    for (int e = threadIdx.x; e < nrows * W; e += NT) xs[e] = fc[(size_t)r_base * W + e];
    __syncthreads();

    const float sc = a.squeeze ? 1.0f : *a.scale;
    const float denom = (float)(h * w);
    const size_t plane = (size_t)H * W;
    float *op = a.squeeze ? a.work + ((size_t)u * a.C + c) * plane
                          : a.out + ((size_t)u * a.C + c) * plane;
    float *rp = (a.relu_out && !a.squeeze) ? a.relu_out + ((size_t)u * a.C + c) * plane : nullptr;

    // zero border of this band (rows outside the valid range, cols outside)
    if (!a.squeeze) {
        for (int e = threadIdx.x; e < (yb1 - yb0) * W; e += NT) {
            int yo = yb0 + e / W, xo = e % W;
            bool valid = yo >= ya && yo < yz && xo >= pw && xo < pw + Wo;
            if (!valid) {
                op[(size_t)yo * W + xo] = 0.0f;
                if (rp) rp[(size_t)yo * W + xo] = 0.0f;
            }
        }
    }

    const int ngroups = (nv + RY - 1) / RY;
    for (int task = threadIdx.x; task < Wo * ngroups; task += NT) {
        const int x = task % Wo, r0 = (task / Wo) * RY;
        float acc[RY];
#pragma unroll
        for (int r = 0; r < RY; ++r) acc[r] = 0.0f;
        for (int ii = 0; ii < RY + h - 1; ++ii) {
            const float *xr = xs + (r0 + ii) * W + x;
            for (int j0 = 0; j0 < w; j0 += JC) {
                float xv[JC];
#pragma unroll
                for (int jj = 0; jj < JC; ++jj) xv[jj] = (j0 + jj < w) ? xr[j0 + jj] : 0.0f;
#pragma unroll
                for (int r = 0; r < RY; ++r) {
                    const int i = ii - r;
                    if (i < 0 || i >= h) continue;
                    const float *tr = tc + i * w + j0;
#pragma unroll
                    for (int jj = 0; jj < JC; ++jj)
                        if (j0 + jj < w) acc[r] = fmaf(xv[jj], tr[jj], acc[r]);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RY; ++r) {
            const int yl = r0 + r;
            if (yl >= nv) break;
            const size_t o = (size_t)(ya + yl) * W + x + pw;
            const float v = (acc[r] / denom) * sc;
            op[o] = v;
            if (rp) rp[o] = v > 0.0f ? v : 0.0f;
        }
    }
}

// squeeze (template_matching.py:34-35): sum over channels, pad, scale
__global__ void xcorr_squeeze_kernel(const float *__restrict__ work, const tmr_unit_t *__restrict__ units,
                                     int U, int C, int H, int W, const float *__restrict__ scale,
                                     float *__restrict__ out, float *__restrict__ relu_out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)U * H * W) return;
    const int u = (int)(i / ((int64_t)H * W));
    const int p = (int)(i % ((int64_t)H * W));
    const int y = p / W, x = p % W;
    const tmr_unit_t un = units[u];
    const int ph = un.ht / 2, pw = un.wt / 2, Ho = H - un.ht + 1, Wo = W - un.wt + 1;
    float v = 0.0f;
    if (y >= ph && y < ph + Ho && x >= pw && x < pw + Wo) {
        const float *wp = work + (size_t)u * C * H * W + p;
        float s = 0.0f;
        for (int c = 0; c < C; ++c) s += wp[(size_t)c * H * W];
        v = s * *scale;
    }
    out[i] = v;
    if (relu_out) relu_out[i] = v > 0.0f ? v : 0.0f;
}

}  // namespace

extern "C" int tmr_xcorr(const float *f, int B, int C, int H, int W, const float *templates,
                         const tmr_unit_t *units, int U, int max_ht, int max_wt,
                         const float *scale, int squeeze, float *out, float *relu_out, float *work,
                         void *stream) {
    TMR_REQUIRE(f && templates && units && scale && out && B > 0 && C > 0 && U > 0);
    TMR_REQUIRE(max_ht >= 1 && max_wt >= 1 && max_ht <= H && max_wt <= W);
    TMR_REQUIRE(!squeeze || work);
    const int max_rows = (150 * 1024) / (4 * W);
    const int RB = min(32, max_rows - (max_ht - 1) - RY);
    if (RB < 1) return TMR_E_UNSUPPORTED;
    XArgs a;
    a.f = f;
    a.tmpl = templates;
    a.units = units;
    a.scale = scale;
    a.out = out;
    a.relu_out = relu_out;
    a.work = work;
    a.C = C;
    a.H = H;
    a.W = W;
    a.RB = RB;
    a.squeeze = squeeze;
    const size_t lds = (size_t)(RB + max_ht - 1 + RY) * W * sizeof(float);
    hipStream_t s = tmr_stream(stream);
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void *)xcorr_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
        return TMR_E_HIP;
    dim3 grid((unsigned)tmr_cdiv(H, RB), (unsigned)C, (unsigned)U);
    TMR_REQUIRE(C < 65536 && U < 65536);
    hipLaunchKernelGGL(xcorr_kernel, grid, dim3(NT), lds, s, a);
    TMR_CHECK_LAUNCH();
    if (squeeze) {
        int64_t tot = (int64_t)U * H * W;
        hipLaunchKernelGGL(xcorr_squeeze_kernel, dim3((unsigned)tmr_cdiv(tot, 256)), dim3(256), 0, s,
                           work, units, U, C, H, W, scale, out, relu_out);
        TMR_CHECK_LAUNCH();
    }
    return TMR_OK;
}
