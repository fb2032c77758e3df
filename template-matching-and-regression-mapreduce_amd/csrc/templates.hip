// Exemplar templates (gfx950): RoIAlign (torchvision 0.19 semantics, as
// called at models/template_matching.py:75 with aligned=True,
// sampling_ratio=-1, spatial_scale=1) and the prototype average
// (template_matching.py:43-53).  Workgroups per (unit, channel group); the
// sampling grid is computed once per workgroup into LDS and reused by every
// channel, like torchvision's CPU pre_calc.  Built with -ffp-contract=off: every product and
// sum is a separately rounded fp32 op, as in the reference's CPU kernel.
#include <algorithm>

#include "tmr_common.h"

namespace {

constexpr int NT = 256;
constexpr int MAX_SAMPLES = 1536;  // (ph,pw,iy,ix) samples cached per unit (48 KB)

struct Samp {
    int p[4];
    float w[4];
};

__global__ __launch_bounds__(NT) void roi_align_kernel(const float *__restrict__ f, int C, int H,
                                                       int W, const tmr_unit_t *__restrict__ units,
                                                       float *__restrict__ tmpl) {
    __shared__ Samp samp[MAX_SAMPLES];
    const tmr_unit_t un = units[blockIdx.x];
    if (un.type != TMR_TEMPLATE_ROI_ALIGN) return;
    const int PH = un.ht, PW = un.wt;
    const float off = 0.5f;
    const float sw = un.roi[0] - off, sh = un.roi[1] - off;
    const float ew = un.roi[2] - off, eh = un.roi[3] - off;
    const float rw = ew - sw, rh = eh - sh;
    const float bin_h = rh / (float)PH, bin_w = rw / (float)PW;
    const int gh = (int)ceilf(rh / (float)PH);
    const int gw = (int)ceilf(rw / (float)PW);
    const int g = gh * gw;
    const float count = (float)(g > 1 ? g : 1);
    const int ns = g * PH * PW;
    const bool cached = ns <= MAX_SAMPLES;

    auto make = [&](int k) -> Samp {
        Samp s;
        int ix = k % gw, iy = (k / gw) % gh, pw = (k / g) % PW, ph = k / (g * PW);
        float y = sh + (float)ph * bin_h + ((float)iy + 0.5f) * bin_h / (float)gh;
        float x = sw + (float)pw * bin_w + ((float)ix + 0.5f) * bin_w / (float)gw;
        if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) {
            for (int q = 0; q < 4; ++q) { s.p[q] = 0; s.w[q] = 0.0f; }
            return s;
        }
        if (y <= 0) y = 0;
        if (x <= 0) x = 0;
        int yl = (int)y, xl = (int)x, yh, xh;
        if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
        if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
        float ly = y - (float)yl, lx = x - (float)xl;
        float hy = 1.0f - ly, hx = 1.0f - lx;
        s.w[0] = hy * hx; s.w[1] = hy * lx; s.w[2] = ly * hx; s.w[3] = ly * lx;
        s.p[0] = yl * W + xl; s.p[1] = yl * W + xh; s.p[2] = yh * W + xl; s.p[3] = yh * W + xh;
        return s;
    };
    if (cached)
        for (int k = threadIdx.x; k < ns; k += NT) samp[k] = make(k);
    __syncthreads();

    const float *fb = f + (size_t)un.image * C * H * W;
    float *out = tmpl + un.tmpl_offset;
    const int per_c = PH * PW;
    // this block's channel range (grid.y splits the unit's channels)
    const int c0 = (int)((int64_t)C * blockIdx.y / gridDim.y), c1 = (int)((int64_t)C * (blockIdx.y + 1) / gridDim.y);
    for (int e = c0 * per_c + threadIdx.x; e < c1 * per_c; e += NT) {
        const int c = e / per_c, q0 = (e % per_c) * g;
        const float *fc = fb + (size_t)c * H * W;
        float acc = 0.0f;
        for (int s = 0; s < g; ++s) {
            Samp sp = cached ? samp[q0 + s] : make(q0 + s);
            float v = sp.w[0] * fc[sp.p[0]] + sp.w[1] * fc[sp.p[1]];
            v = v + sp.w[2] * fc[sp.p[2]];
            v = v + sp.w[3] * fc[sp.p[3]];
            acc += v;
        }
        out[e] = acc / count;
    }
}

// AdaptiveAvgPool2d(1) over the integer-snapped box, one wave per channel.
__global__ __launch_bounds__(NT) void prototype_kernel(const float *__restrict__ f, int C, int H,
                                                       int W, const tmr_unit_t *__restrict__ units,
                                                       float *__restrict__ tmpl) {
    const tmr_unit_t un = units[blockIdx.x];
    if (un.type != TMR_TEMPLATE_PROTOTYPE) return;
    const int x1 = un.pbox[0], y1 = un.pbox[1], x2 = un.pbox[2], y2 = un.pbox[3];
    const int bw = x2 - x1, n = (y2 - y1) * bw;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float *fb = f + (size_t)un.image * C * H * W;
    for (int c = blockIdx.y * (NT / 64) + wave; c < C; c += gridDim.y * (NT / 64)) {
        const float *fc = fb + (size_t)c * H * W;
        double acc = 0.0;
        for (int i = lane; i < n; i += 64) acc += fc[(y1 + i / bw) * W + x1 + i % bw];
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0) tmpl[un.tmpl_offset + c] = (float)(acc / (double)n);
    }
}

}  // namespace

extern "C" int tmr_templates(const float *f, int B, int C, int H, int W, const tmr_unit_t *units,
                             int U, int max_ht, int max_wt, float *templates, void *stream) {
    TMR_REQUIRE(f && units && templates && B > 0 && C > 0 && H > 0 && W > 0 && U > 0);
    TMR_REQUIRE(max_ht > 0 && max_wt > 0);
    hipStream_t s = tmr_stream(stream);
    // channel groups per unit: enough workgroups for the chip at small U
    // (the module API runs one unit per call), >= 8 channels each
    const int cg = (int)std::max<int64_t>(1, std::min<int64_t>(C / 8, tmr_cdiv(1024, U)));
    hipLaunchKernelGGL(roi_align_kernel, dim3(U, cg), dim3(NT), 0, s, f, C, H, W, units, templates);
    TMR_CHECK_LAUNCH();
    hipLaunchKernelGGL(prototype_kernel, dim3(U, (unsigned)tmr_cdiv(C, NT / 64) > 64 ? 64 : (unsigned)tmr_cdiv(C, NT / 64)),
                       dim3(NT), 0, s, f, C, H, W, units, templates);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}
