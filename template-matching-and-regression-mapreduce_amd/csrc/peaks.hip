// Peak finder + box decode (gfx950): Get_pred_boxes for one level
// (utils/TM_utils.py:245-282) with adaptive_kernel_generater's 3x3 mask
// (:363-377) and custom_shape_3x3_maxpool2d (:337-361, zero padding).
//
//   1. prob_kernel:  p = sigmoid(o) (near-correctly rounded) or p = o.
//   2. peaks_kernel: one 1024-thread workgroup per unit; each lane owns a
//      contiguous run of pixels, flags p >= thr && p == masked 3x3 max,
//      a workgroup prefix sum gives each candidate its row-major slot
//      (torch.where order, no cap), and the candidate is decoded in place:
//      ref = (x/W, y/H); xy = ref + r[:2]*s; wh = exp(r[2:])*(bw,bh);
//      box = (xy - wh/2, xy + wh/2).
// exp: the reference's torch.exp (ATen CPU -> MKL VML vsExp, high accuracy)
// restated as the correctly rounded value except at the inputs recorded in
// the reference-exp table (tmr_amd/exp_table.py), where MKL rounds to the
// other neighbour; without a table, correctly rounded.
// Built with -ffp-contract=off so every op is separately rounded as in the
// reference's elementwise torch ops.
#include "tmr_common.h"

namespace {

constexpr int NT = 1024;
constexpr int EXP_HEADER = 128;  // tmr_amd/exp_table.py

struct ExpTable {
    const uint32_t *off;  // [65537] by the input's upper 16 bits
    const uint16_t *lo;   // sorted lower 16 bits of the recorded inputs
};

__device__ __forceinline__ float expf_ref(float x, ExpTable t) {
    const double e = exp((double)x);
    float y = (float)e;
    if (!t.off) return y;
    const uint32_t b = __float_as_uint(x);
    const uint32_t hb = b >> 16, key = b & 0xffffu;
    uint32_t s = t.off[hb], n = t.off[hb + 1];
    const uint32_t end = n;
    while (s < n) {  // lower bound of key in lo[s, end)
        const uint32_t m = (s + n) >> 1;
        if (t.lo[m] < key) s = m + 1; else n = m;
    }
    if (s < end && t.lo[s] == key)  // MKL rounded to the exact value's other side
        y = e > (double)y ? nextafterf(y, __builtin_inff()) : nextafterf(y, -__builtin_inff());
    return y;
}

__global__ void prob_kernel(const float *__restrict__ o, int64_t n, int is_prob,
                            float *__restrict__ p) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = o[i];
    p[i] = is_prob ? v : tmr_sigmoid_cr(v);
}

// custom_shape_3x3_maxpool2d (TM_utils.py:337-361): per element, the max of
// the masked 3x3 neighbourhood (F.unfold's zero padding), taps in row-major
// order; a NaN propagates (torch.max) and a tie keeps the earlier tap.
__global__ void maxpool3x3_kernel(const float *__restrict__ x, int64_t n, int H, int W, int mask,
                                  float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t hw = (int64_t)H * W;
    const int64_t pl = i / hw;
    const int r = (int)(i - pl * hw), y = r / W, xx = r % W;
    const float *p = x + pl * hw;
    float mx = 0.0f;
    bool first = true;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
            if (!((mask >> ((dy + 1) * 3 + dx + 1)) & 1)) continue;
            const int yy = y + dy, xc = xx + dx;
            const float q = (yy < 0 || yy >= H || xc < 0 || xc >= W) ? 0.0f : p[yy * W + xc];
            if (first || q > mx || (q != q && mx == mx)) { mx = q; first = false; }
        }
    out[i] = mx;
}

__device__ __forceinline__ bool is_peak(const float *__restrict__ p, int H, int W, int y, int x,
                                        int mask, float thr) {
    const float v = p[y * W + x];
    if (!(v >= thr)) return false;
    float mx = 0.0f;
    bool first = true;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
            if (!((mask >> ((dy + 1) * 3 + dx + 1)) & 1)) continue;
            const int yy = y + dy, xx = x + dx;
            const float q = (yy < 0 || yy >= H || xx < 0 || xx >= W) ? 0.0f : p[yy * W + xx];
            if (first || q > mx) { mx = q; first = false; }
        }
    return mx == v;
}

__global__ __launch_bounds__(NT) void peaks_kernel(const float *__restrict__ prob,
                                                   const float *__restrict__ reg, int H, int W,
                                                   const tmr_peak_param_t *__restrict__ params,
                                                   float *__restrict__ logits, float *__restrict__ box,
                                                   float *__restrict__ ref, int32_t *__restrict__ counts,
                                                   ExpTable et) {
    __shared__ int wsum[NT / 64];
    const int u = blockIdx.x;
    const tmr_peak_param_t pp = params[u];
    const int HW = H * W;
    const float *p = prob + (size_t)u * HW;
    const int per = (HW + NT - 1) / NT;
    const int beg = min(threadIdx.x * per, HW), end = min(beg + per, HW);
    // pass 1: count (bits of up to 64 owned pixels kept in a register mask)
    int cnt = 0;
    for (int i = beg; i < end; ++i) cnt += is_peak(p, H, W, i / W, i % W, pp.mask, pp.thr);
    // workgroup exclusive scan
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = cnt;
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int wbase = 0, total = 0;
    for (int k = 0; k < NT / 64; ++k) {
        int s = wsum[k];
        if (k < wave) wbase += s;
        total += s;
    }
    int pos = wbase + incl - cnt;
    const size_t cap = (size_t)HW;
    if (threadIdx.x == 0) {
        counts[u] = total;
        if (total == 0) {  // the empty unit's dummy row (TM_utils.py:288-291) at row 0
            *reinterpret_cast<float2 *>(logits + (size_t)u * cap * 2) = float2{0.0f, 0.0f};
            *reinterpret_cast<float4 *>(box + (size_t)u * cap * 4) = float4{0.0f, 0.0f, 1e-14f, 1e-14f};
            *reinterpret_cast<float2 *>(ref + (size_t)u * cap * 2) = float2{0.0f, 0.0f};
        }
    }
    if (cnt == 0) return;
    const float *r = reg ? reg + (size_t)u * 4 * HW : nullptr;
    for (int i = beg; i < end; ++i) {
        const int y = i / W, x = i % W;
        if (!is_peak(p, H, W, y, x, pp.mask, pp.thr)) continue;
        const size_t k = (size_t)u * cap + pos++;
        const float v = p[i];
        const float rx = (float)x / (float)W, ry = (float)y / (float)H;
        float r0 = 0.0f, r1 = 0.0f, r2 = 0.0f, r3 = 0.0f;
        if (pp.mode != 2 && r) {
            r0 = r[i]; r1 = r[HW + i]; r2 = r[2 * HW + i]; r3 = r[3 * HW + i];
        }
        const float sx = pp.mode == 1 ? 1.0f : pp.scale_w, sy = pp.mode == 1 ? 1.0f : pp.scale_h;
        const float cx = rx + r0 * sx, cy = ry + r1 * sy;
        const float w = expf_ref(r2, et) * pp.scale_w, h = expf_ref(r3, et) * pp.scale_h;
        const float hw2 = w / 2.0f, hh2 = h / 2.0f;
        logits[2 * k + 0] = v;
        logits[2 * k + 1] = 0.0f;
        box[4 * k + 0] = cx - hw2;
        box[4 * k + 1] = cy - hh2;
        box[4 * k + 2] = cx + hw2;
        box[4 * k + 3] = cy + hh2;
        ref[2 * k + 0] = rx;
        ref[2 * k + 1] = ry;
    }
}

}  // namespace

extern "C" int tmr_maxpool3x3(const float *x, int64_t planes, int H, int W, int mask9, float *out,
                              void *stream) {
    if (planes < 0 || H < 0 || W < 0 || (mask9 & 0x1ff) == 0 || (mask9 & ~0x1ff) != 0) return TMR_E_INVALID;
    const int64_t n = planes * H * W;
    if (n == 0) return TMR_OK;
    if (!x || !out) return TMR_E_INVALID;
    hipLaunchKernelGGL(maxpool3x3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       x, n, H, W, mask9, out);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int tmr_peaks_decode(const float *o, int input_is_prob, const float *reg, int U, int H,
                                int W, const tmr_peak_param_t *params, float *prob, float *logits,
                                float *box, float *ref, int32_t *counts, const void *exp_table,
                                void *stream) {
    TMR_REQUIRE(o && params && prob && logits && box && ref && counts && U > 0 && H > 0 && W > 0);
    hipStream_t s = tmr_stream(stream);
    ExpTable et = {nullptr, nullptr};
    if (exp_table) {
        const char *base = reinterpret_cast<const char *>(exp_table);
        et.off = reinterpret_cast<const uint32_t *>(base + EXP_HEADER);
        et.lo = reinterpret_cast<const uint16_t *>(base + EXP_HEADER + 4 * 65537);
    }
    int64_t n = (int64_t)U * H * W;
    hipLaunchKernelGGL(prob_kernel, dim3((unsigned)tmr_cdiv(n, 256)), dim3(256), 0, s, o, n,
                       input_is_prob, prob);
    TMR_CHECK_LAUNCH();
    hipLaunchKernelGGL(peaks_kernel, dim3(U), dim3(NT), 0, s, prob, reg, H, W, params, logits, box, ref,
                       counts, et);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}
