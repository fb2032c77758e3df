// Peak finder + box decode (gfx950): Get_pred_boxes for one level
// (utils/TM_utils.py:245-282) with adaptive_kernel_generater's 3x3 mask
// (:363-377) and custom_shape_3x3_maxpool2d (:337-361, zero padding).
//
//   peaks_kernel: one workgroup per unit, one pass: p = sigmoid(o)
//   (near-correctly rounded; or p = o) staged in LDS by row chunks, flags
//   p >= thr && p == masked 3x3 max, wave ballots + mbcnt + a workgroup scan
//   give each candidate its row-major slot (torch.where order, no cap), and
//   the candidate is decoded in place: ref = (x/W, y/H); xy = ref + r[:2]*s;
//   wh = exp(r[2:])*(bw,bh); box = (xy - wh/2, xy + wh/2).
// exp: the reference's torch.exp (ATen CPU -> MKL VML vsExp, high accuracy)
// restated as the correctly rounded value except at the inputs recorded in
// the reference-exp table (tmr_amd/exp_table.py), where MKL rounds to the
// other neighbour; without a table, correctly rounded.
// Built with -ffp-contract=off so every op is separately rounded as in the
// reference's elementwise torch ops.
#include "tmr_common.h"

namespace {

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

// The probability map, chip-wide (one thread per 4 pixels): p = sigmoid(o)
// (near-correctly rounded), or o itself when the input is already p.  With
// TMR_PEAKS_PROB_SCRATCH the caller does not want the map: a logit whose
// sigmoid cannot round to thr or above is written as -1 without its sigmoid
// -- it can neither be a candidate nor beat one (its p < thr <= the
// candidate's p) -- and NaN stays NaN.  (Computing the sigmoid inside the
// one-workgroup-per-unit finder left a single unit's map to one CU: 25 us
// at config A.)
__global__ __launch_bounds__(256) void prob_kernel(const float *__restrict__ o, int is_prob, int scratch, int64_t n,
                                                   int64_t HW, const tmr_peak_param_t *__restrict__ params,
                                                   float *__restrict__ prob) {
    const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    int64_t ulast = -1;
    float olo = -INFINITY;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = i0 + k;
        if (i >= n) break;
        const float x = o[i];
        float v = x;
        if (!is_prob) {
            const int64_t u = i / HW;
            if (scratch && u != ulast) {
                ulast = u;
                const float thr = params[u].thr;
                olo = -INFINITY;
                if (thr > 0.0f) {
                    // p = (float)sigmoid(x) reaches thr only when the exact sigmoid is at least
                    // the midpoint between thr and the float below it; a logit under that
                    // midpoint's logit (less a margin far above the double sigmoid's error and
                    // olo's own fp32 rounding) cannot round up to thr, even for thr near 1
                    const float tq = fminf(thr, 1.0f);
                    const double mid = 0.5 * ((double)tq + (double)nextafterf(tq, 0.0f));
                    const double lg = log(mid / (1.0 - mid));
                    olo = (float)(lg - 1e-5 * (1.0 + fabs(lg)));
                }
            }
            v = x < olo ? -1.0f : tmr_sigmoid_cr(x);
        }
        prob[i] = v;
    }
}

// One workgroup per unit, one pass (north_star kernel 4, "wavefront-ballot"):
// the unit's probability map is walked in chunks of R whole rows; each chunk
// and its two halo rows (zero outside the image: F.unfold's padding) are
// staged in LDS.  Every wave takes 64 consecutive row-major pixels per step
// and keeps the step's is_peak ballot in LDS; after ONE barrier every lane
// finds its slot from the ballots of the steps and waves before it (+ mbcnt),
// so the candidates leave in row-major (torch.where) order, three barriers
// per chunk (round 5's first ballot kernel synchronised twice per 512-pixel
// step: 72 barriers per 128x128 unit).
constexpr int PNT = 1024;               // threads per unit block (16 waves: one unit per CU at most)
constexpr int PNW = PNT / 64;           // waves
constexpr int PCHUNK = 16384;           // staged pixels per chunk (whole rows): a 128 x 128 map in one
constexpr int PSTEPS = PCHUNK / PNT;    // PNT-pixel steps per chunk at most (W <= PCHUNK / 2)

__host__ __device__ inline int peak_rows(int W) { return W >= PCHUNK ? 1 : PCHUNK / W; }

__device__ __forceinline__ void decode_one(const float *__restrict__ reg, int HW, const tmr_peak_param_t &pp,
                                           int u, int i, const float *__restrict__ ref, float *__restrict__ box,
                                           ExpTable et);

__global__ __launch_bounds__(PNT) void peaks_kernel(const float *__restrict__ pm, int H, int W,
                                                    const tmr_peak_param_t *__restrict__ params,
                                                    float *__restrict__ logits, float *__restrict__ box,
                                                    float *__restrict__ ref, int32_t *__restrict__ counts,
                                                    const float *__restrict__ reg, int fuse_decode, ExpTable et) {
    extern __shared__ float sp[];  // [R + 2][W] probabilities, row 0 = image row r0 - 1
    __shared__ uint64_t bal[PSTEPS][PNW];
    const int u = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const tmr_peak_param_t pp = params[u];
    const int HW = H * W, R = peak_rows(W);
    // e / W by one multiply: exact while e < (R + 2) W <= 2 * PCHUNK (far below 2^22)
    const float rW = 1.0f / (float)W;
    const float *pmu = pm + (size_t)u * HW;
    const size_t cap = (size_t)HW;
    const uint64_t lt = (1ull << lane) - 1ull;  // lanes below this one
    int base = 0;  // candidates so far (block-uniform)
    for (int r0 = 0; r0 < H; r0 += R) {
        const int rn = min(R, H - r0), np = rn * W, ns = (np + PNT - 1) / PNT;
#pragma unroll 4
        for (int e = tid; e < (rn + 2) * W; e += PNT) {
            const int lr = (int)(((float)e + 0.5f) * rW), c = e - lr * W, y = r0 - 1 + lr;
            sp[e] = (y >= 0 && y < H) ? pmu[(size_t)y * W + c] : 0.0f;
        }
        __syncthreads();  // (1) the chunk is staged
        uint32_t fb = 0;  // bit s: this lane's pixel of step s is a candidate
        for (int st = 0; st < ns; ++st) {
            const int i = st * PNT + tid;  // pixel of the chunk
            bool f = false;
            if (i < np) {
                const int ly = (int)(((float)i + 0.5f) * rW) + 1, x = i - (ly - 1) * W;
                const float v = sp[ly * W + x];
                if (v >= pp.thr) {  // masked 3x3 max (TM_utils.py:337-361): first tap, then strict >;
                    float mx = 0.0f;  // a NaN tap sticks (torch.max, :359), so `pooled == p` (:253) fails
                    bool first = true;
#pragma unroll
                    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                        for (int dx = -1; dx <= 1; ++dx) {
                            if (!((pp.mask >> ((dy + 1) * 3 + dx + 1)) & 1)) continue;
                            const int xx = x + dx;
                            const float q = (xx < 0 || xx >= W) ? 0.0f : sp[(ly + dy) * W + xx];
                            if (first || q > mx || q != q) { mx = q; first = false; }
                        }
                    f = mx == v;
                }
            }
            const uint64_t bw = __ballot(f);
            if (lane == 0) bal[st][wave] = bw;
            fb |= (uint32_t)f << st;
        }
        __syncthreads();  // (2) every step's ballots are in
        int before = 0, tot = 0;  // candidates of the chunk before this wave's step st
        for (int st = 0; st < ns; ++st) {
            int cw = 0;
#pragma unroll
            for (int k = 0; k < PNW; ++k) {
                const int c = __popcll(bal[st][k]);
                cw += k < wave ? c : 0;
                tot += c;
            }
            if ((fb >> st) & 1u) {  // the slot's pixel index rides in the box row until decode_kernel
                const int i = st * PNT + tid, ly = (int)(((float)i + 0.5f) * rW) + 1, x = i - (ly - 1) * W;
                const int y = r0 + ly - 1;
                const size_t k = (size_t)u * cap + base + before + cw + __popcll(bal[st][wave] & lt);
                *reinterpret_cast<float2 *>(logits + 2 * k) = float2{sp[ly * W + x], 0.0f};
                reinterpret_cast<int *>(box)[4 * k] = y * W + x;
                *reinterpret_cast<float2 *>(ref + 2 * k) = float2{(float)x / (float)W, (float)y / (float)H};
            }
            before = tot;
        }
        base += tot;
        __syncthreads();  // (3) sp and the ballots free again
    }
    if (fuse_decode) {  // the block's own candidates (written above; visible after the barrier)
        for (int i = tid; i < base; i += PNT) decode_one(reg, HW, pp, u, i, ref, box, et);
    }
    if (tid == 0) {
        counts[u] = base;
        if (base == 0) {  // the empty unit's dummy row (TM_utils.py:288-291) at row 0
            *reinterpret_cast<float2 *>(logits + (size_t)u * cap * 2) = float2{0.0f, 0.0f};
            *reinterpret_cast<float4 *>(box + (size_t)u * cap * 4) = float4{0.0f, 0.0f, 1e-14f, 1e-14f};
            *reinterpret_cast<float2 *>(ref + (size_t)u * cap * 2) = float2{0.0f, 0.0f};
        }
    }
}

// The box decode of candidate i of unit u (TM_utils.py:264-278): the slot's
// pixel index rides in the box row until here.
__device__ __forceinline__ void decode_one(const float *__restrict__ reg, int HW, const tmr_peak_param_t &pp,
                                           int u, int i, const float *__restrict__ ref, float *__restrict__ box,
                                           ExpTable et) {
    const float *r = reg ? reg + (size_t)u * 4 * HW : nullptr;
    const float sx = pp.mode == 1 ? 1.0f : pp.scale_w, sy = pp.mode == 1 ? 1.0f : pp.scale_h;
    const size_t k = (size_t)u * HW + i;
    const int pi = reinterpret_cast<const int *>(box)[4 * k];
    const float2 rf = *reinterpret_cast<const float2 *>(ref + 2 * k);
    float r0v = 0.0f, r1 = 0.0f, r2 = 0.0f, r3 = 0.0f;
    if (pp.mode != 2 && r) {
        r0v = r[pi]; r1 = r[HW + pi]; r2 = r[2 * HW + pi]; r3 = r[3 * HW + pi];
    }
    const float cx = rf.x + r0v * sx, cy = rf.y + r1 * sy;
    const float w = expf_ref(r2, et) * pp.scale_w, h = expf_ref(r3, et) * pp.scale_h;
    const float hw2 = w / 2.0f, hh2 = h / 2.0f;
    *reinterpret_cast<float4 *>(box + 4 * k) = float4{cx - hw2, cy - hh2, cx + hw2, cy + hh2};
}

// Every candidate's decode, chip-wide: one thread per candidate, so the
// reference-exp table's binary search (a chain of dependent loads) overlaps
// across thousands of threads instead of serialising the finder's steps.
// (Launches of a few units decode inside peaks_kernel instead: one launch
// less, config A.)
__global__ __launch_bounds__(256) void decode_kernel(const float *__restrict__ reg, int H, int W,
                                                     const tmr_peak_param_t *__restrict__ params,
                                                     const int32_t *__restrict__ counts, const float *__restrict__ ref,
                                                     float *__restrict__ box, ExpTable et) {
    const int u = blockIdx.x;
    const int n = counts[u];
    const tmr_peak_param_t pp = params[u];
    for (int i = blockIdx.y * 256 + threadIdx.x; i < n; i += gridDim.y * 256)
        decode_one(reg, H * W, pp, u, i, ref, box, et);
}

constexpr int kFuseDecodeUnits = 8;

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
    TMR_REQUIRE((input_is_prob & ~(1 | TMR_PEAKS_PROB_SCRATCH)) == 0);
    const int is_prob = input_is_prob & 1, scratch = (input_is_prob & TMR_PEAKS_PROB_SCRATCH) != 0;
    hipStream_t s = tmr_stream(stream);
    ExpTable et = {nullptr, nullptr};
    if (exp_table) {
        const char *base = reinterpret_cast<const char *>(exp_table);
        et.off = reinterpret_cast<const uint32_t *>(base + EXP_HEADER);
        et.lo = reinterpret_cast<const uint16_t *>(base + EXP_HEADER + 4 * 65537);
    }
    TMR_REQUIRE(W <= PCHUNK / 2);  // (R + 2) W floats of LDS <= 3 * 8192 * 4 B
    const size_t lds = (size_t)(peak_rows(W) + 2) * W * sizeof(float);
    if (lds > 64 * 1024 && tmr_set_max_lds((const void *)peaks_kernel, lds) != hipSuccess) return TMR_E_HIP;
    const float *pm = o;
    if (!(is_prob && scratch)) {  // the map (or its scratch form) into prob
        const int64_t n = (int64_t)U * H * W;
        TMR_REQUIRE(tmr_cdiv(n, 1024) < (1LL << 31));
        hipLaunchKernelGGL(prob_kernel, dim3((unsigned)tmr_cdiv(n, 1024)), dim3(256), 0, s, o, is_prob, scratch, n,
                           (int64_t)H * W, params, prob);
        TMR_CHECK_LAUNCH();
        pm = prob;
    }
    // a few units: decode inside the finder (one launch less); many: chip-wide
    const int fuse = U <= kFuseDecodeUnits;
    hipLaunchKernelGGL(peaks_kernel, dim3(U), dim3(PNT), lds, s, pm, H, W, params, logits, box, ref, counts, reg,
                       fuse, et);
    TMR_CHECK_LAUNCH();
    if (!fuse) {
        const int ny = (int)std::min<int64_t>(tmr_cdiv((int64_t)H * W, 256), 32);
        hipLaunchKernelGGL(decode_kernel, dim3(U, ny), dim3(256), 0, s, reg, H, W, params, counts, ref, box, et);
        TMR_CHECK_LAUNCH();
    }
    return TMR_OK;
}
