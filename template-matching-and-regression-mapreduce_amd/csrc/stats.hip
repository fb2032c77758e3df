// Per-image feature statistics of the streaming mapper (gfx950): the four
// numbers mapper.py:97-101 computes from each image's backbone feature,
//   mean = np.mean(f), std = np.std(f), max = np.max(f), spar = np.mean(f <= 0),
// for a batch of images already resident in HBM (the features the matching
// path consumes), so the mapper's line protocol (mapper.py:134-138) needs no
// host copy of the features.
//
//   1. stats_partial_kernel: grid (slices, images); each workgroup streams a
//      contiguous slice with 16-B loads and keeps, in fp64, the sum and sum of
//      squares of d = x - x0 (x0 = the image's first element: a shift that
//      makes the one-pass variance exact to ~1e-10 relative), the fp32 max and
//      the count of x <= 0.  Partials go to a [B][slices][4] fp64 workspace.
//   2. stats_final_kernel: one wave per image reduces the slices in a fixed
//      order (deterministic) and writes out[b] = {mean, std, max, spar}:
//      mean and std rounded once to fp32 (the mapper's values are float32),
//      max exact, spar = count / n exactly as numpy's fp64 mean of a bool array.
#include "tmr_common.h"

namespace {

constexpr int NT = 256;
constexpr int SLICES = 64;

__global__ __launch_bounds__(NT) void stats_partial_kernel(const float *__restrict__ x, int64_t n,
                                                           double *__restrict__ part) {
    const int s = blockIdx.x, b = blockIdx.y;
    const float *img = x + (size_t)b * n;
    const double x0 = (double)img[0];
    const int64_t per = ((n + SLICES - 1) / SLICES + 3) / 4 * 4;  // 16-B aligned slices
    const int64_t beg = min((int64_t)s * per, n), end = min(beg + per, n);
    double sum = 0.0, sq = 0.0;
    float mx = -INFINITY;
    int64_t cnt = 0;
    auto take = [&](float v) {
        const double d = (double)v - x0;
        sum += d;
        sq = fma(d, d, sq);
        mx = fmaxf(mx, v);
        cnt += v <= 0.0f;
    };
    // the image base is 16-B aligned when n % 4 == 0 (checked on the host)
    const bool vec = (n & 3) == 0;
    if (vec) {
        const float4 *v4 = reinterpret_cast<const float4 *>(img + beg);
        const int64_t n4 = (end - beg) / 4;
        for (int64_t i = threadIdx.x; i < n4; i += NT) {
            const float4 v = v4[i];
            take(v.x); take(v.y); take(v.z); take(v.w);
        }
        for (int64_t i = beg + n4 * 4 + threadIdx.x; i < end; i += NT) take(img[i]);
    } else {
        for (int64_t i = beg + threadIdx.x; i < end; i += NT) take(img[i]);
    }
    // wave reduction, then the 4 waves in order
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o);
        sq += __shfl_xor(sq, o);
        mx = fmaxf(mx, __shfl_xor(mx, o));
        cnt += __shfl_xor(cnt, o);
    }
    __shared__ double ws[NT / 64][4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        ws[w][0] = sum; ws[w][1] = sq; ws[w][2] = (double)mx; ws[w][3] = (double)cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double r[4] = {ws[0][0], ws[0][1], ws[0][2], ws[0][3]};
        for (int i = 1; i < NT / 64; ++i) {
            r[0] += ws[i][0]; r[1] += ws[i][1]; r[2] = fmax(r[2], ws[i][2]); r[3] += ws[i][3];
        }
        double *p = part + ((size_t)b * SLICES + s) * 4;
        p[0] = r[0]; p[1] = r[1]; p[2] = r[2]; p[3] = r[3];
    }
}

__global__ __launch_bounds__(64) void stats_final_kernel(const float *__restrict__ x, int64_t n,
                                                         const double *__restrict__ part,
                                                         double *__restrict__ out) {
    const int b = blockIdx.x, l = threadIdx.x;
    const double *p = part + ((size_t)b * SLICES + l) * 4;
    double sum = p[0], sq = p[1], mx = p[2], cnt = p[3];
    for (int o = 1; o < 64; o <<= 1) {  // fixed butterfly order: deterministic
        sum += __shfl_xor(sum, o);
        sq += __shfl_xor(sq, o);
        mx = fmax(mx, __shfl_xor(mx, o));
        cnt += __shfl_xor(cnt, o);
    }
    if (l == 0) {
        const double x0 = (double)x[(size_t)b * n];
        const double dn = (double)n;
        const double md = sum / dn;
        const double var = fmax(sq / dn - md * md, 0.0);
        double *o = out + (size_t)b * 4;
        o[0] = (double)(float)(x0 + md);
        o[1] = (double)(float)sqrt(var);
        o[2] = mx;
        o[3] = cnt / dn;
    }
}

}  // namespace

int64_t tmr_stats_work_bytes(int B) {
    if (B < 0) return -1;
    return (int64_t)B * SLICES * 4 * (int64_t)sizeof(double);
}

extern "C" int tmr_feature_stats(const float *x, int B, int64_t n, void *work, double *out,
                                 void *stream) {
    TMR_REQUIRE(B >= 0 && n > 0 && n < (1ll << 40));
    if (B == 0) return TMR_OK;
    TMR_REQUIRE(x && work && out);
    TMR_REQUIRE(B <= 65535);
    hipStream_t s = tmr_stream(stream);
    double *part = static_cast<double *>(work);
    hipLaunchKernelGGL(stats_partial_kernel, dim3(SLICES, B), dim3(NT), 0, s, x, n, part);
    TMR_CHECK_LAUNCH();
    hipLaunchKernelGGL(stats_final_kernel, dim3(B), dim3(64), 0, s, x, n, part, out);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}
