// Two small bandwidth kernels around the decoder GEMM (conv_split.hip):
//   * the bilinear x2 upsample (models/matching_net.py:50-51): up2x of the
//     projection at the SAM features' size, and the module API's f[0] (:81);
//   * the head reduction: the fused decoder kernel's per-128-channel-tile
//     partial sums of the 1x1 ObjectnessHead / BboxesHead
//     (regression_head.py:31,50) summed over tiles, plus the head biases.
#include <algorithm>

#include "tmr_common.h"

namespace {

constexpr int NHEAD = 5;  // 4 ltrbs outputs + 1 objectness

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

}  // namespace

extern "C" int tmr_upsample2x(const float *feat, int BC, int Hin, int Win, float *out, void *stream) {
    TMR_REQUIRE(feat && out && BC > 0 && Hin > 0 && Win > 0);
    return launch_upsample2x(feat, BC, Hin, Win, out, tmr_stream(stream));
}

int64_t tmr_heads_partials_floats(int N, int U, int H, int W) {
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
