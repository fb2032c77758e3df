// Shared helpers for the libtmr.so HIP sources (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/tmr.h"

#define TMR_CHECK_LAUNCH()                                  \
    do {                                                    \
        hipError_t e_ = hipGetLastError();                  \
        if (e_ != hipSuccess) return TMR_E_HIP;             \
    } while (0)

#define TMR_REQUIRE(cond)                                   \
    do {                                                    \
        if (!(cond)) return TMR_E_INVALID;                  \
    } while (0)

static inline hipStream_t tmr_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

static inline int64_t tmr_cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// host-side A/B switch of a measured variant (documented where it is read)
static inline int tmr_env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

// Near-correctly-rounded fp32 exp / sigmoid: double evaluation, one rounding.
// The reference's torch.exp / torch.sigmoid bits depend on the backend and on
// the element's position (vector body vs scalar tail on CPU); the path's
// decode contract is defined on these ("bit-exactness").
__device__ __forceinline__ float tmr_expf_cr(float x) { return (float)exp((double)x); }
__device__ __forceinline__ float tmr_sigmoid_cr(float x) {
    return (float)(1.0 / (1.0 + exp(-(double)x)));
}

// Bilinear x2 (align_corners=False) of a half-resolution plane at output
// (y, x); the fma nesting reproduces ATen's CPU kernel.
__device__ __forceinline__ void up_coord(int d, int L, int &i0, int &i1, float &l0, float &l1) {
    float src = 0.5f * ((float)d + 0.5f) - 0.5f;
    src = src < 0.0f ? 0.0f : src;
    int a = (int)src;
    i0 = a;
    i1 = a + ((a < L - 1) ? 1 : 0);
    l1 = src - (float)a;
    l0 = 1.0f - l1;
}

__device__ __forceinline__ float up_value(const float *plane, int Hin, int Win, int y, int x) {
    int y0, y1, x0, x1;
    float ly0, ly1, lx0, lx1;
    up_coord(y, Hin, y0, y1, ly0, ly1);
    up_coord(x, Win, x0, x1, lx0, lx1);
    float a = plane[y0 * Win + x0], b = plane[y0 * Win + x1];
    float c = plane[y1 * Win + x0], d = plane[y1 * Win + x1];
    float top = fmaf(lx0, a, lx1 * b);
    float bot = fmaf(lx0, c, lx1 * d);
    return fmaf(ly0, top, ly1 * bot);
}

// The same upsample from the two input rows r0, r1 (rows y0, y1 of
// up_coord(y)) at output column x: up_value's arithmetic.
__device__ __forceinline__ float up_rows(const float *r0, const float *r1, float ly0, float ly1, int Win,
                                         int x) {
    int x0, x1;
    float lx0, lx1;
    up_coord(x, Win, x0, x1, lx0, lx1);
    const float top = fmaf(lx0, r0[x0], lx1 * r0[x1]);
    const float bot = fmaf(lx0, r1[x0], lx1 * r1[x1]);
    return fmaf(ly0, top, ly1 * bot);
}

// Output columns 4q .. 4q+3, bit-identical to four up_rows calls: away from
// the left/right edge they read input columns 2q-1 .. 2q+2 with the exact
// weights up_coord yields there (x = 4q: 0.25/0.75, 4q+1: 0.75/0.25,
// 4q+2: 0.25/0.75, 4q+3: 0.75/0.25).
__device__ __forceinline__ float4 up_rows4(const float *r0, const float *r1, float ly0, float ly1, int Win,
                                           int q) {
    if (q > 0 && 2 * q + 2 < Win) {
        const float *p0 = r0 + 2 * q - 1, *p1 = r1 + 2 * q - 1;
        const float a0 = p0[0], a1 = p0[1], a2 = p0[2], a3 = p0[3];
        const float b0 = p1[0], b1 = p1[1], b2 = p1[2], b3 = p1[3];
        const float t0 = fmaf(0.25f, a0, 0.75f * a1), u0 = fmaf(0.25f, b0, 0.75f * b1);
        const float t1 = fmaf(0.75f, a1, 0.25f * a2), u1 = fmaf(0.75f, b1, 0.25f * b2);
        const float t2 = fmaf(0.25f, a1, 0.75f * a2), u2 = fmaf(0.25f, b1, 0.75f * b2);
        const float t3 = fmaf(0.75f, a2, 0.25f * a3), u3 = fmaf(0.75f, b2, 0.25f * b3);
        return float4{fmaf(ly0, t0, ly1 * u0), fmaf(ly0, t1, ly1 * u1), fmaf(ly0, t2, ly1 * u2),
                      fmaf(ly0, t3, ly1 * u3)};
    }
    return float4{up_rows(r0, r1, ly0, ly1, Win, 4 * q), up_rows(r0, r1, ly0, ly1, Win, 4 * q + 1),
                  up_rows(r0, r1, ly0, ly1, Win, 4 * q + 2), up_rows(r0, r1, ly0, ly1, Win, 4 * q + 3)};
}

// Outputs (y, 4q .. 4q+3) of up2x(plane), bit-identical to four up_value calls.
__device__ __forceinline__ float4 up_value4(const float *plane, int Hin, int Win, int y, int q) {
    int y0, y1;
    float ly0, ly1;
    up_coord(y, Hin, y0, y1, ly0, ly1);
    return up_rows4(plane + (size_t)y0 * Win, plane + (size_t)y1 * Win, ly0, ly1, Win, q);
}
