// Shared helpers for the libtmr.so HIP sources (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <utility>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/tmr.h"

// Library-internal functions shared between the sources (not part of the
// ABI: hidden, the one sizing entry point tmr_size dispatches to them).
#define TMR_INTERNAL __attribute__((visibility("hidden")))
TMR_INTERNAL int64_t tmr_template_split_bytes(int U, int C, int64_t total_rows);
TMR_INTERNAL int64_t tmr_heads_partials_floats(int N, int U, int H, int W);
TMR_INTERNAL int64_t tmr_xpack_bytes(int S, int C, int H, int W, int ks, int prec);
TMR_INTERNAL int64_t tmr_wpack_bytes(int N, int C0, int C1, int ks, int prec);
TMR_INTERNAL int64_t tmr_acc_floats(int U, int N, int H, int W);
TMR_INTERNAL int64_t tmr_nms_work_bytes(int64_t total_cand, int64_t sum_nb, int64_t max_cand, int G);
TMR_INTERNAL int64_t tmr_stats_work_bytes(int B);

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

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (device, kernel):
// the attribute is idempotent and the call is no stream operation, so a
// launch replayed inside a HIP graph capture must not re-issue it (the
// runtime refuses non-stream calls during a global-mode capture).  The only
// process-wide state of the library: a cache of an idempotent setting.
static inline hipError_t tmr_set_max_lds(const void *fn, size_t bytes) {
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, size_t> done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lock(mu);
    auto it = done.find({dev, fn});
    if (it != done.end() && it->second >= bytes) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) done[{dev, fn}] = bytes;
    return e;
}

// Near-correctly-rounded fp32 exp / sigmoid: double evaluation, one rounding.
// The reference's torch.exp / torch.sigmoid bits depend on the backend and on
// the element's position (vector body vs scalar tail on CPU); the path's
// decode contract is defined on these ("bit-exactness").
// f rounded to `bits` significant bits (round to nearest even on the fp32 bit
// pattern; inf/NaN unchanged): the sparse hi part of the 3-term split records
// (conv_split.hip WH_BITS, xcorr.hip TH_BITS)
__device__ __forceinline__ float tmr_round_sig_bits(float f, int bits) {
    uint32_t u = __float_as_uint(f);
    const uint32_t drop = 24u - (uint32_t)bits;
    if (drop == 0u || (u & 0x7f800000u) == 0x7f800000u) return f;
    const uint32_t half = 1u << (drop - 1u);
    u = (u + half - 1u + ((u >> drop) & 1u)) & ~((1u << drop) - 1u);
    return __uint_as_float(u);
}

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
