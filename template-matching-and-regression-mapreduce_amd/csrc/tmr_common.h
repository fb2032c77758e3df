// Shared helpers for the libtmr.so HIP sources (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

// Near-correctly-rounded fp32 exp / sigmoid: double evaluation, one rounding.
// The reference's torch.exp / torch.sigmoid bits depend on the backend and on
// the element's position (vector body vs scalar tail on CPU); the path's
// decode contract is defined on these ("bit-exactness").
__device__ __forceinline__ float tmr_expf_cr(float x) { return (float)exp((double)x); }
__device__ __forceinline__ float tmr_sigmoid_cr(float x) {
    return (float)(1.0 / (1.0 + exp(-(double)x)));
}
