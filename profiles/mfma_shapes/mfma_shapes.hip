// 16-bit MFMA shape study for the correlation's row-Toeplitz GEMM (VERDICT r5
// #2): cycles per instruction and FLOP/s of every gfx950 16-bit MFMA form that
// could carry it, measured the same way for each -- operands in registers,
// random fp16 / bf16 values (the power-limited clock depends on bit density,
// MI355X_MICROARCH.md), 16 independent accumulator chains per wave (8 / 4 for the
// 16- / 32-register accumulators; -DCH4=4 for 4), 2 waves per
// SIMD on every CU.  Per shape: wall (HIP events, best of 5) -> TFLOP/s, and
// per wave s_memtime ticks -> cycles per MFMA per SIMD.  Prints one JSON line
// per shape (results/*.jsonl, round 6); profiles/mfma_shapes/toeplitz.py turns
// them into the useful-FLOP table of the Toeplitz formulations (toeplitz_table.md).
//
//   hipcc --offload-arch=gfx950 -O3 mfma_shapes.hip -o mfma_shapes && ./mfma_shapes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#ifndef CH4
#define CH4 16  // chains per wave for the 4-register accumulators
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x32 __attribute__((ext_vector_type(32)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b4 __attribute__((ext_vector_type(4)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

__device__ __forceinline__ float urand(unsigned &s) {  // xorshift32 -> [-1, 1)
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    return (float)(s >> 8) * (2.0f / 16777216.0f) - 1.0f;
}

template <class V, int N> __device__ __forceinline__ V fill(unsigned &s) {
    V v;
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = (decltype(v[0] + v[0]))urand(s);
    return v;
}

// one shape: A, B operand vector types, accumulator type, the builtin call
#define SHAPE(NAME, AV, NA, CV, NC, CALL, MACS)                                              \
    struct NAME {                                                                            \
        typedef AV A;                                                                        \
        typedef CV C;                                                                        \
        static constexpr int na = NA, nc = NC;                                               \
        static constexpr double macs = MACS;                                                 \
        static constexpr const char *name = #NAME;                                           \
        __device__ static __forceinline__ C mma(A a, A b, C c) { return CALL(a, b, c, 0, 0, 0); } \
    };

SHAPE(f16_16x16x32, h8, 8, f32x4, 4, __builtin_amdgcn_mfma_f32_16x16x32_f16, 16.0 * 16 * 32)
SHAPE(f16_16x16x16, h4, 4, f32x4, 4, __builtin_amdgcn_mfma_f32_16x16x16f16, 16.0 * 16 * 16)
SHAPE(f16_32x32x16, h8, 8, f32x16, 16, __builtin_amdgcn_mfma_f32_32x32x16_f16, 32.0 * 32 * 16)
SHAPE(f16_32x32x8, h4, 4, f32x16, 16, __builtin_amdgcn_mfma_f32_32x32x8f16, 32.0 * 32 * 8)
SHAPE(f16_16x16x4_4b, h4, 4, f32x16, 16, __builtin_amdgcn_mfma_f32_16x16x4f16, 4.0 * 16 * 16 * 4)
SHAPE(f16_32x32x4_2b, h4, 4, f32x32, 32, __builtin_amdgcn_mfma_f32_32x32x4f16, 2.0 * 32 * 32 * 4)
SHAPE(f16_4x4x4_16b, h4, 4, f32x4, 4, __builtin_amdgcn_mfma_f32_4x4x4f16, 16.0 * 4 * 4 * 4)
SHAPE(bf16_16x16x32, b8, 8, f32x4, 4, __builtin_amdgcn_mfma_f32_16x16x32_bf16, 16.0 * 16 * 32)
SHAPE(bf16_16x16x16, s4, 4, f32x4, 4, __builtin_amdgcn_mfma_f32_16x16x16bf16_1k, 16.0 * 16 * 16)
SHAPE(bf16_4x4x4_16b, s4, 4, f32x4, 4, __builtin_amdgcn_mfma_f32_4x4x4bf16_1k, 16.0 * 4 * 4 * 4)

template <class S> __device__ __forceinline__ typename S::A operand(unsigned &s) {
    if constexpr (S::na == 8) {
        return fill<typename S::A, 8>(s);
    } else {
        typename S::A v;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if constexpr (sizeof(v[0]) == 2 && __is_same(decltype(v[0] + v[0]), int)) {
                // bf16 bits in a short vector (the _1k builtins' operand type)
                const float f = urand(s);
                v[q] = (short)(__float_as_uint(f) >> 16);
            } else {
                v[q] = (decltype(v[0] + v[0]))urand(s);
            }
        }
        return v;
    }
}

// accumulator chains per wave: CHAINS, or 4 for the 32-register accumulators
template <class S> constexpr int chains() { return S::nc >= 32 ? 4 : S::nc >= 16 ? 8 : CH4; }

template <class S> __global__ __launch_bounds__(256) void shape_loop(float *out, unsigned long long *ticks, int iters) {
    unsigned s = 0x9e3779b9u * (blockIdx.x * 256 + threadIdx.x + 1);
    typename S::A a[2], b[2];
    a[0] = operand<S>(s); a[1] = operand<S>(s);
    b[0] = operand<S>(s); b[1] = operand<S>(s);
    constexpr int CHAINS = chains<S>();
    typename S::C acc[CHAINS];
#pragma unroll
    for (int k = 0; k < CHAINS; ++k)
#pragma unroll
        for (int q = 0; q < S::nc; ++q) acc[k][q] = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int k = 0; k < CHAINS; ++k) acc[k] = S::mma(a[k & 1], b[(k >> 1) & 1], acc[k]);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float r = 0.0f;
#pragma unroll
    for (int k = 0; k < CHAINS; ++k)
#pragma unroll
        for (int q = 0; q < S::nc; ++q) r += acc[k][q];
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) ticks[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <class S> static void run(int cus, float *out, unsigned long long *ticks, unsigned long long *hticks) {
    const int blocks = cus * 2;  // 8 waves per CU: 2 per SIMD
    const int iters = 20000;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(shape_loop<S>, dim3(blocks), dim3(256), 0, 0, out, ticks, iters);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(shape_loop<S>, dim3(blocks), dim3(256), 0, 0, out, ticks, iters);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    CHECK(hipMemcpy(hticks, ticks, sizeof(unsigned long long) * blocks * 4, hipMemcpyDeviceToHost));
    double tsum = 0;
    for (int i = 0; i < blocks * 4; ++i) tsum += (double)hticks[i];
    const double tmean = tsum / (blocks * 4);
    const double n_mfma = (double)iters * chains<S>();  // per wave
    const double flop = 2.0 * S::macs * n_mfma * blocks * 4;
    // two waves share a SIMD: cycles per MFMA per SIMD = wave ticks / (2 x MFMAs per wave)
    printf("{\"shape\": \"%s\", \"macs_per_instr\": %.0f, \"tflops\": %.1f, \"ms\": %.4f, "
           "\"cycles_per_mfma_per_simd\": %.2f, \"clock_ghz_est\": %.3f, \"chains\": %d}\n",
           S::name, S::macs, flop / best / 1e9, best, tmean / (2.0 * n_mfma), tmean / (best * 1e6), chains<S>());
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    float *out;
    unsigned long long *ticks;
    CHECK(hipMalloc(&out, sizeof(float) * cus * 2 * 256));
    CHECK(hipMalloc(&ticks, sizeof(unsigned long long) * cus * 2 * 4));
    unsigned long long *h = (unsigned long long *)malloc(sizeof(unsigned long long) * cus * 2 * 4);
    run<f16_16x16x32>(cus, out, ticks, h);
    run<f16_16x16x16>(cus, out, ticks, h);
    run<f16_32x32x16>(cus, out, ticks, h);
    run<f16_32x32x8>(cus, out, ticks, h);
    run<f16_16x16x4_4b>(cus, out, ticks, h);
    run<f16_32x32x4_2b>(cus, out, ticks, h);
    run<f16_4x4x4_16b>(cus, out, ticks, h);
    run<bf16_16x16x32>(cus, out, ticks, h);
    run<bf16_16x16x16>(cus, out, ticks, h);
    run<bf16_4x4x4_16b>(cus, out, ticks, h);
    return 0;
}
