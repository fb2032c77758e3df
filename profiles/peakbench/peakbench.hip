// Peak microbenchmarks of the MI355X this runs on ("re-measure
// all peaks on the box"): dense 16-bit MFMA (v_mfma_f32_16x16x32_bf16 / _f16,
// operands in registers, 8 independent accumulator chains per wave, 2 waves
// per SIMD), packed fp32 VALU FMA (v_pk_fma_f32, 8 independent chains), and
// HBM streaming read and copy over 4 GiB buffers (16-B lane accesses).  HIP
// events around each launch; the best of 5 runs.  Prints one JSON object.
//
//   hipcc --offload-arch=gfx950 -O3 peakbench.hip -o peakbench && ./peakbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

template <int BF>
__global__ __launch_bounds__(256) void mfma_peak(float *out, int iters) {
    const int t = threadIdx.x;
    f32x4 acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if constexpr (BF) {
        b8 a, b;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            a[q] = (__bf16)(1.0f + 1e-3f * (t + q));
            b[q] = (__bf16)(1.0f - 1e-3f * (t - q));
        }
        for (int i = 0; i < iters; ++i)
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[k], 0, 0, 0);
    } else {
        h8 a, b;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            a[q] = (_Float16)(1.0f + 1e-3f * (t + q));
            b[q] = (_Float16)(1.0f - 1e-3f * (t - q));
        }
        for (int i = 0; i < iters; ++i)
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[k], 0, 0, 0);
    }
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * 256 + t] = s;
}

__global__ __launch_bounds__(256) void valu_peak(float *out, int iters) {
    const int t = threadIdx.x;
    f32x2 x[8];
    const f32x2 m = {1.0000001f, 0.9999999f}, c = {1e-7f, -1e-7f};
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = f32x2{(float)(t + k), (float)(t - k)};
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = __builtin_elementwise_fma(x[k], m, c);
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += x[k][0] + x[k][1];
    out[blockIdx.x * 256 + t] = s;
}

__global__ __launch_bounds__(256) void hbm_read(const f32x4 *__restrict__ src, size_t n4, float *out) {
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        acc += __builtin_nontemporal_load(src + i);
    if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.0f) out[0] = acc[0];  // keeps the loads
}

__global__ __launch_bounds__(256) void hbm_copy(const f32x4 *__restrict__ src, f32x4 *__restrict__ dst, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

template <class F>
static float best_ms(F launch, int reps = 5) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch();  // warm
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a));
        launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    return best;
}

int main() {
    int dev = 0, cus = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = cus * 8;  // 4 waves each: 8 waves per CU, 2 per SIMD
    float *out;
    CHECK(hipMalloc(&out, sizeof(float) * blocks * 256));
    const int it = 20000;
    const double mfma_flop = (double)blocks * 4 * it * 8 * (16.0 * 16 * 32 * 2);
    const float ms_bf = best_ms([&] { hipLaunchKernelGGL(mfma_peak<1>, dim3(blocks), dim3(256), 0, 0, out, it); });
    const float ms_f16 = best_ms([&] { hipLaunchKernelGGL(mfma_peak<0>, dim3(blocks), dim3(256), 0, 0, out, it); });
    const int vit = 20000;
    const double valu_flop = (double)blocks * 256 * vit * 8 * 4;  // 2 lanes x FMA per v_pk_fma
    const float ms_valu = best_ms([&] { hipLaunchKernelGGL(valu_peak, dim3(blocks), dim3(256), 0, 0, out, vit); });
    const size_t bytes = (size_t)4 << 30;
    f32x4 *src, *dst;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&dst, bytes));
    CHECK(hipMemset(src, 0, bytes));
    const size_t n4 = bytes / 16;
    const int sblocks = cus * 16;
    const float ms_rd = best_ms([&] { hipLaunchKernelGGL(hbm_read, dim3(sblocks), dim3(256), 0, 0, src, n4, out); });
    const float ms_cp = best_ms([&] { hipLaunchKernelGGL(hbm_copy, dim3(sblocks), dim3(256), 0, 0, src, dst, n4); });
    CHECK(hipGetLastError());
    printf("{\"cus\": %d, \"mfma_bf16_tflops\": %.1f, \"mfma_f16_tflops\": %.1f, \"valu_fp32_tflops\": %.1f, "
           "\"hbm_read_gbs\": %.0f, \"hbm_copy_gbs\": %.0f, \"basis\": \"best of 5 launches; MFMA: "
           "v_mfma_f32_16x16x32 with register operands, 8 chains per wave, 2 waves per SIMD, %d iterations; "
           "VALU: v_pk_fma_f32, 8 chains; HBM: 4 GiB, 16-B nontemporal lane accesses, read = bytes read, "
           "copy = bytes read + written\"}\n",
           cus, mfma_flop / ms_bf / 1e9, mfma_flop / ms_f16 / 1e9, valu_flop / ms_valu / 1e9,
           bytes / ms_rd / 1e6, 2.0 * bytes / ms_cp / 1e6, it);
    return 0;
}
