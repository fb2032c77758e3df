// Per-image greedy NMS over the exemplar-ordered candidate union (gfx950).
// Reference: NMS / NMS_process (utils/TM_utils.py:307-323) ->
// torchvision.ops.nms (0.19 CPU semantics: stable descending score order,
// fp32 IoU, `(double)ovr > iou_threshold`), applied after the per-exemplar
// Get_pred_boxes results are concatenated (demo.py:123-130,
// trainer.py:111-118), dummy rows included (TM_utils.py:288-291).
//
//   gather : union per image in unit order, dummy row for empty units
//   rank   : stable descending rank by counting (ties -> lower index)
//   mask   : upper-triangular 64-bit IoU suppression words per sorted row
//   reduce : one wave per image walks 64-row blocks; the in-block greedy
//            chain is resolved from registers (readlane), then the kept rows
//            are OR-ed into the LDS "removed" bitmap in parallel.  The keep
//            list equals the sequential torchvision loop because IoU(i,j) is
//            bitwise symmetric and suppression only flows from kept rows.
// Built with -ffp-contract=off.
#include "tmr_common.h"

namespace {

constexpr int RANK_NT = 256;

struct NmsWork {
    float *s;       // [T]
    float *b;       // [T][4]
    float *r;       // [T][2]
    int32_t *order; // [T] sorted position -> local index
    uint64_t *mask; // [mask_words]
};

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

__host__ __device__ inline NmsWork carve(void *work, int64_t T) {
    NmsWork w;
    char *p = (char *)work;
    w.s = (float *)p; p += align256(sizeof(float) * T);
    w.b = (float *)p; p += align256(sizeof(float) * 4 * T);
    w.r = (float *)p; p += align256(sizeof(float) * 2 * T);
    w.order = (int32_t *)p; p += align256(sizeof(int32_t) * T);
    w.mask = (uint64_t *)p;
    return w;
}

__global__ void gather_kernel(const float *__restrict__ logits, const float *__restrict__ box,
                              const float *__restrict__ ref, const int32_t *__restrict__ counts,
                              const int64_t *__restrict__ unit_off,
                              const int32_t *__restrict__ seg_units,
                              const int64_t *__restrict__ cand_off, NmsWork w) {
    const int g = blockIdx.x;
    int64_t pos = cand_off[g];
    for (int u = seg_units[g]; u < seg_units[g + 1]; ++u) {
        const int n = counts[u];
        if (n == 0) {
            if (threadIdx.x == 0) {
                w.s[pos] = 0.0f;
                w.b[4 * pos + 0] = 0.0f; w.b[4 * pos + 1] = 0.0f;
                w.b[4 * pos + 2] = 1e-14f; w.b[4 * pos + 3] = 1e-14f;
                w.r[2 * pos + 0] = 0.0f; w.r[2 * pos + 1] = 0.0f;
            }
            pos += 1;
            continue;
        }
        const size_t src = (size_t)unit_off[u];
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            w.s[pos + i] = logits[2 * (src + i)];
            const float4 bb = reinterpret_cast<const float4 *>(box)[src + i];
            reinterpret_cast<float4 *>(w.b)[pos + i] = bb;
            w.r[2 * (pos + i) + 0] = ref[2 * (src + i) + 0];
            w.r[2 * (pos + i) + 1] = ref[2 * (src + i) + 1];
        }
        pos += n;
    }
}

__global__ __launch_bounds__(RANK_NT) void rank_kernel(const int64_t *__restrict__ cand_off, NmsWork w) {
    __shared__ float ss[RANK_NT];
    const int g = blockIdx.y;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    if ((int)blockIdx.x * RANK_NT >= n) return;
    const int i = blockIdx.x * RANK_NT + threadIdx.x;
    const float si = i < n ? w.s[off + i] : 0.0f;
    int rank = 0;
    for (int j0 = 0; j0 < n; j0 += RANK_NT) {
        __syncthreads();
        ss[threadIdx.x] = (j0 + threadIdx.x < n) ? w.s[off + j0 + threadIdx.x] : 0.0f;
        __syncthreads();
        const int m = min(RANK_NT, n - j0);
        for (int k = 0; k < m; ++k) {
            const float sj = ss[k];
            const int j = j0 + k;
            rank += (sj > si) || (sj == si && j < i);
        }
    }
    if (i < n) w.order[off + rank] = i;
}

__global__ __launch_bounds__(64) void mask_kernel(const int64_t *__restrict__ cand_off,
                                                  const int64_t *__restrict__ mask_off, double thr,
                                                  NmsWork w) {
    __shared__ float jb_box[64][4];
    __shared__ float jb_area[64];
    const int jb = blockIdx.x, ib = blockIdx.y, g = blockIdx.z;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    const int nb = (n + 63) / 64;
    if (ib >= nb || jb >= nb || jb < ib) return;
    const int t = threadIdx.x;
    const int j = jb * 64 + t;
    if (j < n) {
        const int lj = min(max(w.order[off + j], 0), n - 1);  // NaN-safe
        const float4 bj = reinterpret_cast<const float4 *>(w.b)[off + lj];
        jb_box[t][0] = bj.x; jb_box[t][1] = bj.y; jb_box[t][2] = bj.z; jb_box[t][3] = bj.w;
        jb_area[t] = (bj.z - bj.x) * (bj.w - bj.y);
    }
    __syncthreads();
    const int i = ib * 64 + t;
    if (i >= n) return;
    const int li = min(max(w.order[off + i], 0), n - 1);
    const float4 bi = reinterpret_cast<const float4 *>(w.b)[off + li];
    const float ai = (bi.z - bi.x) * (bi.w - bi.y);
    uint64_t bits = 0;
    const int kmax = min(64, n - jb * 64);
    for (int k = 0; k < kmax; ++k) {
        if (jb * 64 + k <= i) continue;
        const float xx1 = fmaxf(bi.x, jb_box[k][0]), yy1 = fmaxf(bi.y, jb_box[k][1]);
        const float xx2 = fminf(bi.z, jb_box[k][2]), yy2 = fminf(bi.w, jb_box[k][3]);
        float ww = xx2 - xx1, hh = yy2 - yy1;
        ww = ww > 0.0f ? ww : 0.0f;
        hh = hh > 0.0f ? hh : 0.0f;
        const float inter = ww * hh;
        const float ovr = inter / (ai + jb_area[k] - inter);
        if ((double)ovr > thr) bits |= (1ull << k);
    }
    w.mask[mask_off[g] + (int64_t)i * nb + jb] = bits;
}

__global__ __launch_bounds__(64) void reduce_kernel(const int64_t *__restrict__ cand_off,
                                                    const int64_t *__restrict__ mask_off, NmsWork w,
                                                    float *__restrict__ out_logits,
                                                    float *__restrict__ out_boxes,
                                                    float *__restrict__ out_refs,
                                                    int64_t *__restrict__ out_keep,
                                                    int32_t *__restrict__ kept_out) {
    extern __shared__ uint64_t removed[];
    const int g = blockIdx.x, lane = threadIdx.x;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    const int nb = (n + 63) / 64;
    const uint64_t *mask = w.mask + mask_off[g];
    for (int k = lane; k < nb; k += 64) {
        const int rem = n - k * 64;
        removed[k] = rem >= 64 ? 0ull : ~((1ull << rem) - 1);  // rows past n never kept
    }
    __syncthreads();
    int cnt = 0;
    for (int ib = 0; ib < nb; ++ib) {
        const int i = ib * 64 + lane;
        const uint64_t diag = i < n ? mask[(int64_t)i * nb + ib] : 0ull;
        uint64_t word = removed[ib];
        uint64_t kept = 0;
        const uint32_t dlo = (uint32_t)diag, dhi = (uint32_t)(diag >> 32);
        for (int bit = 0; bit < 64; ++bit) {
            if ((word >> bit) & 1ull) continue;
            kept |= 1ull << bit;
            const uint32_t lo = __builtin_amdgcn_readlane(dlo, bit);
            const uint32_t hi = __builtin_amdgcn_readlane(dhi, bit);
            word |= ((uint64_t)hi << 32) | lo;
        }
        if ((kept >> lane) & 1ull) {
            const int pos = cnt + __popcll(kept & ((1ull << lane) - 1));
            const int li = min(max(w.order[off + i], 0), n - 1);
            const int64_t src = off + li, dst = off + pos;
            out_logits[2 * dst + 0] = w.s[src];
            out_logits[2 * dst + 1] = 0.0f;
            reinterpret_cast<float4 *>(out_boxes)[dst] = reinterpret_cast<const float4 *>(w.b)[src];
            out_refs[2 * dst + 0] = w.r[2 * src + 0];
            out_refs[2 * dst + 1] = w.r[2 * src + 1];
            if (out_keep) out_keep[dst] = li;
        }
        cnt += __popcll(kept);
        // OR the kept rows' words into the later blocks: lane k gathers
        // column block k (coalesced across lanes); the kept rows (a
        // wave-uniform set) are walked 8 at a time so 8 independent loads are
        // in flight per wait instead of one load latency per kept row
        for (int k = ib + 1 + lane; k < nb; k += 64) {
            uint64_t acc = 0;
            uint64_t kb = kept;
            while (kb) {
                uint64_t v[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    v[t] = 0;
                    if (kb) {
                        const int b = __builtin_ctzll(kb);
                        kb &= kb - 1;
                        v[t] = mask[(int64_t)(ib * 64 + b) * nb + k];
                    }
                }
                acc |= ((v[0] | v[1]) | (v[2] | v[3])) | ((v[4] | v[5]) | (v[6] | v[7]));
            }
            removed[k] |= acc;
        }
        __syncthreads();
    }
    if (lane == 0) kept_out[g] = cnt;
}

}  // namespace

extern "C" int64_t tmr_nms_work_size(int64_t total_cand, int64_t mask_words) {
    if (total_cand < 0 || mask_words < 0) return -1;
    const int64_t T = total_cand;
    return (int64_t)(align256(sizeof(float) * T) + align256(sizeof(float) * 4 * T) +
                     align256(sizeof(float) * 2 * T) + align256(sizeof(int32_t) * T) +
                     sizeof(uint64_t) * (size_t)mask_words + 256);
}

extern "C" int tmr_nms(const float *logits, const float *box, const float *ref,
                       const int32_t *counts, const int64_t *unit_off, const int32_t *seg_units,
                       const int64_t *cand_off, const int64_t *mask_off, int G,
                       int64_t total_cand, int64_t max_cand, double iou_threshold,
                       float *out_logits, float *out_boxes, float *out_refs, int64_t *out_keep,
                       int32_t *kept, void *work, void *stream) {
    TMR_REQUIRE(logits && box && ref && counts && unit_off && seg_units && cand_off && mask_off);
    TMR_REQUIRE(work && out_logits && out_boxes && out_refs && kept && G > 0);
    TMR_REQUIRE(total_cand >= G && max_cand >= 1);
    const int64_t max_nb = (max_cand + 63) / 64;
    TMR_REQUIRE(max_nb < 65536 && G < 65536);
    TMR_REQUIRE(max_nb * 8 <= 150 * 1024);
    hipStream_t s = tmr_stream(stream);
    NmsWork w = carve(work, total_cand);
    hipLaunchKernelGGL(gather_kernel, dim3(G), dim3(256), 0, s, logits, box, ref, counts, unit_off,
                       seg_units, cand_off, w);
    TMR_CHECK_LAUNCH();
    hipLaunchKernelGGL(rank_kernel, dim3((unsigned)tmr_cdiv(max_cand, RANK_NT), G), dim3(RANK_NT), 0, s,
                       cand_off, w);
    TMR_CHECK_LAUNCH();
    hipLaunchKernelGGL(mask_kernel, dim3((unsigned)max_nb, (unsigned)max_nb, G), dim3(64), 0, s, cand_off,
                       mask_off, iou_threshold, w);
    TMR_CHECK_LAUNCH();
    const size_t lds = sizeof(uint64_t) * (size_t)max_nb;
    auto rk = reduce_kernel;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void *)rk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
            hipSuccess)
        return TMR_E_HIP;
    hipLaunchKernelGGL(rk, dim3(G), dim3(64), lds, s, cand_off, mask_off, w, out_logits, out_boxes,
                       out_refs, out_keep, kept);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}
