// Per-image greedy NMS over the exemplar-ordered candidate union (gfx950).
// Reference: NMS / NMS_process (utils/TM_utils.py:307-323) ->
// torchvision.ops.nms (0.19 CPU semantics: stable descending score order,
// fp32 IoU, `(double)ovr > iou_threshold`), applied after the per-exemplar
// Get_pred_boxes results are concatenated (demo.py:123-130,
// trainer.py:111-118), dummy rows included (TM_utils.py:288-291).
//
//   gather : union per image in unit order (dummy row for an empty unit)
//            + the local index of every row
//   sort   : rocprim segmented radix sort of (score, index) pairs, descending
//            and stable: ties keep the lower index first, as torchvision's
//            stable sort (O(n log) per image instead of O(n^2) rank counting)
//   strips : the 64-bit IoU suppression words of a STRIP of S row blocks
//            (64 sorted rows each) against every later column block are
//            computed (mask_strip) and consumed (reduce_strip) strip after
//            strip.  One workgroup per image keeps the running "removed"
//            bitmap (one bit per sorted row, in LDS, parked in HBM between
//            strips): a row block's in-block greedy chain is resolved from
//            registers (readlane over the surviving rows), then its kept
//            rows' words are OR-ed into the later blocks by all its threads.  Memory is O(n) per image plus ONE strip buffer whose
//            size is bounded (TMR_NMS_STRIP_WORDS) independently of n^2; the
//            keep list equals the sequential torchvision loop because IoU(i,j)
//            is bitwise symmetric and suppression only flows from kept rows.
// Built with -ffp-contract=off.
#include <algorithm>

#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "tmr_common.h"

namespace {

// strip buffer budget: 32 Mi 64-bit words (256 MiB) across all images of a
// call; a strip holds S row blocks of every image (S >= 1)
constexpr int64_t STRIP_WORDS = 32ll << 20;
// rocprim's temporary storage beyond its key/value double buffers
constexpr int64_t SORT_SLACK = 1 << 20;

struct NmsWork {
    float *s;        // [T] scores (unit order)
    float *skeys;    // [T] sorted scores (unused beyond the sort)
    float *b;        // [T][4]
    float *r;        // [T][2]
    int32_t *idx;    // [T] local row index (sort values in)
    int32_t *order;  // [T] sorted position -> local index
    float *sb;       // [T][4] boxes in sorted order (the strips' row and column operands)
    uint64_t *removed;  // [sum_nb] running suppression bitmap per image
    uint64_t *strip;    // [strip_words]
    char *temp;         // rocprim temporary storage
    int64_t temp_bytes;
};

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

inline int64_t sort_temp_bound(int64_t T, int G) { return 8 * T + SORT_SLACK + 64 * (int64_t)(G + 1); }

// S (row blocks per strip) and the strip buffer's words for these sizes
inline void strip_plan(int64_t sum_nb, int64_t max_nb, int64_t &S, int64_t &words) {
    S = std::max<int64_t>(1, std::min<int64_t>(max_nb, STRIP_WORDS / std::max<int64_t>(1, 64 * sum_nb)));
    words = S * 64 * sum_nb;
}

inline NmsWork carve(void *work, int64_t T, int64_t sum_nb, int64_t strip_words, int G) {
    NmsWork w;
    char *p = (char *)work;
    w.s = (float *)p; p += align256(sizeof(float) * T);
    w.skeys = (float *)p; p += align256(sizeof(float) * T);
    w.b = (float *)p; p += align256(sizeof(float) * 4 * T);
    w.r = (float *)p; p += align256(sizeof(float) * 2 * T);
    w.idx = (int32_t *)p; p += align256(sizeof(int32_t) * T);
    w.order = (int32_t *)p; p += align256(sizeof(int32_t) * T);
    w.sb = (float *)p; p += align256(sizeof(float) * 4 * T);
    w.removed = (uint64_t *)p; p += align256(sizeof(uint64_t) * sum_nb);
    w.strip = (uint64_t *)p; p += align256(sizeof(uint64_t) * strip_words);
    w.temp = p;
    w.temp_bytes = sort_temp_bound(T, G);
    return w;
}

inline int64_t work_bytes(int64_t T, int64_t sum_nb, int64_t strip_words, int G) {
    const NmsWork w = carve(nullptr, T, sum_nb, strip_words, G);
    return (int64_t)(w.temp - (char *)nullptr) + w.temp_bytes + 256;
}

__global__ void gather_kernel(const float *__restrict__ logits, const float *__restrict__ box,
                              const float *__restrict__ ref, const int32_t *__restrict__ counts,
                              const int64_t *__restrict__ unit_off,
                              const int32_t *__restrict__ seg_units,
                              const int64_t *__restrict__ cand_off, NmsWork w) {
    const int g = blockIdx.x;
    const int64_t off = cand_off[g];
    int64_t pos = off;
    for (int u = seg_units[g]; u < seg_units[g + 1]; ++u) {
        const int n = counts[u];
        if (n == 0) {
            if (threadIdx.x == 0) {
                w.s[pos] = 0.0f;
                w.b[4 * pos + 0] = 0.0f; w.b[4 * pos + 1] = 0.0f;
                w.b[4 * pos + 2] = 1e-14f; w.b[4 * pos + 3] = 1e-14f;
                w.r[2 * pos + 0] = 0.0f; w.r[2 * pos + 1] = 0.0f;
                w.idx[pos] = (int32_t)(pos - off);
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
            w.idx[pos + i] = (int32_t)(pos + i - off);
        }
        pos += n;
    }
}

// Boxes in sorted order, once per call: the strips then read rows and
// columns contiguously instead of through the order indirection.
__global__ void sort_boxes_kernel(const int64_t *__restrict__ cand_off, int G, NmsWork w) {
    const int g = blockIdx.y;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const int li = min(max(w.order[off + p], 0), n - 1);  // NaN-safe
        reinterpret_cast<float4 *>(w.sb)[off + p] = reinterpret_cast<const float4 *>(w.b)[off + li];
    }
}

// IoU words of row block ib = s*S + blockIdx.y (64 sorted rows, one per lane)
// x column blocks jb0 .. jb0 + NJ - 1 (those >= ib): bit k of word (i, jb) =
// IoU(row i, column jb*64 + k) > thr for columns after i.  A block of MW
// waves shares the row block: wave w computes column blocks jb0 + w, jb0 + w
// + MW, ... with the column boxes staged in LDS (read as broadcasts); the
// NJ words of each row are then written row-contiguously through an LDS
// transpose (8 rows x 64 B per store instruction instead of 64 scattered 8-B
// words per column block), and blocks wholly below the diagonal exit first.
constexpr int NJ = 8, MW = 4;

__global__ __launch_bounds__(64 * MW) void mask_strip_kernel(const int64_t *__restrict__ cand_off,
                                                             const int64_t *__restrict__ nb_off, double thr,
                                                             int64_t S, int64_t s, NmsWork w) {
    __shared__ float4 cb[NJ * 64];
    __shared__ float ca[NJ * 64];
    __shared__ uint64_t tw[64][NJ + 1];
    const int g = blockIdx.z;
    const int64_t ib = s * S + blockIdx.y;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    const int nb = (n + 63) / 64;
    const int jb0 = blockIdx.x * NJ;
    if (ib >= nb || jb0 >= nb || jb0 + NJ <= ib) return;  // block-uniform
    const int tid = threadIdx.x, t = tid & 63, wv = tid >> 6;
    const int jlo = max(jb0, (int)ib), jhi = min(jb0 + NJ, nb);  // column blocks of this block
    const float4 *sb = reinterpret_cast<const float4 *>(w.sb) + off;
    for (int e = tid; e < (jhi - jlo) * 64; e += 64 * MW) {
        const int j = jlo * 64 + e;
        if (j < n) {
            const float4 bj = sb[j];
            cb[e] = bj;
            ca[e] = (bj.z - bj.x) * (bj.w - bj.y);
        }
    }
    __syncthreads();
    const int i = (int)ib * 64 + t;
    const float4 bi = i < n ? sb[i] : float4{0.0f, 0.0f, 0.0f, 0.0f};
    const float ai = (bi.z - bi.x) * (bi.w - bi.y);
    for (int jb = jlo + wv; jb < jhi; jb += MW) {
        uint64_t bits = 0;
        const int kmax = min(64, n - jb * 64);
        const int kmin = jb == ib ? t + 1 : 0;  // columns after row i only
        const int base = (jb - jlo) * 64;
#pragma unroll 4
        for (int k = 0; k < kmax; ++k) {
            const float4 bj = cb[base + k];
            const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
            const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
            float ww = xx2 - xx1, hh = yy2 - yy1;
            ww = ww > 0.0f ? ww : 0.0f;
            hh = hh > 0.0f ? hh : 0.0f;
            const float inter = ww * hh;
            const float ovr = inter / (ai + ca[base + k] - inter);
            if (k >= kmin && (double)ovr > thr) bits |= (1ull << k);
        }
        tw[t][jb - jb0] = i < n ? bits : 0ull;
    }
    __syncthreads();
    // strip layout per image: [S*64 rows][nb words]; lanes (8 rows x 8 words)
    uint64_t *dst = w.strip + S * 64 * nb_off[g] + (int64_t)(blockIdx.y * 64) * nb;
    const int wq = t & 7, rq = t >> 3;
    const int jb = jb0 + wq;
    for (int r0 = 8 * wv; r0 < 64; r0 += 8 * MW) {
        const int r = r0 + rq;
        if (jb >= jlo && jb < jhi && (int)ib * 64 + r < n) dst[(int64_t)r * nb + jb] = tw[r][wq];
    }
}

// One block of RT threads per image.  Every wave resolves the block's greedy
// chain itself (the same 64 diagonal words and the same removed word, so the
// same kept mask, with no barrier to broadcast it); wave 0 writes the kept
// rows; the OR of the kept rows' words into the later column blocks -- the
// bulk of the work, (nb - ib) words per kept row -- is spread over all RT
// threads (one wave per image left 8 waves running chip-wide at config E).
constexpr int RT = 256;

__global__ __launch_bounds__(RT) void reduce_strip_kernel(const int64_t *__restrict__ cand_off,
                                                          const int64_t *__restrict__ nb_off, int64_t S,
                                                          int64_t s, NmsWork w, float *__restrict__ out_logits,
                                                          float *__restrict__ out_boxes,
                                                          float *__restrict__ out_refs,
                                                          int64_t *__restrict__ out_keep,
                                                          int32_t *__restrict__ kept_out) {
    extern __shared__ uint64_t removed[];
    const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const bool w0 = tid < 64;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    const int nb = (n + 63) / 64;
    const int64_t ib0 = s * S;
    if (ib0 >= nb) return;  // this image has no rows in the strip (block-uniform)
    uint64_t *grem = w.removed + nb_off[g];
    const uint64_t *mask = w.strip + S * 64 * nb_off[g];
    for (int k = tid; k < nb; k += RT) {
        if (s == 0) {
            const int rem = n - k * 64;
            removed[k] = rem >= 64 ? 0ull : ~((1ull << rem) - 1);  // rows past n never kept
        } else {
            removed[k] = grem[k];
        }
    }
    int cnt = s == 0 ? 0 : kept_out[g];
    __syncthreads();
    const int ib1 = (int)std::min<int64_t>(ib0 + S, nb);
    // the row block's diagonal words do not depend on the chain: each is
    // loaded one row block ahead, so its latency overlaps the previous
    // block's OR loads instead of opening every block
    uint64_t diag_next = (int)ib0 < ib1 && (int)ib0 * 64 + lane < n ? mask[(int64_t)lane * nb + ib0] : 0ull;
    for (int ib = (int)ib0; ib < ib1; ++ib) {
        const int i = ib * 64 + lane;
        const int64_t row = (int64_t)(ib - ib0) * 64;
        const uint64_t diag = diag_next;
        if (ib + 1 < ib1)
            diag_next = i + 64 < n ? mask[(row + 64 + lane) * nb + ib + 1] : 0ull;
        uint64_t word = removed[ib];
        uint64_t kept = 0;
        const uint32_t dlo = (uint32_t)diag, dhi = (uint32_t)(diag >> 32);
        // walk the surviving rows only (lowest first): each kept row's
        // diagonal word suppresses later rows of the block
        for (uint64_t avail = ~word; avail;) {
            const int bit = __builtin_ctzll(avail);
            kept |= 1ull << bit;
            const uint32_t lo = __builtin_amdgcn_readlane(dlo, bit);
            const uint32_t hi = __builtin_amdgcn_readlane(dhi, bit);
            word |= ((uint64_t)hi << 32) | lo;
            avail = bit == 63 ? 0ull : ~word & (~0ull << (bit + 1));
        }
        if (w0 && ((kept >> lane) & 1ull)) {
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
        // OR the kept rows' words into the later blocks: thread t gathers
        // column block ib+1+t (coalesced across lanes); the kept rows (a
        // block-uniform set) are walked 8 at a time so 8 independent loads
        // are in flight per wait instead of one load latency per kept row
        for (int k = ib + 1 + tid; k < nb; k += RT) {
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
                        v[t] = mask[(row + b) * nb + k];
                    }
                }
                acc |= ((v[0] | v[1]) | (v[2] | v[3])) | ((v[4] | v[5]) | (v[6] | v[7]));
            }
            removed[k] |= acc;
        }
        __syncthreads();
    }
    for (int k = tid; k < nb; k += RT) grem[k] = removed[k];
    if (tid == 0) kept_out[g] = cnt;
}

// Calls whose every image has at most SMALL_N candidates (the module API's
// one image of a few exemplars, demo.py:123-130): the whole NMS of an image
// in ONE workgroup -- gather, the stable descending sort as a rank count over
// rocprim's float key order (so the same order as the radix sort: -0.0 ==
// +0.0, ties by local index), the IoU words in LDS with mask_strip's
// arithmetic, and the greedy chain -- one launch instead of gather + sort
// + strips, no work buffer.  Same keep lists by construction.
constexpr int SMALL_N = TMR_NMS_SMALL;

__device__ __forceinline__ uint32_t radix_key(float f) {
    uint32_t b = __float_as_uint(f);
    if (b == 0x80000000u) b = 0u;  // rocprim's digit extractor: -0.0 sorts as +0.0
    return b ^ ((b & 0x80000000u) ? 0xffffffffu : 0x80000000u);
}

// one image's union (units u_beg..u_end-1, n <= SMALL_N rows) -> kept rows at
// out[off ...], kept_out[g]; one workgroup of SMALL_N threads
__device__ __forceinline__ void nms_small_image(
    const float *__restrict__ logits, const float *__restrict__ box, const float *__restrict__ ref,
    const int32_t *__restrict__ counts, const int64_t *__restrict__ unit_off, int u_beg, int u_end, int n,
    int64_t off, double thr, float *__restrict__ out_logits, float *__restrict__ out_boxes,
    float *__restrict__ out_refs, int64_t *__restrict__ out_keep, int32_t *__restrict__ kept_out, int g) {
    __shared__ float ss[SMALL_N];
    __shared__ float4 ub[SMALL_N];   // unit order
    __shared__ float2 ur[SMALL_N];
    __shared__ uint32_t key[SMALL_N];
    __shared__ int order[SMALL_N];   // sorted position -> local index
    __shared__ float4 sb[SMALL_N];   // sorted order
    __shared__ float sa[SMALL_N];
    __shared__ uint64_t mask[SMALL_N][SMALL_N / 64];
    const int tid = threadIdx.x;
    int pos = 0;
    for (int u = u_beg; u < u_end; ++u) {  // gather_kernel's union
        const int c = counts[u];
        if (c == 0) {
            if (tid == 0 && pos < n) {
                ss[pos] = 0.0f;
                ub[pos] = float4{0.0f, 0.0f, 1e-14f, 1e-14f};
                ur[pos] = float2{0.0f, 0.0f};
            }
            pos += 1;
            continue;
        }
        const size_t src = (size_t)unit_off[u];
        for (int i = tid; i < c && pos + i < n; i += SMALL_N) {  // (n from the host's counts)
            ss[pos + i] = logits[2 * (src + i)];
            ub[pos + i] = reinterpret_cast<const float4 *>(box)[src + i];
            ur[pos + i] = float2{ref[2 * (src + i) + 0], ref[2 * (src + i) + 1]};
        }
        pos += c;
    }
    __syncthreads();
    if (tid < n) key[tid] = radix_key(ss[tid]);
    __syncthreads();
    if (tid < n) {
        const uint32_t k = key[tid];
        int r = 0;
        for (int j = 0; j < n; ++j) {
            const uint32_t kj = key[j];
            r += (kj > k) | ((kj == k) & (j < tid));
        }
        order[r] = tid;
    }
    __syncthreads();
    if (tid < n) {
        const float4 b = ub[order[tid]];
        sb[tid] = b;
        sa[tid] = (b.z - b.x) * (b.w - b.y);
    }
    __syncthreads();
    const int nb = (n + 63) / 64;
    for (int t = tid; t < n * nb; t += SMALL_N) {  // word q of sorted row i
        const int i = t / nb, q = t - i * nb;
        const float4 bi = sb[i];
        const float ai = sa[i];
        uint64_t bits = 0;
        const int jhi = min(64, n - q * 64);
        for (int k = 0; k < jhi; ++k) {
            const int j = q * 64 + k;
            const float4 bj = sb[j];
            const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
            const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
            float ww = xx2 - xx1, hh = yy2 - yy1;
            ww = ww > 0.0f ? ww : 0.0f;
            hh = hh > 0.0f ? hh : 0.0f;
            const float inter = ww * hh;
            const float ovr = inter / (ai + sa[j] - inter);
            if (j > i && (double)ovr > thr) bits |= (1ull << k);
        }
        mask[i][q] = bits;
    }
    __syncthreads();
    if (tid < 64) {  // wave 0: lane q < nb holds word q of the removed bitmap
        uint64_t rem = 0;
        int cnt = 0;
        for (int i = 0; i < n; ++i) {
            const uint64_t mine = tid == (i >> 6) ? rem : 0ull;
            const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)mine, i >> 6);
            const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(mine >> 32), i >> 6);
            const uint64_t w = ((uint64_t)hi << 32) | lo;
            if ((w >> (i & 63)) & 1ull) continue;  // wave-uniform
            if (tid == 0) {
                const int li = order[i];
                const int64_t dst = off + cnt;
                out_logits[2 * dst + 0] = ss[li];
                out_logits[2 * dst + 1] = 0.0f;
                reinterpret_cast<float4 *>(out_boxes)[dst] = ub[li];
                out_refs[2 * dst + 0] = ur[li].x;
                out_refs[2 * dst + 1] = ur[li].y;
                if (out_keep) out_keep[dst] = li;
            }
            ++cnt;
            if (tid < nb) rem |= mask[i][tid];
        }
        if (tid == 0) kept_out[g] = cnt;
    }
}

__global__ __launch_bounds__(SMALL_N) void nms_small_kernel(
    const float *__restrict__ logits, const float *__restrict__ box, const float *__restrict__ ref,
    const int32_t *__restrict__ counts, const int64_t *__restrict__ unit_off,
    const int32_t *__restrict__ seg_units, const int64_t *__restrict__ cand_off, double thr,
    float *__restrict__ out_logits, float *__restrict__ out_boxes, float *__restrict__ out_refs,
    int64_t *__restrict__ out_keep, int32_t *__restrict__ kept_out) {
    const int g = blockIdx.x;
    const int64_t off = cand_off[g];
    const int n = min((int)(cand_off[g + 1] - off), SMALL_N);
    nms_small_image(logits, box, ref, counts, unit_off, seg_units[g], seg_units[g + 1], n, off, thr,
                    out_logits, out_boxes, out_refs, out_keep, kept_out, g);
}

// The same with the union sizes taken from the DEVICE counts (no host sync
// first): image g's rows go to g * SMALL_N; an image whose union exceeds
// SMALL_N rows gets kept[g] = -1 and is left to tmr_nms.
__global__ __launch_bounds__(SMALL_N) void nms_small_dev_kernel(
    const float *__restrict__ logits, const float *__restrict__ box, const float *__restrict__ ref,
    const int32_t *__restrict__ counts, const int64_t *__restrict__ unit_off,
    const int32_t *__restrict__ seg_units, double thr, float *__restrict__ out_logits,
    float *__restrict__ out_boxes, float *__restrict__ out_refs, int64_t *__restrict__ out_keep,
    int32_t *__restrict__ kept_out) {
    const int g = blockIdx.x;
    const int u_beg = seg_units[g], u_end = seg_units[g + 1];
    int64_t n = 0;
    for (int u = u_beg; u < u_end; ++u) n += max(counts[u], 1);  // (block-uniform)
    if (n > SMALL_N) {
        if (threadIdx.x == 0) kept_out[g] = -1;
        return;
    }
    nms_small_image(logits, box, ref, counts, unit_off, u_beg, u_end, (int)n, (int64_t)g * SMALL_N, thr,
                    out_logits, out_boxes, out_refs, out_keep, kept_out, g);
}

}  // namespace

extern "C" int64_t tmr_nms_work_size(int64_t total_cand, int64_t sum_nb, int64_t max_cand, int G) {
    if (total_cand < 0 || sum_nb < 0 || max_cand < 0 || G <= 0) return -1;
    int64_t S, words;
    strip_plan(sum_nb, (max_cand + 63) / 64, S, words);
    return work_bytes(total_cand, sum_nb, words, G);
}

extern "C" int tmr_nms_small(const float *logits, const float *box, const float *ref, const int32_t *counts,
                             const int64_t *unit_off, const int32_t *seg_units, int G, double iou_threshold,
                             float *out_logits, float *out_boxes, float *out_refs, int64_t *out_keep,
                             int32_t *kept, void *stream) {
    TMR_REQUIRE(logits && box && ref && counts && unit_off && seg_units && out_logits && out_boxes && out_refs);
    TMR_REQUIRE(kept && G > 0 && G < 65536);
    hipLaunchKernelGGL(nms_small_dev_kernel, dim3(G), dim3(SMALL_N), 0, tmr_stream(stream), logits, box, ref,
                       counts, unit_off, seg_units, iou_threshold, out_logits, out_boxes, out_refs, out_keep,
                       kept);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}

extern "C" int tmr_nms(const float *logits, const float *box, const float *ref,
                       const int32_t *counts, const int64_t *unit_off, const int32_t *seg_units,
                       const int64_t *cand_off, const int64_t *nb_off, int G,
                       int64_t total_cand, int64_t max_cand, int64_t sum_nb, double iou_threshold,
                       float *out_logits, float *out_boxes, float *out_refs, int64_t *out_keep,
                       int32_t *kept, void *work, void *stream) {
    TMR_REQUIRE(logits && box && ref && counts && unit_off && seg_units && cand_off && nb_off);
    TMR_REQUIRE(work && out_logits && out_boxes && out_refs && kept && G > 0);
    TMR_REQUIRE(total_cand >= G && max_cand >= 1 && sum_nb >= G);
    TMR_REQUIRE(total_cand < (1ll << 31));
    const int64_t max_nb = (max_cand + 63) / 64;
    TMR_REQUIRE(max_nb < (1 << 20) && G < 65536);
    TMR_REQUIRE(max_nb * 8 <= 150 * 1024);  // the removed bitmap in LDS
    hipStream_t s = tmr_stream(stream);
    if (max_cand <= SMALL_N) {  // every image fits one workgroup
        hipLaunchKernelGGL(nms_small_kernel, dim3(G), dim3(SMALL_N), 0, s, logits, box, ref, counts, unit_off,
                           seg_units, cand_off, iou_threshold, out_logits, out_boxes, out_refs, out_keep, kept);
        TMR_CHECK_LAUNCH();
        return TMR_OK;
    }
    int64_t S, strip_words;
    strip_plan(sum_nb, max_nb, S, strip_words);
    NmsWork w = carve(work, total_cand, sum_nb, strip_words, G);
    hipLaunchKernelGGL(gather_kernel, dim3(G), dim3(256), 0, s, logits, box, ref, counts, unit_off,
                       seg_units, cand_off, w);
    TMR_CHECK_LAUNCH();
    size_t tb = 0;
    if (rocprim::segmented_radix_sort_pairs_desc(nullptr, tb, w.s, w.skeys, w.idx, w.order,
                                                 (unsigned)total_cand, (unsigned)G, cand_off, cand_off + 1,
                                                 0, 32, s) != hipSuccess)
        return TMR_E_HIP;
    if ((int64_t)tb > w.temp_bytes) return TMR_E_INVALID;
    if (rocprim::segmented_radix_sort_pairs_desc(w.temp, tb, w.s, w.skeys, w.idx, w.order,
                                                 (unsigned)total_cand, (unsigned)G, cand_off, cand_off + 1,
                                                 0, 32, s) != hipSuccess)
        return TMR_E_HIP;
    const size_t lds = sizeof(uint64_t) * (size_t)max_nb;
    auto rk = reduce_strip_kernel;
    if (lds > 64 * 1024 &&
        tmr_set_max_lds((const void *)rk, lds) !=
            hipSuccess)
        return TMR_E_HIP;
    hipLaunchKernelGGL(sort_boxes_kernel, dim3((unsigned)std::min<int64_t>(tmr_cdiv(max_cand, 256), 1024), G),
                       dim3(256), 0, s, cand_off, G, w);
    TMR_CHECK_LAUNCH();
    for (int64_t st = 0; st * S < max_nb; ++st) {
        hipLaunchKernelGGL(mask_strip_kernel, dim3((unsigned)tmr_cdiv(max_nb, NJ), (unsigned)S, G), dim3(64 * MW), 0, s,
                           cand_off, nb_off, iou_threshold, S, st, w);
        TMR_CHECK_LAUNCH();
        hipLaunchKernelGGL(rk, dim3(G), dim3(RT), lds, s, cand_off, nb_off, S, st, w, out_logits, out_boxes,
                           out_refs, out_keep, kept);
        TMR_CHECK_LAUNCH();
    }
    return TMR_OK;
}
