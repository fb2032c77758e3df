// Per-image greedy NMS over the exemplar-ordered candidate union (gfx950).
// Reference: NMS / NMS_process (utils/TM_utils.py:307-323) ->
// torchvision.ops.nms (0.19 CPU semantics: stable descending score order,
// fp32 IoU, `(double)ovr > iou_threshold`), applied after the per-exemplar
// Get_pred_boxes results are concatenated (demo.py:123-130,
// trainer.py:111-118), dummy rows included (TM_utils.py:288-291).
//
//   gather : union per image in unit order (dummy row for an empty unit)
//            + the local index of every row
//   sort   : ONE device-wide rocprim radix sort of (image, score) keys --
//            the image in the high bits, the score's descending radix key
//            below -- with the local index as value: stable, so ties keep the
//            lower index first, as torchvision's stable sort (a segmented
//            sort of a few large images ran a workgroup per image: 0.75 ms
//            at config E)
//   bins   : the sorted boxes are binned by their top-left corner on a
//            per-image grid (<= 64 x 64 cells); two boxes can only overlap
//            (and so only suppress, for iou_threshold >= 0) when each one's
//            corner lies within the other's extent + the image's largest box
//            extent, so a box's partners are found in a small window of cells
//   pairs  : one thread per box, in cell order (neighbours in a wave scan the
//            same cells): the exact IoU against the boxes of its window that
//            are in earlier 64-row blocks (its possible suppressors: a list of
//            up to CAP) or later in its own block (a diagonal word)
//   greedy : one wave per image walks the 64-row blocks in score order: a row
//            is removed when a listed suppressor is in the kept bitmap (LDS),
//            then the block's chain is resolved from the diagonal words in
//            registers (a row with more than CAP suppressors, none listed kept,
//            rescans its window).  Memory is O(candidates); the work is the
//            spatial pairs, not n^2/2 (round 4's dense strips: 4.3e9 IoU
//            pairs per config-E step, 2.9 ms of mask + 2.0 ms of strip
//            reduction).  The keep list equals the sequential torchvision
//            loop: IoU(i, j) is evaluated with the same expression, pairs
//            outside a window have no intersection (ovr = 0 or NaN, never
//            > a threshold >= 0), and suppression only flows from kept rows.
//            A negative threshold or a non-finite box puts the image in ONE
//            cell (every pair evaluated).
// Built with -ffp-contract=off.
#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>

#include "tmr_common.h"

namespace {

// rocprim's temporary storage beyond its key/value double buffers
constexpr int64_t SORT_SLACK = 1 << 20;
constexpr int GB = 64;            // bins per axis (at most)
constexpr int NCELL = GB * GB;
constexpr int CAP = 128;          // listed earlier-block suppressors per row (config E: p99 68, max ~100;
                                  // at 96 the overflow rescans cost 0.24 ms of 1.42, profiles/r05m)
constexpr int LUNR = 32;          // list entries tested per step of the greedy (CAP % LUNR == 0)

struct BinHdr {
    float x0, y0, icx, icy, wmax, hmax;
    float tq;  // the threshold the windows are narrowed by (0: overlap only)
    int gx, gy;
};

struct NmsWork {
    float *s;        // [T] scores (unit order)
    uint64_t *key;   // [T] (image << 32) | descending score key
    uint64_t *skey;  // [T] sorted keys (unused beyond the sort)
    float *b;        // [T][4]
    float *r;        // [T][2]
    int32_t *idx;    // [T] local row index (sort values in)
    int32_t *order;  // [T] sorted position -> local index
    float *sb;       // [T][4] boxes in sorted order
    BinHdr *hdr;     // [G]
    int32_t *cnt;    // [G][NCELL] per-cell counts, then fill cursors
    int32_t *cst;    // [G][NCELL + 1] cell starts (local)
    int32_t *clist;  // [T] sorted positions in cell order
    float *cbox;     // [T][4] their boxes
    uint64_t *diag;  // [T] in-block suppression word of each sorted row (later rows it suppresses)
    int32_t *lcnt;   // [T] earlier-block suppressors of each sorted row
    uint64_t *keptw; // [sum_nb] kept word of each 64-row block
    int32_t *kbase;  // [sum_nb] kept rows before each block
    int32_t *lst;    // [sum_nb][CAP][64] the first CAP of them found (sorted positions),
                     // per 64-row block entry-major: entry e of row i at
                     // ((nb_off[g] + i/64) * CAP + e) * 64 + i%64
    char *temp;      // rocprim temporary storage
    int64_t temp_bytes;
    int64_t lbuf_words;  // greedy_kernel: 64-bit words of LDS before its list buffers
};

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// rocprim's radix sort keeps its own key + value double buffers in the
// temporary storage (12 B per candidate) beside its histograms
inline int64_t sort_temp_bound(int64_t T, int G) { return 16 * T + SORT_SLACK + 64 * (int64_t)(G + 1); }

inline NmsWork carve(void *work, int64_t T, int64_t sum_nb, int G) {
    NmsWork w;
    char *p = (char *)work;
    w.s = (float *)p; p += align256(sizeof(float) * T);
    w.key = (uint64_t *)p; p += align256(sizeof(uint64_t) * T);
    w.skey = (uint64_t *)p; p += align256(sizeof(uint64_t) * T);
    w.b = (float *)p; p += align256(sizeof(float) * 4 * T);
    w.r = (float *)p; p += align256(sizeof(float) * 2 * T);
    w.idx = (int32_t *)p; p += align256(sizeof(int32_t) * T);
    w.order = (int32_t *)p; p += align256(sizeof(int32_t) * T);
    w.sb = (float *)p; p += align256(sizeof(float) * 4 * T);
    w.hdr = (BinHdr *)p; p += align256(sizeof(BinHdr) * G);
    w.cnt = (int32_t *)p; p += align256(sizeof(int32_t) * NCELL * (size_t)G);
    w.cst = (int32_t *)p; p += align256(sizeof(int32_t) * (NCELL + 1) * (size_t)G);
    w.clist = (int32_t *)p; p += align256(sizeof(int32_t) * T);
    w.cbox = (float *)p; p += align256(sizeof(float) * 4 * T);
    w.diag = (uint64_t *)p; p += align256(sizeof(uint64_t) * T);
    w.lcnt = (int32_t *)p; p += align256(sizeof(int32_t) * T);
    w.keptw = (uint64_t *)p; p += align256(sizeof(uint64_t) * sum_nb);
    w.kbase = (int32_t *)p; p += align256(sizeof(int32_t) * sum_nb);
    w.lst = (int32_t *)p; p += align256(sizeof(int32_t) * CAP * 64 * sum_nb);
    w.temp = p;
    w.temp_bytes = sort_temp_bound(T, G);
    return w;
}

inline int64_t work_bytes(int64_t T, int64_t sum_nb, int G) {
    const NmsWork w = carve(nullptr, T, sum_nb, G);
    return (int64_t)(w.temp - (char *)nullptr) + w.temp_bytes + 256;
}

// Ascending float order as torch.sort compares (descending = its complement):
// -0.0 == +0.0, and every NaN, of either sign and any payload, above +inf and
// equal to each other -- so the stable descending sort puts NaN scores first
// in index order, as scores.sort(stable=True, descending=True) in
// torchvision's nms_kernel.cpp does.
__device__ __forceinline__ uint32_t radix_key(float f) {
    uint32_t b = __float_as_uint(f);
    if (f != f) return 0xffffffffu;
    if (b == 0x80000000u) b = 0u;
    return b ^ ((b & 0x80000000u) ? 0xffffffffu : 0x80000000u);
}

// the sort key of candidate (image g, score f): images ascending, scores
// descending in rocprim's float key order
__device__ __forceinline__ uint64_t sort_key(int g, float f) {
    return ((uint64_t)(uint32_t)g << 32) | (uint64_t)(~radix_key(f));
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
                w.key[pos] = sort_key(g, 0.0f);
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
            const float sc = logits[2 * (src + i)];
            w.s[pos + i] = sc;
            w.key[pos + i] = sort_key(g, sc);
            const float4 bb = reinterpret_cast<const float4 *>(box)[src + i];
            reinterpret_cast<float4 *>(w.b)[pos + i] = bb;
            w.r[2 * (pos + i) + 0] = ref[2 * (src + i) + 0];
            w.r[2 * (pos + i) + 1] = ref[2 * (src + i) + 1];
            w.idx[pos + i] = (int32_t)(pos + i - off);
        }
        pos += n;
    }
}

// Boxes in sorted order, once per call: the bins and pairs then read rows
// contiguously instead of through the order indirection.
__global__ void sort_boxes_kernel(const int64_t *__restrict__ cand_off, int G, NmsWork w) {
    const int g = blockIdx.y;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const int li = min(max(w.order[off + p], 0), n - 1);  // NaN-safe
        reinterpret_cast<float4 *>(w.sb)[off + p] = reinterpret_cast<const float4 *>(w.b)[off + li];
    }
}

// the IoU test of torchvision's CPU kernel (fp32 IoU, `(double)ovr > thr`);
// with `prune` (thr >= 0) a pair without intersection is decided without
// the division: ovr is then 0 or NaN, never > thr
__device__ __forceinline__ bool iou_over(float4 bi, float ai, float4 bj, float aj, double thr, bool prune) {
    const float xx1 = fmaxf(bi.x, bj.x), yy1 = fmaxf(bi.y, bj.y);
    const float xx2 = fminf(bi.z, bj.z), yy2 = fminf(bi.w, bj.w);
    float ww = xx2 - xx1, hh = yy2 - yy1;
    ww = ww > 0.0f ? ww : 0.0f;
    hh = hh > 0.0f ? hh : 0.0f;
    const float inter = ww * hh;
    if (prune && !(inter > 0.0f)) return false;
    const float ovr = inter / (ai + aj - inter);
    return (double)ovr > thr;
}

__device__ __forceinline__ float box_area(float4 b) { return (b.z - b.x) * (b.w - b.y); }

// per image: the grid over the boxes' top-left corners (x1, y1).  Cells are
// at least 2^-16 of the coordinates' magnitude wide, so the one-cell slack of
// the windows covers the fp32 rounding of the cell arithmetic; a non-finite
// coordinate or a negative threshold gives one cell (every pair evaluated).
__global__ __launch_bounds__(256) void bin_setup_kernel(const int64_t *__restrict__ cand_off, double thr,
                                                        NmsWork w) {
    __shared__ float red[8][4];
    __shared__ int bad[4];
    const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    const float4 *sb = reinterpret_cast<const float4 *>(w.sb) + off;
    // x1 min, y1 min, x1 max, y1 max, w max, h max, w min, h min
    float v[8] = {INFINITY, INFINITY, -INFINITY, -INFINITY, 0.0f, 0.0f, INFINITY, INFINITY};
    int nf = 0;
    for (int p = tid; p < n; p += 256) {
        const float4 bb = sb[p];
        nf |= !(isfinite(bb.x) && isfinite(bb.y) && isfinite(bb.z) && isfinite(bb.w));
        v[0] = fminf(v[0], bb.x); v[1] = fminf(v[1], bb.y);
        v[2] = fmaxf(v[2], bb.x); v[3] = fmaxf(v[3], bb.y);
        v[4] = fmaxf(v[4], bb.z - bb.x); v[5] = fmaxf(v[5], bb.w - bb.y);
        v[6] = fminf(v[6], bb.z - bb.x); v[7] = fminf(v[7], bb.w - bb.y);
    }
    for (int o = 32; o > 0; o >>= 1) {
        v[0] = fminf(v[0], __shfl_xor(v[0], o)); v[1] = fminf(v[1], __shfl_xor(v[1], o));
        v[2] = fmaxf(v[2], __shfl_xor(v[2], o)); v[3] = fmaxf(v[3], __shfl_xor(v[3], o));
        v[4] = fmaxf(v[4], __shfl_xor(v[4], o)); v[5] = fmaxf(v[5], __shfl_xor(v[5], o));
        v[6] = fminf(v[6], __shfl_xor(v[6], o)); v[7] = fminf(v[7], __shfl_xor(v[7], o));
        nf |= __shfl_xor(nf, o);
    }
    if (lane == 0) {
        for (int k = 0; k < 8; ++k) red[k][wv] = v[k];
        bad[wv] = nf;
    }
    __syncthreads();
    if (tid != 0) return;
    for (int q = 1; q < 4; ++q) {
        v[0] = fminf(v[0], red[0][q]); v[1] = fminf(v[1], red[1][q]);
        v[2] = fmaxf(v[2], red[2][q]); v[3] = fmaxf(v[3], red[3][q]);
        v[4] = fmaxf(v[4], red[4][q]); v[5] = fmaxf(v[5], red[5][q]);
        v[6] = fminf(v[6], red[6][q]); v[7] = fminf(v[7], red[7][q]);
        nf |= bad[q];
    }
    BinHdr h;
    h.x0 = v[0]; h.y0 = v[1];
    h.wmax = v[4]; h.hmax = v[5];
    h.gx = h.gy = 1;
    h.icx = h.icy = 0.0f;
    // IoU > t needs |x1_i - x1_j| < (1 - t) max(w_i, w_j) and w_j < w_i / t
    // (window()); that bound holds for the fp32 IoU too while no area or
    // intersection can underflow or overflow to change the quotient by more
    // than 2^-16 of t: box sides in [2^-60, 2^60], corners below 2^60 and
    // t >= 2^-12.  Otherwise the windows bound overlap only (exact for fp32).
    const bool narrow = thr >= 0x1p-12 && v[6] >= 0x1p-60f && v[7] >= 0x1p-60f && v[4] <= 0x1p60f &&
                        v[5] <= 0x1p60f && fmaxf(fabsf(v[0]), fabsf(v[2])) <= 0x1p60f &&
                        fmaxf(fabsf(v[1]), fabsf(v[3])) <= 0x1p60f;
    h.tq = narrow ? (float)thr * (1.0f - 0x1p-16f) : 0.0f;
    if (!nf && thr >= 0.0 && n > 0) {
        const float rx = v[2] - v[0], ry = v[3] - v[1];
        const float mx = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[2])), 1e-30f);
        const float my = fmaxf(fmaxf(fabsf(v[1]), fabsf(v[3])), 1e-30f);
        const float minc_x = mx * 0x1p-16f, minc_y = my * 0x1p-16f;
        h.gx = rx > 0.0f ? (int)fminf((float)GB, fmaxf(1.0f, floorf(rx / minc_x))) : 1;
        h.gy = ry > 0.0f ? (int)fminf((float)GB, fmaxf(1.0f, floorf(ry / minc_y))) : 1;
        h.icx = rx > 0.0f ? (float)h.gx / rx : 0.0f;
        h.icy = ry > 0.0f ? (float)h.gy / ry : 0.0f;
    }
    w.hdr[g] = h;
}

__device__ __forceinline__ int cell_of(float v, float v0, float ic, int gn) {
    const float c = floorf((v - v0) * ic);
    if (!(c >= 0.0f)) return 0;  // (below the grid, or NaN)
    return c >= (float)(gn - 1) ? gn - 1 : (int)c;
}

// per sorted box: its cell; counting pass (MODE 0) or the fill (MODE 1)
template <int MODE>
__global__ void bin_kernel(const int64_t *__restrict__ cand_off, NmsWork w) {
    const int g = blockIdx.y;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    const BinHdr h = w.hdr[g];
    int32_t *cnt = w.cnt + (size_t)g * NCELL;
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const float4 bb = reinterpret_cast<const float4 *>(w.sb)[off + p];
        const int c = cell_of(bb.y, h.y0, h.icy, h.gy) * h.gx + cell_of(bb.x, h.x0, h.icx, h.gx);
        if (MODE == 0) {
            atomicAdd(cnt + c, 1);
        } else {
            const int e = w.cst[(size_t)g * (NCELL + 1) + c] + atomicAdd(cnt + c, 1);
            w.clist[off + e] = p;
            reinterpret_cast<float4 *>(w.cbox)[off + e] = bb;
        }
    }
}

// exclusive scan of the cell counts per image (one block per image); the
// counts are reset to 0 for the fill's cursors
__global__ __launch_bounds__(256) void bin_scan_kernel(NmsWork w) {
    __shared__ int part[256];
    const int g = blockIdx.x, tid = threadIdx.x;
    int32_t *cnt = w.cnt + (size_t)g * NCELL;
    int32_t *cst = w.cst + (size_t)g * (NCELL + 1);
    constexpr int PER = NCELL / 256;
    int loc[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        loc[k] = cnt[tid * PER + k];
        sum += loc[k];
    }
    part[tid] = sum;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // Hillis-Steele inclusive scan
        const int t = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += t;
        __syncthreads();
    }
    int run = part[tid] - sum;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        cst[tid * PER + k] = run;
        run += loc[k];
        cnt[tid * PER + k] = 0;
    }
    if (tid == 255) cst[NCELL] = part[255];
}

// the cells a box's partners can lie in: with t = hdr.tq,
//   x1_j in (x1_i - f min(wmax, w_i / t), x1_i + f w_i),  f = 1 - t (+ 2^-16)
// (IoU > t: the intersection is wider than t w_i and t w_j, so w_j < w_i / t
// and |x1_i - x1_j| < (1 - t) max(w_i, w_j)); t = 0 is plain overlap,
// x1_j in (x1_i - wmax, x2_i).  y likewise; one cell of slack each way.
// Config E: 2680 -> 802 boxes per window at t = 0.5 (profiles/r05g dumps).
__device__ __forceinline__ void window(const BinHdr &h, float4 bi, int &ax0, int &ax1, int &ay0, int &ay1) {
    if (h.gx == 1 && h.gy == 1) {
        ax0 = ax1 = ay0 = ay1 = 0;
        return;
    }
    const float f = (1.0f - h.tq) + 0x1p-16f;
    const float bw = bi.z - bi.x, bh = bi.w - bi.y;
    const float mw = h.tq > 0.0f ? fminf(h.wmax, bw / h.tq) : h.wmax;
    const float mh = h.tq > 0.0f ? fminf(h.hmax, bh / h.tq) : h.hmax;
    ax0 = max(cell_of(bi.x - f * mw, h.x0, h.icx, h.gx) - 1, 0);
    ax1 = min(cell_of(bi.x + f * bw, h.x0, h.icx, h.gx) + 1, h.gx - 1);
    ay0 = max(cell_of(bi.y - f * mh, h.y0, h.icy, h.gy) - 1, 0);
    ay1 = min(cell_of(bi.y + f * bh, h.y0, h.icy, h.gy) + 1, h.gy - 1);
    if (!(bw >= 0.0f)) { ax0 = 0; ax1 = h.gx - 1; }  // inverted / NaN extents: the whole row of cells
    if (!(bh >= 0.0f)) { ay0 = 0; ay1 = h.gy - 1; }
}

__device__ __forceinline__ float rdl(float v, int q) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), q));
}

// One thread per box of image blockIdx.y, taken in cell order, and the
// window scanned per WAVE: the 64 rows of a wave lie in a few neighbouring
// cells of one grid row, so the wave walks the union of their windows once.
// The entries of each window row come 64 at a time by one coalesced load
// (lane l holds entry eb + l) and are broadcast by readlane, so the loads of
// a batch are in flight together (one scalar load per entry had left the
// kernel waiting on their latency: 2.9 ms at config E, profiles/r05f).  Every
// lane tests each entry against its own row.  The lanes of a wave that spans
// grid rows are taken one grid row at a time.
__global__ __launch_bounds__(256) void pairs_kernel(const int64_t *__restrict__ cand_off,
                                                    const int64_t *__restrict__ nb_off, double thr, NmsWork w) {
    const int g = blockIdx.y;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (__builtin_amdgcn_readfirstlane(k) >= n) return;  // whole waves past the image
    const int lane = threadIdx.x & 63;
    const bool live = k < n;
    const BinHdr h = w.hdr[g];
    const bool prune = thr >= 0.0;
    const int i = live ? w.clist[off + k] : 0;
    const float4 bi = live ? reinterpret_cast<const float4 *>(w.sb)[off + i] : float4{0.0f, 0.0f, 0.0f, 0.0f};
    const float ai = box_area(bi);
    const int blk0 = i & ~63, blk1 = blk0 + 64;  // this row's 64-row block
    const int32_t *__restrict__ cst = w.cst + (size_t)g * (NCELL + 1);
    const int32_t *__restrict__ cl = w.clist + off;
    const float4 *__restrict__ cb = reinterpret_cast<const float4 *>(w.cbox) + off;
    // entry e of this row's list at lst[e * 64]
    int32_t *__restrict__ lst = w.lst + (size_t)(nb_off[g] + (i >> 6)) * CAP * 64 + (i & 63);
    uint64_t diag = 0;
    int cnt = 0;
    int ax0 = 0, ax1 = -1, ay0 = 0, ay1 = -1;
    if (live) window(h, bi, ax0, ax1, ay0, ay1);
    // the grid row of each lane's own cell (the grouping key)
    const int myrow = live ? cell_of(bi.y, h.y0, h.icy, h.gy) : -1;
    uint64_t todo = __ballot(live);
    while (todo) {
        const int lead = __builtin_ctzll(todo);
        const int grp = __shfl(myrow, lead);
        const bool in = live && myrow == grp;
        todo &= ~__ballot(in);
        // the group's union window (wave-uniform)
        int x0 = in ? ax0 : 1 << 30, x1 = in ? ax1 : -1, y0 = in ? ay0 : 1 << 30, y1 = in ? ay1 : -1;
        for (int o = 32; o > 0; o >>= 1) {
            x0 = min(x0, __shfl_xor(x0, o)); x1 = max(x1, __shfl_xor(x1, o));
            y0 = min(y0, __shfl_xor(y0, o)); y1 = max(y1, __shfl_xor(y1, o));
        }
        x0 = __builtin_amdgcn_readfirstlane(x0); x1 = __builtin_amdgcn_readfirstlane(x1);
        y0 = __builtin_amdgcn_readfirstlane(y0); y1 = __builtin_amdgcn_readfirstlane(y1);
        for (int ay = y0; ay <= y1; ++ay) {
            const bool rowin = in && ay >= ay0 && ay <= ay1;
            if (!__ballot(rowin)) continue;
            const int e0 = __builtin_amdgcn_readfirstlane(cst[ay * h.gx + x0]);
            const int e1 = __builtin_amdgcn_readfirstlane(cst[ay * h.gx + x1 + 1]);
            for (int eb = e0; eb < e1; eb += 64) {
                const int el = eb + lane;
                int jl = 0;
                float4 bl = float4{0.0f, 0.0f, 0.0f, 0.0f};
                if (el < e1) {
                    jl = cl[el];
                    bl = cb[el];
                }
                const int nq = min(64, e1 - eb);
                for (int q = 0; q < nq; ++q) {  // wave-uniform entry
                    const int j = __builtin_amdgcn_readlane(jl, q);
                    const float4 bj = float4{rdl(bl.x, q), rdl(bl.y, q), rdl(bl.z, q), rdl(bl.w, q)};
                    // earlier blocks: j may suppress i; later rows of this block: i may
                    // suppress j (the chain); the rest is the other row's business
                    if (!rowin || j >= blk1 || (j >= blk0 && j <= i)) continue;
                    if (!iou_over(bi, ai, bj, box_area(bj), thr, prune)) continue;
                    if (j > i) {
                        diag |= 1ull << (j & 63);
                    } else {
                        if (cnt < CAP) lst[cnt * 64] = j;
                        ++cnt;
                    }
                }
            }
        }
    }
    if (live) {
        w.diag[off + i] = diag;
        w.lcnt[off + i] = cnt;
    }
}

// One wave per image: the greedy pass over the 64-row blocks in score order.
// A row is removed when one of its earlier-block suppressors was kept (a
// bitmap of the kept rows in LDS; each lane tests its own row's list, LDS
// reads, no scatter), then the block's chain is resolved from the diagonal
// words.  A block's lists (CAP x 64 entries, entry-major, so lane r reads
// column r conflict free), diagonal words and list counts arrive in LDS by
// buffer-to-LDS DMA GP blocks ahead into GP slots, so the wave's serial path
// waits on no memory latency (the kept rows, once written inside the loop,
// put two dependent global loads on every block: 1.83 -> 1.58 ms at config
// E without them; a third block of look-ahead measured 1.58 -> 1.46).  The DMA count per block is fixed, so one
// s_waitcnt vmcnt(N) waits for exactly the block about to be read.  A row
// with more than CAP earlier suppressors, none of its listed ones kept, is
// settled by the wave rescanning its window (rare).
typedef __attribute__((address_space(3))) void *lds_ptr_t;
constexpr int LBLK = CAP * 64;                  // list entries per 64-row block
constexpr int GP = 2;                           // look-ahead (blocks) = slots
constexpr int SLOT_W = LBLK + 128 + 64;         // int32 words per slot: lists, 64 diag words, 64 counts
constexpr int DMA_PER_BLOCK = CAP / 4 + 3;      // 1-KB list pieces + 2 diag + 1 count instructions
static_assert(CAP % LUNR == 0 && CAP % 4 == 0, "list steps and 1-KB DMA pieces");
static_assert((GP - 1) * DMA_PER_BLOCK <= 63, "vmcnt range");

__device__ __forceinline__ void block_dma(__amdgpu_buffer_rsrc_t rl, __amdgpu_buffer_rsrc_t rd,
                                          __amdgpu_buffer_rsrc_t rc, int32_t *slot, int ib, int lane) {
#pragma unroll
    for (int q = 0; q < CAP / 4; ++q)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rl, (lds_ptr_t)(slot + q * 256), 16, lane * 16,
                                                 (uint32_t)ib * (LBLK * 4) + q * 1024, 0, 0);
    // rows past the image read out of range: zero (and masked anyway)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (lds_ptr_t)(slot + LBLK), 4, lane * 4, (uint32_t)ib * 512, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (lds_ptr_t)(slot + LBLK + 64), 4, lane * 4,
                                             (uint32_t)ib * 512 + 256, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (lds_ptr_t)(slot + LBLK + 128), 4, lane * 4, (uint32_t)ib * 256, 0,
                                             0);
}

__global__ __launch_bounds__(64) void greedy_kernel(const int64_t *__restrict__ cand_off,
                                                    const int64_t *__restrict__ nb_off, double thr, NmsWork w,
                                                    int32_t *__restrict__ kept_out) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long keptb[];  // [lbuf_words], then GP slots
    const int g = blockIdx.x, lane = threadIdx.x;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    const int nb = (n + 63) / 64;
    int32_t *slots = reinterpret_cast<int32_t *>(keptb + w.lbuf_words);  // [GP][SLOT_W], 16-B aligned
    const int zw = (int)w.lbuf_words - 1;  // a word that stays zero (past the kept bitmap)
    const uint32_t *kept32 = reinterpret_cast<const uint32_t *>(keptb);
    if (lane == 0) keptb[zw] = 0ull;
    const BinHdr h = w.hdr[g];
    const bool prune = thr >= 0.0;
    const int32_t *cst = w.cst + (size_t)g * (NCELL + 1);
    const int32_t *cl = w.clist + off;
    const float4 *cb = reinterpret_cast<const float4 *>(w.cbox) + off;
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(w.lst + (size_t)nb_off[g] * LBLK), (short)0, (int)((size_t)nb * LBLK * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc((void *)(w.diag + off), (short)0, (int)((size_t)n * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t rc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(w.lcnt + off), (short)0, (int)((size_t)n * 4), 0x00020000);
    int cnt = 0;
    for (int q = 0; q < GP && q < nb; ++q) block_dma(rl, rd, rc, slots + q * SLOT_W, q, lane);
    for (int ib = 0; ib < nb; ++ib) {
        const int i = ib * 64 + lane;
        // block ib's DMA is done once at most the later blocks' are in flight
        if (ib + GP <= nb)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((GP - 1) * DMA_PER_BLOCK) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int32_t *slot = slots + (ib % GP) * SLOT_W;
        const uint64_t diag = i < n ? reinterpret_cast<const uint64_t *>(slot + LBLK)[lane] : 0ull;
        const int lc = i < n ? slot[LBLK + 128 + lane] : 0;
        // removed by a kept earlier-block suppressor?  LUNR list entries per
        // step, all LDS reads unconditional so they are in flight together
        // (e0 + LUNR <= CAP whenever e0 < m <= CAP; an entry past the count
        // reads the always-zero word keptb[zw])
        const int32_t *lb = slot + lane;
        const int m = min(lc, CAP);
        uint32_t rem32 = 0;
        for (int e0 = 0; __ballot(!rem32 && e0 < m); e0 += LUNR) {
            int jj[LUNR];
#pragma unroll
            for (int t = 0; t < LUNR; ++t) jj[t] = lb[(e0 + t) * 64];
#pragma unroll
            for (int t = 0; t < LUNR; ++t) {
                const int j = e0 + t < m ? jj[t] : zw * 64;
                rem32 |= (kept32[j >> 5] >> (j & 31)) & 1u;  // 32-bit halves: 4-B reads
            }
        }
        bool rem = rem32 != 0;
        // more suppressors than listed and none of the listed kept: rescan
        for (uint64_t ovf = __ballot(i < n && lc > CAP && !rem); ovf; ovf &= ovf - 1) {
            const int r = __builtin_ctzll(ovf);
            const float4 bi = reinterpret_cast<const float4 *>(w.sb)[off + ib * 64 + r];
            const float ai = box_area(bi);
            int ax0, ax1, ay0, ay1;
            window(h, bi, ax0, ax1, ay0, ay1);
            bool hit = false;
            for (int ay = ay0; ay <= ay1; ++ay) {
                const int e0 = cst[ay * h.gx + ax0], e1 = cst[ay * h.gx + ax1 + 1];
                for (int e = e0 + lane; e < e1; e += 64) {
                    const int j = cl[e];
                    if (j >= ib * 64 || !((keptb[j >> 6] >> (j & 63)) & 1ull)) continue;
                    hit |= iou_over(bi, ai, cb[e], box_area(cb[e]), thr, prune);
                }
            }
            if (__ballot(hit) && lane == r) rem = true;
        }
        uint64_t word = __ballot(rem);
        const int rows = n - ib * 64;
        if (rows < 64) word |= ~((1ull << rows) - 1);  // rows past n never kept
        uint64_t kept = 0;
        const uint32_t dlo = (uint32_t)diag, dhi = (uint32_t)(diag >> 32);
        for (uint64_t avail = ~word; avail;) {  // the surviving rows, lowest first
            const int bit = __builtin_ctzll(avail);
            kept |= 1ull << bit;
            const uint32_t lo = __builtin_amdgcn_readlane(dlo, bit);
            const uint32_t hi = __builtin_amdgcn_readlane(dhi, bit);
            word |= ((uint64_t)hi << 32) | lo;
            avail = bit == 63 ? 0ull : ~word & (~0ull << (bit + 1));
        }
        if (lane == 0) keptb[ib] = kept;
        cnt += __popcll(kept);
        // keptb[ib] before the next block's reads; this slot's reads before
        // the DMA that refills it
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (ib + GP < nb) block_dma(rl, rd, rc, slot, ib + GP, lane);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int q = lane; q < nb; q += 64) w.keptw[nb_off[g] + q] = keptb[q];
    if (lane == 0) kept_out[g] = cnt;
}

// kept rows before each 64-row block (exclusive scan of the kept words'
// popcounts), one workgroup per image
__global__ __launch_bounds__(256) void kept_scan_kernel(const int64_t *__restrict__ cand_off,
                                                        const int64_t *__restrict__ nb_off, NmsWork w) {
    __shared__ int part[256];
    const int g = blockIdx.x, tid = threadIdx.x;
    const int n = (int)(cand_off[g + 1] - cand_off[g]);
    const int nb = (n + 63) / 64;
    const int per = (nb + 255) / 256, q0 = min(tid * per, nb), q1 = min(q0 + per, nb);
    const uint64_t *kw = w.keptw + nb_off[g];
    int32_t *kb = w.kbase + nb_off[g];
    int sum = 0;
    for (int q = q0; q < q1; ++q) sum += __popcll(kw[q]);
    part[tid] = sum;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // Hillis-Steele inclusive scan
        const int t = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += t;
        __syncthreads();
    }
    int run = part[tid] - sum;
    for (int q = q0; q < q1; ++q) {
        kb[q] = run;
        run += __popcll(kw[q]);
    }
}

// The kept rows out, chip-wide: one thread per sorted row, its slot from the
// block's kept word and running count (greedy_kernel).  Writing them inside
// the greedy wave had put two dependent global loads (order, then the row)
// on every block's serial path.
__global__ __launch_bounds__(256) void emit_kernel(const int64_t *__restrict__ cand_off,
                                                   const int64_t *__restrict__ nb_off, NmsWork w,
                                                   float *__restrict__ out_logits, float *__restrict__ out_boxes,
                                                   float *__restrict__ out_refs, int64_t *__restrict__ out_keep) {
    const int g = blockIdx.y;
    const int64_t off = cand_off[g];
    const int n = (int)(cand_off[g + 1] - off);
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int64_t wb = nb_off[g] + (p >> 6);
    const uint64_t kept = w.keptw[wb];
    const int lane = p & 63;
    if (!((kept >> lane) & 1ull)) return;
    const int pos = w.kbase[wb] + __popcll(kept & ((1ull << lane) - 1));
    const int li = min(max(w.order[off + p], 0), n - 1);
    const int64_t src = off + li, dst = off + pos;
    out_logits[2 * dst + 0] = w.s[src];
    out_logits[2 * dst + 1] = 0.0f;
    reinterpret_cast<float4 *>(out_boxes)[dst] = reinterpret_cast<const float4 *>(w.b)[src];
    out_refs[2 * dst + 0] = w.r[2 * src + 0];
    out_refs[2 * dst + 1] = w.r[2 * src + 1];
    if (out_keep) out_keep[dst] = li;
}

// Calls whose every image has at most SMALL_N candidates (the module API's
// one image of a few exemplars, demo.py:123-130): the whole NMS of an image
// in ONE workgroup -- gather, the stable descending sort as a rank count over
// rocprim's float key order (so the same order as the radix sort: -0.0 ==
// +0.0, ties by local index), the IoU words in LDS with mask_strip's
// arithmetic, and the greedy chain -- one launch instead of gather + sort
// + strips, no work buffer.  Same keep lists by construction.
constexpr int SMALL_N = TMR_NMS_SMALL;


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

int64_t tmr_nms_work_bytes(int64_t total_cand, int64_t sum_nb, int64_t max_cand, int G) {
    if (total_cand < 0 || sum_nb < 0 || max_cand < 0 || G <= 0) return -1;
    return work_bytes(total_cand, sum_nb, G);
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
    TMR_REQUIRE(max_nb * 8 <= 80 * 1024);  // the kept bitmap in LDS (beside ~66 KB of list slots)
    hipStream_t s = tmr_stream(stream);
    if (max_cand <= SMALL_N) {  // every image fits one workgroup
        hipLaunchKernelGGL(nms_small_kernel, dim3(G), dim3(SMALL_N), 0, s, logits, box, ref, counts, unit_off,
                           seg_units, cand_off, iou_threshold, out_logits, out_boxes, out_refs, out_keep, kept);
        TMR_CHECK_LAUNCH();
        return TMR_OK;
    }
    NmsWork w = carve(work, total_cand, sum_nb, G);
    hipLaunchKernelGGL(gather_kernel, dim3(G), dim3(256), 0, s, logits, box, ref, counts, unit_off,
                       seg_units, cand_off, w);
    TMR_CHECK_LAUNCH();
    size_t tb = 0;
    int gbits = 0;
    while ((1 << gbits) < G) ++gbits;
    const unsigned end_bit = 32u + (unsigned)gbits;  // the image bits only as far as G needs
    if (rocprim::radix_sort_pairs(nullptr, tb, w.key, w.skey, w.idx, w.order, (unsigned)total_cand, 0u, end_bit,
                                  s) != hipSuccess)
        return TMR_E_HIP;
    if ((int64_t)tb > w.temp_bytes) return TMR_E_INVALID;
    if (rocprim::radix_sort_pairs(w.temp, tb, w.key, w.skey, w.idx, w.order, (unsigned)total_cand, 0u, end_bit,
                                  s) != hipSuccess)
        return TMR_E_HIP;
    const dim3 per_box((unsigned)std::min<int64_t>(tmr_cdiv(max_cand, 256), 1024), G);
    hipLaunchKernelGGL(sort_boxes_kernel, per_box, dim3(256), 0, s, cand_off, G, w);
    TMR_CHECK_LAUNCH();
    hipLaunchKernelGGL(bin_setup_kernel, dim3(G), dim3(256), 0, s, cand_off, iou_threshold, w);
    TMR_CHECK_LAUNCH();
    if (hipMemsetAsync(w.cnt, 0, sizeof(int32_t) * NCELL * (size_t)G, s) != hipSuccess) return TMR_E_HIP;
    hipLaunchKernelGGL(bin_kernel<0>, per_box, dim3(256), 0, s, cand_off, w);
    TMR_CHECK_LAUNCH();
    hipLaunchKernelGGL(bin_scan_kernel, dim3(G), dim3(256), 0, s, w);
    TMR_CHECK_LAUNCH();
    hipLaunchKernelGGL(bin_kernel<1>, per_box, dim3(256), 0, s, cand_off, w);
    TMR_CHECK_LAUNCH();
    hipLaunchKernelGGL(pairs_kernel, dim3((unsigned)tmr_cdiv(max_cand, 256), G), dim3(256), 0, s, cand_off,
                       nb_off, iou_threshold, w);
    TMR_CHECK_LAUNCH();
    // LDS: the kept bitmap (max_nb words + the zero word, rounded to 16 B) + GP slots
    w.lbuf_words = (max_nb + 2) & ~int64_t(1);
    const size_t lds = sizeof(uint64_t) * (size_t)w.lbuf_words + GP * sizeof(int32_t) * SLOT_W;
    TMR_REQUIRE(lds <= 160 * 1024);
    if (lds > 64 * 1024 && tmr_set_max_lds((const void *)greedy_kernel, lds) != hipSuccess) return TMR_E_HIP;
    hipLaunchKernelGGL(greedy_kernel, dim3(G), dim3(64), lds, s, cand_off, nb_off, iou_threshold, w, kept);
    TMR_CHECK_LAUNCH();
    hipLaunchKernelGGL(kept_scan_kernel, dim3(G), dim3(256), 0, s, cand_off, nb_off, w);
    TMR_CHECK_LAUNCH();
    hipLaunchKernelGGL(emit_kernel, dim3((unsigned)tmr_cdiv(max_cand, 256), G), dim3(256), 0, s, cand_off, nb_off,
                       w, out_logits, out_boxes, out_refs, out_keep);
    TMR_CHECK_LAUNCH();
    return TMR_OK;
}
