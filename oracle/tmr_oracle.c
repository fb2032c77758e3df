/*
 * TEST INFRASTRUCTURE ONLY -- CPU oracle for the TMR hot path.
 *
 * Plain-C restatement of the reference algorithm (mFinn27/Template-Matching-
 * and-Regression-MapReduce @ 2026-01-16) for the integer / index / bit-exact
 * parts of the path, plus the small fp32 ops whose exact arithmetic we pin.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker.  The product path
 * (template-matching-and-regression-mapreduce_amd/) never links it.
 *
 * Compile with -ffp-contract=off: the reference's CPU kernels perform every
 * multiply and add as a separately rounded fp32 operation.
 *
 * Pinning: the functions restating the reference's own Python (template
 * sizing, cross-correlation, peak finder, box decode) are pinned against
 * golden vectors produced by importing /root/reference (oracle/make_golden.py,
 * tests/golden/).  roi_align / nms restate torchvision==0.19.0 (a third-party
 * dependency absent from this image): parity there is UNPINNED (see
 * DESIGN.md "Oracle").
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------
 * Exemplar box clamp + template sizing.
 * reference: models/template_matching.py:55-73 (extract_template)
 *   x1, y1 = min(1., max(0., x1)), ...     (:58-59) -- Python min/max
 *   x1, x2 = x1*Wf, x2*Wf                  (:61-62) -- fp32 0-d tensor ops
 *   Wt = ceil(x2) - floor(x1); even -> -1  (:66-73)
 * Python's max(0., v) returns v iff v > 0., min(1., v) returns v iff v < 1.
 * ------------------------------------------------------------------------ */
static float clamp01(float v) {
    float m = (v > 0.0f) ? v : 0.0f;   /* max(0., v)  (NaN -> 0.) */
    return (m < 1.0f) ? m : 1.0f;      /* min(1., m) */
}

void orc_clamp_box(const float in[4], float out[4]) {
    for (int i = 0; i < 4; ++i) out[i] = clamp01(in[i]);
}

/* returns 0 on success, -1 when the reference would build an invalid
 * (non-positive) roi_align output size. */
int orc_template_size(const float box[4], int H, int W, float roi[4], int *Ht, int *Wt) {
    float c[4];
    orc_clamp_box(box, c);
    volatile float x1 = c[0] * (float)W, x2 = c[2] * (float)W;  /* :61 */
    volatile float y1 = c[1] * (float)H, y2 = c[3] * (float)H;  /* :62 */
    roi[0] = x1; roi[1] = y1; roi[2] = x2; roi[3] = y2;         /* :63 */
    int wt = (int)ceilf(x2) - (int)floorf(x1);                  /* :66,70 */
    int ht = (int)ceilf(y2) - (int)floorf(y1);                  /* :67,71 */
    if (wt % 2 == 0) wt -= 1;                                   /* :72 */
    if (ht % 2 == 0) ht -= 1;                                   /* :73 */
    *Ht = ht; *Wt = wt;
    return (ht > 0 && wt > 0) ? 0 : -1;
}

/* Integer-snapped prototype box, models/template_matching.py:43-53. */
void orc_prototype_box(const float box[4], int H, int W, int out[4]) {
    float c[4];
    orc_clamp_box(box, c);
    /* Python floats (double) here: x1*Wf with x1 a 0-d fp32 tensor -> fp32 */
    volatile float x1 = c[0] * (float)W, x2 = c[2] * (float)W;
    volatile float y1 = c[1] * (float)H, y2 = c[3] * (float)H;
    out[0] = (int)floorf(x1); out[1] = (int)floorf(y1);
    out[2] = (int)ceilf(x2);  out[3] = (int)ceilf(y2);
}

/* ------------------------------------------------------------------------
 * RoIAlign, torchvision 0.19.0 CPU kernel semantics (third-party, UNPINNED),
 * called at models/template_matching.py:75 as
 *   roi_align(f[1,C,H,W], [[x1,y1,x2,y2]], (Ht,Wt), aligned=True)
 * spatial_scale = 1, sampling_ratio = -1 (adaptive), aligned offset 0.5.
 * SURVEY.md Appendix A.
 * ------------------------------------------------------------------------ */
void orc_roi_align(const float *f, int C, int H, int W, const float roi[4],
                   int PH, int PW, float *out) {
    const float off = 0.5f;
    float sw = roi[0] - off, sh = roi[1] - off;
    float ew = roi[2] - off, eh = roi[3] - off;
    float rw = ew - sw, rh = eh - sh;
    float bin_h = rh / (float)PH, bin_w = rw / (float)PW;
    int gh = (int)ceilf(rh / (float)PH);
    int gw = (int)ceilf(rw / (float)PW);
    int cnt_i = gh * gw; if (cnt_i < 1) cnt_i = 1;
    float count = (float)cnt_i;
    int ns = gh * gw * PH * PW;
    int *pos = (int *)malloc(sizeof(int) * 4 * (ns > 0 ? ns : 1));
    float *wt = (float *)malloc(sizeof(float) * 4 * (ns > 0 ? ns : 1));
    int k = 0;
    for (int ph = 0; ph < PH; ++ph)
        for (int pw = 0; pw < PW; ++pw)
            for (int iy = 0; iy < gh; ++iy)
                for (int ix = 0; ix < gw; ++ix, ++k) {
                    float y = sh + (float)ph * bin_h + ((float)iy + 0.5f) * bin_h / (float)gh;
                    float x = sw + (float)pw * bin_w + ((float)ix + 0.5f) * bin_w / (float)gw;
                    if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) {
                        for (int q = 0; q < 4; ++q) { pos[4 * k + q] = 0; wt[4 * k + q] = 0.0f; }
                        continue;
                    }
                    if (y <= 0) y = 0;
                    if (x <= 0) x = 0;
                    int yl = (int)y, xl = (int)x, yh, xh;
                    if (yl >= H - 1) { yh = yl = H - 1; y = (float)yl; } else yh = yl + 1;
                    if (xl >= W - 1) { xh = xl = W - 1; x = (float)xl; } else xh = xl + 1;
                    float ly = y - (float)yl, lx = x - (float)xl;
                    float hy = 1.0f - ly, hx = 1.0f - lx;
                    wt[4 * k + 0] = hy * hx; wt[4 * k + 1] = hy * lx;
                    wt[4 * k + 2] = ly * hx; wt[4 * k + 3] = ly * lx;
                    pos[4 * k + 0] = yl * W + xl; pos[4 * k + 1] = yl * W + xh;
                    pos[4 * k + 2] = yh * W + xl; pos[4 * k + 3] = yh * W + xh;
                }
    for (int c = 0; c < C; ++c) {
        const float *fc = f + (size_t)c * H * W;
        int q = 0;
        for (int ph = 0; ph < PH; ++ph)
            for (int pw = 0; pw < PW; ++pw) {
                float acc = 0.0f;
                for (int s = 0; s < gh * gw; ++s, ++q) {
                    float v = wt[4 * q + 0] * fc[pos[4 * q + 0]] + wt[4 * q + 1] * fc[pos[4 * q + 1]];
                    v = v + wt[4 * q + 2] * fc[pos[4 * q + 2]];
                    v = v + wt[4 * q + 3] * fc[pos[4 * q + 3]];
                    acc += v;
                }
                out[((size_t)c * PH + ph) * PW + pw] = acc / count;
            }
    }
    free(pos); free(wt);
}

/* Prototype template: AdaptiveAvgPool2d(1) over the snapped box,
 * models/template_matching.py:52.  Double accumulation. */
void orc_prototype(const float *f, int C, int H, int W, const int b[4], float *out) {
    int n = (b[3] - b[1]) * (b[2] - b[0]);
    for (int c = 0; c < C; ++c) {
        const float *fc = f + (size_t)c * H * W;
        double acc = 0.0;  /* ATen's reduction order is not ours: sum exactly-ish */
        for (int y = b[1]; y < b[3]; ++y)
            for (int x = b[0]; x < b[2]; ++x) acc += fc[y * W + x];
        out[c] = (float)(acc / (double)n);
    }
}

/* ------------------------------------------------------------------------
 * Depthwise cross-correlation, models/template_matching.py:23-41, then the
 * learned scale at :97.
 *   out = pad( conv2d(f, t, groups=C) / fl32(h*w) ) * scale
 * The divide is an IEEE fp32 divide by fl32(h*w) (the Python scalar
 * h*w + 1e-14 rounds to h*w in fp32).  squeeze=1 sums over C (:34-35).
 * Summation order (row-major over the template) is ours; parity with the
 * reference's mkldnn order is to fp32 tolerance.
 * ------------------------------------------------------------------------ */
void orc_xcorr(const float *f, int C, int H, int W, const float *t, int h, int w,
               float scale, int squeeze, float *out) {
    int Ho = H - h + 1, Wo = W - w + 1, ph = h / 2, pw = w / 2;
    float denom = (float)(h * w);
    int Co = squeeze ? 1 : C;
    memset(out, 0, sizeof(float) * (size_t)Co * H * W);
    float *tmp = squeeze ? (float *)calloc((size_t)H * W, sizeof(float)) : NULL;
    for (int c = 0; c < C; ++c) {
        const float *fc = f + (size_t)c * H * W;
        const float *tc = t + (size_t)c * h * w;
        for (int y = 0; y < Ho; ++y)
            for (int x = 0; x < Wo; ++x) {
                float acc = 0.0f;
                for (int i = 0; i < h; ++i)
                    for (int j = 0; j < w; ++j) acc += fc[(y + i) * W + x + j] * tc[i * w + j];
                float v = acc / denom;
                if (squeeze) tmp[(y + ph) * W + x + pw] += v;
                else out[((size_t)c * H + y + ph) * W + x + pw] = v * scale;
            }
    }
    if (squeeze) {
        for (int y = 0; y < Ho; ++y)
            for (int x = 0; x < Wo; ++x) {
                size_t o = (size_t)(y + ph) * W + x + pw;
                out[o] = tmp[o] * scale;
            }
        free(tmp);
    }
}

/* ------------------------------------------------------------------------
 * Bilinear x2 upsample, align_corners=False, models/matching_net.py:50-51
 * (ATen upsample_bilinear2d).  SURVEY.md Appendix C: with the source index
 * src = max(0, 0.5*(d+0.5)-0.5) the fma nesting below reproduces torch's
 * AVX-512 CPU kernel bit for bit.
 * ------------------------------------------------------------------------ */
static void up_index(int d, int L, int *i0, int *i1, float *l0, float *l1) {
    float src = 0.5f * ((float)d + 0.5f) - 0.5f;
    if (src < 0.0f) src = 0.0f;
    int a = (int)src;
    int off = (a < L - 1) ? 1 : 0;
    float lam = src - (float)a;
    *i0 = a; *i1 = a + off; *l1 = lam; *l0 = 1.0f - lam;
}

void orc_upsample2x(const float *f, int C, int H, int W, float *out) {
    int H2 = 2 * H, W2 = 2 * W;
    for (int c = 0; c < C; ++c) {
        const float *fc = f + (size_t)c * H * W;
        float *oc = out + (size_t)c * H2 * W2;
        for (int oy = 0; oy < H2; ++oy) {
            int y0, y1; float ly0, ly1;
            up_index(oy, H, &y0, &y1, &ly0, &ly1);
            for (int ox = 0; ox < W2; ++ox) {
                int x0, x1; float lx0, lx1;
                up_index(ox, W, &x0, &x1, &lx0, &lx1);
                float a = fc[y0 * W + x0], b = fc[y0 * W + x1];
                float c2 = fc[y1 * W + x0], d = fc[y1 * W + x1];
                float top = fmaf(lx0, a, lx1 * b);
                float bot = fmaf(lx0, c2, lx1 * d);
                oc[oy * W2 + ox] = fmaf(ly0, top, ly1 * bot);
            }
        }
    }
}

/* ------------------------------------------------------------------------
 * Peak finder + box decode, utils/TM_utils.py:224-305 (Get_pred_boxes) with
 * adaptive_kernel_generater (:363-377) and custom_shape_3x3_maxpool2d
 * (:337-361).  Input is the probability map p = sigmoid(o) (:246); the
 * bit-exact contract is defined on p.
 * ------------------------------------------------------------------------ */

/* :363-377.  ex_h / ex_w are fp32 (0-d tensor arithmetic), compared with the
 * Python doubles k/H cast to fp32 (torch wraps the scalar). mask row-major. */
void orc_adaptive_kernel(float ex_h, float ex_w, int H, int W, uint8_t mask[9]) {
    double nh = 1.0 / (double)H, nw = 1.0 / (double)W;
    float h3 = (float)(nh * 3), w3 = (float)(nw * 3);
    float h2 = (float)(nh * 2), w2 = (float)(nw * 2);
    static const uint8_t full[9] = {1, 1, 1, 1, 1, 1, 1, 1, 1};
    static const uint8_t ctr[9] = {0, 0, 0, 0, 1, 0, 0, 0, 0};
    static const uint8_t vert[9] = {0, 1, 0, 0, 1, 0, 0, 1, 0};
    static const uint8_t horz[9] = {0, 0, 0, 1, 1, 1, 0, 0, 0};
    static const uint8_t cross[9] = {0, 1, 0, 1, 1, 1, 0, 1, 0};
    const uint8_t *m;
    if (ex_h >= h3 && ex_w >= w3) m = full;
    else if (ex_h < h2 && ex_w < w2) m = ctr;
    else if (ex_h < h2 && ex_w >= w2) m = vert;
    else if (ex_h >= h2 && ex_w < w2) m = horz;
    else m = cross;
    memcpy(mask, m, 9);
}

/* Exemplar-derived decode scalars (:236-243).  box_w = x2-x1 (fp32). */
void orc_exemplar_scalars(const float box[4], int ablation_b, float out[4]) {
    float c[4];
    orc_clamp_box(box, c);
    volatile float bw = c[2] - c[0], bh = c[3] - c[1];
    out[0] = bh; out[1] = bw;                /* ex size for the adaptive kernel (:252) */
    out[2] = ablation_b ? 1.0f : bw;         /* decode scale (:239,242-243) */
    out[3] = ablation_b ? 1.0f : bh;
}

/* Correctly rounded expf (double exp rounded once).  The reference's
 * torch.exp is position-dependent on CPU (vector body vs scalar tail); the
 * decode contract is defined on this correctly rounded exp. */
static float cr_expf(float x) { return (float)exp((double)x); }

/* Returns the number of candidates written (no cap, row-major order).
 * outputs (each may be NULL): idx[n] = y*W+x, logits[2n], boxes[4n], refs[2n].
 * mode: 0 = box regression (:264-272), 1 = regression_ablation_c (:268-269),
 *       2 = no box regression / template-size predictions (:273-276). */
int64_t orc_peaks_decode(const float *p, const float *reg, int H, int W,
                         const uint8_t mask[9], float thr, float bw, float bh,
                         int mode, int64_t cap, int64_t *idx, float *logits,
                         float *boxes, float *refs) {
    int64_t n = 0;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            float v = p[y * W + x];
            if (!(v >= thr)) continue;
            /* pooled = selected_positions.max(dim=2) (:359): torch.max propagates
             * NaN, so a NaN anywhere among the masked taps makes pooled NaN and
             * `pooled == p` (:253) False -- the pixel is never a peak. */
            float mx = -INFINITY;
            int first = 1, nan = 0;
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    if (!mask[(dy + 1) * 3 + dx + 1]) continue;
                    int yy = y + dy, xx = x + dx;
                    float q = (yy < 0 || yy >= H || xx < 0 || xx >= W) ? 0.0f : p[yy * W + xx];
                    if (q != q) nan = 1;
                    if (first || q > mx) { mx = q; first = 0; }
                }
            if (nan || !(mx == v)) continue;
            if (n < cap) {
                int64_t i = n;
                if (idx) idx[i] = (int64_t)y * W + x;
                volatile float rx = (float)x / (float)W, ry = (float)y / (float)H;  /* :257 */
                if (refs) { refs[2 * i] = rx; refs[2 * i + 1] = ry; }
                if (logits) { logits[2 * i] = v; logits[2 * i + 1] = 0.0f; }  /* :260-261 */
                if (boxes) {
                    float r0 = 0, r1 = 0, r2 = 0, r3 = 0;
                    if (mode != 2) {
                        size_t o = (size_t)y * W + x, hw = (size_t)H * W;
                        r0 = reg[o]; r1 = reg[hw + o]; r2 = reg[2 * hw + o]; r3 = reg[3 * hw + o];
                    }
                    float sx = (mode == 1) ? 1.0f : bw, sy = (mode == 1) ? 1.0f : bh;
                    volatile float tx = r0 * sx, ty = r1 * sy;
                    volatile float cx = rx + tx, cy = ry + ty;
                    volatile float w = cr_expf(r2) * bw, h = cr_expf(r3) * bh;
                    volatile float hw2 = w / 2.0f, hh2 = h / 2.0f;           /* :278 */
                    boxes[4 * i + 0] = cx - hw2; boxes[4 * i + 1] = cy - hh2;
                    boxes[4 * i + 2] = cx + hw2; boxes[4 * i + 3] = cy + hh2;
                }
            }
            ++n;
        }
    return n;
}

/* ------------------------------------------------------------------------
 * Greedy NMS, torchvision 0.19.0 CPU nms kernel semantics (third-party,
 * UNPINNED), called at utils/TM_utils.py:322.  SURVEY.md Appendix B:
 * stable descending sort on score, IoU in fp32, compared in double.
 * ------------------------------------------------------------------------ */
static const float *g_sort_scores;
/* scores.sort(stable=true, descending=true): torch orders NaN (either sign)
 * above +inf, all NaNs equal; -0.0 == +0.0; ties keep the lower index. */
static int cmp_desc_stable(const void *a, const void *b) {
    int64_t i = *(const int64_t *)a, j = *(const int64_t *)b;
    float si = g_sort_scores[i], sj = g_sort_scores[j];
    int ni = si != si, nj = sj != sj;
    if (ni != nj) return ni ? -1 : 1;
    if (!ni) {
        if (si > sj) return -1;
        if (si < sj) return 1;
    }
    return (i < j) ? -1 : (i > j);
}

int64_t orc_nms(const float *boxes, const float *scores, int64_t n, double thr, int64_t *keep) {
    if (n <= 0) return 0;
    int64_t *order = (int64_t *)malloc(sizeof(int64_t) * n);
    float *areas = (float *)malloc(sizeof(float) * n);
    uint8_t *sup = (uint8_t *)calloc(n, 1);
    for (int64_t i = 0; i < n; ++i) {
        order[i] = i;
        const float *b = boxes + 4 * i;
        areas[i] = (b[2] - b[0]) * (b[3] - b[1]);
    }
    g_sort_scores = scores;
    qsort(order, n, sizeof(int64_t), cmp_desc_stable);
    int64_t nk = 0;
    for (int64_t _i = 0; _i < n; ++_i) {
        int64_t i = order[_i];
        if (sup[i]) continue;
        keep[nk++] = i;
        const float *bi = boxes + 4 * i;
        for (int64_t _j = _i + 1; _j < n; ++_j) {
            int64_t j = order[_j];
            if (sup[j]) continue;
            const float *bj = boxes + 4 * j;
            /* std::max(ix1, x1[j]) = ix1 < x1[j] ? x1[j] : ix1, std::min likewise
             * (a NaN coordinate makes an area NaN, so ovr is NaN and never > thr) */
            float xx1 = bi[0] < bj[0] ? bj[0] : bi[0];
            float yy1 = bi[1] < bj[1] ? bj[1] : bi[1];
            float xx2 = bj[2] < bi[2] ? bj[2] : bi[2];
            float yy2 = bj[3] < bi[3] ? bj[3] : bi[3];
            float w = xx2 - xx1; if (!(0.0f < w)) w = 0.0f;
            float h = yy2 - yy1; if (!(0.0f < h)) h = 0.0f;
            float inter = w * h;
            float ovr = inter / (areas[i] + areas[j] - inter);
            if ((double)ovr > thr) sup[j] = 1;
        }
    }
    free(order); free(areas); free(sup);
    return nk;
}

/* Test-infrastructure helper for oracle/agreement.py: over the n candidates two
 * runs share (row i of a and of b is the same (unit, pixel)), count the pairs
 * whose NMS sort order (stable descending, by the run's own row positions) or
 * IoU decision ((double)IoU > thr, the arithmetic of orc_nms) differ between
 * the runs.  margin[0] = max |IoU_a - thr| over the IoU flips. */
static float iou_f32(const float *bi, const float *bj) {
    float ai = (bi[2] - bi[0]) * (bi[3] - bi[1]);
    float aj = (bj[2] - bj[0]) * (bj[3] - bj[1]);
    float xx1 = bi[0] > bj[0] ? bi[0] : bj[0];
    float yy1 = bi[1] > bj[1] ? bi[1] : bj[1];
    float xx2 = bi[2] < bj[2] ? bi[2] : bj[2];
    float yy2 = bi[3] < bj[3] ? bi[3] : bj[3];
    float w = xx2 - xx1; if (!(w > 0.0f)) w = 0.0f;
    float h = yy2 - yy1; if (!(h > 0.0f)) h = 0.0f;
    float inter = w * h;
    return inter / (ai + aj - inter);
}

void orc_decision_flips(int64_t n, const float *boxes_a, const float *scores_a, const int64_t *rows_a,
                        const float *boxes_b, const float *scores_b, const int64_t *rows_b, double thr,
                        int64_t *order_flips, int64_t *iou_flips, double *margin) {
    int64_t of = 0, qf = 0;
    double mg = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        for (int64_t j = i + 1; j < n; ++j) {
            int ba = scores_a[i] > scores_a[j] || (scores_a[i] == scores_a[j] && rows_a[i] < rows_a[j]);
            int bb = scores_b[i] > scores_b[j] || (scores_b[i] == scores_b[j] && rows_b[i] < rows_b[j]);
            of += ba != bb;
            const float *ai = boxes_a + 4 * i, *aj = boxes_a + 4 * j;
            const float *bi = boxes_b + 4 * i, *bj = boxes_b + 4 * j;
            /* no overlap in either run: both IoUs are 0 */
            if (!(ai[0] < aj[2] && aj[0] < ai[2] && ai[1] < aj[3] && aj[1] < ai[3]) &&
                !(bi[0] < bj[2] && bj[0] < bi[2] && bi[1] < bj[3] && bj[1] < bi[3]))
                continue;
            double qa = (double)iou_f32(ai, aj), qb = (double)iou_f32(bi, bj);
            if ((qa > thr) != (qb > thr)) {
                ++qf;
                double d = qa > thr ? qa - thr : thr - qa;
                if (d > mg) mg = d;
            }
        }
    }
    *order_flips = of; *iou_flips = qf; *margin = mg;
}

int orc_version(void) { return 1; }
