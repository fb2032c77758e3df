/*
 * tmr.h -- C ABI of libtmr.so, the MI355X-native TMR hot path.
 *
 * Every entry point replaces one reference operation on the path named by
 * BASELINE.json north_star (file:line into mFinn27/Template-Matching-and-
 * Regression-MapReduce @ 2026-01-16).  The reference
 * is pure Python over ATen/torchvision, so the "FFI" a maintainer binds is
 * Python ctypes (INTEGRATION.md shows the stub); no torch types cross this
 * boundary.
 *
 * Conventions
 *  - All tensor pointers are DEVICE pointers owned by the caller; the library
 *    never allocates or frees device memory.  fp32, NCHW, contiguous.
 *  - Every call is asynchronous on `stream` (a hipStream_t, passed as void*;
 *    NULL = the null stream) and returns 0 or a negative TMR_E* code; nothing
 *    throws across the ABI.  tmr_strerror() names the code.
 *  - No global mutable state (beyond an idempotent per-(device, kernel) cache of
 *    the LDS-size attribute): calls are reentrant across streams/devices.
 *  - "units" are (image, exemplar) matching units, described by a device
 *    array of tmr_unit_t built on the host (the reference sizes templates on
 *    the host too: template_matching.py:56-73 runs Python math on 0-d
 *    tensors).
 */
#ifndef TMR_H_
#define TMR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TMR_ABI_VERSION 3  /* 2: per-unit out_absmax, per-sample activation scales;
                            * 3: one correlation entry point (tmr_xcorr_args_t), one
                            * sizing query (tmr_size), one split conv entry point,
                            * no subset launches (tmr_unit_t.out_unit removed) */

enum {
    TMR_OK = 0,
    TMR_E_INVALID = -1,    /* bad argument / shape */
    TMR_E_HIP = -2,        /* a HIP runtime error (launch failure) */
    TMR_E_UNSUPPORTED = -3 /* configuration not built into this library */
};

enum { TMR_TEMPLATE_ROI_ALIGN = 0, TMR_TEMPLATE_PROTOTYPE = 1 };

/* One (image, exemplar) matching unit.  Built by the host from the exemplar
 * box exactly as models/template_matching.py:43-76 does. */
typedef struct tmr_unit {
    int32_t image;         /* index into the feature batch                        */
    int32_t type;          /* TMR_TEMPLATE_*                                      */
    int32_t ht, wt;        /* template size (odd; 1x1 for prototype)              */
    float roi[4];          /* roi_align box in feature px (x1,y1,x2,y2), :61-63   */
    int32_t pbox[4];       /* prototype snapped box (x1,y1,x2,y2), :49-50         */
    int64_t tmpl_offset;   /* float offset of this unit's [C,ht,wt] template      */
    int32_t row_offset;    /* sum of ht * tsplit_nk(wt) over the units before this */
                           /* one (the MFMA correlation's split-template rows,    */
                           /* tmr_template_split)                                  */
    int32_t pad_;
} tmr_unit_t;

/* Per-unit peak-finder parameters (utils/TM_utils.py:236-278). */
typedef struct tmr_peak_param {
    float thr;             /* fl32(cls_ths), compared p >= thr (:254)             */
    float scale_w, scale_h;/* decode scale: clamped exemplar w,h or 1 (:239-243)  */
    int32_t mask;          /* 9-bit 3x3 kernel, bit (dy+1)*3+(dx+1) (:363-377)    */
    int32_t mode;          /* 0 box regression, 1 ablation_c, 2 no regression      */
    int32_t pad_;
} tmr_peak_param_t;

int tmr_version(void);
const char *tmr_strerror(int rc);

/* ---- sizes of the caller-provided buffers ---------------------------------
 * tmr_size(kind, d0..d5) returns the size of a buffer the caller allocates
 * (bytes, or floats where noted), or -1 for invalid dimensions; unused
 * dimensions are 0.
 *   TMR_SIZE_TEMPLATE_SPLIT (U, C, total_rows)          bytes, tmr_template_split
 *   TMR_SIZE_HEADS_PARTIALS (N, U, H, W)                floats, tmr_split_conv heads
 *   TMR_SIZE_XPACK          (S, C, H, W, ks, prec)      bytes, tmr_split_xpack (H, W at
 *                                                       the output resolution)
 *   TMR_SIZE_WPACK          (N, C0, C1, ks, prec)       bytes, tmr_split_wpack
 *   TMR_SIZE_ACC            (U, N, H, W)                floats, TMR_SPLIT_TILED_OUT slabs
 *   TMR_SIZE_NMS_WORK       (total_cand, sum_nb, max_cand, G)  bytes, tmr_nms
 *   TMR_SIZE_STATS_WORK     (B)                         bytes, tmr_feature_stats */
enum {
    TMR_SIZE_TEMPLATE_SPLIT = 1,
    TMR_SIZE_HEADS_PARTIALS = 2,
    TMR_SIZE_XPACK = 3,
    TMR_SIZE_WPACK = 4,
    TMR_SIZE_ACC = 5,
    TMR_SIZE_NMS_WORK = 6,
    TMR_SIZE_STATS_WORK = 7
};
int64_t tmr_size(int kind, int64_t d0, int64_t d1, int64_t d2, int64_t d3, int64_t d4, int64_t d5);

/* ---- (a2+a13) bilinear x2 upsample ---------------------------------------
 * f[0] = F.interpolate(feat, scale_factor=2, mode='bilinear',
 * align_corners=False) alone (matching_net.py:50-51, the API output :81):
 * feat [BC][Hin][Win] -> out [BC][2 Hin][2 Win], bit-exact with ATen's CPU
 * kernel's fma nesting. */
int tmr_upsample2x(const float *feat, int BC, int Hin, int Win, float *out, void *stream);

/* ---- (a6+a7+a8) exemplar templates --------------------------------------
 * torchvision.ops.roi_align(f, [roi], (ht,wt), aligned=True) per unit
 * (models/template_matching.py:75) or the prototype AdaptiveAvgPool2d(1)
 * (:52).  f [B,C,H,W]; templates written at units[u].tmpl_offset as [C,ht,wt]. */
int tmr_templates(const float *f, int B, int C, int H, int W, const tmr_unit_t *units, int U,
                  int max_ht, int max_wt, float *templates, void *stream);

/* ---- (a9+a4) depthwise cross-correlation + pad + scale -------------------
 * out[u] = pad(conv2d(f[img(u)], T_u, groups=C) / fl32(ht*wt)) * scale
 * (models/template_matching.py:23-41, :97), one launch over all units:
 *  f [B,C,H,W] (the projected features fp); templates from tmr_templates;
 *  units [U] sorted by image, img_units (device int32[B+1]) each image's unit
 *  range (an image's feature band is staged once for all of its exemplars);
 *  scale: device scalar (matcher.scale).
 *  squeeze != 0: out is [U,1,H,W] = pad(sum_c ...) * scale (:34-35) and `work`
 *  holds U*C*H*W floats; otherwise out is [U,C,H,W] and work may be NULL.
 *  relu_out (nullable) receives relu(out) (matching_net.py:79).
 *  out_absmax (nullable, device float[U], zeroed by the caller): raised to
 *  max |out[u]| per unit (the split decoder's per-unit activation scale
 *  source, TMR_SPLIT_XMAX_PER_UNIT), with no extra pass over out.
 *  algo: TMR_XCORR_VALU (fp32 LDS-blocked wavefront kernels), TMR_XCORR_MFMA
 *  (2-D window Toeplitz implicit GEMM on v_mfma_f32_16x16x32_{f16,bf16}:
 *  W % 64 == 0, W <= 256, templates <= 31x31, the staged band fits,
 *  tmpl_split given; TMR_E_UNSUPPORTED
 *  otherwise) or TMR_XCORR_AUTO (MFMA when it fits, tmpl_split is given and
 *  min_k -- the smallest template side of the launch -- reaches the
 *  crossover; VALU otherwise).
 *  tmpl_split / total_rows: tmr_template_split of the same templates and prec.
 *  prec (TMR_PREC_*, below): the MFMA operands -- TMR_PREC_F16X3 the fp32
 *  path's 3-term split (1e-5 contract); TMR_PREC_BF16 / TMR_PREC_F16 one
 *  16-bit term with fp32 accumulation (config C's bf16 contract, 1e-2).  The
 *  VALU kernels are fp32 whatever prec says.
 *  out_bf16 = 1: out is bf16 [U][C][H][W], each element the round-to-nearest-
 *  even bf16 of the fp32 value (the bf16 contract's detect path, whose decoder
 *  records are those bf16 values); needs algo TMR_XCORR_MFMA, prec
 *  TMR_PREC_BF16, squeeze 0 and relu_out NULL. */
#define TMR_XCORR_AUTO 0
#define TMR_XCORR_VALU 1
#define TMR_XCORR_MFMA 2
typedef struct tmr_xcorr_args {
    const float *f;
    const float *templates;
    const tmr_unit_t *units;
    const int32_t *img_units;
    const float *scale;
    void *out;
    float *relu_out;
    float *work;
    float *out_absmax;
    const void *tmpl_split;
    int64_t total_rows;
    int32_t B, C, H, W;
    int32_t U, max_ht, max_wt;
    int32_t squeeze;
    int32_t algo, min_k, prec, out_bf16;
} tmr_xcorr_args_t;
int tmr_xcorr(const tmr_xcorr_args_t *args, void *stream);
/* Operand prep of the MFMA correlation: per (unit u, channel c) template
 * T = templates[units[u].tmpl_offset + c*ht*wt ...], t * 2^-e = th + tl with
 * fp16 hi/lo parts and 2^-e the power-of-two scale of max |T| (max |t| 2^-e <
 * 2^14), written as the kernel's MFMA A fragments: with nk(wt) = 1 if
 * 16 + s + wt - 1 <= 32 else 2 (pw = wt/2, s = 8*ceil(pw/8) - pw) K blocks
 * per template row, the 1-KB fragment (64 lanes x 8 fp16; lane m + 16 g holds
 * T[i][8g + 32b + q - m - s], q = 0..7, zero outside [0, wt)) of row i, block
 * b, term k (0 hi, 1 lo) of (u, c) is fragment number
 * (C * row_offset(u) + c * ht * nk) * 2 + (i * nk + b) * 2 + k; then e
 * int32[U][C].  row_offset(u) = sum over earlier units of ht * nk(wt) and
 * total_rows = that sum over all units (tmr_unit_t.row_offset, set by the
 * host); size from tmr_size(TMR_SIZE_TEMPLATE_SPLIT, U, C, total_rows).
 * prec: TMR_PREC_F16X3 writes hi and lo; the one-term precisions the hi
 * fragments only (TMR_PREC_BF16: bf16; TMR_PREC_F16: the fp16 hi). */
int tmr_template_split(const float *templates, const tmr_unit_t *units, int U, int C,
                       int64_t total_rows, int prec, void *out, void *stream);

/* ---- (a10+a11+a12) conv stack: head partials ------------------------------
 * tmr_split_conv with headw (below) never stores the decoder activations:
 * each 128-channel tile t of the fused decoder_b || decoder_o GEMM writes
 *   partials[t][j][u][h][w] = sum_{n in tile t} act(conv)[n] * headw[n][j], j < 5
 * (headw [ceil(N/128)*128][5] fp32, zero padded; j 0-3 = ltrbs_head,
 * 4 = objectness_head, regression_head.py:31,50), and tmr_heads_reduce() sums
 * the tiles and adds the head biases.  Size: TMR_SIZE_HEADS_PARTIALS floats. */
/* o [U,1,H,W] = head_bias[4] + sum_t partials[t][4];  b [U,4,H,W] (nullable) =
 * head_bias[j] + sum_t partials[t][j], t over ceil(N/tile_n) channel tiles
 * (tile_n = 128, the split kernel's tile; 64 is accepted too). */
int tmr_heads_reduce(const float *partials, int N, int tile_n, int U, int H, int W,
                     const float *head_bias, float *o, float *b, void *stream);

/* ---- (a11) the decoder conv: split-precision 16-bit MFMA -------------------
 * Direct implicit-GEMM kxk conv (ks 1/3/5/7, pad ks/2) over the virtual
 * channel concat x_u = cat([src0[unit_image[u]] (C0 ch), src1[u] (C1 ch)])
 * (matching_net.py:64) with bias and optional LeakyReLU(0.01)
 * (regression_head.py:7-8) on v_mfma_f32_16x16x32_{f16,bf16}; unit_image
 * (device int32[U]) may be NULL (identity).  Operands are pre-packed 16-bit
 * records:
 *   TMR_PREC_F16X3: x*s = xh + xl, w*s' = wh + wl (fp16, power-of-two scales
 *                   from the tensors' max |.|), x.w = (wh xh + wl xh + wh xl)
 *                   / (s s') with fp32 accumulation: the fp32 path's 1e-5
 *                   normwise contract (config B);
 *   TMR_PREC_BF16:  one bf16 term, fp32 accumulation (config C, 1e-2 contract);
 *   TMR_PREC_F16:   one scaled fp16 term.
 * tmr_absmax_rows: out[s] = max |x[s][0..n)| for x [S][n] (or max(out[s], ...)
 * when accumulate), the scale sources for the packs and the conv (F16X3 /
 * F16; NULL allowed for BF16).  tmr_scale_merge: out_img[b] = max(img_max[b] (nullable: 0),
 * unit_max[u] over the units with unit_image[u] == b), out_unit[u] =
 * out_img[unit_image[u]] (out_img nullable) -- one scale per image for a
 * launch whose tiles read an image's src0 records and its units' src1
 * records together.
 * tmr_split_xpack: x [S][C][H][W] fp32 -> [S][ceil(C/32)*halves][Hp][Wp][64 B]
 * (halves 2 for F16X3: hi, lo), zero padded to whole 16x32 tiles plus the ks
 * halo (size TMR_SIZE_XPACK).  `up` bit TMR_XPACK_UPSAMPLE: the records are
 * of up2x(x) (H, W are x's; the records' are 2H, 2W); bit TMR_XPACK_ONES: a
 * constant-1 channel is appended (C + 1 channels; see tmr_split_fold_proj).
 * xmax_per_sample = 0: one scale source *xmax for
 * every sample; 1: xmax[s] for sample s (float[S]); 2: xmax[s][y][x] per
 * (output-resolution) pixel, for TMR_SPLIT_XMAX_PER_PIXEL 1x1 convs.
 * Per-sample scales make a unit's arithmetic independent of the other units
 * of the batch: its hi/lo parts never go subnormal because another sample is
 * 2^20 larger (a power-of-two rescale is exact otherwise, so results equal
 * the single-unit run's bit for bit).
 * tmr_split_wpack: w [N][C0+C1][ks][ks] -> [ks*ks][ceil(C0/32)+ceil(C1/32)]
 * [ceil(N/128)*128][rec]; the conv's src0 (per image, C0 channels, packed by
 * xpack with S = images) and src1 (per unit, C1) may both be present.
 * Records: one 64-B record per pixel per 32-channel chunk (F16X3: a hi and a
 * lo record); weights [ks*ks][chunks][ceil(N/128)*128][128 B (wh, wl) |
 * 64 B].  Head partials use 128-channel tiles (tmr_heads_reduce tile_n = 128). */
#define TMR_PREC_F16X3 0
#define TMR_PREC_BF16 1
#define TMR_PREC_F16 2
int tmr_absmax_rows(const float *x, int S, int64_t n, int accumulate, float *out, void *stream);
int tmr_scale_merge(const float *img_max, const float *unit_max, const int32_t *unit_image, int B, int U,
                    float *out_img, float *out_unit, void *stream);
#define TMR_XPACK_UPSAMPLE 1
#define TMR_XPACK_ONES 2
int tmr_split_xpack(const float *x, int S, int C, int H, int W, int up, int ks, int prec,
                    const float *xmax, int xmax_per_sample, void *out, void *stream);
/* tmr_split_xpack16: the TMR_PREC_BF16 records of a bf16 x [S][C][H][W]
 * (tmr_xcorr's bf16 f_TM; W % 8 == 0): bit-identical to tmr_split_xpack
 * of the fp32 values those bf16 elements round. */
int tmr_split_xpack16(const void *x, int S, int C, int H, int W, int ks, int prec, void *out,
                      void *stream);
/* tmr_split_fold_proj: with tmr_split_xpack's TMR_XPACK_UPSAMPLE | ONES
 * records of the SAM features it feeds the decoder's fp half without
 * materialising fp: conv(input_proj(x))
 * = conv'([x; 1]), W'[n][c] = sum_k Wd[n][k] P[k][c], W'[n][Cin] = sum_k
 * Wd[n][k] b[k] per tap (matching_net.py:27-30,56,63-69), fp64 accumulation;
 * out [N][Cin+1][ks][ks] from wd [N][Cw][ks][ks] (first Cp channels = fp). */
int tmr_split_fold_proj(const float *wd, int N, int Cw, int Cp, int ks, const float *proj_w,
                        const float *proj_b, int Cin, float *out, void *stream);
int tmr_split_wpack(const float *w, int N, int C0, int C1, int ks, int prec, const float *wmax,
                    void *out, void *stream);
/* tmr_split_conv: headw NULL -- `out` [U][N][H][W] receives act(conv + bias);
 * headw given -- `out` receives the head partials (above, TMR_SIZE_HEADS_PARTIALS
 * floats) and the activations are never stored.
 * flags: TMR_SPLIT_TILED_OUT (headw NULL only): `out` receives the raw conv
 * result (no bias / activation) in the kernel's tiled accumulator layout,
 * TMR_SIZE_ACC(U, N, H, W) floats; TMR_SPLIT_TILED_INIT: `acc_init` is
 * in that layout (indexed by unit_image), e.g. the per-image fp half. */
#define TMR_SPLIT_TILED_OUT 1
#define TMR_SPLIT_TILED_INIT 2
#define TMR_SPLIT_INIT_BCAST 4  /* acc_init is ONE slab shared by every unit
                                 * (e.g. the folded projection bias plane) */
/* the tiled `out` (TMR_SPLIT_OUT_BF16) / tiled `acc_init` (TMR_SPLIT_INIT_BF16)
 * hold bf16 values (round to nearest even) in the first half of the same
 * allocation: one-term precisions only (the per-image fp half under the bf16
 * contract; halves the heads launch's initial-value read) */
#define TMR_SPLIT_OUT_BF16 8
#define TMR_SPLIT_INIT_BF16 16
/* xmax is float[U], one activation scale source per unit u (the output slab;
 * the image index for a per-image store): both record sets a tile reads must
 * have been packed with that unit's value (tmr_split_xpack xmax_per_sample,
 * tmr_scale_merge when src0 is per image) */
#define TMR_SPLIT_XMAX_PER_UNIT 32
/* 1x1 plain stores (no acc_init, no tiled out): xmax is float[U][H][W], one
 * scale source per output pixel -- the max over that pixel's input channels
 * (tmr_pixel_absmax), the records packed with tmr_split_xpack(_up)
 * xmax_per_sample = 2 -- so every pixel is fp32-grade relative to its own
 * magnitude (the projection: templates cut from a quiet region of an image
 * are renormalised by the correlation, template_matching.py:75,31) */
#define TMR_SPLIT_XMAX_PER_PIXEL 64
/* flags bits 8..15: E, the units per image (unit u of image u / E; U % E ==
 * 0) -- the launch then runs an image's E units' blocks of one output tile
 * back to back (image-major order; 0 or 1: unit-major).  Results are the
 * same either way; only the order, and so the cache reuse, changes. */
#define TMR_SPLIT_UNITS_PER_IMAGE_SHIFT 8
/* out[s][p] = max_c |x[s][c][p]| for x [S][C][HW] */
int tmr_pixel_absmax(const float *x, int S, int C, int64_t HW, float *out, void *stream);
int tmr_split_conv(const void *xp0, int C0, const int32_t *unit_image, const void *xp1, int C1, int U,
                   int H, int W, int ks, int prec, const void *wpack, const float *wmax, const float *xmax,
                   const float *bias, int N, int leaky, const float *headw, const float *acc_init,
                   float *out, int flags, void *stream);

/* ---- (a16) custom_shape_3x3_maxpool2d -----------------------------------
 * utils/TM_utils.py:337-361 on device fp32 planes x [planes][H][W]: out[e] =
 * the max over the 3x3 neighbourhood taps selected by mask9 (bit 3*r + c is
 * kernel[r][c]; zero padding as F.unfold), taps in row-major order, a NaN
 * propagates and ties keep the earlier tap.  mask9 == 0 (an empty selection,
 * which torch.max rejects) or bits above 8 return TMR_E_INVALID. */
int tmr_maxpool3x3(const float *x, int64_t planes, int H, int W, int mask9, float *out, void *stream);

/* ---- (a14-a16) peak finder + box decode ------------------------------------
 * Get_pred_boxes per unit (utils/TM_utils.py:245-282): p = sigmoid(o) (or o
 * itself when input_is_prob), masked 3x3 local max with zero padding,
 * p >= thr, row-major compaction (no cap), decode.  Outputs per unit u at
 * stride cap = H*W: logits[(u*cap+i)*2] = (p, 0) (TM_utils.py:260-261),
 * box[(u*cap+i)*4] (normalised xyxy), ref[(u*cap+i)*2], counts[u]; a unit
 * with no peak (counts[u] = 0) gets the reference's dummy row at its row 0
 * (logits (0,0), box (0,0,1e-14,1e-14), ref (0,0); TM_utils.py:288-291).
 * prob [U,H,W] receives the probability map (required).  With
 * TMR_PEAKS_PROB_SCRATCH or-ed into input_is_prob it is scratch only: a
 * pixel whose logit lies well below its unit's threshold holds -1 there (its
 * sigmoid is skipped); the candidates are the same.
 * exp_table (device, nullable): the reference-exp table (tmr_amd/exp_table.py:
 * 128-B header, uint32 offsets[65537], sorted uint16 low halves).  The decode's
 * exp (TM_utils.py:272) is the correctly rounded value except at the table's
 * inputs, where it is the other neighbour, as the reference's torch.exp (MKL
 * vsExp) rounds; NULL = correctly rounded everywhere. */
#define TMR_PEAKS_PROB_SCRATCH 2  /* input_is_prob flag: prob is scratch (see above) */
int tmr_peaks_decode(const float *o, int input_is_prob, const float *reg, int U, int H, int W,
                     const tmr_peak_param_t *params, float *prob, float *logits, float *box,
                     float *ref, int32_t *counts, const void *exp_table, void *stream);

/* ---- (a17-a19) per-image greedy NMS over the exemplar-ordered union --------
 * torchvision.ops.nms (utils/TM_utils.py:317-323) on, per image g, the
 * concatenation (in unit order seg_units[g] .. seg_units[g+1]-1) of each
 * unit's candidates, or of the dummy row [0,0,1e-14,1e-14]/score 0 when the
 * unit has none (TM_utils.py:288-291).  Unit u's counts[u] candidates start
 * at row unit_off[u] (device int64[U]) of logits [.,2] / box [.,4] /
 * ref [.,2]; the score is logits[.,0] (:319).  seg_units (device int32[G+1]),
 * cand_off (device int64[G+1], the offsets of those unions) and nb_off
 * (device int64[G+1], prefix sums of ceil(n_g/64)) are computed on the
 * host from the candidate counts (one sync, as the reference's torch.where);
 * sum_nb = nb_off[G], max_cand = max n_g.
 * Outputs are written per image at cand_off[g]: keep-ordered logits [n,2] =
 * (score, 0), boxes [n,4], refs [n,2], optionally the keep indices (int64,
 * local to the image's union, = torchvision's return value) and kept[g].
 * `work` holds TMR_SIZE_NMS_WORK(total_cand, sum_nb, max_cand, G) bytes:
 * linear in the candidates, at most ~640 B per candidate (the suppressor
 * lists take 512 B of it: 128 entries per row, sized per 64-row block), so
 * the worst case -- every pixel of 16 units at 192^2 a candidate of one
 * image, 589,824 rows -- needs ~0.38 GB.  An image of more than 655,360
 * candidates is refused with TMR_E_INVALID (the greedy wave's LDS holds the
 * kept bitmap), never truncated. */
int tmr_nms(const float *logits, const float *box, const float *ref, const int32_t *counts,
            const int64_t *unit_off, const int32_t *seg_units, const int64_t *cand_off,
            const int64_t *nb_off,
            int G, int64_t total_cand, int64_t max_cand, int64_t sum_nb, double iou_threshold,
            float *out_logits, float *out_boxes, float *out_refs, int64_t *out_keep,
            int32_t *kept, void *work, void *stream);
/* tmr_nms for images of at most TMR_NMS_SMALL candidates, sized on the
 * DEVICE from counts (no host sync before it, so it can follow the peak
 * finder inside one captured forward): image g's kept rows are written at
 * row g * TMR_NMS_SMALL of out_logits [G*TMR_NMS_SMALL,2] / out_boxes [.,4] /
 * out_refs [.,2] (+ out_keep, nullable), kept[g] = their count -- the same
 * rows and order tmr_nms produces -- or kept[g] = -1 when the image's union
 * exceeds TMR_NMS_SMALL rows (then nothing is written for it: run tmr_nms).
 * One workgroup per image, no work memory. */
#define TMR_NMS_SMALL 256
int tmr_nms_small(const float *logits, const float *box, const float *ref, const int32_t *counts,
                  const int64_t *unit_off, const int32_t *seg_units, int G, double iou_threshold,
                  float *out_logits, float *out_boxes, float *out_refs, int64_t *out_keep,
                  int32_t *kept, void *stream);

/* ---- (§8f f1) streaming mapper statistics ---------------------------------
 * Per image b of x [B][n] fp32 (the backbone feature the mapper computes,
 * mapper.py:94), out[b] = {mean, std, max, sparsity} (fp64), as
 * mapper.py:97-101 computes them with numpy: mean = np.mean(f) and
 * std = np.std(f) (population) each correctly rounded to fp32 from an fp64
 * evaluation (numpy's float32 pairwise sums differ by a few fp32 ulps),
 * max = np.max(f) exactly, sparsity = np.mean(f <= 0) = count / n exactly.
 * Deterministic (fixed reduction order).  `work` holds
 * TMR_SIZE_STATS_WORK(B) bytes. */
int tmr_feature_stats(const float *x, int B, int64_t n, void *work, double *out, void *stream);

/* ---- the decode's reference-exp table, compact form ------------------------
 * Host-only (no device pointers, no stream).  The table of fp32 inputs where
 * the reference's torch.exp (utils/TM_utils.py:272, MKL vsExp on the golden
 * host) is not the correctly rounded exp (tmr_amd/exp_table.py) is committed
 * as a range-coded candidate bitmap (csrc/exp_codec.cpp).
 * tmr_exp_table_encode: `exc` = the n recorded fp32 bit patterns, sorted
 * (positive x first); out = NULL returns the blob size; else writes it and
 * returns its size (< 0: TMR_E_INVALID, or TMR_E_UNSUPPORTED when an input
 * lies outside the codec's candidate set).
 * tmr_exp_table_decode: out = NULL returns the recorded count; else writes
 * the sorted bit patterns and returns the count (< 0 on a malformed blob). */
int64_t tmr_exp_table_encode(const uint32_t *exc, int64_t n, uint8_t *out, int64_t cap);
int64_t tmr_exp_table_decode(const uint8_t *blob, int64_t nbytes, uint32_t *out, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif /* TMR_H_ */
