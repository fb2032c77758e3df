// Version, error strings and the one sizing query of the libtmr.so C ABI
// (include/tmr.h).
#include <stdint.h>

#include "../../include/tmr.h"

// the per-buffer size functions of the sources (hidden; tmr_common.h)
#define TMR_INTERNAL __attribute__((visibility("hidden")))
TMR_INTERNAL int64_t tmr_template_split_bytes(int U, int C, int64_t total_rows);
TMR_INTERNAL int64_t tmr_heads_partials_floats(int N, int U, int H, int W);
TMR_INTERNAL int64_t tmr_xpack_bytes(int S, int C, int H, int W, int ks, int prec);
TMR_INTERNAL int64_t tmr_wpack_bytes(int N, int C0, int C1, int ks, int prec);
TMR_INTERNAL int64_t tmr_acc_floats(int U, int N, int H, int W);
TMR_INTERNAL int64_t tmr_nms_work_bytes(int64_t total_cand, int64_t sum_nb, int64_t max_cand, int G);
TMR_INTERNAL int64_t tmr_stats_work_bytes(int B);

extern "C" int tmr_version(void) { return TMR_ABI_VERSION; }

extern "C" const char *tmr_strerror(int rc) {
    switch (rc) {
        case TMR_OK: return "ok";
        case TMR_E_INVALID: return "tmr: invalid argument or shape";
        case TMR_E_HIP: return "tmr: HIP runtime error (kernel launch failed)";
        case TMR_E_UNSUPPORTED: return "tmr: configuration not supported by this build";
        default: return "tmr: unknown error";
    }
}

static bool fits_int(int64_t v) { return v >= INT32_MIN && v <= INT32_MAX; }

extern "C" int64_t tmr_size(int kind, int64_t d0, int64_t d1, int64_t d2, int64_t d3, int64_t d4, int64_t d5) {
    const bool small = fits_int(d0) && fits_int(d1) && fits_int(d2) && fits_int(d3) && fits_int(d4) && fits_int(d5);
    switch (kind) {
        case TMR_SIZE_TEMPLATE_SPLIT:
            return fits_int(d0) && fits_int(d1) ? tmr_template_split_bytes((int)d0, (int)d1, d2) : -1;
        case TMR_SIZE_HEADS_PARTIALS:
            return small ? tmr_heads_partials_floats((int)d0, (int)d1, (int)d2, (int)d3) : -1;
        case TMR_SIZE_XPACK: return small ? tmr_xpack_bytes((int)d0, (int)d1, (int)d2, (int)d3, (int)d4, (int)d5) : -1;
        case TMR_SIZE_WPACK: return small ? tmr_wpack_bytes((int)d0, (int)d1, (int)d2, (int)d3, (int)d4) : -1;
        case TMR_SIZE_ACC: return small ? tmr_acc_floats((int)d0, (int)d1, (int)d2, (int)d3) : -1;
        case TMR_SIZE_NMS_WORK: return fits_int(d3) ? tmr_nms_work_bytes(d0, d1, d2, (int)d3) : -1;
        case TMR_SIZE_STATS_WORK: return fits_int(d0) ? tmr_stats_work_bytes((int)d0) : -1;
        default: return -1;
    }
}
