// Version / error strings of the libtmr.so C ABI (include/tmr.h).
#include "../../include/tmr.h"

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
