// gemm.hip -- batched (prefill) quantized mat-mul.
#include "kcpp_common.h"
#include "kcpp_internal.h"

int gemv_cols(int type, const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, int64_t Mtot,
              int64_t c0, float *Y, int64_t ldy, const float *res, int64_t ldr, int mode, void *stream);

extern "C" {

int64_t kcpp_gemm_workspace_bytes(int type, int64_t K, int64_t N, int64_t M) { return 0; }

int kcpp_gemm(int type, const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, float *Y,
              int64_t ldy, const float *res, int64_t ldr, int mode, void *ws, void *stream) {
    for (int64_t c0 = 0; c0 < M; c0 += 8) {
        const int64_t mc = M - c0 < 8 ? M - c0 : 8;
        int rc = gemv_cols(type, W, W2, K, N, act, mc, M, c0, Y, ldy, res, ldr, mode, stream);
        if (rc) return rc;
    }
    return 0;
}

}  // extern "C"
