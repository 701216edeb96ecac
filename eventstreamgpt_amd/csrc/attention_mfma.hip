// bf16 MFMA flash attention for gfx950 — placeholder until the MFMA kernels land; the generic path serves.
#include "common.h"

int esgpt_attn_fwd_mfma(const void*, const void*, const void*, int64_t, int64_t, void*, int64_t, float*,
                        const uint8_t*, const uint8_t*, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                        hipStream_t) {
  return ESGPT_ERR_UNSUPPORTED;
}
int esgpt_attn_bwd_mfma(const void*, const void*, const void*, int64_t, int64_t, const void*, int64_t, const void*,
                        int64_t, const float*, const uint8_t*, const uint8_t*, void*, void*, void*, int64_t, int64_t,
                        int64_t, int64_t, int64_t, int64_t, int64_t, float*, hipStream_t) {
  return ESGPT_ERR_UNSUPPORTED;
}
bool esgpt_attn_mfma_supported(int64_t, int64_t, int64_t, int64_t, int64_t, int64_t) { return false; }
