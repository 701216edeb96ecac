// KV-cache decode attention for generation (InnerSelfAttention.forward with layer_past / use_cache,
// transformer.py:245-282; the cache branch is :261-268, the masked softmax :171-217).
//
// The reference grows its cache with torch.cat((past_key, key), dim=-2) every generated event: O(L^2) copies per
// sequence. Here the cache is a preallocated token-major buffer per layer, k/v: [B, cap, D] (D = H*hd, the same
// row layout the packed QKV projection writes), and a step
//   1. appends the Lq new key/value rows from the packed qkv buffer into rows [past, past + Lq)  (esgpt_kv_append)
//   2. attends each new query to rows [0, past + Lq) of the cache                                 (esgpt_attn_decode)
// Query i sits at key position p_i = past + i; key j is visible iff j <= p_i, (local) p_i - j < window, and
// key_mask[b, j] (the full-length event mask, the reference's expand_mask(batch.event_mask) computed before the batch
// is trimmed to its last event, conditionally_independent_model.py:226-238). Scores q.k in f32 without 1/sqrt(hd)
// scaling, softmax in f32; with bf16 data the probabilities are rounded to bf16 before P.V as the reference casts
// attn_weights to value.dtype (:207). Rows whose query is padded, or that see no valid key, are zeros (the reference
// zeroes them one op later, transformer.py:818-823).
//
// Decode is HBM-bound: every visible cached row is read once per (query, head) -> 2*hd*s bytes per visible pair.
// One workgroup (4 waves) per (b, h, query); the waves take interleaved 64-key blocks, each lane scores one key
// (q broadcast from LDS, the key row read as 16-B vectors), P.V runs lane-per-dimension over the block with the
// probabilities broadcast from LDS (coalesced value rows, a whole 64-key block in flight, issued with the key rows),
// and the four partial softmax states merge through LDS.
#include "common.h"

using namespace esgpt;

namespace {

constexpr int DEC_WAVES = 4;
constexpr int PV_ROWS = 64;  // value elements per lane in flight per P.V step (64 rows for hd <= 64)

template <typename T>
__global__ __launch_bounds__(256) void kv_append_kernel(const T* __restrict__ qkv, int64_t ld_qkv, T* __restrict__ kc,
                                                         T* __restrict__ vc, int64_t B, int64_t Lq, int64_t past,
                                                         int64_t cap, int64_t D) {
  const int64_t n = B * Lq * D;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = e % D;
    const int64_t t = e / D;
    const int64_t i = t % Lq, b = t / Lq;
    const T* src = qkv + (b * Lq + i) * ld_qkv;
    const int64_t dst = (b * cap + past + i) * D + d;
    kc[dst] = src[D + d];
    vc[dst] = src[2 * D + d];
  }
}

__device__ __forceinline__ float round_like(float p, float) { return p; }
__device__ __forceinline__ float round_like(float p, bf16) { return __bfloat162float(__float2bfloat16(p)); }

template <typename T, int HDP>
__device__ __forceinline__ float dot_row(const float* __restrict__ qs, const T* __restrict__ kp, int hd) {
  float s = 0.f;
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int d = 0; d < HDP; d += 4) {
      if (d < hd) {
        const float4 kv = *reinterpret_cast<const float4*>(kp + d);
        s = fmaf(qs[d], kv.x, s);
        s = fmaf(qs[d + 1], kv.y, s);
        s = fmaf(qs[d + 2], kv.z, s);
        s = fmaf(qs[d + 3], kv.w, s);
      }
    }
  } else {
#pragma unroll
    for (int d = 0; d < HDP; d += 8) {
      if (d < hd) {
        const uint4 raw = *reinterpret_cast<const uint4*>(kp + d);
        const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          s = fmaf(qs[d + 2 * u], bf16_bits_to_f32((uint16_t)(w[u] & 0xffffu)), s);
          s = fmaf(qs[d + 2 * u + 1], bf16_bits_to_f32((uint16_t)(w[u] >> 16)), s);
        }
      }
    }
  }
  return s;
}

// HDP: head dim rounded up to a multiple of 8 (<= 128); DPL = dims per lane in P.V.
template <typename T, int HDP>
__global__ __launch_bounds__(256) void attn_decode_kernel(const T* __restrict__ q, int64_t ld_q,
                                                          const T* __restrict__ kc, const T* __restrict__ vc,
                                                          const uint8_t* __restrict__ kmask,
                                                          const uint8_t* __restrict__ qmask, T* __restrict__ o,
                                                          int64_t ld_o, int64_t H, int64_t Lq, int64_t Lk, int64_t cap,
                                                          int hd, int64_t window) {
  constexpr int DPL = (HDP + 63) / 64;
  __shared__ float qs[HDP];
  __shared__ float ps[DEC_WAVES][64];
  __shared__ float wm[DEC_WAVES], wl[DEC_WAVES];
  __shared__ float wacc[DEC_WAVES][DPL * 64];

  const int64_t gid = blockIdx.x;  // (b, h, i) with i fastest
  const int64_t i = gid % Lq;
  const int64_t bh = gid / Lq;
  const int64_t h = bh % H, b = bh / H;
  const int64_t D = H * hd;
  const int lane = lane_id();
  const int w = threadIdx.x >> 6;
  const int64_t pos = (Lk - Lq) + i;
  const bool qvalid = qmask ? (qmask[b * Lq + i] != 0) : true;

  const T* qp = q + (b * Lq + i) * ld_q + h * hd;
  for (int d = threadIdx.x; d < HDP; d += blockDim.x) qs[d] = (d < hd) ? to_f32(qp[d]) : 0.f;
  __syncthreads();

  const int64_t jlo = (window > 0) ? max((int64_t)0, pos - window + 1) : 0;
  const int64_t nkeys = qvalid ? (pos - jlo + 1) : 0;
  const int64_t nblk = (nkeys + 63) / 64;
  const T* kbase = kc + b * cap * D + h * hd;
  const T* vbase = vc + b * cap * D + h * hd;
  const uint8_t* km = kmask ? kmask + b * Lk : nullptr;

  float m = -INFINITY, l = 0.f;
  float acc[DPL];
#pragma unroll
  for (int u = 0; u < DPL; ++u) acc[u] = 0.f;

  constexpr int PVU = PV_ROWS / DPL;  // value rows per P.V step (registers: PVU * DPL)
  for (int64_t blk = w; blk < nblk; blk += DEC_WAVES) {
    const int64_t j0 = jlo + blk * 64;
    const int64_t j = j0 + lane;
    const int64_t nb = min((int64_t)64, pos + 1 - j0);
    // The first P.V step's value rows are loaded together with the key rows (one memory round trip per block for
    // hd <= 64); rows past the block clamp to its last row and get p = 0.
    float vv[PVU][DPL];
#pragma unroll
    for (int x = 0; x < PVU; ++x) {
      const T* vp = vbase + (j0 + min(x, (int)nb - 1)) * D;
#pragma unroll
      for (int u = 0; u < DPL; ++u) {
        const int d = lane + 64 * u;
        vv[x][u] = (d < hd) ? to_f32(vp[d]) : 0.f;
      }
    }
    float s = -INFINITY;
    if (lane < nb && (!km || km[j])) s = dot_row<T, HDP>(qs, kbase + j * D, hd);
    const float mb = wave_max(s);
    const float mn = fmaxf(m, mb);
    if (mn == -INFINITY) continue;  // wave-uniform: the whole block is masked
    const float c = (m == -INFINITY) ? 0.f : __expf(m - mn);
    const float p = (s == -INFINITY) ? 0.f : __expf(s - mn);
    l = l * c + wave_sum(p);
    m = mn;
    ps[w][lane] = round_like(p, T{});
    // ps is private to this wave; a wave executes in lockstep, so only an LDS fence is needed.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < DPL; ++u) acc[u] *= c;
    // P.V: PVU value rows in flight per step, so the row loads overlap instead of forming one chain per key.
    for (int t0 = 0; t0 < nb; t0 += PVU) {
      if (t0 > 0) {
#pragma unroll
        for (int x = 0; x < PVU; ++x) {
          const T* vp = vbase + (j0 + min(t0 + x, (int)nb - 1)) * D;
#pragma unroll
          for (int u = 0; u < DPL; ++u) {
            const int d = lane + 64 * u;
            vv[x][u] = (d < hd) ? to_f32(vp[d]) : 0.f;
          }
        }
      }
#pragma unroll
      for (int x = 0; x < PVU; ++x) {
        const float pt = (t0 + x < nb) ? ps[w][t0 + x] : 0.f;
#pragma unroll
        for (int u = 0; u < DPL; ++u) acc[u] = fmaf(pt, vv[x][u], acc[u]);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  if (lane == 0) {
    wm[w] = m;
    wl[w] = l;
  }
#pragma unroll
  for (int u = 0; u < DPL; ++u) wacc[w][lane + 64 * u] = acc[u];
  __syncthreads();
  if (w != 0) return;
  float M = -INFINITY;
#pragma unroll
  for (int x = 0; x < DEC_WAVES; ++x) M = fmaxf(M, wm[x]);
  float Ls = 0.f;
  float out[DPL];
#pragma unroll
  for (int u = 0; u < DPL; ++u) out[u] = 0.f;
  if (M != -INFINITY) {
#pragma unroll
    for (int x = 0; x < DEC_WAVES; ++x) {
      if (wm[x] == -INFINITY) continue;
      const float c = __expf(wm[x] - M);
      Ls = fmaf(wl[x], c, Ls);
#pragma unroll
      for (int u = 0; u < DPL; ++u) out[u] = fmaf(wacc[x][lane + 64 * u], c, out[u]);
    }
  }
  const float inv = (Ls > 0.f) ? 1.f / Ls : 0.f;
  T* op = o + (b * Lq + i) * ld_o + h * hd;
#pragma unroll
  for (int u = 0; u < DPL; ++u) {
    const int d = lane + 64 * u;
    if (d < hd) op[d] = from_f32<T>(out[u] * inv);
  }
}

template <typename T>
int launch_decode(const void* q, int64_t ld_q, const void* kc, const void* vc, const uint8_t* kmask,
                  const uint8_t* qmask, void* o, int64_t ld_o, int64_t B, int64_t H, int64_t Lq, int64_t Lk,
                  int64_t cap, int64_t hd, int64_t window, hipStream_t st) {
  const dim3 grid((unsigned)(B * H * Lq)), block(64 * DEC_WAVES);
#define DEC(HD)                                                                                                     \
  hipLaunchKernelGGL((attn_decode_kernel<T, HD>), grid, block, 0, st, (const T*)q, ld_q, (const T*)kc,             \
                     (const T*)vc, kmask, qmask, (T*)o, ld_o, H, Lq, Lk, cap, (int)hd, window)
  if (hd <= 8) DEC(8);
  else if (hd <= 16) DEC(16);
  else if (hd <= 32) DEC(32);
  else if (hd <= 64) DEC(64);
  else DEC(128);
#undef DEC
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

}  // namespace

extern "C" {

int esgpt_kv_append(const void* qkv, int64_t ld_qkv, void* k_cache, void* v_cache, int64_t B, int64_t Lq,
                    int64_t past, int64_t cap, int64_t D, int dtype, void* stream) {
  ESGPT_REQUIRE(qkv && k_cache && v_cache && B >= 0 && Lq >= 0 && past >= 0 && D > 0 && past + Lq <= cap);
  ESGPT_REQUIRE(ld_qkv >= 3 * D && (dtype == ESGPT_F32 || dtype == ESGPT_BF16));
  const int64_t n = B * Lq * D;
  if (n == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  const int64_t blocks = min(cdiv(n, 256), (int64_t)8192);
  if (dtype == ESGPT_F32)
    hipLaunchKernelGGL((kv_append_kernel<float>), dim3((unsigned)blocks), dim3(256), 0, st, (const float*)qkv, ld_qkv,
                       (float*)k_cache, (float*)v_cache, B, Lq, past, cap, D);
  else
    hipLaunchKernelGGL((kv_append_kernel<bf16>), dim3((unsigned)blocks), dim3(256), 0, st, (const bf16*)qkv, ld_qkv,
                       (bf16*)k_cache, (bf16*)v_cache, B, Lq, past, cap, D);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_attn_decode(const void* q, int64_t ld_q, const void* k_cache, const void* v_cache, const uint8_t* key_mask,
                      const uint8_t* query_mask, void* o, int64_t ld_o, int64_t B, int64_t H, int64_t Lq, int64_t Lk,
                      int64_t cap, int64_t hd, int64_t window, int dtype, void* stream) {
  ESGPT_REQUIRE(q && k_cache && v_cache && o && hd > 0 && hd <= 128 && Lq >= 0 && Lq <= Lk && Lk <= cap);
  ESGPT_REQUIRE(window >= 0 && ld_q >= H * hd && ld_o >= H * hd && (dtype == ESGPT_F32 || dtype == ESGPT_BF16));
  // 16-B row loads: rows and head slices must stay 16-B aligned.
  ESGPT_REQUIRE(dtype == ESGPT_F32 ? (hd % 4 == 0) : (hd % 8 == 0));
  if (B * H * Lq == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  if (dtype == ESGPT_F32)
    return launch_decode<float>(q, ld_q, k_cache, v_cache, key_mask, query_mask, o, ld_o, B, H, Lq, Lk, cap, hd,
                                window, st);
  return launch_decode<bf16>(q, ld_q, k_cache, v_cache, key_mask, query_mask, o, ld_o, B, H, Lq, Lk, cap, hd, window,
                             st);
}

}  // extern "C"
