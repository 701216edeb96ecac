// Nested-attention glue for gfx950: the tensor shuffles of StructuredAttention.forward
// (EventStream/transformer/structured_attention.py:28-219, training path: history prepended, the last graph element
// replaced by the contextualised event) and the InnerBlock residual (transformer.py:409-461) as single-pass kernels,
// in place of ATen where / pad / cat / slice copies / dropout / add launches and their zero-filled backward slices.
//
//   residual      h[r]  = mask(r) ? x[xr(r)] + dropout(y[r]) : 0              (mask(r) = row_mask[r / mask_div])
//                 xr(r) = r, or with static_kv_first (skip_T = T) the rows of x = [Bs, T, D] after each first one
//   na_split      per[e] = event_mask[e] ? x[e, G-1] : 0                       (x = [B·L, G, D]: the whole-event element)
//   na_assemble   seq[e] = [ctx[e-1] (zeros for an event at l = 0), x[e, 0 .. G-2], ctx[e]]   ([B·L, G+1, D])
//   na_head_split head = x[:, 0 .. G-2], last = x[:, G-1] in the head GEMM's dtype (the NA output layer's operands)
// and their backwards. Every kernel is an f32 streaming pass (HBM-bound: algorithmic bytes = what it reads + writes
// once); 16-B accesses, one float4 per thread per iteration, grid-stride. Dropout: the library's counter hash of
// (seed, r·D + c) (common.h), regenerated in the backward.
#include "common.h"

using namespace esgpt;

namespace {

constexpr int kThreads = 256;

inline unsigned grid_for(int64_t n4) {
  const int64_t g = cdiv(n4, kThreads);
  return (unsigned)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

template <typename TY>
__device__ __forceinline__ float4 ld4y(const TY* p) {
  if constexpr (sizeof(TY) == 4) {
    return ld4(reinterpret_cast<const float*>(p));
  } else {
    const uint2 w = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
                       __uint_as_float(w.y & 0xffff0000u));
  }
}

template <typename TY>
__device__ __forceinline__ void st4y(TY* p, float4 v) {
  if constexpr (sizeof(TY) == 4) {
    st4(reinterpret_cast<float*>(p), v);
  } else {
    const uint32_t lo = (uint32_t)f32_to_bf16_bits(v.x) | ((uint32_t)f32_to_bf16_bits(v.y) << 16);
    const uint32_t hi = (uint32_t)f32_to_bf16_bits(v.z) | ((uint32_t)f32_to_bf16_bits(v.w) << 16);
    *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
  }
}

__device__ __forceinline__ int64_t x_row(int64_t r, int64_t skip_T) {
  return skip_T ? (r / (skip_T - 1)) * skip_T + 1 + r % (skip_T - 1) : r;
}

// h = mask ? x + dropout(y) : 0 (x NULL: 0 — a plain dropout, e.g. the NA input layer's)
template <typename TY>
__global__ __launch_bounds__(kThreads) void residual_fwd_kernel(const float* __restrict__ x, const TY* __restrict__ y,
                                                               const uint8_t* __restrict__ mask, int64_t mask_div,
                                                               int64_t skip_T, float p, const uint64_t* seed,
                                                               int64_t N, int64_t D, float* __restrict__ h) {
  const DropoutSpec dr = make_dropout(p, seed);
  const bool i32 = (uint64_t)N * (uint64_t)D <= 0xffffffffull;  // 32-bit dropout element indices
  const int64_t n4 = N * D / 4, D4 = D / 4;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
    const int64_t r = i / D4, c = (i - r * D4) * 4;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    if (mask == nullptr || mask[r / mask_div]) {
      const float4 xv = x ? ld4(x + x_row(r, skip_T) * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 yv = ld4y(y + r * D + c);
      if (p > 0.f) {
        float z0, z1, z2, z3;
        dropout_pair_rc(dr, i32, r, D, c, z0, z1);
        dropout_pair_rc(dr, i32, r, D, c + 2, z2, z3);
        yv.x *= z0, yv.y *= z1, yv.z *= z2, yv.w *= z3;
      }
      o = make_float4(xv.x + yv.x, xv.y + yv.y, xv.z + yv.z, xv.w + yv.w);
    }
    st4(h + r * D + c, o);
  }
}

// dy = mask ? dropout'(dh) : 0 over the N output rows; dx (optional) over the x rows: mask ? dh : 0, and zeros for the
// rows of x no output reads (the first row of each sequence under skip_T)
template <typename TY>
__global__ __launch_bounds__(kThreads) void residual_bwd_kernel(const float* __restrict__ dh,
                                                               const uint8_t* __restrict__ mask, int64_t mask_div,
                                                               int64_t skip_T, float p, const uint64_t* seed,
                                                               int64_t N, int64_t D, float* __restrict__ dx,
                                                               TY* __restrict__ dy) {
  const DropoutSpec dr = make_dropout(p, seed);
  const bool i32 = (uint64_t)N * (uint64_t)D <= 0xffffffffull;  // 32-bit dropout element indices
  const int64_t D4 = D / 4, n4 = N * D4;
  const int64_t xN = skip_T ? N / (skip_T - 1) * skip_T : N;
  const int64_t total = n4 + (dx ? xN * D4 : 0);
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kThreads) {
    if (i < n4) {
      const int64_t r = i / D4, c = (i - r * D4) * 4;
      float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
      if (mask == nullptr || mask[r / mask_div]) {
        g = ld4(dh + r * D + c);
        if (p > 0.f) {
          float z0, z1, z2, z3;
          dropout_pair_rc(dr, i32, r, D, c, z0, z1);
          dropout_pair_rc(dr, i32, r, D, c + 2, z2, z3);
          g.x *= z0, g.y *= z1, g.z *= z2, g.w *= z3;
        }
      }
      st4y(dy + r * D + c, g);
    } else {
      const int64_t j = i - n4, xr = j / D4, c = (j - xr * D4) * 4;
      float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
      int64_t r = xr;
      bool live = true;
      if (skip_T) {
        const int64_t t = xr % skip_T;
        live = t != 0;
        r = (xr / skip_T) * (skip_T - 1) + t - 1;
      }
      if (live && (mask == nullptr || mask[r / mask_div])) g = ld4(dh + r * D + c);
      st4(dx + xr * D + c, g);
    }
  }
}

// per[e] = m[e] ? x[e, G-1] : 0
__global__ __launch_bounds__(kThreads) void na_split_fwd_kernel(const float* __restrict__ x,
                                                               const uint8_t* __restrict__ m, int64_t BL, int64_t G,
                                                               int64_t D, float* __restrict__ per) {
  const int64_t D4 = D / 4, n4 = BL * D4;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
    const int64_t e = i / D4, c = (i - e * D4) * 4;
    st4(per + e * D + c, m[e] ? ld4(x + (e * G + G - 1) * D + c) : make_float4(0.f, 0.f, 0.f, 0.f));
  }
}

// dx[e, G-1] = m[e] ? dper[e] : 0 (the other levels of dx are na_assemble_bwd's)
__global__ __launch_bounds__(kThreads) void na_split_bwd_kernel(const float* __restrict__ dper,
                                                               const uint8_t* __restrict__ m, int64_t BL, int64_t G,
                                                               int64_t D, float* __restrict__ dx) {
  const int64_t D4 = D / 4, n4 = BL * D4;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
    const int64_t e = i / D4, c = (i - e * D4) * 4;
    st4(dx + (e * G + G - 1) * D + c, m[e] ? ld4(dper + e * D + c) : make_float4(0.f, 0.f, 0.f, 0.f));
  }
}

// seq[e, 0] = l > 0 ? ctx[e-1] : 0 ; seq[e, 1 .. G-1] = x[e, 0 .. G-2] ; seq[e, G] = ctx[e]   (e = b·L + l)
__global__ __launch_bounds__(kThreads) void na_assemble_fwd_kernel(const float* __restrict__ ctx,
                                                                  const float* __restrict__ x, int64_t B, int64_t L,
                                                                  int64_t G, int64_t D, float* __restrict__ seq) {
  const int64_t D4 = D / 4, n4 = B * L * (G + 1) * D4;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
    const int64_t row = i / D4, c = (i - row * D4) * 4;
    const int64_t e = row / (G + 1), j = row - e * (G + 1);
    float4 v;
    if (j == 0) v = (e % L) ? ld4(ctx + (e - 1) * D + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    else if (j == G) v = ld4(ctx + e * D + c);
    else v = ld4(x + (e * G + j - 1) * D + c);
    st4(seq + row * D + c, v);
  }
}

// dctx[e] = dseq[e, G] + (l + 1 < L ? dseq[e+1, 0] : 0) ; dx[e, 0 .. G-2] = dseq[e, 1 .. G-1]
__global__ __launch_bounds__(kThreads) void na_assemble_bwd_kernel(const float* __restrict__ dseq, int64_t B,
                                                                  int64_t L, int64_t G, int64_t D,
                                                                  float* __restrict__ dctx, float* __restrict__ dx) {
  const int64_t D4 = D / 4, BL = B * L, nc = BL * D4, n4 = nc + BL * (G - 1) * D4;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
    if (i < nc) {
      const int64_t e = i / D4, c = (i - e * D4) * 4;
      float4 v = ld4(dseq + (e * (G + 1) + G) * D + c);
      if ((e % L) + 1 < L) {
        const float4 w = ld4(dseq + (e + 1) * (G + 1) * D + c);
        v.x += w.x, v.y += w.y, v.z += w.z, v.w += w.w;
      }
      st4(dctx + e * D + c, v);
    } else {
      const int64_t k = i - nc, row = k / D4, c = (k - row * D4) * 4;  // row over B·L·(G-1)
      const int64_t e = row / (G - 1), j = row - e * (G - 1);
      st4(dx + (e * G + j) * D + c, ld4(dseq + (e * (G + 1) + j + 1) * D + c));
    }
  }
}

// NA output-layer operands (model_output.py NA heads: content heads on levels 0..G-2, TTE on level G-1):
// head[e, 0 .. G-2] = x[e, 0 .. G-2], last[e] = x[e, G-1], cast to the head GEMM's dtype in the same pass
template <typename TO>
__global__ __launch_bounds__(kThreads) void na_head_split_fwd_kernel(const float* __restrict__ x, int64_t BL,
                                                                    int64_t G, int64_t D, TO* __restrict__ head,
                                                                    TO* __restrict__ last) {
  const int64_t D4 = D / 4, n4 = BL * G * D4;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
    const int64_t row = i / D4, c = (i - row * D4) * 4;
    const int64_t e = row / G, j = row - e * G;
    const float4 v = ld4(x + row * D + c);
    if (j + 1 < G) st4y(head + (e * (G - 1) + j) * D + c, v);
    else st4y(last + e * D + c, v);
  }
}

// dx[e, 0 .. G-2] = dhead[e, 0 .. G-2], dx[e, G-1] = dlast[e] (f32; a NULL gradient reads as zeros)
template <typename TI>
__global__ __launch_bounds__(kThreads) void na_head_split_bwd_kernel(const TI* __restrict__ dhead,
                                                                    const TI* __restrict__ dlast, int64_t BL,
                                                                    int64_t G, int64_t D, float* __restrict__ dx) {
  const int64_t D4 = D / 4, n4 = BL * G * D4;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
    const int64_t row = i / D4, c = (i - row * D4) * 4;
    const int64_t e = row / G, j = row - e * G;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j + 1 < G) {
      if (dhead) v = ld4y(dhead + (e * (G - 1) + j) * D + c);
    } else if (dlast) {
      v = ld4y(dlast + e * D + c);
    }
    st4(dx + row * D + c, v);
  }
}

}  // namespace

// Row-tile mask of a token matrix whose event e owns rows [e·rpe, (e+1)·rpe): byte t = 1 iff some event overlapping
// rows [64t, 64t + 64) is not padded (esgpt_gemm_row_tiles).
__global__ __launch_bounds__(256) void row_tiles_kernel(const uint8_t* __restrict__ em, int64_t n_events, int64_t rpe,
                                                        uint8_t* __restrict__ tiles, int64_t nt) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= nt) return;
  const int64_t e0 = (64 * t) / rpe, e1 = min(n_events - 1, (64 * t + 63) / rpe);
  uint8_t any = 0;
  for (int64_t e = e0; e <= e1; ++e) any |= em[e] != 0;
  tiles[t] = any;
}

extern "C" {

int esgpt_residual_fwd(const float* x, const void* y, int y_dtype, const uint8_t* row_mask, int64_t mask_div,
                       int64_t skip_T, float dropout_p, const uint64_t* seed, int64_t N, int64_t D, float* h,
                       void* stream) {
  ESGPT_REQUIRE(y && h && N >= 0 && D > 0 && D % 4 == 0 && mask_div >= 1 && (skip_T == 0 || skip_T >= 2));
  ESGPT_REQUIRE(x || skip_T == 0);
  ESGPT_REQUIRE(y_dtype == ESGPT_F32 || y_dtype == ESGPT_BF16);
  ESGPT_REQUIRE(skip_T == 0 || N % (skip_T - 1) == 0);
  ESGPT_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || seed));
  ESGPT_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)h % 16) == 0 && ((uintptr_t)y % 8) == 0);
  if (N == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  const unsigned g = grid_for(N * D / 4);
  if (y_dtype == ESGPT_F32)
    residual_fwd_kernel<float><<<g, kThreads, 0, st>>>(x, (const float*)y, row_mask, mask_div, skip_T, dropout_p,
                                                       seed, N, D, h);
  else
    residual_fwd_kernel<bf16><<<g, kThreads, 0, st>>>(x, (const bf16*)y, row_mask, mask_div, skip_T, dropout_p, seed,
                                                      N, D, h);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_residual_bwd(const float* dh, const uint8_t* row_mask, int64_t mask_div, int64_t skip_T, float dropout_p,
                       const uint64_t* seed, int64_t N, int64_t D, float* dx, void* dy, int y_dtype, void* stream) {
  ESGPT_REQUIRE(dh && dy && N >= 0 && D > 0 && D % 4 == 0 && mask_div >= 1 && (skip_T == 0 || skip_T >= 2));
  ESGPT_REQUIRE(y_dtype == ESGPT_F32 || y_dtype == ESGPT_BF16);
  ESGPT_REQUIRE(skip_T == 0 || N % (skip_T - 1) == 0);
  ESGPT_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || seed));
  ESGPT_REQUIRE(((uintptr_t)dh % 16) == 0 && ((uintptr_t)dx % 16) == 0 && ((uintptr_t)dy % 8) == 0);
  if (N == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  const int64_t xN = skip_T ? N / (skip_T - 1) * skip_T : N;
  const unsigned g = grid_for((N + (dx ? xN : 0)) * D / 4);
  if (y_dtype == ESGPT_F32)
    residual_bwd_kernel<float><<<g, kThreads, 0, st>>>(dh, row_mask, mask_div, skip_T, dropout_p, seed, N, D, dx,
                                                       (float*)dy);
  else
    residual_bwd_kernel<bf16><<<g, kThreads, 0, st>>>(dh, row_mask, mask_div, skip_T, dropout_p, seed, N, D, dx,
                                                      (bf16*)dy);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_na_split_fwd(const float* x, const uint8_t* event_mask, int64_t BL, int64_t G, int64_t D, float* per,
                       void* stream) {
  ESGPT_REQUIRE(x && event_mask && per && BL >= 0 && G >= 1 && D > 0 && D % 4 == 0);
  ESGPT_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)per % 16) == 0);
  if (BL == 0) return ESGPT_OK;
  na_split_fwd_kernel<<<grid_for(BL * D / 4), kThreads, 0, as_stream(stream)>>>(x, event_mask, BL, G, D, per);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_na_split_bwd(const float* dper, const uint8_t* event_mask, int64_t BL, int64_t G, int64_t D, float* dx,
                       void* stream) {
  ESGPT_REQUIRE(dper && event_mask && dx && BL >= 0 && G >= 1 && D > 0 && D % 4 == 0);
  ESGPT_REQUIRE(((uintptr_t)dper % 16) == 0 && ((uintptr_t)dx % 16) == 0);
  if (BL == 0) return ESGPT_OK;
  na_split_bwd_kernel<<<grid_for(BL * D / 4), kThreads, 0, as_stream(stream)>>>(dper, event_mask, BL, G, D, dx);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_na_assemble_fwd(const float* ctx, const float* x, int64_t B, int64_t L, int64_t G, int64_t D, float* seq,
                          void* stream) {
  ESGPT_REQUIRE(ctx && x && seq && B >= 0 && L >= 0 && G >= 1 && D > 0 && D % 4 == 0);
  ESGPT_REQUIRE(((uintptr_t)ctx % 16) == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)seq % 16) == 0);
  if (B * L == 0) return ESGPT_OK;
  na_assemble_fwd_kernel<<<grid_for(B * L * (G + 1) * D / 4), kThreads, 0, as_stream(stream)>>>(ctx, x, B, L, G, D,
                                                                                                  seq);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_na_assemble_bwd(const float* dseq, int64_t B, int64_t L, int64_t G, int64_t D, float* dctx, float* dx,
                          void* stream) {
  ESGPT_REQUIRE(dseq && dctx && dx && B >= 0 && L >= 0 && G >= 1 && D > 0 && D % 4 == 0);
  ESGPT_REQUIRE(((uintptr_t)dseq % 16) == 0 && ((uintptr_t)dctx % 16) == 0 && ((uintptr_t)dx % 16) == 0);
  if (B * L == 0) return ESGPT_OK;
  na_assemble_bwd_kernel<<<grid_for(B * L * G * D / 4), kThreads, 0, as_stream(stream)>>>(dseq, B, L, G, D, dctx,
                                                                                           dx);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_na_head_split_fwd(const float* x, int64_t BL, int64_t G, int64_t D, void* head, void* last, int out_dtype,
                            void* stream) {
  ESGPT_REQUIRE(x && head && last && BL >= 0 && G >= 2 && D > 0 && D % 4 == 0);
  ESGPT_REQUIRE(out_dtype == ESGPT_F32 || out_dtype == ESGPT_BF16);
  ESGPT_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)head % 8) == 0 && ((uintptr_t)last % 8) == 0);
  if (BL == 0) return ESGPT_OK;
  const unsigned g = grid_for(BL * G * D / 4);
  if (out_dtype == ESGPT_F32)
    na_head_split_fwd_kernel<float><<<g, kThreads, 0, as_stream(stream)>>>(x, BL, G, D, (float*)head, (float*)last);
  else
    na_head_split_fwd_kernel<bf16><<<g, kThreads, 0, as_stream(stream)>>>(x, BL, G, D, (bf16*)head, (bf16*)last);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_na_head_split_bwd(const void* dhead, const void* dlast, int in_dtype, int64_t BL, int64_t G, int64_t D,
                            float* dx, void* stream) {
  ESGPT_REQUIRE(dx && BL >= 0 && G >= 2 && D > 0 && D % 4 == 0);
  ESGPT_REQUIRE(in_dtype == ESGPT_F32 || in_dtype == ESGPT_BF16);
  ESGPT_REQUIRE(((uintptr_t)dx % 16) == 0 && ((uintptr_t)dhead % 8) == 0 && ((uintptr_t)dlast % 8) == 0);
  if (BL == 0) return ESGPT_OK;
  const unsigned g = grid_for(BL * G * D / 4);
  if (in_dtype == ESGPT_F32)
    na_head_split_bwd_kernel<float><<<g, kThreads, 0, as_stream(stream)>>>((const float*)dhead, (const float*)dlast,
                                                                          BL, G, D, dx);
  else
    na_head_split_bwd_kernel<bf16><<<g, kThreads, 0, as_stream(stream)>>>((const bf16*)dhead, (const bf16*)dlast, BL,
                                                                         G, D, dx);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_row_tiles(const uint8_t* event_mask, int64_t n_events, int64_t rows_per_event, uint8_t* tiles,
                    void* stream) {
  ESGPT_REQUIRE(event_mask && tiles && n_events >= 0 && rows_per_event >= 1);
  const int64_t nt = cdiv(n_events * rows_per_event, 64);
  if (nt == 0) return ESGPT_OK;
  row_tiles_kernel<<<dim3((unsigned)cdiv(nt, 256)), dim3(256), 0, as_stream(stream)>>>(event_mask, n_events,
                                                                                        rows_per_event, tiles, nt);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

}  // extern "C"
