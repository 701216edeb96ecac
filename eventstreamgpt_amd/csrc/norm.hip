// Fused elementwise stages of the transformer block for gfx950 (InnerBlock, transformer.py:394-461, and the
// CI encoder's per-block event mask, :818-823):
//
//   residual_ln_fwd   h   = rowmask ? x + dropout(y + bias) : 0          (f32 residual stream)
//                     out = LayerNorm(h) * w + b                         (f32 or bf16: the next GEMM's operand)
//   residual_ln_bwd   dh  = rowmask ? dh_in + LN'(dout) : 0 ; dx = dh ; dy = dropout'(dh)
//                     per-block column partials of dgamma, dbeta, dbias
//   bias_act_fwd/bwd  g = act(f + bias) (exact-erf GELU, tanh GELU or ReLU), dbias partials
//
// One wave per row (D <= 1024: each lane owns D/64 columns), statistics in registers (two-pass mean / variance,
// biased variance as torch.nn.LayerNorm). HBM-bound: fwd reads x (4B), y (2-4B), writes h (4B) + out (2-4B) per
// element; the backward reads dh_in, dout, h and writes dx, dy.
#include "common.h"

using namespace esgpt;

namespace {

constexpr int kRowsPerWave = 4;
constexpr int kWaves = 4;
constexpr int kMaxPerLane = 16;  // D <= 1024

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i) { return to_f32(p[i]); }

__device__ __forceinline__ uint64_t drop_idx(int64_t row, int64_t D, int64_t col) { return (uint64_t)(row * D + col); }

template <typename TY, typename TO>
__global__ __launch_bounds__(256) void residual_ln_fwd_kernel(const float* __restrict__ x, const TY* __restrict__ y,
                                                              const float* __restrict__ bias,
                                                              const uint8_t* __restrict__ rmask, float drop_p,
                                                              const uint64_t* __restrict__ seed,
                                                              const float* __restrict__ w, const float* __restrict__ b,
                                                              float eps, int64_t N, int64_t D, float* __restrict__ h,
                                                              TO* __restrict__ out, float* __restrict__ mean_o,
                                                              float* __restrict__ rstd_o) {
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int per = (int)((D + 63) / 64);
  for (int rr = 0; rr < kRowsPerWave; ++rr) {
    const int64_t row = ((int64_t)blockIdx.x * kWaves + wave) * kRowsPerWave + rr;
    if (row >= N) return;
    const bool keep_row = rmask == nullptr || rmask[row] != 0;
    float v[kMaxPerLane];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxPerLane; ++k) {
      const int64_t c = lane + 64 * k;
      v[k] = 0.f;
      if (k < per && c < D && keep_row) {
        float a = x ? x[row * D + c] : 0.f;
        if (y) {
          float t = ld(y, row * D + c) + (bias ? bias[c] : 0.f);
          if (dr.p > 0.f) t *= dropout_mult(dr, drop_idx(row, D, c));
          a += t;
        }
        v[k] = a;
      }
      s += v[k];
    }
    const float mean = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxPerLane; ++k) {
      const int64_t c = lane + 64 * k;
      if (k < per && c < D) {
        const float d = v[k] - mean;
        q += d * d;
      }
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
    for (int k = 0; k < kMaxPerLane; ++k) {
      const int64_t c = lane + 64 * k;
      if (k < per && c < D) {
        if (h) h[row * D + c] = v[k];
        out[row * D + c] = from_f32<TO>((v[k] - mean) * rstd * w[c] + b[c]);
      }
    }
    if (lane == 0) {
      mean_o[row] = mean;
      rstd_o[row] = rstd;
    }
  }
}

// Backward. part: f32 [gridDim.x, 3, D] column partials (dgamma, dbeta, dbias) of this block's rows.
template <typename TY, typename TO>
__global__ __launch_bounds__(256) void residual_ln_bwd_kernel(
    const float* __restrict__ dh_in, const TO* __restrict__ dout, const float* __restrict__ h,
    const float* __restrict__ mean_i, const float* __restrict__ rstd_i, const float* __restrict__ w,
    const uint8_t* __restrict__ rmask, float drop_p, const uint64_t* __restrict__ seed, int64_t N, int64_t D,
    float* __restrict__ dx, TY* __restrict__ dy, float* __restrict__ part) {
  __shared__ float s_part[kWaves][3][256];
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int per = (int)((D + 63) / 64);
  float pg[kMaxPerLane], pb[kMaxPerLane], py[kMaxPerLane];
#pragma unroll
  for (int k = 0; k < kMaxPerLane; ++k) pg[k] = pb[k] = py[k] = 0.f;
  for (int rr = 0; rr < kRowsPerWave; ++rr) {
    const int64_t row = ((int64_t)blockIdx.x * kWaves + wave) * kRowsPerWave + rr;
    if (row >= N) break;
    const float mean = mean_i[row], rstd = rstd_i[row];
    const bool keep_row = rmask == nullptr || rmask[row] != 0;
    float xh[kMaxPerLane], g[kMaxPerLane];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxPerLane; ++k) {
      const int64_t c = lane + 64 * k;
      xh[k] = g[k] = 0.f;
      if (k < per && c < D) {
        const float dv = ld(dout, row * D + c);
        xh[k] = (h[row * D + c] - mean) * rstd;
        g[k] = dv * w[c];
        pg[k] += dv * xh[k];
        pb[k] += dv;
        sg += g[k];
        sgx += g[k] * xh[k];
      }
    }
    sg = wave_sum(sg) / (float)D;
    sgx = wave_sum(sgx) / (float)D;
#pragma unroll
    for (int k = 0; k < kMaxPerLane; ++k) {
      const int64_t c = lane + 64 * k;
      if (k < per && c < D) {
        float d = rstd * (g[k] - sg - xh[k] * sgx);
        if (dh_in) d += dh_in[row * D + c];
        if (!keep_row) d = 0.f;
        if (dx) dx[row * D + c] = d;
        if (dy) {
          const float t = dr.p > 0.f ? d * dropout_mult(dr, drop_idx(row, D, c)) : d;
          dy[row * D + c] = from_f32<TY>(t);
          py[k] += t;
        }
      }
    }
  }
  // combine the 4 waves' column partials, one row of partials per (block, quantity)
  for (int k = 0; k < per; ++k) {
    const int64_t c0 = 64 * k;
    s_part[wave][0][lane] = pg[k];
    s_part[wave][1][lane] = pb[k];
    s_part[wave][2][lane] = py[k];
    __syncthreads();
    if (wave == 0) {
      for (int qd = 0; qd < 3; ++qd) {
        const float t = s_part[0][qd][lane] + s_part[1][qd][lane] + s_part[2][qd][lane] + s_part[3][qd][lane];
        if (c0 + lane < D) part[((int64_t)blockIdx.x * 3 + qd) * D + c0 + lane] = t;
      }
    }
    __syncthreads();
  }
}

// Column sums of part[nb, 3, D] -> sums[3, D] (deterministic: fixed block order).
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, int64_t nb, int64_t Q, int64_t D,
                                                     float* __restrict__ sums) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Q * D) return;
  const int64_t qd = i / D, c = i % D;
  float s = 0.f;
  for (int64_t b = 0; b < nb; ++b) s += part[(b * Q + qd) * D + c];
  sums[i] = s;
}

__device__ __forceinline__ float act_f(float z, int act) {
  if (act == 0) return 0.5f * z * (1.f + erff(z * 0.70710678118654752440f));
  if (act == 1) {
    const float k = 0.79788456080286535588f;  // sqrt(2/pi)
    return 0.5f * z * (1.f + tanhf(k * (z + 0.044715f * z * z * z)));
  }
  return z > 0.f ? z : 0.f;
}

__device__ __forceinline__ float act_d(float z, int act) {
  if (act == 0) {
    const float cdf = 0.5f * (1.f + erff(z * 0.70710678118654752440f));
    const float pdf = 0.39894228040143267794f * expf(-0.5f * z * z);
    return cdf + z * pdf;
  }
  if (act == 1) {
    const float k = 0.79788456080286535588f;
    const float u = k * (z + 0.044715f * z * z * z);
    const float t = tanhf(u);
    return 0.5f * (1.f + t) + 0.5f * z * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * z * z);
  }
  return z > 0.f ? 1.f : 0.f;
}

template <typename T>
__global__ __launch_bounds__(256) void bias_act_fwd_kernel(const T* __restrict__ f, const float* __restrict__ bias,
                                                           int act, int64_t N, int64_t F, T* __restrict__ g) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= N * F) return;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t j = i + k;
    if (j < N * F) g[j] = from_f32<T>(act_f(to_f32(f[j]) + bias[j % F], act));
  }
}

// dz = dg * act'(f + bias); part[blockIdx.x, F] column partials of dz over this block's rows.
constexpr int kActRows = 32;
template <typename T>
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(const T* __restrict__ dg, const T* __restrict__ f,
                                                           const float* __restrict__ bias, int act, int64_t N,
                                                           int64_t F, T* __restrict__ dz, float* __restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.x * kActRows;
  for (int64_t c = threadIdx.x; c < F; c += blockDim.x) {
    float s = 0.f;
    const float bc = bias[c];
    for (int64_t r = r0; r < min(N, r0 + kActRows); ++r) {
      const float z = to_f32(f[r * F + c]) + bc;
      const float d = to_f32(dg[r * F + c]) * act_d(z, act);
      dz[r * F + c] = from_f32<T>(d);
      s += d;
    }
    part[(int64_t)blockIdx.x * F + c] = s;
  }
}

template <typename TY, typename TO>
void launch_ln_fwd(const float* x, const void* y, const float* bias, const uint8_t* rmask, float p, const uint64_t* seed,
                   const float* w, const float* b, float eps, int64_t N, int64_t D, float* h, void* out, float* mean,
                   float* rstd, hipStream_t st) {
  const unsigned grid = (unsigned)cdiv(N, kWaves * kRowsPerWave);
  residual_ln_fwd_kernel<TY, TO><<<grid, 256, 0, st>>>(x, (const TY*)y, bias, rmask, p, seed, w, b, eps, N, D, h,
                                                       (TO*)out, mean, rstd);
}

template <typename TY, typename TO>
void launch_ln_bwd(const float* dh_in, const void* dout, const float* h, const float* mean, const float* rstd,
                   const float* w, const uint8_t* rmask, float p, const uint64_t* seed, int64_t N, int64_t D, float* dx,
                   void* dy, float* part, hipStream_t st) {
  const unsigned grid = (unsigned)cdiv(N, kWaves * kRowsPerWave);
  residual_ln_bwd_kernel<TY, TO><<<grid, 256, 0, st>>>(dh_in, (const TO*)dout, h, mean, rstd, w, rmask, p, seed, N,
                                                       D, dx, (TY*)dy, part);
}

}  // namespace

extern "C" {

int64_t esgpt_residual_ln_partials(int64_t N) { return cdiv(N, kWaves * kRowsPerWave); }

int esgpt_residual_ln_fwd(const float* x, const void* y, int y_dtype, const float* bias, const uint8_t* row_mask,
                          float dropout_p, const uint64_t* seed, const float* ln_w, const float* ln_b, float eps,
                          int64_t N, int64_t D, float* h, void* out, int out_dtype, float* mean, float* rstd,
                          void* stream) {
  ESGPT_REQUIRE(ln_w && ln_b && out && mean && rstd && D > 0 && D <= 64 * kMaxPerLane && (x || y));
  ESGPT_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || seed));
  if (N == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  const bool yb = y_dtype == ESGPT_BF16, ob = out_dtype == ESGPT_BF16;
  if (!yb && !ob) launch_ln_fwd<float, float>(x, y, bias, row_mask, dropout_p, seed, ln_w, ln_b, eps, N, D, h, out,
                                             mean, rstd, st);
  else if (!yb && ob) launch_ln_fwd<float, bf16>(x, y, bias, row_mask, dropout_p, seed, ln_w, ln_b, eps, N, D, h, out,
                                                mean, rstd, st);
  else if (yb && !ob) launch_ln_fwd<bf16, float>(x, y, bias, row_mask, dropout_p, seed, ln_w, ln_b, eps, N, D, h, out,
                                                mean, rstd, st);
  else launch_ln_fwd<bf16, bf16>(x, y, bias, row_mask, dropout_p, seed, ln_w, ln_b, eps, N, D, h, out, mean, rstd,
                                 st);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_residual_ln_bwd(const float* dh_in, const void* dout, int out_dtype, const float* h, const float* mean,
                          const float* rstd, const float* ln_w, const uint8_t* row_mask, float dropout_p,
                          const uint64_t* seed, int64_t N, int64_t D, float* dx, void* dy, int y_dtype, float* part,
                          float* sums, void* stream) {
  ESGPT_REQUIRE(dout && h && mean && rstd && ln_w && part && sums && D > 0 && D <= 64 * kMaxPerLane);
  ESGPT_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || seed));
  if (N == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  const bool yb = y_dtype == ESGPT_BF16, ob = out_dtype == ESGPT_BF16;
  if (!yb && !ob) launch_ln_bwd<float, float>(dh_in, dout, h, mean, rstd, ln_w, row_mask, dropout_p, seed, N, D, dx,
                                             dy, part, st);
  else if (!yb && ob) launch_ln_bwd<float, bf16>(dh_in, dout, h, mean, rstd, ln_w, row_mask, dropout_p, seed, N, D,
                                                dx, dy, part, st);
  else if (yb && !ob) launch_ln_bwd<bf16, float>(dh_in, dout, h, mean, rstd, ln_w, row_mask, dropout_p, seed, N, D,
                                                dx, dy, part, st);
  else launch_ln_bwd<bf16, bf16>(dh_in, dout, h, mean, rstd, ln_w, row_mask, dropout_p, seed, N, D, dx, dy, part,
                                 st);
  const int64_t nb = esgpt_residual_ln_partials(N);
  colsum_kernel<<<(unsigned)cdiv(3 * D, 256), 256, 0, st>>>(part, nb, 3, D, sums);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_bias_act_fwd(const void* f, const float* bias, int act, int64_t N, int64_t F, void* g, int dtype,
                       void* stream) {
  ESGPT_REQUIRE(f && bias && g && (dtype == ESGPT_F32 || dtype == ESGPT_BF16) && act >= 0 && act <= 2);
  if (N * F == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)cdiv(cdiv(N * F, 4), 256);
  if (dtype == ESGPT_F32) bias_act_fwd_kernel<float><<<grid, 256, 0, st>>>((const float*)f, bias, act, N, F, (float*)g);
  else bias_act_fwd_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)f, bias, act, N, F, (bf16*)g);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int64_t esgpt_bias_act_partials(int64_t N) { return cdiv(N, kActRows); }

int esgpt_bias_act_bwd(const void* dg, const void* f, const float* bias, int act, int64_t N, int64_t F, void* dz,
                       float* part, float* dbias, int dtype, void* stream) {
  ESGPT_REQUIRE(dg && f && bias && dz && part && dbias && (dtype == ESGPT_F32 || dtype == ESGPT_BF16));
  if (N * F == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  const unsigned grid = (unsigned)esgpt_bias_act_partials(N);
  if (dtype == ESGPT_F32)
    bias_act_bwd_kernel<float><<<grid, 256, 0, st>>>((const float*)dg, (const float*)f, bias, act, N, F, (float*)dz,
                                                     part);
  else
    bias_act_bwd_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)dg, (const bf16*)f, bias, act, N, F, (bf16*)dz, part);
  colsum_kernel<<<(unsigned)cdiv(F, 256), 256, 0, st>>>(part, grid, 1, F, dbias);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

}  // extern "C"
