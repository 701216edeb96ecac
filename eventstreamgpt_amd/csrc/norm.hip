// Fused elementwise stages of the transformer block for gfx950 (InnerBlock, transformer.py:394-461, and the
// CI encoder's per-block event mask, :818-823):
//
//   residual_ln_fwd   h   = rowmask ? x + dropout(y + bias) : 0          (f32 residual stream)
//                     out = LayerNorm(h) * w + b                         (f32 or bf16: the next GEMM's operand)
//   residual_ln_bwd   dh  = rowmask ? dh_in + LN'(dout) : 0 ; dx = dh ; dy = dropout'(dh)
//                     + the column sums dgamma, dbeta, dbias (block partials, then a fixed-order colsum launch)
//   bias_act_fwd/bwd  g = act(f + bias) (erf GELU, tanh GELU or ReLU: common.h), dbias partials -> colsum
//
// Layout: one wave per row; lane l owns the 4-column chunks {4l + 256k}, k < KC = ceil(D / 256) (a template
// parameter: registers sized for the row), loaded as 16-B (f32) / 8-B (bf16) vectors; statistics in registers
// (two-pass mean / variance, biased variance as torch.nn.LayerNorm).
// HBM-bound: fwd reads x (4 B) + y (2-4 B), writes h (4 B) + out (2-4 B) per element; bwd reads dout (2-4 B), h
// (4 B), dh_in (4 B) and writes dx (4 B) + dy (2-4 B) per element.
#include <algorithm>

#include "common.h"

using namespace esgpt;

namespace {

constexpr int kWaves = 4;
constexpr int kMaxChunks = 4;       // 4-column chunks per lane: D <= 1024
constexpr int kBwdRowsPerWave = 2;  // backward default: rows per wave, every load issued before the row reductions

// Backward rows per wave (2, 4 or 8; ESGPT_LN_BWD_ROWS tuning hook, read once).
int bwd_rows() {
  static int r = 0;
  if (r == 0) {
    const char* e = tuning_env("ESGPT_LN_BWD_ROWS");
    const int v = e ? atoi(e) : kBwdRowsPerWave;
#ifdef ESGPT_TUNING_HOOKS
    r = (v == 2 || v == 4 || v == 8) ? v : kBwdRowsPerWave;
#else
    r = (v == 2 || v == 4) ? v : kBwdRowsPerWave;
#endif
  }
  return r;
}

struct V4 {
  float v[4];
};

__device__ __forceinline__ V4 load4(const float* p) {
  const float4 t = *reinterpret_cast<const float4*>(p);
  return V4{{t.x, t.y, t.z, t.w}};
}
__device__ __forceinline__ V4 load4(const bf16* p) {
  const uint2 t = *reinterpret_cast<const uint2*>(p);
  return V4{{bf16_bits_to_f32((uint16_t)(t.x & 0xffff)), bf16_bits_to_f32((uint16_t)(t.x >> 16)),
             bf16_bits_to_f32((uint16_t)(t.y & 0xffff)), bf16_bits_to_f32((uint16_t)(t.y >> 16))}};
}
__device__ __forceinline__ void store4(float* p, const V4& a) {
  *reinterpret_cast<float4*>(p) = make_float4(a.v[0], a.v[1], a.v[2], a.v[3]);
}
__device__ __forceinline__ void store4(bf16* p, const V4& a) {
  uint2 t;
  t.x = (uint32_t)f32_to_bf16_bits(a.v[0]) | ((uint32_t)f32_to_bf16_bits(a.v[1]) << 16);
  t.y = (uint32_t)f32_to_bf16_bits(a.v[2]) | ((uint32_t)f32_to_bf16_bits(a.v[3]) << 16);
  *reinterpret_cast<uint2*>(p) = t;
}

__device__ __forceinline__ V4 zero4() { return V4{{0.f, 0.f, 0.f, 0.f}}; }


// Row of x under skip_T = T > 1 (static_kv_first residual, transformer.py:437): x = [N / (T-1), T, D] and output row r
// reads the rows after each sequence's first one.
__device__ __forceinline__ int64_t skip_row(int64_t r, int64_t skip_T) {
  return skip_T ? (r / (skip_T - 1)) * skip_T + 1 + r % (skip_T - 1) : r;
}

// Forward rows per wave (1, 2 or 4; ESGPT_LN_FWD_ROWS tuning hook, read once): every load of the wave's rows is
// issued before the first row reduction.
int fwd_rows() {
  static int r = 0;
  if (r == 0) {
    const char* e = tuning_env("ESGPT_LN_FWD_ROWS");
    const int v = e ? atoi(e) : 1;
    r = (v == 1 || v == 2 || v == 4) ? v : 1;
  }
  return r;
}

template <typename TY, typename TO, int KC, int R>
__global__ __launch_bounds__(256) void residual_ln_fwd_kernel(const float* __restrict__ x, const TY* __restrict__ y,
                                                              const float* __restrict__ bias,
                                                              const uint8_t* __restrict__ rmask, float drop_p,
                                                              const uint64_t* __restrict__ seed,
                                                              const float* __restrict__ w, const float* __restrict__ b,
                                                              float eps, int64_t N, int64_t D, float* __restrict__ h,
                                                              TO* __restrict__ out, float* __restrict__ mean_o,
                                                              float* __restrict__ rstd_o, int64_t skip_T) {
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const bool i32 = (uint64_t)N * (uint64_t)D <= 0xffffffffull;  // 32-bit dropout element indices
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row0 = ((int64_t)blockIdx.x * kWaves + wave) * R;
  if (row0 >= N) return;
  // loads of every row first (rows past N clamped, results dropped), with the LayerNorm weight / bias chunks (read
  // before the row reductions, not after them: one memory round trip per row instead of two)
  V4 xv[R][KC], yv[R][KC], wv[KC], bv[KC], yb[KC];
  bool keep[R];
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int64_t c = 4 * lane + 256 * k;
    wv[k] = bv[k] = yb[k] = zero4();
    if (c < D) {
      wv[k] = load4(w + c), bv[k] = load4(b + c);
      if (bias) yb[k] = load4(bias + c);
    }
  }
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
    const int64_t row = min(row0 + rr, N - 1), xrow = skip_row(row, skip_T);
    keep[rr] = rmask == nullptr || rmask[row] != 0;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int64_t c = 4 * lane + 256 * k;
      xv[rr][k] = yv[rr][k] = zero4();
      if (c < D) {
        if (x) xv[rr][k] = load4(x + xrow * D + c);
        if (y) yv[rr][k] = load4(y + row * D + c);
      }
    }
  }
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
    const int64_t row = row0 + rr;
    if (row >= N) break;  // wave-uniform
    V4 v[KC];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int64_t c = 4 * lane + 256 * k;
      v[k] = zero4();
      if (c < D && keep[rr]) {
        v[k] = xv[rr][k];
        if (y) {
          float z[4] = {1.f, 1.f, 1.f, 1.f};
          if (dr.p > 0.f) {  // row * D + c is even (D % 4 == 0): two element pairs
            dropout_pair_rc(dr, i32, row, D, c, z[0], z[1]);
            dropout_pair_rc(dr, i32, row, D, c + 2, z[2], z[3]);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float u = yv[rr][k].v[j] + yb[k].v[j];  // (+0 without a bias: exact)
            if (dr.p > 0.f) u *= z[j];
            v[k].v[j] += u;
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) s += v[k].v[j];
      }
    }
    const float mean = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int64_t c = 4 * lane + 256 * k;
      if (c < D) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = v[k].v[j] - mean;
          q += d * d;
        }
      }
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int64_t c = 4 * lane + 256 * k;
      if (c < D) {
        if (h) store4(h + row * D + c, v[k]);
        V4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o.v[j] = (v[k].v[j] - mean) * rstd * wv[k].v[j] + bv[k].v[j];
        store4(out + row * D + c, o);
      }
    }
    if (lane == 0) {
      mean_o[row] = mean;
      rstd_o[row] = rstd;
    }
  }
}

// Backward. Each wave owns kBwdRowsPerWave consecutive rows and issues every load of them before the row
// reductions. Column partials (dgamma, dbeta, dbias) of the block's rows go to part[blockIdx.x][3][D]; a second
// small launch (ln_colsum_kernel) sums them in a fixed order (deterministic). An in-launch last-arriver tail was
// measured at ~10 us of the 17.6 us launch (two write-through drains + ticket round trips); the kernel boundary
// costs ~1.3 us.
template <typename TY, typename TO, int KC, int R>
__global__ __launch_bounds__(256) void residual_ln_bwd_kernel(
    const float* __restrict__ dh_in, const TO* __restrict__ dout, const float* __restrict__ h,
    const float* __restrict__ mean_i, const float* __restrict__ rstd_i, const float* __restrict__ w,
    const uint8_t* __restrict__ rmask, float drop_p, const uint64_t* __restrict__ seed, int64_t N, int64_t D,
    float* __restrict__ dx, TY* __restrict__ dy, float* __restrict__ part, int64_t skip_T) {
  __shared__ float s_part[kWaves][3][4 * 64];
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const bool i32 = (uint64_t)N * (uint64_t)D <= 0xffffffffull;  // 32-bit dropout element indices
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  V4 pg[KC], pb[KC], py[KC], wv[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    pg[k] = pb[k] = py[k] = zero4();
    const int64_t c = 4 * lane + 256 * k;
    wv[k] = (c < D) ? load4(w + c) : zero4();
  }
  // ---- every load of the wave's rows first (rows past N clamped to a valid row, results dropped) ----
  const int64_t row0 = ((int64_t)blockIdx.x * kWaves + wave) * R;
  V4 dv[R][KC], hv[R][KC], di[R][KC];
  float mean[R], rstd[R];
  bool keep[R];
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
    const int64_t row = min(row0 + rr, N - 1);
    mean[rr] = mean_i[row];
    rstd[rr] = rstd_i[row];
    keep[rr] = rmask == nullptr || rmask[row] != 0;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int64_t c = 4 * lane + 256 * k;
      dv[rr][k] = hv[rr][k] = di[rr][k] = zero4();
      if (c < D) {
        dv[rr][k] = load4(dout + row * D + c);
        hv[rr][k] = load4(h + row * D + c);
        if (dh_in) di[rr][k] = load4(dh_in + row * D + c);
      }
    }
  }
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
    const int64_t row = row0 + rr;
    if (row >= N) break;  // wave-uniform
    V4 xh[KC], g[KC];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int64_t c = 4 * lane + 256 * k;
      xh[k] = g[k] = zero4();
      if (c < D) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          xh[k].v[j] = (hv[rr][k].v[j] - mean[rr]) * rstd[rr];
          g[k].v[j] = dv[rr][k].v[j] * wv[k].v[j];
          pg[k].v[j] += dv[rr][k].v[j] * xh[k].v[j];
          pb[k].v[j] += dv[rr][k].v[j];
          sg += g[k].v[j];
          sgx += g[k].v[j] * xh[k].v[j];
        }
      }
    }
    sg = wave_sum(sg) / (float)D;
    sgx = wave_sum(sgx) / (float)D;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int64_t c = 4 * lane + 256 * k;
      if (c < D) {
        V4 d;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float t = rstd[rr] * (g[k].v[j] - sg - xh[k].v[j] * sgx) + di[rr][k].v[j];
          d.v[j] = keep[rr] ? t : 0.f;
        }
        if (dx) {
          const int64_t xrow = skip_row(row, skip_T);
          store4(dx + xrow * D + c, d);
          // the x row before each sequence's first output row is read by no output: its gradient is zero
          if (skip_T && row % (skip_T - 1) == 0) store4(dx + (xrow - 1) * D + c, zero4());
        }
        if (dy) {
          V4 e;
          float z[4] = {1.f, 1.f, 1.f, 1.f};
          if (dr.p > 0.f) {
            dropout_pair_rc(dr, i32, row, D, c, z[0], z[1]);
            dropout_pair_rc(dr, i32, row, D, c + 2, z[2], z[3]);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            e.v[j] = dr.p > 0.f ? d.v[j] * z[j] : d.v[j];
            py[k].v[j] += e.v[j];
          }
          store4(dy + row * D + c, e);
        }
      }
    }
  }
  // ---- combine the 4 waves' column partials ----
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const int64_t c0 = 256 * k;
    if (c0 >= D) break;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s_part[wave][0][4 * lane + j] = pg[k].v[j];
      s_part[wave][1][4 * lane + j] = pb[k].v[j];
      s_part[wave][2][4 * lane + j] = py[k].v[j];
    }
    __syncthreads();
    if (threadIdx.x < 3 * 64) {
      const int qd = threadIdx.x / 64, cc = 4 * (threadIdx.x % 64);
      if (c0 + cc < D) {
        float4 t;
        t.x = s_part[0][qd][cc + 0] + s_part[1][qd][cc + 0] + s_part[2][qd][cc + 0] + s_part[3][qd][cc + 0];
        t.y = s_part[0][qd][cc + 1] + s_part[1][qd][cc + 1] + s_part[2][qd][cc + 1] + s_part[3][qd][cc + 1];
        t.z = s_part[0][qd][cc + 2] + s_part[1][qd][cc + 2] + s_part[2][qd][cc + 2] + s_part[3][qd][cc + 2];
        t.w = s_part[0][qd][cc + 3] + s_part[1][qd][cc + 3] + s_part[2][qd][cc + 3] + s_part[3][qd][cc + 3];
        *reinterpret_cast<float4*>(part + ((int64_t)blockIdx.x * 3 + qd) * D + c0 + cc) = t;
      }
    }
    __syncthreads();
  }
}

// sums[i] = sum_b part[b * QD + i] (QD % 4 == 0): 16 threads x 4 columns = 64 columns per block, 16 row groups
// each summing partials b = g, g + 16, ... in order, then the 16 group sums in order (deterministic). (A 1024-thread
// form with 64 row groups measured 0.5 us slower at N = 8192, D = 256.)
__global__ __launch_bounds__(256) void ln_colsum_kernel(const float* __restrict__ part, int64_t nb, int64_t QD,
                                                        float* __restrict__ sums) {
  __shared__ float4 s[16][16];
  const int c4 = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t i = (int64_t)blockIdx.x * 64 + 4 * c4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < QD) {
#pragma unroll 8
    for (int64_t b = grp; b < nb; b += 16) {
      const float4 v = *reinterpret_cast<const float4*>(part + b * QD + i);
      a.x += v.x;
      a.y += v.y;
      a.z += v.z;
      a.w += v.w;
    }
  }
  s[grp][c4] = a;
  __syncthreads();
  if (grp == 0 && i < QD) {
    float4 t = s[0][c4];
#pragma unroll
    for (int g = 1; g < 16; ++g) {
      t.x += s[g][c4].x;
      t.y += s[g][c4].y;
      t.z += s[g][c4].z;
      t.w += s[g][c4].w;
    }
    *reinterpret_cast<float4*>(sums + i) = t;
  }
}

// Many independent column sums in ONE launch (the deferred LayerNorm-backward sums of a whole backward pass):
// block -> (job, 64-column group) through a prefix table; each block is ln_colsum_kernel's block (16 row groups in
// a fixed order): the same sums bit for bit as one ln_colsum launch per job.
constexpr int kMaxColsumJobs = 48;
struct ColsumJobs {
  esgpt_colsum_job j[kMaxColsumJobs];
  int start[kMaxColsumJobs + 1];  // first block of each job
  int n;
};

__global__ __launch_bounds__(256) void colsum_jobs_kernel(ColsumJobs a) {
  __shared__ float4 s[16][16];
  int job = 0;
  while (job + 1 < a.n && (int)blockIdx.x >= a.start[job + 1]) ++job;  // block-uniform
  const esgpt_colsum_job& jb = a.j[job];
  const int c4 = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t i = (int64_t)(blockIdx.x - a.start[job]) * 64 + 4 * c4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < jb.width) {
#pragma unroll 8
    for (int64_t b = grp; b < jb.n_parts; b += 16) {
      const float4 v = *reinterpret_cast<const float4*>(jb.part + b * jb.width + i);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  s[grp][c4] = acc;
  __syncthreads();
  if (grp == 0 && i < jb.width) {
    float4 t = s[0][c4];
#pragma unroll
    for (int g = 1; g < 16; ++g) {
      t.x += s[g][c4].x;
      t.y += s[g][c4].y;
      t.z += s[g][c4].z;
      t.w += s[g][c4].w;
    }
    *reinterpret_cast<float4*>(jb.sums + i) = t;
  }
}

// sums[q, c] = sum_b part[b, q, c]. Block: 64 columns x 16 row groups (1024 threads); fixed order -> deterministic.
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ part, int64_t nb, int64_t QD,
                                                      float* __restrict__ sums) {
  __shared__ float s[16][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + cl;
  float a = 0.f;
  if (i < QD) {
#pragma unroll 4
    for (int64_t b = grp; b < nb; b += 16) a += part[b * QD + i];
  }
  s[grp][cl] = a;
  __syncthreads();
  if (grp == 0 && i < QD) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += s[g][cl];
    sums[i] = t;
  }
}

// 4 consecutive elements per thread (F % 4 == 0).
template <typename T>
__global__ __launch_bounds__(256) void bias_act_fwd_kernel(const T* __restrict__ f, const float* __restrict__ bias,
                                                           int act, int64_t N, int64_t F, T* __restrict__ g) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= N * F) return;
  const int64_t c = i % F;
  const V4 z = load4(f + i);
  const V4 bv = load4(bias + c);
  V4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o.v[j] = act_fwd(z.v[j] + bv.v[j], act);
  store4(g + i, o);
}

// dz = dg * act'(f + bias); part[blockIdx.y, F] column partials of dz over this block's kActRows rows.
// Block: 64 threads x 4 columns = 256 columns, 4 row groups (LDS combine); grid (F/256, N/kActRows).
constexpr int kActRows = 32;
template <typename T>
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(const T* __restrict__ dg, const T* __restrict__ f,
                                                           const float* __restrict__ bias, int act, int64_t N,
                                                           int64_t F, T* __restrict__ dz, float* __restrict__ part) {
  __shared__ float s_part[4][256];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 256 + 4 * cl;
  const int64_t r0 = (int64_t)blockIdx.y * kActRows, r1 = min(N, r0 + kActRows);
  V4 s{{0.f, 0.f, 0.f, 0.f}};
  if (c < F) {
    const V4 bv = load4(bias + c);
#pragma unroll 2
    for (int64_t r = r0 + grp; r < r1; r += 4) {
      const V4 z = load4(f + r * F + c);
      const V4 d = load4(dg + r * F + c);
      V4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o.v[j] = d.v[j] * act_grad(z.v[j] + bv.v[j], act);
        s.v[j] += o.v[j];
      }
      store4(dz + r * F + c, o);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) s_part[grp][4 * cl + j] = s.v[j];
  __syncthreads();
  const int64_t cc = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (cc < F)
    part[(int64_t)blockIdx.y * F + cc] =
        s_part[0][threadIdx.x] + s_part[1][threadIdx.x] + s_part[2][threadIdx.x] + s_part[3][threadIdx.x];
}

// part[blockIdx.y, c] = sum over this block's kColRows rows of x[:, c]; thread per column (coalesced along c).
constexpr int kColRows = 64;
template <typename T>
__global__ __launch_bounds__(256) void column_partial_kernel(const T* __restrict__ x, int64_t N, int64_t F,
                                                             float* __restrict__ part) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= F) return;
  const int64_t r0 = (int64_t)blockIdx.y * kColRows, r1 = min(N, r0 + kColRows);
  float s = 0.f;
#pragma unroll 8
  for (int64_t r = r0; r < r1; ++r) s += to_f32(x[r * F + c]);
  part[(int64_t)blockIdx.y * F + c] = s;
}

template <typename TY, typename TO>
void launch_ln_fwd(const float* x, const void* y, const float* bias, const uint8_t* rmask, float p, const uint64_t* seed,
                   const float* w, const float* b, float eps, int64_t N, int64_t D, float* h, void* out, float* mean,
                   float* rstd, int64_t skip_T, hipStream_t st) {
  const int R = fwd_rows();
  const unsigned grid = (unsigned)cdiv(N, kWaves * R);
#define LN_FWD(KC, RR)                                                                                             \
  residual_ln_fwd_kernel<TY, TO, KC, RR><<<grid, 256, 0, st>>>(x, (const TY*)y, bias, rmask, p, seed, w, b, eps, N, D, \
                                                               h, (TO*)out, mean, rstd, skip_T)
#define LN_FWD_R(KC)                 \
  do {                               \
    if (R == 2) LN_FWD(KC, 2);       \
    else if (R == 4) LN_FWD(KC, 4);  \
    else LN_FWD(KC, 1);              \
  } while (0)
  switch (cdiv(D, 256)) {
    case 1: LN_FWD_R(1); break;
    case 2: LN_FWD_R(2); break;
    case 3: LN_FWD_R(3); break;
    default: LN_FWD_R(4); break;
  }
#undef LN_FWD_R
#undef LN_FWD
}

template <typename TY, typename TO>
void launch_ln_bwd(const float* dh_in, const void* dout, const float* h, const float* mean, const float* rstd,
                   const float* w, const uint8_t* rmask, float p, const uint64_t* seed, int64_t N, int64_t D, float* dx,
                   void* dy, float* part, float* sums, int64_t skip_T, hipStream_t st) {
  const int R = bwd_rows();
  const unsigned grid = (unsigned)cdiv(N, kWaves * R);
#define LN_BWD(KC, RR)                                                                                             \
  residual_ln_bwd_kernel<TY, TO, KC, RR><<<grid, 256, 0, st>>>(dh_in, (const TO*)dout, h, mean, rstd, w, rmask, p, \
                                                               seed, N, D, dx, (TY*)dy, part, skip_T)
#ifdef ESGPT_TUNING_HOOKS
#define LN_BWD_R(KC)              \
  do {                            \
    if (R == 2) LN_BWD(KC, 2);    \
    else if (R == 8) LN_BWD(KC, 8); \
    else LN_BWD(KC, 4);           \
  } while (0)
#else  // 8 rows per wave (measured slower; spills at D > 768) in the tools build only
#define LN_BWD_R(KC)              \
  do {                            \
    if (R == 2) LN_BWD(KC, 2);    \
    else LN_BWD(KC, 4);           \
  } while (0)
#endif
  switch (cdiv(D, 256)) {
    case 1: LN_BWD_R(1); break;
    case 2: LN_BWD_R(2); break;
    case 3: LN_BWD_R(3); break;
    default: LN_BWD_R(4); break;
  }
#undef LN_BWD_R
#undef LN_BWD
  if (sums) ln_colsum_kernel<<<(unsigned)cdiv(3 * D, 64), 256, 0, st>>>(part, grid, 3 * D, sums);
}

}  // namespace

extern "C" {

int64_t esgpt_residual_ln_partials(int64_t N) { return cdiv(N, kWaves * bwd_rows()); }

int64_t esgpt_residual_ln_counters(int64_t N) {
  (void)N;
  return 0;
}

int esgpt_residual_ln_fwd(const float* x, const void* y, int y_dtype, const float* bias, const uint8_t* row_mask,
                          float dropout_p, const uint64_t* seed, const float* ln_w, const float* ln_b, float eps,
                          int64_t N, int64_t D, float* h, void* out, int out_dtype, float* mean, float* rstd,
                          void* stream) {
  return esgpt_residual_ln_fwd_ex(x, y, y_dtype, bias, row_mask, dropout_p, seed, ln_w, ln_b, eps, N, D, 0, h, out,
                                  out_dtype, mean, rstd, stream);
}

int esgpt_residual_ln_fwd_ex(const float* x, const void* y, int y_dtype, const float* bias, const uint8_t* row_mask,
                             float dropout_p, const uint64_t* seed, const float* ln_w, const float* ln_b, float eps,
                             int64_t N, int64_t D, int64_t skip_T, float* h, void* out, int out_dtype, float* mean,
                             float* rstd, void* stream) {
  ESGPT_REQUIRE(ln_w && ln_b && out && mean && rstd && D > 0 && D % 4 == 0 && D <= 256 * kMaxChunks && (x || y));
  ESGPT_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || seed));
  ESGPT_REQUIRE(skip_T == 0 || (skip_T >= 2 && x && N % (skip_T - 1) == 0));
  if (N == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  const bool yb = y_dtype == ESGPT_BF16, ob = out_dtype == ESGPT_BF16;
  if (!yb && !ob) launch_ln_fwd<float, float>(x, y, bias, row_mask, dropout_p, seed, ln_w, ln_b, eps, N, D, h, out,
                                             mean, rstd, skip_T, st);
  else if (!yb && ob) launch_ln_fwd<float, bf16>(x, y, bias, row_mask, dropout_p, seed, ln_w, ln_b, eps, N, D, h, out,
                                                mean, rstd, skip_T, st);
  else if (yb && !ob) launch_ln_fwd<bf16, float>(x, y, bias, row_mask, dropout_p, seed, ln_w, ln_b, eps, N, D, h, out,
                                                mean, rstd, skip_T, st);
  else launch_ln_fwd<bf16, bf16>(x, y, bias, row_mask, dropout_p, seed, ln_w, ln_b, eps, N, D, h, out, mean, rstd,
                                 skip_T, st);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_residual_ln_bwd(const float* dh_in, const void* dout, int out_dtype, const float* h, const float* mean,
                          const float* rstd, const float* ln_w, const uint8_t* row_mask, float dropout_p,
                          const uint64_t* seed, int64_t N, int64_t D, float* dx, void* dy, int y_dtype, float* part,
                          float* sums, int32_t* counters, void* stream) {
  (void)counters;
  return esgpt_residual_ln_bwd_ex(dh_in, dout, out_dtype, h, mean, rstd, ln_w, row_mask, dropout_p, seed, N, D, 0, dx,
                                  dy, y_dtype, part, sums, stream);
}

int esgpt_residual_ln_bwd_ex(const float* dh_in, const void* dout, int out_dtype, const float* h, const float* mean,
                             const float* rstd, const float* ln_w, const uint8_t* row_mask, float dropout_p,
                             const uint64_t* seed, int64_t N, int64_t D, int64_t skip_T, float* dx, void* dy,
                             int y_dtype, float* part, float* sums, void* stream) {
  ESGPT_REQUIRE(dout && h && mean && rstd && ln_w && part && D > 0 && D % 4 == 0 && D <= 256 * kMaxChunks);
  ESGPT_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || seed));
  ESGPT_REQUIRE(esgpt_residual_ln_partials(N) * 3 * D * 4 < (1ll << 31) && ((uintptr_t)sums % 16) == 0);
  ESGPT_REQUIRE(skip_T == 0 || (skip_T >= 2 && N % (skip_T - 1) == 0));
  hipStream_t st = as_stream(stream);
  if (N == 0) {  // no rows: zero sums (or, deferred, zero partials: one all-zero block)
    if (sums) return zero_async(sums, sizeof(float) * 3 * D, st) == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
    return zero_async(part, sizeof(float) * 3 * D, st) == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
  }
  const bool yb = y_dtype == ESGPT_BF16, ob = out_dtype == ESGPT_BF16;
  if (!yb && !ob) launch_ln_bwd<float, float>(dh_in, dout, h, mean, rstd, ln_w, row_mask, dropout_p, seed, N, D, dx,
                                             dy, part, sums, skip_T, st);
  else if (!yb && ob) launch_ln_bwd<float, bf16>(dh_in, dout, h, mean, rstd, ln_w, row_mask, dropout_p, seed, N, D,
                                                dx, dy, part, sums, skip_T, st);
  else if (yb && !ob) launch_ln_bwd<bf16, float>(dh_in, dout, h, mean, rstd, ln_w, row_mask, dropout_p, seed, N, D,
                                                dx, dy, part, sums, skip_T, st);
  else launch_ln_bwd<bf16, bf16>(dh_in, dout, h, mean, rstd, ln_w, row_mask, dropout_p, seed, N, D, dx, dy, part,
                                 sums, skip_T, st);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_colsum_jobs(const esgpt_colsum_job* jobs, int64_t n_jobs, void* stream) {
  ESGPT_REQUIRE(n_jobs >= 0 && (n_jobs == 0 || jobs != nullptr));
  hipStream_t st = as_stream(stream);
  for (int64_t j0 = 0; j0 < n_jobs; j0 += kMaxColsumJobs) {
    ColsumJobs a{};
    a.n = (int)std::min<int64_t>(kMaxColsumJobs, n_jobs - j0);
    a.start[0] = 0;
    for (int i = 0; i < a.n; ++i) {
      const esgpt_colsum_job& jb = jobs[j0 + i];
      ESGPT_REQUIRE(jb.part && jb.sums && jb.n_parts >= 1 && jb.width > 0 && jb.width % 4 == 0 &&
                    ((uintptr_t)jb.part % 16) == 0 && ((uintptr_t)jb.sums % 16) == 0);
      a.j[i] = jb;
      a.start[i + 1] = a.start[i] + (int)cdiv(jb.width, 64);
    }
    if (a.start[a.n] == 0) continue;
    colsum_jobs_kernel<<<(unsigned)a.start[a.n], 256, 0, st>>>(a);
    ESGPT_LAUNCH_CHECK();
  }
  return ESGPT_OK;
}

int esgpt_bias_act_fwd(const void* f, const float* bias, int act, int64_t N, int64_t F, void* g, int dtype,
                       void* stream) {
  ESGPT_REQUIRE(f && bias && g && (dtype == ESGPT_F32 || dtype == ESGPT_BF16) && act >= 0 && act <= 2 && F % 4 == 0);
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
  ESGPT_REQUIRE(dg && f && bias && dz && part && dbias && (dtype == ESGPT_F32 || dtype == ESGPT_BF16) && F % 4 == 0);
  if (N * F == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  const int64_t nb = esgpt_bias_act_partials(N);
  dim3 grid((unsigned)cdiv(F, 256), (unsigned)nb);
  if (dtype == ESGPT_F32)
    bias_act_bwd_kernel<float><<<grid, 256, 0, st>>>((const float*)dg, (const float*)f, bias, act, N, F, (float*)dz,
                                                     part);
  else
    bias_act_bwd_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)dg, (const bf16*)f, bias, act, N, F, (bf16*)dz, part);
  colsum_kernel<<<(unsigned)cdiv(F, 64), 1024, 0, st>>>(part, nb, F, dbias);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int64_t esgpt_column_sum_partials(int64_t N) { return cdiv(N, kColRows); }

int esgpt_column_sum(const void* x, int dtype, int64_t N, int64_t F, float* part, float* out, void* stream) {
  ESGPT_REQUIRE(x && part && out && (dtype == ESGPT_F32 || dtype == ESGPT_BF16) && N >= 0 && F >= 0);
  if (F == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  if (N == 0) {
    if (zero_async(out, F * sizeof(float), st) != hipSuccess) return ESGPT_ERR_LAUNCH;
    return ESGPT_OK;
  }
  const int64_t nb = esgpt_column_sum_partials(N);
  dim3 grid((unsigned)cdiv(F, 256), (unsigned)nb);
  if (dtype == ESGPT_F32) column_partial_kernel<float><<<grid, 256, 0, st>>>((const float*)x, N, F, part);
  else column_partial_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)x, N, F, part);
  colsum_kernel<<<(unsigned)cdiv(F, 64), 1024, 0, st>>>(part, nb, F, out);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

}  // extern "C"
