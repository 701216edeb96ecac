// Causal / local-window attention for gfx950 (InnerSelfAttention._attn, transformer.py:171-217).
//
// Three implementations behind one entry point:
//   * attn_*_generic  — one lane per query (forward, dQ) or per key (dK/dV), f32 arithmetic, any head dim up to
//     128, f32 or bf16 I/O. Lanes of a wave hold consecutive queries of one (batch, head), so every K/V (or Q/dO)
//     row load in the key loop is wave-uniform (a broadcast). Used for head dims / layouts without an MFMA path.
//   * attn_*_small — Lk <= 16 (the NA model's dependency-graph sequences, Lk = G + 1): one wave per (sequence,
//     head), lane = head dimension, K / V in registers, one fused backward pass.
//   * attn_*_mfma (attention_mfma.hip) — bf16 v_mfma_f32_32x32x16_bf16 flash kernels for hd in {16, 32, 64, 128};
//     attn_*_f32 (attention_f32.hip) — the f32 path on v_mfma_f32_32x32x2_f32 (exact f32), same head dims.
//
// Semantics (all): s_ij = q_i . k_j in f32 with NO 1/sqrt(hd) scaling; key j is visible to query i (at key
// position p_i = i + Lk - Lq) iff j <= p_i, (local) p_i - j < window, and key_mask[j]; softmax in f32; the
// attention-probability dropout of the reference (transformer.py:208, nn.Dropout on attn_weights) multiplies
// p_ij by keep_ij / (1 - p) with keep regenerated from a counter hash of (seed, (bh*Lq + i)*Lk + j);
// rows of padded queries (query_mask[i] == 0) are zeros and carry no gradient.
#include <stdlib.h>

#include <initializer_list>

#include "common.h"

using namespace esgpt;

namespace {

__device__ __forceinline__ uint64_t elem_index(int64_t bh, int64_t Lq, int64_t Lk, int64_t qi, int64_t kj) {
  return ((uint64_t)(bh * Lq + qi)) * (uint64_t)Lk + (uint64_t)kj;
}

template <typename T, int HDP>
__global__ __launch_bounds__(256) void attn_fwd_generic(const T* __restrict__ q, const T* __restrict__ k,
                                                        const T* __restrict__ v, int64_t ld_in, int64_t tq,
                                                        T* __restrict__ o, int64_t ld_o, float* __restrict__ lse,
                                                        const uint8_t* __restrict__ kmask,
                                                        const uint8_t* __restrict__ qmask, int64_t B, int64_t H,
                                                        int64_t Lq, int64_t Lk, int hd, int64_t window, float drop_p,
                                                        const uint64_t* __restrict__ seed) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = B * H * Lq;
  if (tid >= total) return;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const int64_t qi = tid % Lq;
  const int64_t bh = tid / Lq;
  const int64_t h = bh % H, b = bh / H;
  const int64_t pos = qi + (Lk - Lq);
  const bool qvalid = qmask ? (qmask[b * Lq + qi] != 0) : true;

  float qr[HDP], acc[HDP];
  const T* qp = q + (b * tq + qi) * ld_in + h * hd;
#pragma unroll
  for (int d = 0; d < HDP; ++d) {
    qr[d] = (d < hd) ? to_f32(qp[d]) : 0.f;
    acc[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  const int64_t jlo = (window > 0) ? max((int64_t)0, pos - window + 1) : 0;
  if (qvalid) {
    for (int64_t j = jlo; j <= pos; ++j) {
      if (kmask && !kmask[b * Lk + j]) continue;
      const T* kp = k + (b * Lk + j) * ld_in + h * hd;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < HDP; ++d)
        if (d < hd) s = fmaf(qr[d], to_f32(kp[d]), s);
      float p;
      if (s > m) {
        const float c = expf(m - s);  // m = -inf on the first key -> c = 0
        l *= c;
#pragma unroll
        for (int d = 0; d < HDP; ++d) acc[d] *= c;
        m = s;
        p = 1.f;
      } else {
        p = expf(s - m);
      }
      l += p;  // the softmax normaliser uses the undropped probabilities
      const float pd = dr.p > 0.f ? p * dropout_mult(dr, elem_index(bh, Lq, Lk, qi, j)) : p;
      const T* vp = v + (b * Lk + j) * ld_in + h * hd;
#pragma unroll
      for (int d = 0; d < HDP; ++d)
        if (d < hd) acc[d] = fmaf(pd, to_f32(vp[d]), acc[d]);
    }
  }
  const bool ok = qvalid && l > 0.f;
  const float inv = ok ? 1.f / l : 0.f;
  T* op = o + (b * Lq + qi) * ld_o + h * hd;
#pragma unroll
  for (int d = 0; d < HDP; ++d)
    if (d < hd) op[d] = from_f32<T>(acc[d] * inv);
  lse[bh * Lq + qi] = ok ? m + logf(l) : 0.f;
}

// dQ (and delta = rowsum(dO * O)) — one lane per query. With dropout: dS = P o (dP_drop o keep / (1-p) - delta).
template <typename T, int HDP>
__global__ __launch_bounds__(256) void attn_bwd_dq_generic(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, int64_t ld_in, int64_t tq,
    const T* __restrict__ o, int64_t ld_o, const T* __restrict__ dout, int64_t ld_do, const float* __restrict__ lse,
    const uint8_t* __restrict__ kmask, const uint8_t* __restrict__ qmask, T* __restrict__ dq, int64_t ld_d,
    float* __restrict__ delta, int64_t B, int64_t H, int64_t Lq, int64_t Lk, int hd, int64_t window, float drop_p,
    const uint64_t* __restrict__ seed) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = B * H * Lq;
  if (tid >= total) return;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const int64_t qi = tid % Lq;
  const int64_t bh = tid / Lq;
  const int64_t h = bh % H, b = bh / H;
  const int64_t pos = qi + (Lk - Lq);
  const bool qvalid = qmask ? (qmask[b * Lq + qi] != 0) : true;
  float qr[HDP], dor[HDP], acc[HDP];
  const T* qp = q + (b * tq + qi) * ld_in + h * hd;
  const T* dp_ = dout + (b * Lq + qi) * ld_do + h * hd;
  const T* op = o + (b * Lq + qi) * ld_o + h * hd;
  float dl = 0.f;
#pragma unroll
  for (int d = 0; d < HDP; ++d) {
    qr[d] = (d < hd) ? to_f32(qp[d]) : 0.f;
    dor[d] = (d < hd) ? to_f32(dp_[d]) : 0.f;
    if (d < hd) dl = fmaf(dor[d], to_f32(op[d]), dl);
    acc[d] = 0.f;
  }
  if (!qvalid) dl = 0.f;
  delta[bh * Lq + qi] = dl;
  const float ls = lse[bh * Lq + qi];
  const int64_t jlo = (window > 0) ? max((int64_t)0, pos - window + 1) : 0;
  if (qvalid) {
    for (int64_t j = jlo; j <= pos; ++j) {
      if (kmask && !kmask[b * Lk + j]) continue;
      const T* kp = k + (b * Lk + j) * ld_in + h * hd;
      const T* vp = v + (b * Lk + j) * ld_in + h * hd;
      float s = 0.f, dpv = 0.f;
#pragma unroll
      for (int d = 0; d < HDP; ++d) {
        if (d < hd) {
          s = fmaf(qr[d], to_f32(kp[d]), s);
          dpv = fmaf(dor[d], to_f32(vp[d]), dpv);
        }
      }
      if (dr.p > 0.f) dpv *= dropout_mult(dr, elem_index(bh, Lq, Lk, qi, j));
      const float p = expf(s - ls);
      const float ds = p * (dpv - dl);
#pragma unroll
      for (int d = 0; d < HDP; ++d)
        if (d < hd) acc[d] = fmaf(ds, to_f32(kp[d]), acc[d]);
    }
  }
  T* dqp = dq + (b * tq + qi) * ld_d + h * hd;
#pragma unroll
  for (int d = 0; d < HDP; ++d)
    if (d < hd) dqp[d] = from_f32<T>(acc[d]);
}

// dK, dV — one lane per key; loops over the queries that can see it.
template <typename T, int HDP>
__global__ __launch_bounds__(256) void attn_bwd_dkv_generic(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, int64_t ld_in, int64_t tq,
    const T* __restrict__ dout, int64_t ld_do, const float* __restrict__ lse, const float* __restrict__ delta,
    const uint8_t* __restrict__ kmask, const uint8_t* __restrict__ qmask, T* __restrict__ dk, T* __restrict__ dv,
    int64_t ld_d, int64_t B, int64_t H, int64_t Lq, int64_t Lk, int hd, int64_t window, float drop_p,
    const uint64_t* __restrict__ seed) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = B * H * Lk;
  if (tid >= total) return;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const int64_t kj = tid % Lk;
  const int64_t bh = tid / Lk;
  const int64_t h = bh % H, b = bh / H;
  const bool kvalid = kmask ? (kmask[b * Lk + kj] != 0) : true;
  float kr[HDP], vr[HDP], dka[HDP], dva[HDP];
  const T* kp = k + (b * Lk + kj) * ld_in + h * hd;
  const T* vp = v + (b * Lk + kj) * ld_in + h * hd;
#pragma unroll
  for (int d = 0; d < HDP; ++d) {
    kr[d] = (d < hd) ? to_f32(kp[d]) : 0.f;
    vr[d] = (d < hd) ? to_f32(vp[d]) : 0.f;
    dka[d] = 0.f;
    dva[d] = 0.f;
  }
  const int64_t off = Lk - Lq;
  // queries i with p_i = i + off in [kj, kj + window - 1] (local) or [kj, Lk-1] (global)
  const int64_t ilo = max((int64_t)0, kj - off);
  const int64_t ihi = (window > 0) ? min(Lq - 1, kj + window - 1 - off) : Lq - 1;
  if (kvalid) {
    for (int64_t i = ilo; i <= ihi; ++i) {
      if (qmask && !qmask[b * Lq + i]) continue;
      const T* qp = q + (b * tq + i) * ld_in + h * hd;
      const T* dop = dout + (b * Lq + i) * ld_do + h * hd;
      float s = 0.f, dpv = 0.f;
#pragma unroll
      for (int d = 0; d < HDP; ++d) {
        if (d < hd) {
          s = fmaf(to_f32(qp[d]), kr[d], s);
          dpv = fmaf(to_f32(dop[d]), vr[d], dpv);
        }
      }
      const float keep = dr.p > 0.f ? dropout_mult(dr, elem_index(bh, Lq, Lk, i, kj)) : 1.f;
      const float p = expf(s - lse[bh * Lq + i]);
      const float ds = p * (dpv * keep - delta[bh * Lq + i]);
      const float pd = p * keep;
#pragma unroll
      for (int d = 0; d < HDP; ++d) {
        if (d < hd) {
          dva[d] = fmaf(pd, to_f32(dop[d]), dva[d]);
          dka[d] = fmaf(ds, to_f32(qp[d]), dka[d]);
        }
      }
    }
  }
  T* dkp = dk + (b * Lk + kj) * ld_d + h * hd;
  T* dvp = dv + (b * Lk + kj) * ld_d + h * hd;
#pragma unroll
  for (int d = 0; d < HDP; ++d) {
    if (d < hd) {
      dkp[d] = from_f32<T>(dka[d]);
      dvp[d] = from_f32<T>(dva[d]);
    }
  }
}

// ---- short sequences (Lk <= 16: the NA dependency graph, G + 1 tokens) ----------------------------------------
// One wave per (sequence, head), lane = head dimension (DPL dims per lane): every row load is one coalesced wave
// load, the whole sequence's K / V (and dK / dV) stay in registers, scores and dP are wave reductions, and the
// backward is ONE pass (dQ, dK, dV without the generic kernels' per-lane row walks or a second launch). Same
// visibility, masking, dropout-hash and zero-row semantics as the generic kernels above.
constexpr int kSmallLk = 16;

template <typename T, int DPL, int LKM>
__global__ __launch_bounds__(256) void attn_fwd_small(const T* __restrict__ q, const T* __restrict__ k,
                                                      const T* __restrict__ v, int64_t ld_in, int64_t tq,
                                                      T* __restrict__ o, int64_t ld_o, float* __restrict__ lse,
                                                      const uint8_t* __restrict__ kmask,
                                                      const uint8_t* __restrict__ qmask, int64_t B, int64_t H,
                                                      int64_t Lq, int64_t Lk, int hd, int64_t window, float drop_p,
                                                      const uint64_t* __restrict__ seed) {
  const int64_t bh = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bh >= B * H) return;  // wave-uniform
  const int lane = lane_id();
  const int64_t h = bh % H, b = bh / H;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  float kr[LKM][DPL], vr[LKM][DPL];
  bool kv[LKM];
#pragma unroll
  for (int j = 0; j < LKM; ++j) {
    kv[j] = j < Lk && (!kmask || kmask[b * Lk + j] != 0);
    const T* kp = k + (b * Lk + min((int64_t)j, Lk - 1)) * ld_in + h * hd;
    const T* vp = v + (b * Lk + min((int64_t)j, Lk - 1)) * ld_in + h * hd;
#pragma unroll
    for (int u = 0; u < DPL; ++u) {
      const int d = lane + 64 * u;
      kr[j][u] = (j < Lk && d < hd) ? to_f32(kp[d]) : 0.f;
      vr[j][u] = (j < Lk && d < hd) ? to_f32(vp[d]) : 0.f;
    }
  }
  for (int64_t i = 0; i < Lq; ++i) {
    const int64_t pos = i + (Lk - Lq);
    const int64_t jlo = (window > 0) ? max((int64_t)0, pos - window + 1) : 0;
    const bool qvalid = qmask ? (qmask[b * Lq + i] != 0) : true;
    const T* qp = q + (b * tq + i) * ld_in + h * hd;
    float qr[DPL];
#pragma unroll
    for (int u = 0; u < DPL; ++u) qr[u] = (lane + 64 * u < hd) ? to_f32(qp[lane + 64 * u]) : 0.f;
    float s[LKM];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < LKM; ++j) {
      s[j] = -INFINITY;
      if (qvalid && kv[j] && j >= jlo && j <= pos) {  // wave-uniform
        float t = 0.f;
#pragma unroll
        for (int u = 0; u < DPL; ++u) t = fmaf(qr[u], kr[j][u], t);
        s[j] = wave_sum(t);
        m = fmaxf(m, s[j]);
      }
    }
    float l = 0.f, acc[DPL];
#pragma unroll
    for (int u = 0; u < DPL; ++u) acc[u] = 0.f;
#pragma unroll
    for (int j = 0; j < LKM; ++j) {
      if (s[j] == -INFINITY) continue;
      const float p = expf(s[j] - m);
      l += p;  // normaliser over undropped probabilities
      const float pd = dr.p > 0.f ? p * dropout_mult(dr, elem_index(bh, Lq, Lk, i, j)) : p;
#pragma unroll
      for (int u = 0; u < DPL; ++u) acc[u] = fmaf(pd, vr[j][u], acc[u]);
    }
    const bool ok = qvalid && l > 0.f;
    const float inv = ok ? 1.f / l : 0.f;
    T* op = o + (b * Lq + i) * ld_o + h * hd;
#pragma unroll
    for (int u = 0; u < DPL; ++u)
      if (lane + 64 * u < hd) op[lane + 64 * u] = from_f32<T>(acc[u] * inv);
    if (lane == 0) lse[bh * Lq + i] = ok ? m + logf(l) : 0.f;
  }
}

template <typename T, int DPL, int LKM>
__global__ __launch_bounds__(256) void attn_bwd_small(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, int64_t ld_in, int64_t tq,
    const T* __restrict__ o, int64_t ld_o, const T* __restrict__ dout, int64_t ld_do, const float* __restrict__ lse,
    const uint8_t* __restrict__ kmask, const uint8_t* __restrict__ qmask, T* __restrict__ dq, T* __restrict__ dk,
    T* __restrict__ dv, int64_t ld_d, int64_t B, int64_t H, int64_t Lq, int64_t Lk, int hd, int64_t window,
    float drop_p, const uint64_t* __restrict__ seed, int64_t dq_lead) {
  const int64_t bh = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bh >= B * H) return;  // wave-uniform
  const int lane = lane_id();
  const int64_t h = bh % H, b = bh / H;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  float kr[LKM][DPL], vr[LKM][DPL], dka[LKM][DPL], dva[LKM][DPL];
  bool kv[LKM];
#pragma unroll
  for (int j = 0; j < LKM; ++j) {
    kv[j] = j < Lk && (!kmask || kmask[b * Lk + j] != 0);
    const T* kp = k + (b * Lk + min((int64_t)j, Lk - 1)) * ld_in + h * hd;
    const T* vp = v + (b * Lk + min((int64_t)j, Lk - 1)) * ld_in + h * hd;
#pragma unroll
    for (int u = 0; u < DPL; ++u) {
      const int d = lane + 64 * u;
      kr[j][u] = (j < Lk && d < hd) ? to_f32(kp[d]) : 0.f;
      vr[j][u] = (j < Lk && d < hd) ? to_f32(vp[d]) : 0.f;
      dka[j][u] = dva[j][u] = 0.f;
    }
  }
  for (int64_t i = 0; i < Lq; ++i) {
    const int64_t pos = i + (Lk - Lq);
    const int64_t jlo = (window > 0) ? max((int64_t)0, pos - window + 1) : 0;
    const bool qvalid = qmask ? (qmask[b * Lq + i] != 0) : true;
    const T* qp = q + (b * tq + i) * ld_in + h * hd;
    const T* dop = dout + (b * Lq + i) * ld_do + h * hd;
    const T* opp = o + (b * Lq + i) * ld_o + h * hd;
    float qr[DPL], dor[DPL], dqa[DPL];
    float dl = 0.f;
#pragma unroll
    for (int u = 0; u < DPL; ++u) {
      const int d = lane + 64 * u;
      qr[u] = d < hd ? to_f32(qp[d]) : 0.f;
      dor[u] = d < hd ? to_f32(dop[d]) : 0.f;
      dl = fmaf(dor[u], d < hd ? to_f32(opp[d]) : 0.f, dl);
      dqa[u] = 0.f;
    }
    dl = qvalid ? wave_sum(dl) : 0.f;  // delta = rowsum(dO o O)
    const float ls = lse[bh * Lq + i];
#pragma unroll
    for (int j = 0; j < LKM; ++j) {
      if (!(qvalid && kv[j] && j >= jlo && j <= pos)) continue;  // wave-uniform
      float s = 0.f, dpv = 0.f;
#pragma unroll
      for (int u = 0; u < DPL; ++u) {
        s = fmaf(qr[u], kr[j][u], s);
        dpv = fmaf(dor[u], vr[j][u], dpv);
      }
      s = wave_sum(s);
      dpv = wave_sum(dpv);
      const float keep = dr.p > 0.f ? dropout_mult(dr, elem_index(bh, Lq, Lk, i, j)) : 1.f;
      const float p = expf(s - ls);
      const float ds = p * (dpv * keep - dl);
      const float pd = p * keep;
#pragma unroll
      for (int u = 0; u < DPL; ++u) {
        dqa[u] = fmaf(ds, kr[j][u], dqa[u]);
        dka[j][u] = fmaf(ds, qr[u], dka[j][u]);
        dva[j][u] = fmaf(pd, dor[u], dva[j][u]);
      }
    }
    T* dqp = dq + (b * tq + i) * ld_d + h * hd;
#pragma unroll
    for (int u = 0; u < DPL; ++u)
      if (lane + 64 * u < hd) dqp[lane + 64 * u] = from_f32<T>(dqa[u]);
  }
  // the rows before the first query (static_kv_first: token 0) have no query: their dq is zero
  for (int64_t r = 1; r <= dq_lead; ++r) {
    T* dqp = dq + (b * tq - r) * ld_d + h * hd;
#pragma unroll
    for (int u = 0; u < DPL; ++u)
      if (lane + 64 * u < hd) dqp[lane + 64 * u] = from_f32<T>(0.f);
  }
#pragma unroll
  for (int j = 0; j < LKM; ++j) {
    if (j >= Lk) break;
    T* dkp = dk + (b * Lk + j) * ld_d + h * hd;
    T* dvp = dv + (b * Lk + j) * ld_d + h * hd;
#pragma unroll
    for (int u = 0; u < DPL; ++u) {
      const int d = lane + 64 * u;
      if (d < hd) {
        dkp[d] = from_f32<T>(dka[j][u]);
        dvp[d] = from_f32<T>(dva[j][u]);
      }
    }
  }
}

// ---- short sequences, four queries per wave (Lk <= 8, hd in {16, 32, 64}: the C4 dependency graph) ----------
// One wave per (sequence, head) as above, but the wave is four 16-lane row groups, each owning one query row of the
// current block of four (VE = hd / 16 consecutive dims per lane, one 2..16-byte vector load per row): the queries run
// in parallel (the lane-per-dimension form walks them one after another, each behind its own row loads), scores and
// dP are 16-lane DPP row reductions, and the backward's dK / dV partials are summed over the four groups with two
// permlane swaps at the end. Same visibility, masking, dropout-hash and zero-row semantics.
template <typename T, int VE>
__device__ __forceinline__ void load_vec(const T* p, float (&o)[VE]) {
  if constexpr (sizeof(T) == 4) {
    if constexpr (VE == 4) {
      const float4 t = *reinterpret_cast<const float4*>(p);
      o[0] = t.x, o[1] = t.y, o[2] = t.z, o[3] = t.w;
    } else if constexpr (VE == 2) {
      const float2 t = *reinterpret_cast<const float2*>(p);
      o[0] = t.x, o[1] = t.y;
    } else {
      o[0] = *reinterpret_cast<const float*>(p);
    }
  } else {
    if constexpr (VE == 4) {
      const uint2 t = *reinterpret_cast<const uint2*>(p);
      o[0] = __uint_as_float(t.x << 16), o[1] = __uint_as_float(t.x & 0xffff0000u);
      o[2] = __uint_as_float(t.y << 16), o[3] = __uint_as_float(t.y & 0xffff0000u);
    } else if constexpr (VE == 2) {
      const uint32_t t = *reinterpret_cast<const uint32_t*>(p);
      o[0] = __uint_as_float(t << 16), o[1] = __uint_as_float(t & 0xffff0000u);
    } else {
      o[0] = __uint_as_float((uint32_t)(*reinterpret_cast<const uint16_t*>(p)) << 16);
    }
  }
}

template <typename T, int VE>
__device__ __forceinline__ void store_vec(T* p, const float (&v)[VE]) {
  if constexpr (sizeof(T) == 4) {
    if constexpr (VE == 4) *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    else if constexpr (VE == 2) *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
    else *reinterpret_cast<float*>(p) = v[0];
  } else {
    if constexpr (VE == 4) {
      *reinterpret_cast<uint2*>(p) =
          make_uint2((uint32_t)f32_to_bf16_bits(v[0]) | ((uint32_t)f32_to_bf16_bits(v[1]) << 16),
                     (uint32_t)f32_to_bf16_bits(v[2]) | ((uint32_t)f32_to_bf16_bits(v[3]) << 16));
    } else if constexpr (VE == 2) {
      *reinterpret_cast<uint32_t*>(p) = (uint32_t)f32_to_bf16_bits(v[0]) | ((uint32_t)f32_to_bf16_bits(v[1]) << 16);
    } else {
      *reinterpret_cast<uint16_t*>(p) = f32_to_bf16_bits(v[0]);
    }
  }
}

// Sum over the 16 lanes of each row (every lane of the row ends with it); sum over the 4 rows of the wave.
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}
__device__ __forceinline__ float cross_rows(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

constexpr int kSmall4Lk = 8;

// Dropout multiplier of element (bh, qi, kj): the 32-bit index form when every element index of the launch fits 32
// bits (the same bits as dropout_mult; no 64-bit index products or high-word multiply).
template <bool I32>
__device__ __forceinline__ float small_keep(const DropoutSpec& dr, int64_t bh, int64_t Lq, int64_t Lk, int64_t qi,
                                            int64_t kj) {
  if constexpr (I32)
    return dropout_mult_32(dr, ((uint32_t)bh * (uint32_t)Lq + (uint32_t)qi) * (uint32_t)Lk + (uint32_t)kj);
  return dropout_mult(dr, elem_index(bh, Lq, Lk, qi, kj));
}

// Operands of one (sequence, head) item kept as raw packed words (bf16 pairs: half the registers of f32 copies),
// widened at each use: the wave's register footprint sets how many waves — and row loads — a CU keeps in flight,
// which is what bounds these kernels (a few hundred bytes of rows per wave, ~30 % of HBM at 4-5 waves per SIMD).
// The forward takes NI items per wave with every item's loads issued before the first computes.
template <typename T, int VE>
struct Raw {
  static constexpr int W = (VE * (int)sizeof(T) + 3) / 4;
  uint32_t w[W];
};

template <typename T, int VE>
__device__ __forceinline__ void raw_load(const T* p, Raw<T, VE>& r) {
  if constexpr (sizeof(T) == 4) {
    if constexpr (VE == 4) {
      const uint4 t = *reinterpret_cast<const uint4*>(p);
      r.w[0] = t.x, r.w[1] = t.y, r.w[2] = t.z, r.w[3] = t.w;
    } else if constexpr (VE == 2) {
      const uint2 t = *reinterpret_cast<const uint2*>(p);
      r.w[0] = t.x, r.w[1] = t.y;
    } else {
      r.w[0] = *reinterpret_cast<const uint32_t*>(p);
    }
  } else {
    if constexpr (VE == 4) {
      const uint2 t = *reinterpret_cast<const uint2*>(p);
      r.w[0] = t.x, r.w[1] = t.y;
    } else if constexpr (VE == 2) {
      r.w[0] = *reinterpret_cast<const uint32_t*>(p);
    } else {
      r.w[0] = (uint32_t)(*reinterpret_cast<const uint16_t*>(p)) << 16;
    }
  }
}

template <typename T, int VE>
__device__ __forceinline__ float raw_at(const Raw<T, VE>& r, int e) {
  if constexpr (sizeof(T) == 4) return __uint_as_float(r.w[e]);
  else if constexpr (VE == 1) return __uint_as_float(r.w[0]);
  else return (e & 1) ? __uint_as_float(r.w[e >> 1] & 0xffff0000u) : __uint_as_float(r.w[e >> 1] << 16);
}

template <typename T, int VE, int LKM>
struct S4Item {
  Raw<T, VE> k[LKM], v[LKM];
  Raw<T, VE> q, dout, o;  // the item's first query block (query i = g); bwd: + dO, O rows
  float ls;
  uint32_t km;  // bit j: key j not padded
  bool qm;      // query g not padded
};

template <typename T, int VE, int LKM, bool BWD>
__device__ __forceinline__ void s4_load(const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v,
                                        int64_t ld_in, int64_t tq, const T* __restrict__ o, int64_t ld_o,
                                        const T* __restrict__ dout, int64_t ld_do, const float* __restrict__ lse,
                                        const uint8_t* __restrict__ kmask, const uint8_t* __restrict__ qmask,
                                        int64_t bh, int64_t H, int64_t Lq, int64_t Lk, int hd, int g, int c,
                                        S4Item<T, VE, LKM>& r) {
  const int64_t h = bh % H, b = bh / H;
  r.km = 0;
#pragma unroll
  for (int j = 0; j < LKM; ++j) {
    if (j >= Lk) break;  // wave-uniform: only the sequence's keys are loaded
    if (!kmask || kmask[b * Lk + j] != 0) r.km |= 1u << j;
    raw_load<T, VE>(k + (b * Lk + j) * ld_in + h * hd + c, r.k[j]);
    raw_load<T, VE>(v + (b * Lk + j) * ld_in + h * hd + c, r.v[j]);
  }
  r.qm = false;
  if (Lq > 0) {
    const int64_t ii = min<int64_t>(g, Lq - 1);
    r.qm = !qmask || qmask[b * Lq + ii] != 0;
    raw_load<T, VE>(q + (b * tq + ii) * ld_in + h * hd + c, r.q);
    if constexpr (BWD) {
      raw_load<T, VE>(dout + (b * Lq + ii) * ld_do + h * hd + c, r.dout);
      raw_load<T, VE>(o + (b * Lq + ii) * ld_o + h * hd + c, r.o);
      r.ls = lse[bh * Lq + ii];
    }
  }
}

// item t of the wave: the NI items of a workgroup's wave w are bh = (blockIdx·NI + t)·4 + w (consecutive heads of
// one sequence per t: every row the workgroup reads is read whole)
template <int NI>
__device__ __forceinline__ int64_t s4_item(int t) {
  return ((int64_t)blockIdx.x * NI + t) * 4 + (threadIdx.x >> 6);
}

template <typename T, int VE, int LKM, bool I32, int NI, bool ONE>
__global__ __launch_bounds__(256) void attn_fwd_small4(const T* __restrict__ q, const T* __restrict__ k,
                                                       const T* __restrict__ v, int64_t ld_in, int64_t tq,
                                                       T* __restrict__ o, int64_t ld_o, float* __restrict__ lse,
                                                       const uint8_t* __restrict__ kmask,
                                                       const uint8_t* __restrict__ qmask, int64_t B, int64_t H,
                                                       int64_t Lq, int64_t Lk, int hd, int64_t window, float drop_p,
                                                       const uint64_t* __restrict__ seed) {
  const int64_t W = B * H;
  if (s4_item<NI>(0) >= W) return;  // wave-uniform
  const int lane = lane_id(), g = lane >> 4, c = (lane & 15) * VE;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  S4Item<T, VE, LKM> it[NI];
#pragma unroll
  for (int t = 0; t < NI; ++t)
    if (s4_item<NI>(t) < W)
      s4_load<T, VE, LKM, false>(q, k, v, ld_in, tq, nullptr, 0, nullptr, 0, nullptr, kmask, qmask, s4_item<NI>(t), H,
                                 Lq, Lk, hd, g, c, it[t]);
#pragma unroll
  for (int t = 0; t < NI; ++t) {
    const int64_t bh = s4_item<NI>(t);
    if (bh >= W) break;  // wave-uniform
    const S4Item<T, VE, LKM>& cur = it[t];
    const int64_t h = bh % H, b = bh / H;
    // ONE (Lq <= 4): a single query block, no loop — the packed operands are widened where they are used instead
    // of being hoisted out of a loop as f32 copies
    for (int64_t i0 = 0; i0 < (ONE ? 1 : Lq); i0 += 4) {
      const int64_t i = i0 + g;
      const bool qin = i < Lq;
      const int64_t ii = qin ? i : Lq - 1;
      const int64_t pos = ii + (Lk - Lq);
      const int64_t jlo = (window > 0) ? max((int64_t)0, pos - window + 1) : 0;
      float qr[VE];
      bool qvalid;
      if (i0 == 0) {
#pragma unroll
        for (int e = 0; e < VE; ++e) qr[e] = raw_at<T, VE>(cur.q, e);
        qvalid = qin && cur.qm;
      } else {
        qvalid = qin && (qmask ? (qmask[b * Lq + ii] != 0) : true);
        load_vec<T, VE>(q + (b * tq + ii) * ld_in + h * hd + c, qr);
      }
      float s[LKM];
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < LKM; ++j) {
        s[j] = -INFINITY;
        if (j >= Lk) break;
        float tt = 0.f;
#pragma unroll
        for (int e = 0; e < VE; ++e) tt = fmaf(qr[e], raw_at<T, VE>(cur.k[j], e), tt);
        tt = row_sum16(tt);  // every lane of the wave takes part (DPP)
        const bool ok = qvalid && ((cur.km >> j) & 1u) && j >= jlo && j <= pos;
        s[j] = ok ? tt : -INFINITY;
        m = fmaxf(m, s[j]);
      }
      float l = 0.f, acc[VE];
#pragma unroll
      for (int e = 0; e < VE; ++e) acc[e] = 0.f;
#pragma unroll
      for (int j = 0; j < LKM; ++j) {
        if (j >= Lk) break;
        if (s[j] == -INFINITY) continue;
        const float p = expf(s[j] - m);
        l += p;  // normaliser over undropped probabilities
        const float pd = dr.p > 0.f ? p * small_keep<I32>(dr, bh, Lq, Lk, ii, j) : p;
#pragma unroll
        for (int e = 0; e < VE; ++e) acc[e] = fmaf(pd, raw_at<T, VE>(cur.v[j], e), acc[e]);
      }
      const bool ok = qvalid && l > 0.f;
      const float inv = ok ? 1.f / l : 0.f;
#pragma unroll
      for (int e = 0; e < VE; ++e) acc[e] *= inv;
      if (qin) {
        store_vec<T, VE>(o + (b * Lq + ii) * ld_o + h * hd + c, acc);
        if ((lane & 15) == 0) lse[bh * Lq + ii] = ok ? m + logf(l) : 0.f;
      }
    }
  }
}

template <typename T, int VE, int LKM, bool I32, int NI, bool ONE>
__global__ __launch_bounds__(256) void attn_bwd_small4(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v, int64_t ld_in, int64_t tq,
    const T* __restrict__ o, int64_t ld_o, const T* __restrict__ dout, int64_t ld_do, const float* __restrict__ lse,
    const uint8_t* __restrict__ kmask, const uint8_t* __restrict__ qmask, T* __restrict__ dq, T* __restrict__ dk,
    T* __restrict__ dv, int64_t ld_d, int64_t B, int64_t H, int64_t Lq, int64_t Lk, int hd, int64_t window,
    float drop_p, const uint64_t* __restrict__ seed, int64_t dq_lead) {
  const int64_t W = B * H;
  if (s4_item<NI>(0) >= W) return;  // wave-uniform
  const int lane = lane_id(), g = lane >> 4, c = (lane & 15) * VE;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  S4Item<T, VE, LKM> it[NI];
#pragma unroll
  for (int t = 0; t < NI; ++t)
    if (s4_item<NI>(t) < W)
      s4_load<T, VE, LKM, true>(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, kmask, qmask, s4_item<NI>(t), H, Lq, Lk,
                                hd, g, c, it[t]);
#pragma unroll
  for (int t = 0; t < NI; ++t) {
    const int64_t bh = s4_item<NI>(t);
    if (bh >= W) break;  // wave-uniform
    const S4Item<T, VE, LKM>& cur = it[t];
    const int64_t h = bh % H, b = bh / H;
    float dka[LKM][VE], dva[LKM][VE];
#pragma unroll
    for (int j = 0; j < LKM; ++j)
#pragma unroll
      for (int e = 0; e < VE; ++e) dka[j][e] = dva[j][e] = 0.f;
    // ONE (Lq <= 4): a single query block, no loop — the packed operands are widened where they are used instead
    // of being hoisted out of a loop as f32 copies
    for (int64_t i0 = 0; i0 < (ONE ? 1 : Lq); i0 += 4) {
      const int64_t i = i0 + g;
      const bool qin = i < Lq;
      const int64_t ii = qin ? i : Lq - 1;
      const int64_t pos = ii + (Lk - Lq);
      const int64_t jlo = (window > 0) ? max((int64_t)0, pos - window + 1) : 0;
      float qr[VE], dor[VE], orr[VE], dqa[VE], ls;
      bool qvalid;
      if (i0 == 0) {
#pragma unroll
        for (int e = 0; e < VE; ++e)
          qr[e] = raw_at<T, VE>(cur.q, e), dor[e] = raw_at<T, VE>(cur.dout, e), orr[e] = raw_at<T, VE>(cur.o, e);
        ls = cur.ls;
        qvalid = qin && cur.qm;
      } else {
        qvalid = qin && (qmask ? (qmask[b * Lq + ii] != 0) : true);
        load_vec<T, VE>(q + (b * tq + ii) * ld_in + h * hd + c, qr);
        load_vec<T, VE>(dout + (b * Lq + ii) * ld_do + h * hd + c, dor);
        load_vec<T, VE>(o + (b * Lq + ii) * ld_o + h * hd + c, orr);
        ls = lse[bh * Lq + ii];
      }
      float dl = 0.f;
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        dl = fmaf(dor[e], orr[e], dl);
        dqa[e] = 0.f;
      }
      dl = row_sum16(dl);  // delta = rowsum(dO o O)
      if (!qvalid) dl = 0.f;
#pragma unroll
      for (int j = 0; j < LKM; ++j) {
        if (j >= Lk) break;  // wave-uniform
        float sv = 0.f, dpv = 0.f;
#pragma unroll
        for (int e = 0; e < VE; ++e) {
          sv = fmaf(qr[e], raw_at<T, VE>(cur.k[j], e), sv);
          dpv = fmaf(dor[e], raw_at<T, VE>(cur.v[j], e), dpv);
        }
        sv = row_sum16(sv);
        dpv = row_sum16(dpv);
        if (!(qvalid && ((cur.km >> j) & 1u) && j >= jlo && j <= pos)) continue;  // row-uniform
        const float keep = dr.p > 0.f ? small_keep<I32>(dr, bh, Lq, Lk, ii, j) : 1.f;
        const float p = expf(sv - ls);
        const float ds = p * (dpv * keep - dl);
        const float pd = p * keep;
#pragma unroll
        for (int e = 0; e < VE; ++e) {
          dqa[e] = fmaf(ds, raw_at<T, VE>(cur.k[j], e), dqa[e]);
          dka[j][e] = fmaf(ds, qr[e], dka[j][e]);
          dva[j][e] = fmaf(pd, dor[e], dva[j][e]);
        }
      }
      if (qin) store_vec<T, VE>(dq + (b * tq + ii) * ld_d + h * hd + c, dqa);
    }
    // the rows before the first query (static_kv_first: token 0) have no query: their dq is zero
    if (g < dq_lead) {
      float z[VE];
#pragma unroll
      for (int e = 0; e < VE; ++e) z[e] = 0.f;
      store_vec<T, VE>(dq + (b * tq - 1 - g) * ld_d + h * hd + c, z);
    }
    // dK / dV: the four query groups' partials summed (every group ends with the sums); group g stores the rows
    // j = g, g + 4
#pragma unroll
    for (int j = 0; j < LKM; ++j) {
      if (j >= Lk) break;  // wave-uniform
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        dka[j][e] = cross_rows(dka[j][e]);
        dva[j][e] = cross_rows(dva[j][e]);
      }
      if ((j & 3) == g) {
        store_vec<T, VE>(dk + (b * Lk + j) * ld_d + h * hd + c, dka[j]);
        store_vec<T, VE>(dv + (b * Lk + j) * ld_d + h * hd + c, dva[j]);
      }
    }
  }
}

// Items per wave of the small4 forward / backward (ESGPT_SMALL4_NI = "fwd,bwd" overrides: 1 or 2 each)
static void small4_ni(int& f, int& b) {
  static int nf = -1, nb = -1;
  if (nf < 0) {
    nf = 1, nb = 1;
    const char* e = tuning_env("ESGPT_SMALL4_NI");
    if (e && e[0] && e[1] == ',' && e[2]) nf = e[0] == '1' ? 1 : 2, nb = e[2] == '1' ? 1 : 2;
  }
  f = nf, b = nb;
}

// The four-query form applies (aligned VE-element rows).
template <typename T>
bool small4_ok(int64_t Lk, int64_t hd, std::initializer_list<const void*> ptrs, std::initializer_list<int64_t> lds) {
  if (!(Lk <= kSmall4Lk && (hd == 16 || hd == 32 || hd == 64))) return false;
  const int64_t vb = (hd / 16) * (int64_t)sizeof(T);  // bytes per lane vector
  for (const void* p : ptrs)
    if (p && ((uintptr_t)p % vb)) return false;
  for (int64_t ld : lds)
    if ((ld * (int64_t)sizeof(T)) % vb) return false;
  return true;
}

template <typename T>
int launch_small(bool fwd, const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                 int64_t ld_o, float* lse_w, const float* lse_r, const void* dout, int64_t ld_do,
                 const uint8_t* kmask, const uint8_t* qmask, void* dq, void* dk, void* dv, int64_t ld_d, int64_t B,
                 int64_t H, int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed,
                 int64_t dq_lead, hipStream_t st) {
  const dim3 grid((unsigned)cdiv(B * H, 4)), block(256);
  if (small4_ok<T>(Lk, hd, {q, k, v, o, dout, dq, dk, dv}, {ld_in, ld_o, ld_do, ld_d})) {
    int nif, nib;
    small4_ni(nif, nib);
    const int ni = fwd ? nif : nib;  // items per wave
    const bool one = Lq <= 4;        // one query block per item
    const dim3 grid4((unsigned)cdiv(B * H, 4 * ni));
#define SMALL4_FWD_NI(VE, LKM, I32, NI, ONE)                                                                       \
  attn_fwd_small4<T, VE, LKM, I32, NI, ONE><<<grid4, block, 0, st>>>((const T*)q, (const T*)k, (const T*)v, ld_in,   \
                                                                     tq, (T*)o, ld_o, lse_w, kmask, qmask, B, H, Lq, \
                                                                     Lk, (int)hd, window, drop_p, seed)
#define SMALL4_BWD_NI(VE, LKM, I32, NI, ONE)                                                                       \
  attn_bwd_small4<T, VE, LKM, I32, NI, ONE><<<grid4, block, 0, st>>>(                                                \
      (const T*)q, (const T*)k, (const T*)v, ld_in, tq, (const T*)o, ld_o, (const T*)dout, ld_do, lse_r, kmask,      \
      qmask, (T*)dq, (T*)dk, (T*)dv, ld_d, B, H, Lq, Lk, (int)hd, window, drop_p, seed, dq_lead)
#define SMALL4_FWD(VE, LKM, I32)                                        \
  do {                                                                  \
    if (ni == 2) {                                                      \
      if (one) SMALL4_FWD_NI(VE, LKM, I32, 2, true);                    \
      else SMALL4_FWD_NI(VE, LKM, I32, 2, false);                       \
    } else {                                                            \
      if (one) SMALL4_FWD_NI(VE, LKM, I32, 1, true);                    \
      else SMALL4_FWD_NI(VE, LKM, I32, 1, false);                       \
    }                                                                   \
  } while (0)
#define SMALL4_BWD(VE, LKM, I32)                                        \
  do {                                                                  \
    if (ni == 2) {                                                      \
      if (one) SMALL4_BWD_NI(VE, LKM, I32, 2, true);                    \
      else SMALL4_BWD_NI(VE, LKM, I32, 2, false);                       \
    } else {                                                            \
      if (one) SMALL4_BWD_NI(VE, LKM, I32, 1, true);                    \
      else SMALL4_BWD_NI(VE, LKM, I32, 1, false);                       \
    }                                                                   \
  } while (0)
// key registers sized to the sequence (LKM = 4, 6 or 8 keys): the C4 dependency graph (5 keys) holds 3/4 of the
// 8-key form's K / V / dK / dV registers
#define SMALL4_L(VE, LKM, I32)                                                                                       \
  do {                                                                                                               \
    if (fwd)                                                                                                         \
      SMALL4_FWD(VE, LKM, I32);                                                                                      \
    else                                                                                                             \
      SMALL4_BWD(VE, LKM, I32);                                                                                      \
  } while (0)
  // 32-bit dropout element indices whenever the launch's indices fit (the same keep bits); the 64-bit form only for
  // launches past 2^32 elements
  const bool idx32 = (uint64_t)(B * H) * (uint64_t)Lq * (uint64_t)Lk <= 0xffffffffull;
#define SMALL4(VE)                                     \
  do {                                                 \
    if (!idx32) SMALL4_L(VE, 8, false);                \
    else if (Lk <= 4) SMALL4_L(VE, 4, true);           \
    else if (Lk <= 6) SMALL4_L(VE, 6, true);           \
    else SMALL4_L(VE, 8, true);                        \
  } while (0)
    if (hd == 16) SMALL4(1);
    else if (hd == 32) SMALL4(2);
    else SMALL4(4);
#undef SMALL4
#undef SMALL4_L
#undef SMALL4_FWD
#undef SMALL4_BWD
#undef SMALL4_FWD_NI
#undef SMALL4_BWD_NI
    return hipGetLastError() == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
  }
#define SMALL(DPL, LKM)                                                                                             \
  do {                                                                                                              \
    if (fwd)                                                                                                        \
      attn_fwd_small<T, DPL, LKM><<<grid, block, 0, st>>>((const T*)q, (const T*)k, (const T*)v, ld_in, tq, (T*)o, \
                                                          ld_o, lse_w, kmask, qmask, B, H, Lq, Lk, (int)hd, window,  \
                                                          drop_p, seed);                                           \
    else                                                                                                            \
      attn_bwd_small<T, DPL, LKM><<<grid, block, 0, st>>>(                                                          \
          (const T*)q, (const T*)k, (const T*)v, ld_in, tq, (const T*)o, ld_o, (const T*)dout, ld_do, lse_r, kmask, \
          qmask, (T*)dq, (T*)dk, (T*)dv, ld_d, B, H, Lq, Lk, (int)hd, window, drop_p, seed, dq_lead);               \
  } while (0)
  if (hd <= 64) {
    if (Lk <= 8) SMALL(1, 8);
    else SMALL(1, 16);
  } else {
    if (Lk <= 8) SMALL(2, 8);
    else SMALL(2, 16);
  }
#undef SMALL
  return hipGetLastError() == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
}

template <typename T>
int launch_fwd_generic(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, void* o, int64_t ld_o,
                       float* lse, const uint8_t* kmask, const uint8_t* qmask, int64_t B, int64_t H, int64_t Lq,
                       int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed, hipStream_t st) {
  const int64_t total = B * H * Lq;
  dim3 grid((unsigned)cdiv(total, 256)), block(256);
#define FWD(HDP)                                                                                                  \
  attn_fwd_generic<T, HDP><<<grid, block, 0, st>>>((const T*)q, (const T*)k, (const T*)v, ld_in, tq, (T*)o, ld_o, \
                                                   lse, kmask, qmask, B, H, Lq, Lk, (int)hd, window, drop_p, seed)
  if (hd <= 8) FWD(8);
  else if (hd <= 16) FWD(16);
  else if (hd <= 32) FWD(32);
  else if (hd <= 64) FWD(64);
  else FWD(128);
#undef FWD
  return hipGetLastError() == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
}

template <typename T>
int launch_bwd_generic(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                       int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* kmask,
                       const uint8_t* qmask, void* dq, void* dk, void* dv, int64_t ld_d, int64_t B, int64_t H,
                       int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed,
                       float* delta, hipStream_t st) {
  dim3 gq((unsigned)cdiv(B * H * Lq, 256)), gk((unsigned)cdiv(B * H * Lk, 256)), block(256);
#define BWD(HDP)                                                                                                   \
  do {                                                                                                             \
    attn_bwd_dq_generic<T, HDP><<<gq, block, 0, st>>>((const T*)q, (const T*)k, (const T*)v, ld_in, tq,             \
                                                      (const T*)o, ld_o, (const T*)dout, ld_do, lse, kmask, qmask,  \
                                                      (T*)dq, ld_d, delta, B, H, Lq, Lk, (int)hd, window, drop_p,   \
                                                      seed);                                                       \
    attn_bwd_dkv_generic<T, HDP><<<gk, block, 0, st>>>((const T*)q, (const T*)k, (const T*)v, ld_in, tq,           \
                                                       (const T*)dout, ld_do, lse, delta, kmask, qmask, (T*)dk,     \
                                                       (T*)dv, ld_d, B, H, Lq, Lk, (int)hd, window, drop_p, seed);  \
  } while (0)
  if (hd <= 8) BWD(8);
  else if (hd <= 16) BWD(16);
  else if (hd <= 32) BWD(32);
  else if (hd <= 64) BWD(64);
  else BWD(128);
#undef BWD
  return hipGetLastError() == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
}

// dq rows [-lead, 0) of every sequence <- 0 (the paths whose kernels do not write them: MFMA, generic)
template <typename T>
__global__ __launch_bounds__(256) void dq_lead_zero_kernel(T* __restrict__ dq, int64_t ld_d, int64_t tq, int64_t B,
                                                           int64_t lead, int64_t D) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, n = B * lead * D;
  if (i >= n) return;
  const int64_t b = i / (lead * D), r = (i / D) % lead, d = i % D;
  dq[(b * tq - 1 - r) * ld_d + d] = from_f32<T>(0.f);
}

}  // namespace

// MFMA path (attention_mfma.hip).
int esgpt_attn_fwd_mfma(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, void* o, int64_t ld_o,
                        float* lse, const uint8_t* kmask, const uint8_t* qmask, int64_t B, int64_t H, int64_t Lq,
                        int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed, uint32_t* keep,
                        hipStream_t st);
int esgpt_attn_bwd_mfma(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                        int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* kmask,
                        const uint8_t* qmask, void* dq, void* dk, void* dv, int64_t ld_d, int64_t B, int64_t H,
                        int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed,
                        const uint32_t* keep, float* dq32, int32_t* counters, hipStream_t st);
size_t esgpt_attn_bwd_mfma_workspace(int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t hd);
int64_t esgpt_attn_bwd_mfma_counters(int64_t B, int64_t H, int64_t Lk);
bool esgpt_attn_mfma_supported(int64_t hd, int64_t Lq, int64_t Lk, int64_t tq, int64_t ld_in, int64_t ld_o);
// f32 MFMA path (attention_f32.hip).
bool esgpt_attn_f32_mfma_supported(int64_t hd, int64_t Lq, int64_t Lk, int64_t ld_in, int64_t ld_o);
int esgpt_attn_fwd_f32_mfma(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, void* o,
                            int64_t ld_o, float* lse, const uint8_t* kmask, const uint8_t* qmask, int64_t B, int64_t H,
                            int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed,
                            hipStream_t st);
int esgpt_attn_bwd_f32_mfma(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                            int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* kmask,
                            const uint8_t* qmask, void* dq, void* dk, void* dv, int64_t ld_d, int64_t B, int64_t H,
                            int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed,
                            float* delta, hipStream_t st);

static int g_force_generic = -1;

static bool force_generic() {
  if (g_force_generic < 0) {
    const char* e = tuning_env("ESGPT_ATTN_GENERIC");
    g_force_generic = (e && e[0] == '1') ? 1 : 0;
  }
  return g_force_generic == 1;
}

extern "C" {

int esgpt_attn_fwd(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, void* o, int64_t ld_o,
                   float* lse, const uint8_t* key_mask, const uint8_t* query_mask, int64_t B, int64_t H, int64_t Lq,
                   int64_t Lk, int64_t hd, int64_t window, float dropout_p, const uint64_t* seed, int dtype,
                   void* stream) {
  return esgpt_attn_fwd_ex(q, k, v, ld_in, tq, o, ld_o, lse, key_mask, query_mask, B, H, Lq, Lk, hd, window, dropout_p,
                           seed, dtype, nullptr, stream);
}

int64_t esgpt_attn_keep_words(int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t hd, int64_t tq, int64_t ld_in,
                              int64_t ld_o, int dtype, float dropout_p) {
  if (!(dropout_p > 0.f) || dtype != ESGPT_BF16 || force_generic() ||
      !esgpt_attn_mfma_supported(hd, Lq, Lk, tq, ld_in, ld_o))
    return 0;
  // The keep bits are O(Lq·Lk) activation memory per layer (Lq·⌈Lk/32⌉·4 B per (batch, head): 8 KiB at L = 256,
  // 2 MiB at L = 4096). Above kKeepMaxLk keys, or kKeepMaxBytes per launch, the backward re-hashes the mask instead
  // (the same bits; attention memory stays O(L)).
  constexpr int64_t kKeepMaxLk = 2048, kKeepMaxBytes = 256ll << 20;
  const int64_t words = B * H * Lq * cdiv(Lk, 32);
  if (Lk > kKeepMaxLk || 4 * words > kKeepMaxBytes) return 0;
  return words;
}

int esgpt_attn_fwd_ex(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, void* o, int64_t ld_o,
                      float* lse, const uint8_t* key_mask, const uint8_t* query_mask, int64_t B, int64_t H, int64_t Lq,
                      int64_t Lk, int64_t hd, int64_t window, float dropout_p, const uint64_t* seed, int dtype,
                      uint32_t* keep, void* stream) {
  ESGPT_REQUIRE(q && k && v && o && lse && hd > 0 && hd <= 128 && Lq <= Lk && Lq >= 0 && window >= 0 && tq >= Lq);
  ESGPT_REQUIRE(dtype == ESGPT_F32 || dtype == ESGPT_BF16);
  ESGPT_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || seed));
  if (B * H * Lq == 0) return ESGPT_OK;
  if (esgpt_attn_keep_words(B, H, Lq, Lk, hd, tq, ld_in, ld_o, dtype, dropout_p) == 0) keep = nullptr;
  ESGPT_REQUIRE(keep == nullptr || ((uintptr_t)keep % 4) == 0);
  hipStream_t st = as_stream(stream);
  if (dtype == ESGPT_BF16 && !force_generic() && esgpt_attn_mfma_supported(hd, Lq, Lk, tq, ld_in, ld_o))
    return esgpt_attn_fwd_mfma(q, k, v, ld_in, tq, o, ld_o, lse, key_mask, query_mask, B, H, Lq, Lk, hd, window,
                               dropout_p, seed, keep, st);
  if (dtype == ESGPT_F32 && !force_generic() && esgpt_attn_f32_mfma_supported(hd, Lq, Lk, ld_in, ld_o)) {
    const int rc = esgpt_attn_fwd_f32_mfma(q, k, v, ld_in, tq, o, ld_o, lse, key_mask, query_mask, B, H, Lq, Lk, hd,
                                           window, dropout_p, seed, st);
    if (rc != ESGPT_ERR_UNSUPPORTED) return rc;  // unaligned operands: the generic kernels
  }
  if (Lk <= kSmallLk && !force_generic()) {
    if (dtype == ESGPT_F32)
      return launch_small<float>(true, q, k, v, ld_in, tq, o, ld_o, lse, nullptr, nullptr, 0, key_mask, query_mask,
                                 nullptr, nullptr, nullptr, 0, B, H, Lq, Lk, hd, window, dropout_p, seed, 0, st);
    return launch_small<bf16>(true, q, k, v, ld_in, tq, o, ld_o, lse, nullptr, nullptr, 0, key_mask, query_mask,
                              nullptr, nullptr, nullptr, 0, B, H, Lq, Lk, hd, window, dropout_p, seed, 0, st);
  }
  if (dtype == ESGPT_F32)
    return launch_fwd_generic<float>(q, k, v, ld_in, tq, o, ld_o, lse, key_mask, query_mask, B, H, Lq, Lk, hd, window,
                                     dropout_p, seed, st);
  return launch_fwd_generic<bf16>(q, k, v, ld_in, tq, o, ld_o, lse, key_mask, query_mask, B, H, Lq, Lk, hd, window,
                                  dropout_p, seed, st);
}

int esgpt_attn_path(int64_t hd, int64_t Lq, int64_t Lk, int64_t tq, int64_t ld_in, int64_t ld_o, int dtype) {
  if (dtype == ESGPT_BF16 && !force_generic() && esgpt_attn_mfma_supported(hd, Lq, Lk, tq, ld_in, ld_o))
    return ESGPT_ATTN_PATH_MFMA;
  if (dtype == ESGPT_F32 && !force_generic() && esgpt_attn_f32_mfma_supported(hd, Lq, Lk, ld_in, ld_o))
    return ESGPT_ATTN_PATH_MFMA_F32;  // (16-B aligned operands; otherwise the launch takes the generic kernels)
  if (Lk <= kSmallLk && !force_generic()) return ESGPT_ATTN_PATH_SMALL;
  return ESGPT_ATTN_PATH_GENERIC;
}

int64_t esgpt_attn_bwd_counters(int64_t B, int64_t H, int64_t Lk) { return esgpt_attn_bwd_mfma_counters(B, H, Lk); }

size_t esgpt_attn_bwd_workspace(int64_t B, int64_t H, int64_t Lq, int64_t Lk, int64_t hd) {
  // generic kernels: δ = rowsum(dO∘O) [B*H*Lq]; MFMA kernel: f32 dQ accumulator when Lk > 256, + the dK / dV
  // exchange slabs of the query-split workgroup pairs
  const size_t a = sizeof(float) * (size_t)(B * H * Lq), b = esgpt_attn_bwd_mfma_workspace(B, H, Lq, Lk, hd);
  return a > b ? a : b;
}

int esgpt_attn_bwd(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                   int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* key_mask,
                   const uint8_t* query_mask, void* dq, void* dk, void* dv, int64_t ld_dqkv, int64_t B, int64_t H,
                   int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float dropout_p, const uint64_t* seed,
                   int dtype, void* workspace, size_t workspace_bytes, int32_t* counters, void* stream) {
  return esgpt_attn_bwd_ex(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, key_mask, query_mask, dq, dk, dv, ld_dqkv,
                           B, H, Lq, Lk, hd, window, dropout_p, seed, nullptr, dtype, workspace, workspace_bytes,
                           counters, stream);
}

int esgpt_attn_bwd_ex(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                      int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* key_mask,
                      const uint8_t* query_mask, void* dq, void* dk, void* dv, int64_t ld_dqkv, int64_t B, int64_t H,
                      int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float dropout_p, const uint64_t* seed,
                      const uint32_t* keep, int dtype, void* workspace, size_t workspace_bytes, int32_t* counters,
                      void* stream) {
  return esgpt_attn_bwd_lead(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, key_mask, query_mask, dq, dk, dv,
                             ld_dqkv, B, H, Lq, Lk, hd, window, dropout_p, seed, keep, dtype, workspace,
                             workspace_bytes, counters, 0, stream);
}

int esgpt_attn_bwd_lead(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                        int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* key_mask,
                        const uint8_t* query_mask, void* dq, void* dk, void* dv, int64_t ld_dqkv, int64_t B, int64_t H,
                        int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float dropout_p, const uint64_t* seed,
                        const uint32_t* keep, int dtype, void* workspace, size_t workspace_bytes, int32_t* counters,
                        int64_t dq_lead, void* stream) {
  ESGPT_REQUIRE(q && k && v && o && dout && lse && dq && dk && dv && hd > 0 && hd <= 128 && Lq <= Lk);
  ESGPT_REQUIRE(dq_lead >= 0 && dq_lead <= 4 && Lq + dq_lead <= tq);
  if (esgpt_attn_keep_words(B, H, Lq, Lk, hd, tq, ld_in, ld_o, dtype, dropout_p) == 0) keep = nullptr;
  ESGPT_REQUIRE(keep == nullptr || ((uintptr_t)keep % 4) == 0);
  ESGPT_REQUIRE(dtype == ESGPT_F32 || dtype == ESGPT_BF16);
  ESGPT_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || seed));
  ESGPT_REQUIRE(workspace && workspace_bytes >= esgpt_attn_bwd_workspace(B, H, Lq, Lk, hd));
  if (B * H * Lk == 0) return ESGPT_OK;
  hipStream_t st = as_stream(stream);
  float* delta = (float*)workspace;
  const bool small = Lk <= kSmallLk && !force_generic();
  const bool mfma = dtype == ESGPT_BF16 && !force_generic() && esgpt_attn_mfma_supported(hd, Lq, Lk, tq, ld_in, ld_o);
  const bool mfma32 = dtype == ESGPT_F32 && !force_generic() && esgpt_attn_f32_mfma_supported(hd, Lq, Lk, ld_in, ld_o);
  if (dq_lead > 0 && (mfma || mfma32 || !small)) {  // the small kernels write these rows themselves
    const int64_t n = B * dq_lead * H * hd;
    if (dtype == ESGPT_F32)
      dq_lead_zero_kernel<float><<<(unsigned)cdiv(n, 256), 256, 0, st>>>((float*)dq, ld_dqkv, tq, B, dq_lead, H * hd);
    else
      dq_lead_zero_kernel<bf16><<<(unsigned)cdiv(n, 256), 256, 0, st>>>((bf16*)dq, ld_dqkv, tq, B, dq_lead, H * hd);
    dq_lead = 0;
  }
  if (mfma)
    return esgpt_attn_bwd_mfma(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, key_mask, query_mask, dq, dk, dv,
                               ld_dqkv, B, H, Lq, Lk, hd, window, dropout_p, seed, keep, (float*)workspace,
                               counters, st);
  if (mfma32) {
    const int rc = esgpt_attn_bwd_f32_mfma(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, key_mask, query_mask, dq,
                                           dk, dv, ld_dqkv, B, H, Lq, Lk, hd, window, dropout_p, seed, delta, st);
    if (rc != ESGPT_ERR_UNSUPPORTED) return rc;
  }
  if (small) {
    if (dtype == ESGPT_F32)
      return launch_small<float>(false, q, k, v, ld_in, tq, o, ld_o, nullptr, lse, dout, ld_do, key_mask, query_mask,
                                 dq, dk, dv, ld_dqkv, B, H, Lq, Lk, hd, window, dropout_p, seed, dq_lead, st);
    return launch_small<bf16>(false, q, k, v, ld_in, tq, o, ld_o, nullptr, lse, dout, ld_do, key_mask, query_mask,
                              dq, dk, dv, ld_dqkv, B, H, Lq, Lk, hd, window, dropout_p, seed, dq_lead, st);
  }
  if (dtype == ESGPT_F32)
    return launch_bwd_generic<float>(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, key_mask, query_mask, dq, dk, dv,
                                     ld_dqkv, B, H, Lq, Lk, hd, window, dropout_p, seed, delta, st);
  return launch_bwd_generic<bf16>(q, k, v, ld_in, tq, o, ld_o, dout, ld_do, lse, key_mask, query_mask, dq, dk, dv,
                                  ld_dqkv, B, H, Lq, Lk, hd, window, dropout_p, seed, delta, st);
}

}  // extern "C"
