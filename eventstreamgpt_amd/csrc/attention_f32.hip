// f32 MFMA attention for gfx950: the reference-precision path of InnerSelfAttention._attn (transformer.py:171-217),
// which the reference runs in f32 (scripts/pretrain.py:24). v_mfma_f32_32x32x2_f32 multiplies exact f32 operands
// into f32 accumulators (the FP32 vector rate, 1/16 of bf16 MFMA), hd in {16, 32, 64, 128}; same semantics as the
// generic kernels of attention.hip (visibility, key / query masks, the counter-hash dropout, zero rows for padded
// queries) — results differ from them only by f32 summation order.
//
// Fragment maps (32x32x2 f32): lane l = (r = l&31, h = l>>5) supplies A[row r][k = h] and B[k = h][col r]; C/D
// register i holds row acc_row(i, h) = (i&3) + 8(i>>2) + 4h, column r.
//   * Row-by-row contractions (S = Q·Kᵀ, dP = dO·Vᵀ) run over the head dimension in the permuted order
//     k-step t <-> element 8(t/4) + 4h + t%4, so each lane's operand is its row's float4 chunks (16-B loads):
//     row fragments, HD/2 floats per lane.
//   * Contractions over keys or queries (O += P·V, dQ += dS·K, dV += Pᵀ·dO, dK += dSᵀ·Q) take the probability-like
//     operand straight from an accumulator: k-step s of lane (r, h) is its register s (row acc_row(s, h)); the other
//     operand is read in that same row order, one float per lane per k-step (column fragments: 32 consecutive
//     floats of a row per half-wave, coalesced).
// Every wave works alone (no LDS, no barriers): forward and dQ: one wave per 32 queries of one (batch, head), keys in
// 32-key tiles (Sᵀ layout: key on the register rows, query on the lane, so the softmax statistics of a query are
// lane-local plus one xor-32 exchange); dK / dV: one wave per 32 keys, query tiles in S layout (query rows, key on the
// lane). Fully masked tiles are skipped.
// Roofline: MFMA-bound; algorithmic FLOPs fwd 4·hd·T, bwd 8·hd·T per (batch, head) (T = allowed (q, k) pairs).
#include "common.h"

using namespace esgpt;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ __forceinline__ bool allowed(int key, int qpos, int window) {
  return key <= qpos && (window == 0 || qpos - key < window);
}

// Dropout element counter of the generic kernels: (bh * Lq + q) * Lk + key.
__device__ __forceinline__ uint64_t elem_index(int bh, int Lq, int Lk, int qi, int kj) {
  return ((uint64_t)bh * (uint64_t)Lq + (uint64_t)qi) * (uint64_t)Lk + (uint64_t)kj;
}

// Row fragment of one row (lane r's row, or zeros when !ok): f[4u + j] = row[8u + 4h + j].
template <int HD>
__device__ __forceinline__ void row_frag(float (&f)[HD / 2], const float* row, bool ok, int h) {
#pragma unroll
  for (int u = 0; u < HD / 8; ++u) {
    const float4 x = ok ? *reinterpret_cast<const float4*>(row + 8 * u + 4 * h) : make_float4(0.f, 0.f, 0.f, 0.f);
    f[4 * u] = x.x, f[4 * u + 1] = x.y, f[4 * u + 2] = x.z, f[4 * u + 3] = x.w;
  }
}

// Column fragments: f[dt][s] = M[row0 + acc_row(s, h)][32·dt + r] (rows past rmax and columns past HD read 0).
template <int HD, int ND>
__device__ __forceinline__ void col_frag(float (&f)[ND][16], const float* base, int64_t ld, int row0, int rmax, int r,
                                         int h) {
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int row = row0 + acc_row(s, h), col = 32 * dt + r;
      f[dt][s] = (row <= rmax && col < HD) ? base[(int64_t)row * ld + col] : 0.f;
    }
}

// Stores the transposed accumulators of one lane: acc[dt][i] = X[row r][32·dt + acc_row(i, h)] -> dst[0 .. HD-1]
// (4 consecutive columns per register group: float4 stores), each value times `scale`.
template <int HD, int ND>
__device__ __forceinline__ void store_rowT(float* dst, const f32x16 (&acc)[ND], int h, float scale) {
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * h;
      if (d < HD)
        *reinterpret_cast<float4*>(dst + d) = make_float4(acc[dt][4 * g] * scale, acc[dt][4 * g + 1] * scale,
                                                          acc[dt][4 * g + 2] * scale, acc[dt][4 * g + 3] * scale);
    }
}

constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;

// ---- forward: one wave per 32-query block ---------------------------------------------------------------------
template <int HD, bool DROP>
__global__ __launch_bounds__(256) void attn_fwd_f32_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                           const float* __restrict__ v, int64_t ld_in, int64_t tq,
                                                           float* __restrict__ o, int64_t ld_o, float* __restrict__ lse,
                                                           const uint8_t* __restrict__ kmask,
                                                           const uint8_t* __restrict__ qmask, int BH, int H, int Lq,
                                                           int Lk, int window, float drop_p,
                                                           const uint64_t* __restrict__ seed) {
  constexpr int ND = HD < 32 ? 1 : HD / 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int nqb = (Lq + 31) / 32;
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wave);
  if (gw >= nqb * BH) return;
  const int bh = gw / nqb, qb = (gw % nqb) * 32, b = bh / H, hh = bh % H;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const int off = Lk - Lq, qi = qb + r, qpos = qi + off;
  const bool qin = qi < Lq;
  const bool qvalid = qin && (qmask == nullptr || qmask[(int64_t)b * Lq + qi] != 0);
  float qf[HD / 2];
  row_frag<HD>(qf, q + ((int64_t)b * tq + qi) * ld_in + hh * HD, qin, h);
  const float* kb = k + (int64_t)b * Lk * ld_in + hh * HD;
  const float* vb = v + (int64_t)b * Lk * ld_in + hh * HD;
  const uint8_t* kmb = kmask ? kmask + (int64_t)b * Lk : nullptr;

  f32x16 oacc[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) oacc[dt] = zero16();
  float m = -INFINITY, l = 0.f;  // running max (log2 domain) and normaliser
  const int qhi = min(Lq, qb + 32) - 1;
  const int kmax = min(Lk - 1, qhi + off);
  const int kmin = window ? max(0, qb + off - window + 1) : 0;
  // the next key tile's fragments are loaded while the current tile's MFMAs run
  float kf[HD / 2], vf[ND][16], nkf[HD / 2], nvf[ND][16];
  uint32_t kbits = 0, nbits = 0;
  auto load = [&](int kt, float (&kf_)[HD / 2], float (&vf_)[ND][16], uint32_t& bits) {
    const int kr = kt + r;
    bits = (uint32_t)__ballot(kr <= kmax && (kmb == nullptr || kmb[kr] != 0));
    row_frag<HD>(kf_, kb + (int64_t)kr * ld_in, kr <= kmax, h);
    col_frag<HD, ND>(vf_, vb, ld_in, kt, kmax, r, h);
  };
  const int kt0 = (kmin / 32) * 32;
  if (kt0 <= kmax) load(kt0, kf, vf, kbits);
  for (int kt = kt0; kt <= kmax; kt += 32) {
    if (kt + 32 <= kmax) load(kt + 32, nkf, nvf, nbits);
    if (kbits) {  // (a fully padded key tile is skipped)
      f32x16 s = zero16();  // Sᵀ[key][q]
  #pragma unroll
      for (int t = 0; t < HD / 2; ++t) s = mfma2(kf[t], qf[t], s);
      const bool full = kbits == 0xffffffffu && kt + 31 <= qb + off && (window == 0 || qhi + off - kt < window);
      float mt = -INFINITY;
  #pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (!full) {
          const int kk = acc_row(i, h);
          const bool ok = qvalid && ((kbits >> kk) & 1u) && allowed(kt + kk, qpos, window);
          s[i] = ok ? s[i] : -INFINITY;
        } else if (!qvalid) {
          s[i] = -INFINITY;
        }
        mt = fmaxf(mt, s[i]);
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64)) * kLog2e;
      const float mnew = fmaxf(m, mt);
      const float alpha = (mnew == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f(m - mnew);
      const float msub = (mnew == -INFINITY) ? 0.f : mnew;
      float rs = 0.f;
  #pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[i], kLog2e, -msub));  // exp2(-inf) = 0
        rs += p;  // the normaliser uses the undropped probabilities
        s[i] = DROP ? p * dropout_mult(dr, elem_index(bh, Lq, Lk, qi, kt + acc_row(i, h))) : p;
      }
      rs += __shfl_xor(rs, 32, 64);
      l = l * alpha + rs;
      m = mnew;
      if (__ballot(alpha != 1.f))
  #pragma unroll
        for (int dt = 0; dt < ND; ++dt)
  #pragma unroll
          for (int i = 0; i < 16; ++i) oacc[dt][i] *= alpha;
  #pragma unroll
      for (int dt = 0; dt < ND; ++dt)
  #pragma unroll
        for (int ss = 0; ss < 16; ++ss) oacc[dt] = mfma2(vf[dt][ss], s[ss], oacc[dt]);  // Oᵀ += Vᵀ·Pᵀ
    }
#pragma unroll
    for (int t = 0; t < HD / 2; ++t) kf[t] = nkf[t];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int ss = 0; ss < 16; ++ss) vf[dt][ss] = nvf[dt][ss];
    kbits = nbits;
  }
  const bool ok = qvalid && l > 0.f;
  if (qin) {
    store_rowT<HD, ND>(o + ((int64_t)b * Lq + qi) * ld_o + hh * HD, oacc, h, ok ? 1.f / l : 0.f);
    if (h == 0) lse[(int64_t)bh * Lq + qi] = ok ? m * kLn2 + logf(l) : 0.f;
  }
}

// ---- dQ and δ = rowsum(dO∘O): one wave per 32-query block -------------------------------------------------------
template <int HD, bool DROP>
__global__ __launch_bounds__(256) void attn_dq_f32_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v, int64_t ld_in, int64_t tq,
    const float* __restrict__ o, int64_t ld_o, const float* __restrict__ dout, int64_t ld_do,
    const float* __restrict__ lse, const uint8_t* __restrict__ kmask, const uint8_t* __restrict__ qmask,
    float* __restrict__ dq, int64_t ld_d, float* __restrict__ delta, int BH, int H, int Lq, int Lk, int window,
    float drop_p, const uint64_t* __restrict__ seed) {
  constexpr int ND = HD < 32 ? 1 : HD / 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int nqb = (Lq + 31) / 32;
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wave);
  if (gw >= nqb * BH) return;
  const int bh = gw / nqb, qb = (gw % nqb) * 32, b = bh / H, hh = bh % H;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const int off = Lk - Lq, qi = qb + r, qpos = qi + off;
  const bool qin = qi < Lq;
  const bool qvalid = qin && (qmask == nullptr || qmask[(int64_t)b * Lq + qi] != 0);
  float qf[HD / 2], df[HD / 2];
  row_frag<HD>(qf, q + ((int64_t)b * tq + qi) * ld_in + hh * HD, qin, h);
  row_frag<HD>(df, dout + ((int64_t)b * Lq + qi) * ld_do + hh * HD, qin, h);
  // δ = rowsum(dO∘O) as the diagonal of O·dOᵀ on the same MFMA sequence as dPᵀ = V·dOᵀ below (same B operand,
  // same k order): when a query sees one key (P = 1, O = V exactly) dP − δ cancels exactly, as in the reference's
  // softmax backward, instead of leaving f32 rounding noise in dS
  float dl = 0.f;
  {
    float of[HD / 2];
    row_frag<HD>(of, o + ((int64_t)b * Lq + qi) * ld_o + hh * HD, qin, h);
    f32x16 od = zero16();
#pragma unroll
    for (int t = 0; t < HD / 2; ++t) od = mfma2(of[t], df[t], od);
    // C[q_i][q_r] sits in lane (r, h) register i with acc_row(i, h) = r: h = (r >> 2) & 1, i = (r & 3) + 4 (r >> 3)
    const int hr = (r >> 2) & 1, ir = (r & 3) + 4 * (r >> 3);
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) v = (i == ir) ? od[i] : v;
    v = (h == hr) ? v : 0.f;
    dl = v + __shfl_xor(v, 32, 64);
  }
  if (!qvalid) dl = 0.f;
  if (qin && h == 0) delta[(int64_t)bh * Lq + qi] = dl;
  const float ls2 = qin ? lse[(int64_t)bh * Lq + qi] * kLog2e : 0.f;
  const float* kb = k + (int64_t)b * Lk * ld_in + hh * HD;
  const float* vb = v + (int64_t)b * Lk * ld_in + hh * HD;
  const uint8_t* kmb = kmask ? kmask + (int64_t)b * Lk : nullptr;

  f32x16 acc[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) acc[dt] = zero16();
  const int qhi = min(Lq, qb + 32) - 1;
  const int kmax = min(Lk - 1, qhi + off);
  const int kmin = window ? max(0, qb + off - window + 1) : 0;
  float kf[HD / 2], vf[HD / 2], kc[ND][16], nkf[HD / 2], nvf[HD / 2], nkc[ND][16];
  uint32_t kbits = 0, nbits = 0;
  auto load = [&](int kt, float (&kf_)[HD / 2], float (&vf_)[HD / 2], float (&kc_)[ND][16], uint32_t& bits) {
    const int kr = kt + r;
    bits = (uint32_t)__ballot(kr <= kmax && (kmb == nullptr || kmb[kr] != 0));
    row_frag<HD>(kf_, kb + (int64_t)kr * ld_in, kr <= kmax, h);
    row_frag<HD>(vf_, vb + (int64_t)kr * ld_in, kr <= kmax, h);
    col_frag<HD, ND>(kc_, kb, ld_in, kt, kmax, r, h);
  };
  const int kt0 = (kmin / 32) * 32;
  if (kt0 <= kmax) load(kt0, kf, vf, kc, kbits);
  for (int kt = kt0; kt <= kmax; kt += 32) {
    if (kt + 32 <= kmax) load(kt + 32, nkf, nvf, nkc, nbits);
    if (kbits) {
      f32x16 s = zero16(), dp = zero16();  // Sᵀ, dPᵀ [key][q]
  #pragma unroll
      for (int t = 0; t < HD / 2; ++t) s = mfma2(kf[t], qf[t], s);
  #pragma unroll
      for (int t = 0; t < HD / 2; ++t) dp = mfma2(vf[t], df[t], dp);
  #pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kk = acc_row(i, h);
        const bool ok = qvalid && ((kbits >> kk) & 1u) && allowed(kt + kk, qpos, window);
        const float p = ok ? __builtin_amdgcn_exp2f(fmaf(s[i], kLog2e, -ls2)) : 0.f;
        const float z = DROP ? dropout_mult(dr, elem_index(bh, Lq, Lk, qi, kt + kk)) : 1.f;
        s[i] = p * (dp[i] * z - dl);  // dSᵀ
      }
  #pragma unroll
      for (int dt = 0; dt < ND; ++dt)
  #pragma unroll
        for (int ss = 0; ss < 16; ++ss) acc[dt] = mfma2(kc[dt][ss], s[ss], acc[dt]);  // dQᵀ += Kᵀ·dSᵀ
    }
#pragma unroll
    for (int t = 0; t < HD / 2; ++t) kf[t] = nkf[t], vf[t] = nvf[t];
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int ss = 0; ss < 16; ++ss) kc[dt][ss] = nkc[dt][ss];
    kbits = nbits;
  }
  if (qin) store_rowT<HD, ND>(dq + ((int64_t)b * tq + qi) * ld_d + hh * HD, acc, h, 1.f);
}

// ---- dK, dV: one wave per 32-key block -------------------------------------------------------------------------
template <int HD, bool DROP>
__global__ __launch_bounds__(256) void attn_dkv_f32_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v, int64_t ld_in, int64_t tq,
    const float* __restrict__ dout, int64_t ld_do, const float* __restrict__ lse, const float* __restrict__ delta,
    const uint8_t* __restrict__ kmask, const uint8_t* __restrict__ qmask, float* __restrict__ dk,
    float* __restrict__ dv, int64_t ld_d, int BH, int H, int Lq, int Lk, int window, float drop_p,
    const uint64_t* __restrict__ seed) {
  constexpr int ND = HD < 32 ? 1 : HD / 32;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int nkb = (Lk + 31) / 32;
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wave);
  if (gw >= nkb * BH) return;
  const int bh = gw / nkb, kb0 = (gw % nkb) * 32, b = bh / H, hh = bh % H;
  const DropoutSpec dr = make_dropout(drop_p, seed);
  const int off = Lk - Lq, kj = kb0 + r;
  const bool kin = kj < Lk;
  const bool kvalid = kin && (kmask == nullptr || kmask[(int64_t)b * Lk + kj] != 0);
  float kf[HD / 2], vf[HD / 2];
  row_frag<HD>(kf, k + ((int64_t)b * Lk + kj) * ld_in + hh * HD, kin, h);
  row_frag<HD>(vf, v + ((int64_t)b * Lk + kj) * ld_in + hh * HD, kin, h);
  const float* qbase = q + (int64_t)b * tq * ld_in + hh * HD;
  const float* dbase = dout + (int64_t)b * Lq * ld_do + hh * HD;
  const float* lrow = lse + (int64_t)bh * Lq;
  const float* drow = delta + (int64_t)bh * Lq;
  const uint8_t* qmb = qmask ? qmask + (int64_t)b * Lq : nullptr;

  f32x16 dka[ND], dva[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) dka[dt] = zero16(), dva[dt] = zero16();
  // queries whose position i + off lies in [kb0, kb0 + 31 + window - 1] (local) or [kb0, Lk - 1] (global)
  const int ilo = max(0, kb0 - off);
  const int ihi = window ? min(Lq - 1, kb0 + 31 + window - 1 - off) : Lq - 1;
  if (__ballot(kvalid)) {
    for (int qt = (ilo / 32) * 32; qt <= ihi; qt += 32) {
      const int qr = qt + r;
      float qa[HD / 2], da[HD / 2];
      row_frag<HD>(qa, qbase + (int64_t)qr * ld_in, qr <= ihi, h);
      row_frag<HD>(da, dbase + (int64_t)qr * ld_do, qr <= ihi, h);
      float ls2[16], dl[16];
      bool qok[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qrow = qt + acc_row(i, h);
        const bool in = qrow <= ihi;
        ls2[i] = in ? lrow[qrow] * kLog2e : 0.f;
        dl[i] = in ? drow[qrow] : 0.f;
        qok[i] = in && (qmb == nullptr || qmb[qrow] != 0);
      }
      f32x16 s = zero16(), dp = zero16();  // S, dP [q][key]
#pragma unroll
      for (int t = 0; t < HD / 2; ++t) s = mfma2(qa[t], kf[t], s);
#pragma unroll
      for (int t = 0; t < HD / 2; ++t) dp = mfma2(da[t], vf[t], dp);
      float qc[ND][16], dc[ND][16];
      col_frag<HD, ND>(qc, qbase, ld_in, qt, ihi, r, h);
      col_frag<HD, ND>(dc, dbase, ld_do, qt, ihi, r, h);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qrow = qt + acc_row(i, h);
        const bool ok = kvalid && qok[i] && allowed(kj, qrow + off, window);
        const float p = ok ? __builtin_amdgcn_exp2f(fmaf(s[i], kLog2e, -ls2[i])) : 0.f;
        const float z = DROP ? dropout_mult(dr, elem_index(bh, Lq, Lk, qrow, kj)) : 1.f;
        s[i] = p * z;                   // P∘Z
        dp[i] = p * (dp[i] * z - dl[i]);  // dS
      }
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int ss = 0; ss < 16; ++ss) {
          dva[dt] = mfma2(dc[dt][ss], s[ss], dva[dt]);   // dVᵀ += dOᵀ·(P∘Z)
          dka[dt] = mfma2(qc[dt][ss], dp[ss], dka[dt]);  // dKᵀ += Qᵀ·dS
        }
    }
  }
  if (kin) {
    store_rowT<HD, ND>(dk + ((int64_t)b * Lk + kj) * ld_d + hh * HD, dka, h, 1.f);
    store_rowT<HD, ND>(dv + ((int64_t)b * Lk + kj) * ld_d + hh * HD, dva, h, 1.f);
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

bool esgpt_attn_f32_mfma_supported(int64_t hd, int64_t Lq, int64_t Lk, int64_t ld_in, int64_t ld_o) {
  if (!(hd == 16 || hd == 32 || hd == 64 || hd == 128)) return false;
  if (Lk <= 16 || Lk >= (1ll << 30) || Lq >= (1ll << 30)) return false;  // short sequences: the SMALL kernels
  return ld_in % 4 == 0 && ld_o % 4 == 0;
}

int esgpt_attn_fwd_f32_mfma(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, void* o,
                            int64_t ld_o, float* lse, const uint8_t* kmask, const uint8_t* qmask, int64_t B, int64_t H,
                            int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed,
                            hipStream_t st) {
  if (!aligned16(q) || !aligned16(k) || !aligned16(v) || !aligned16(o)) return ESGPT_ERR_UNSUPPORTED;
  const int64_t waves = cdiv(Lq, 32) * B * H;
  if (waves >= (1ll << 31)) return ESGPT_ERR_UNSUPPORTED;
  const dim3 grid((unsigned)cdiv(waves, 4)), block(256);
#define FWD(HD, DR)                                                                                                 \
  attn_fwd_f32_kernel<HD, DR><<<grid, block, 0, st>>>((const float*)q, (const float*)k, (const float*)v, ld_in, tq, \
                                                      (float*)o, ld_o, lse, kmask, qmask, (int)(B * H), (int)H,     \
                                                      (int)Lq, (int)Lk, (int)window, drop_p, seed)
#define FWD_HD(HD)               \
  do {                           \
    if (drop_p > 0.f) FWD(HD, true); \
    else FWD(HD, false);          \
  } while (0)
  if (hd == 16) FWD_HD(16);
  else if (hd == 32) FWD_HD(32);
  else if (hd == 64) FWD_HD(64);
  else FWD_HD(128);
#undef FWD_HD
#undef FWD
  return hipGetLastError() == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
}

int esgpt_attn_bwd_f32_mfma(const void* q, const void* k, const void* v, int64_t ld_in, int64_t tq, const void* o,
                            int64_t ld_o, const void* dout, int64_t ld_do, const float* lse, const uint8_t* kmask,
                            const uint8_t* qmask, void* dq, void* dk, void* dv, int64_t ld_d, int64_t B, int64_t H,
                            int64_t Lq, int64_t Lk, int64_t hd, int64_t window, float drop_p, const uint64_t* seed,
                            float* delta, hipStream_t st) {
  if (!aligned16(q) || !aligned16(k) || !aligned16(v) || !aligned16(o) || !aligned16(dout) || !aligned16(dq) ||
      !aligned16(dk) || !aligned16(dv) || ld_do % 4 != 0 || ld_d % 4 != 0)
    return ESGPT_ERR_UNSUPPORTED;
  const int64_t wq = cdiv(Lq, 32) * B * H, wk = cdiv(Lk, 32) * B * H;
  if (wq >= (1ll << 31) || wk >= (1ll << 31)) return ESGPT_ERR_UNSUPPORTED;
  const dim3 gq((unsigned)cdiv(wq, 4)), gk((unsigned)cdiv(wk, 4)), block(256);
#define BWD(HD, DR)                                                                                                   \
  do {                                                                                                                \
    attn_dq_f32_kernel<HD, DR><<<gq, block, 0, st>>>((const float*)q, (const float*)k, (const float*)v, ld_in, tq,     \
                                                     (const float*)o, ld_o, (const float*)dout, ld_do, lse, kmask,     \
                                                     qmask, (float*)dq, ld_d, delta, (int)(B * H), (int)H, (int)Lq,    \
                                                     (int)Lk, (int)window, drop_p, seed);                              \
    attn_dkv_f32_kernel<HD, DR><<<gk, block, 0, st>>>((const float*)q, (const float*)k, (const float*)v, ld_in, tq,    \
                                                      (const float*)dout, ld_do, lse, delta, kmask, qmask, (float*)dk, \
                                                      (float*)dv, ld_d, (int)(B * H), (int)H, (int)Lq, (int)Lk,        \
                                                      (int)window, drop_p, seed);                                      \
  } while (0)
#define BWD_HD(HD)                    \
  do {                                \
    if (drop_p > 0.f) BWD(HD, true);  \
    else BWD(HD, false);              \
  } while (0)
  if (hd == 16) BWD_HD(16);
  else if (hd == 32) BWD_HD(32);
  else if (hd == 64) BWD_HD(64);
  else BWD_HD(128);
#undef BWD_HD
#undef BWD
  return hipGetLastError() == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
}
