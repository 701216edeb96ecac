// Fused generative-output losses for gfx950.
//
// Replaces GenerativeOutputLayerBase.get_classification_outputs / get_regression_outputs / get_TTE_outputs
// (EventStream/transformer/model_output.py:1311-1721), the distribution heads (generative_layers.py:6-184) and
// the weighted_loss / safe_weighted_avg reductions (utils.py:134-234) behind ONE forward pass that also emits
// d(total loss)/d(logits), so the backward of the whole output layer is two GEMMs.
//
//   pass 1  count_kernel   one block per (subject, chunk of events): per-term masked event counts (weighted_loss
//                          denominators) and observed-TTE counts, as per-chunk integer partials
//   pass 2  event kernels  one wave per (subject, logit row): every term's per-event loss and logit gradient,
//                          scaled by 1 / (count[b,t] * subjects_with_events[t]); contributions stored (per row, or
//                          per workgroup of rows); ValueError flag for a subject without an observed TTE
//   pass 3  reduce_kernel  one block: deterministic sums of the contributions -> per-term losses, -TTE_LL, total
//
// HBM traffic per logit row: read C logits + write C gradients (+ the event's M entries); HBM-bound.
#include "common.h"

#include <algorithm>
#include <vector>

using namespace esgpt;

namespace {

constexpr int kWaves = 4;
constexpr int kMaxM = 64;
constexpr int kMaxK = 64;  // LNM components


constexpr float kHalfLog2Pi = 0.91893853320467274178f;
constexpr float kTiny = 1.17549435e-38f;  // torch.finfo(torch.float32).tiny

__device__ __forceinline__ float softplus(float x) {  // log(1 + exp(x)), stable
  return fmaxf(x, 0.f) + log1pf(expf(-fabsf(x)));
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float bce_logits(float x, float y) {  // BCEWithLogits, reduction none
  return fmaxf(x, 0.f) - x * y + log1pf(expf(-fabsf(x)));
}
__device__ __forceinline__ float elu1(float z) { return (z > 0.f ? z : expm1f(z)) + 1.f + kTiny; }
__device__ __forceinline__ float delu(float z) { return z > 0.f ? 1.f : expf(z); }

struct Terms {
  esgpt_loss_term t[ESGPT_MAX_TERMS];
  int n;
};

__device__ __forceinline__ int64_t readlane64(int64_t x, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)x, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// ------------------------------------------------------------------------------------------------------------
// Pass 1: one workgroup per (chunk of E events, subject). The chunk's E·M entries are read once, coalesced
// (thread = entry, 4 per thread, loads in flight together), and each entry ORs the bit of every non-MULTI
// term it satisfies into its event's LDS word (SINGLE: measurement present; MVREG / UVREG: measurement with a
// value); then thread = event: term t counts the event when it is an event and (MULTI or bit t set); TTE counts
// events followed by an event. Integer adds: exact, order-free. partial: int32 [B][n_chunks][MAX_TERMS + 1].
// Dynamic LDS: E words.
// The term bits an entry sets depend only on its measurement index (and its value mask): per-index masks built once
// per workgroup in LDS (kLut indices; larger indices take the per-term scan).
constexpr int kLut = 256;
__global__ __launch_bounds__(1024) void count_kernel(esgpt_batch bt, Terms terms, int E, int32_t* __restrict__ partial) {
  extern __shared__ uint32_t s_bits[];
  __shared__ int32_t s_cnt[ESGPT_MAX_TERMS + 1];
  __shared__ uint32_t s_lut_any[kLut], s_lut_val[kLut];
  const int64_t b = blockIdx.y;
  const int ch = blockIdx.x, n_ch = gridDim.x;
  const int T = terms.n;
  const int64_t L = bt.L, M = bt.M;
  const int l0 = ch * E, ne = (int)min((int64_t)E, L - l0);
  if (threadIdx.x <= T) s_cnt[threadIdx.x] = 0;
  for (int l = threadIdx.x; l < ne; l += blockDim.x) s_bits[l] = 0u;
  for (int i = threadIdx.x; i < kLut; i += blockDim.x) s_lut_any[i] = s_lut_val[i] = 0u;
  __syncthreads();
  if (threadIdx.x < T) {
    const esgpt_loss_term& tm = terms.t[threadIdx.x];
    if (tm.kind != ESGPT_TERM_MULTI && tm.meas_idx >= 0 && tm.meas_idx < kLut)
      atomicOr(tm.kind == ESGPT_TERM_SINGLE ? &s_lut_any[tm.meas_idx] : &s_lut_val[tm.meas_idx], 1u << threadIdx.x);
  }
  __syncthreads();
  // this thread's event flags (thread = event in the counting pass below), loaded before the entries so their
  // latency overlaps the entry pass instead of following it
  const uint8_t* em = bt.event_mask + b * L;
  bool ev0 = false, evn0 = false;
  if ((int)threadIdx.x < ne) {
    const int64_t lg = l0 + threadIdx.x;
    ev0 = em[lg] != 0;
    evn0 = lg + 1 < L && em[lg + 1] != 0;
  }
  const int64_t base = (b * L + l0) * M;
  const int64_t* meas = bt.dyn_meas + base;
  const uint8_t* vmask = bt.dyn_vmask + base;
  const int NE = ne * (int)M, Mi = (int)M;  // 32-bit index math (L * M < 2^31, checked on the host)
  constexpr int kU = 4;
  const int stride = (int)blockDim.x;
  for (int i0 = threadIdx.x; i0 < NE; i0 += kU * stride) {
    int64_t mi[kU];
    uint8_t vb[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const int i = min(i0 + k * stride, NE - 1);
      mi[k] = meas[i];
      vb[k] = vmask[i];
    }
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const int i = i0 + k * stride;
      uint32_t bits = 0u;
      if (mi[k] >= 0 && mi[k] < kLut) {
        bits = s_lut_any[mi[k]] | (vb[k] != 0 ? s_lut_val[mi[k]] : 0u);
      } else {
        for (int t = 0; t < T; ++t) {
          const esgpt_loss_term& tm = terms.t[t];
          if (tm.kind != ESGPT_TERM_MULTI && mi[k] == tm.meas_idx && (tm.kind == ESGPT_TERM_SINGLE || vb[k] != 0))
            bits |= 1u << t;
        }
      }
      if (i < NE && bits) atomicOr(&s_bits[i / Mi], bits);
    }
  }
  __syncthreads();
  int32_t c[ESGPT_MAX_TERMS + 1];
#pragma unroll
  for (int t = 0; t <= ESGPT_MAX_TERMS; ++t) c[t] = 0;
  for (int l = threadIdx.x; l < ne; l += blockDim.x) {
    const int64_t lg = l0 + l;
    const bool first = l == (int)threadIdx.x;
    const bool ev = first ? ev0 : em[lg] != 0;
    const uint32_t bits = s_bits[l];
#pragma unroll
    for (int t = 0; t < ESGPT_MAX_TERMS; ++t)
      if (t < T && ev && (terms.t[t].kind == ESGPT_TERM_MULTI || ((bits >> t) & 1u))) ++c[t];
    if (ev && (first ? evn0 : (lg + 1 < L && em[lg + 1] != 0))) ++c[ESGPT_MAX_TERMS];
  }
#pragma unroll
  for (int t = 0; t <= ESGPT_MAX_TERMS; ++t) {
    const int v = (int)wave_sum((float)c[t]);  // < 2^24 events per chunk: exact in f32
    const int slot = t < ESGPT_MAX_TERMS ? t : T;
    if ((t < T || t == ESGPT_MAX_TERMS) && lane_id() == 0 && v) atomicAdd(&s_cnt[slot], v);
  }
  __syncthreads();
  if (threadIdx.x <= T) partial[(b * n_ch + ch) * (ESGPT_MAX_TERMS + 1) + threadIdx.x] = s_cnt[threadIdx.x];
}

// ------------------------------------------------------------------------------------------------------------
// Per-term math shared by both event kernels. `z(col)` reads a logit of the term's row (f32), `put(col, g)` adds
// g to that column's gradient. Every lane of the wave calls these (wave-uniform control flow); returns the
// wave-uniform per-event loss ell of the term. Entry registers: lane m < M holds entry m (e_idx, e_val, e_vm,
// match = entry belongs to the term's measurement); mm / mv = ballots of match / match && value-present.
template <typename ZF, typename GF>
__device__ __forceinline__ float content_term(const esgpt_loss_term& tm, int lane, int64_t M, bool match,
                                              uint64_t mm, uint64_t mv, int64_t e_idx, float e_val, bool e_vm,
                                              bool mk, float scale, int32_t* err, ZF z, GF put) {
  float ell = 0.f;
  if (tm.kind == ESGPT_TERM_SINGLE) {
    const int n = tm.vocab_end - tm.vocab_start;
    int64_t lab = 0;
    const bool has = mm != 0;
    for (uint64_t bits = mm; bits; bits &= bits - 1) lab += readlane64(e_idx, __builtin_ctzll(bits));
    lab = has ? lab - tm.vocab_start : 0;
    if (mk && (lab < 0 || lab >= n)) {
      set_err(err, ESGPT_FLAG_BAD_LABEL);
      lab = 0;
    }
    constexpr int kR = 4;  // n <= 64·kR: the logits read once into registers (same arithmetic, same order)
    if (n <= 64 * kR) {
      float xs[kR], ex[kR];
#pragma unroll
      for (int k = 0; k < kR; ++k) xs[k] = lane + 64 * k < n ? z(tm.col + lane + 64 * k) : -INFINITY;
      const float xl = z(tm.col + lab);
      const float zo = z(tm.obs_col);
      float mx = -INFINITY;
#pragma unroll
      for (int k = 0; k < kR; ++k)
        if (lane + 64 * k < n) mx = fmaxf(mx, xs[k]);
      mx = wave_max(mx);
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < kR; ++k) {
        ex[k] = lane + 64 * k < n ? expf(xs[k] - mx) : 0.f;
        if (lane + 64 * k < n) se += ex[k];
      }
      se = wave_sum(se);
      const float lse = mx + logf(se);
      ell = (lse - xl) + bce_logits(zo, has ? 1.f : 0.f);
      if (scale != 0.f) {
        const float inv = 1.f / se;
#pragma unroll
        for (int k = 0; k < kR; ++k) {
          const int j = lane + 64 * k;
          if (j < n) put(tm.col + j, scale * (ex[k] * inv - (j == lab ? 1.f : 0.f)));
        }
        if (lane == 0) put(tm.obs_col, scale * (sigmoidf_(zo) - (has ? 1.f : 0.f)));
      }
      return ell;
    }
    float mx = -INFINITY;
    for (int j = lane; j < n; j += 64) mx = fmaxf(mx, z(tm.col + j));
    mx = wave_max(mx);
    float se = 0.f;
    for (int j = lane; j < n; j += 64) se += expf(z(tm.col + j) - mx);
    se = wave_sum(se);
    const float lse = mx + logf(se);
    const float xl = z(tm.col + lab);
    const float zo = z(tm.obs_col);
    ell = (lse - xl) + bce_logits(zo, has ? 1.f : 0.f);
    if (scale != 0.f) {
      const float inv = 1.f / se;
      for (int j = lane; j < n; j += 64) {
        const float pj = expf(z(tm.col + j) - mx) * inv;
        put(tm.col + j, scale * (pj - (j == lab ? 1.f : 0.f)));
      }
      if (lane == 0) put(tm.obs_col, scale * (sigmoidf_(zo) - (has ? 1.f : 0.f)));
    }
  } else if (tm.kind == ESGPT_TERM_MULTI) {
    const int n = tm.vocab_end - tm.vocab_start;
    // lane m < M holds entry m's label within this term (-1: another measurement); labels are broadcast
    // with readlane (wave-uniform m) instead of re-reading the staged entries per column
    const int my_lab = match ? (int)(e_idx - tm.vocab_start) : -1;
    float acc = 0.f;
    // passes of kPass column groups: the pass's logits are read before any gradient is written
    constexpr int kPass = 16;
    for (int j1 = 0; j1 < n; j1 += 64 * kPass) {
      float xs[kPass];
#pragma unroll
      for (int it = 0; it < kPass; ++it) {
        const int j = j1 + 64 * it + lane;
        xs[it] = j < n ? z(tm.col + j) : 0.f;
      }
      // multi-hot labels of this pass group: each of the M entries marks the (column group, lane) holding its
      // label — M readlanes per group of 64·kPass columns instead of M per column
      uint32_t ymask = 0;
      for (int m = 0; m < M; ++m) {
        const int rel = __builtin_amdgcn_readlane(my_lab, m) - j1;  // my_lab = -1: not this term's entry
        if (rel >= 0 && rel < 64 * kPass && (rel & 63) == lane) ymask |= 1u << (rel >> 6);
      }
#pragma unroll
      for (int it = 0; it < kPass; ++it) {
        const int j = j1 + 64 * it + lane;
        if (j1 + 64 * it >= n) break;  // wave-uniform
        const bool y = (ymask >> it) & 1u;
        if (j < n) {
          // BCE-with-logits and its gradient from ONE exp2 / log2 / rcp (v_exp_f32, v_log_f32, v_rcp_f32):
          // e = exp(-|x|), loss = max(x, 0) - x·y + log(1 + e), sigmoid(x) = x >= 0 ? 1/(1+e) : e/(1+e)
          const float x = xs[it], yf = y ? 1.f : 0.f;
          const float e = __builtin_amdgcn_exp2f(-fabsf(x) * 1.4426950408889634f);
          const float ope = 1.f + e;
          acc += fmaxf(x, 0.f) - x * yf + __builtin_amdgcn_logf(ope) * 0.6931471805599453f;
          if (scale != 0.f) {
            const float inv = __builtin_amdgcn_rcpf(ope);
            put(tm.col + j, scale / (float)n * ((x >= 0.f ? inv : e * inv) - yf));
          }
        }
      }
    }
    ell = wave_sum(acc) / (float)n;
  } else if (tm.kind == ESGPT_TERM_MVREG) {
    // lanes 0..M-1: one entry each; duplicates of a target index accumulate into one gradient pair.
    const int n_targets = tm.vocab_end - tm.vocab_start;
    const bool sel = match && e_vm;
    int64_t j = 0;
    float nll = 0.f, gmu = 0.f, grho = 0.f;
    if (sel) {
      j = e_idx - tm.vocab_start;
      if (j < 0 || j >= n_targets) {
        set_err(err, ESGPT_FLAG_BAD_LABEL);
        j = 0;
      }
      const float mu = z(tm.col + 2 * j);
      const float rho = z(tm.col + 2 * j + 1);
      const float sd = elu1(rho);
      const float x = e_val;
      const float zz = (x - mu) / sd;
      nll = 0.5f * zz * zz + logf(sd) + kHalfLog2Pi;
      gmu = -(x - mu) / (sd * sd);
      grho = (1.f / sd - (x - mu) * (x - mu) / (sd * sd * sd)) * delu(rho);
    }
    const float nsel = (float)__popcll(mv);
    ell = nsel > 0.f ? wave_sum(nll) / nsel : 0.f;
    if (scale != 0.f && nsel > 0.f) {
      const float s2 = scale / nsel;
      // combine duplicate targets: the first lane of each target sums its group, then writes once
      float sm = 0.f, sr = 0.f;
      bool first = sel;
      for (uint64_t bits = mv; bits; bits &= bits - 1) {  // the selected entries, in lane order
        const int m = __builtin_ctzll(bits);
        const int64_t jm = readlane64(j, m);
        const float gm = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gmu), m));
        const float gr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(grho), m));
        if (sel && jm == j) {
          sm += gm;
          sr += gr;
          if (m < lane) first = false;
        }
      }
      if (first) {
        put(tm.col + 2 * j, s2 * sm);
        put(tm.col + 2 * j + 1, s2 * sr);
      }
    }
  } else if (tm.kind == ESGPT_TERM_UVREG) {
    const bool has_meas = mm != 0, has_val = mv != 0;
    float x = 0.f;
    for (uint64_t bits = mv; bits; bits &= bits - 1)
      x += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e_val), __builtin_ctzll(bits)));
    if (!has_val) x = 0.f;
    const float mu = z(tm.col);
    const float rho = z(tm.col + 1);
    const float sd = elu1(rho);
    const float zz = (x - mu) / sd;
    const float zo = z(tm.obs_col);
    ell = 0.5f * zz * zz + logf(sd) + kHalfLog2Pi + bce_logits(zo, has_meas ? 1.f : 0.f);
    if (scale != 0.f && lane == 0) {
      put(tm.col, scale * (-(x - mu) / (sd * sd)));
      put(tm.col + 1, scale * (1.f / sd - (x - mu) * (x - mu) / (sd * sd * sd)) * delu(rho));
      put(tm.obs_col, scale * (sigmoidf_(zo) - (has_meas ? 1.f : 0.f)));
    }
  }
  return ell;
}

// Time-to-event log-likelihood of one observed delta x; z(k) / put(k, g) address the TTE columns relative to
// tte.col. `scale` = d(-LL)/d ll for this event (0: no gradient). Returns ll (wave-uniform).
template <typename ZF, typename GF>
__device__ __forceinline__ float tte_term(const esgpt_tte_spec& tte, int lane, float x, float scale, ZF z, GF put) {
  float ll = 0.f;
  if (tte.kind == ESGPT_TTE_EXP) {
    const float zz = z(0);
    const float rate = elu1(zz);
    ll = logf(rate) - rate * x;
    if (lane == 0 && scale != 0.f) put(0, scale * (1.f / rate - x) * delu(zz));
  } else {
    // LogNormalMixture (third-party pytorch_lognormal_mixture, restated): lanes = components.
    const int K = tte.K;
    const bool affine = !(tte.mean_log == 0.f && tte.std_log == 1.f);
    const float lx = logf(x);
    const float y = affine ? (lx - tte.mean_log) / tte.std_log : lx;
    float loc = 0.f, ls = 0.f, lw = -INFINITY, a = -INFINITY;
    if (lane < K) {
      loc = z(3 * lane);
      ls = z(3 * lane + 1);
      lw = z(3 * lane + 2);
    }
    const float wmax = wave_max(lw);
    const float wse = wave_sum(lane < K ? expf(lw - wmax) : 0.f);
    const float lsm = lw - (wmax + logf(wse));  // log_softmax(weights)
    if (lane < K) {
      const float sd = expf(ls);
      const float zz = (y - loc) / sd;
      a = lsm - 0.5f * zz * zz - ls - kHalfLog2Pi;
    }
    const float amax = wave_max(a);
    const float ase = wave_sum(lane < K ? expf(a - amax) : 0.f);
    ll = amax + logf(ase) - lx - (affine ? logf(fabsf(tte.std_log)) : 0.f);
    if (scale != 0.f && lane < K) {
      const float resp = expf(a - amax) / ase;  // posterior responsibility
      const float pi = expf(lsm);
      const float sd = expf(ls);
      const float dz = (y - loc) / sd;
      put(3 * lane, scale * resp * dz / sd);
      put(3 * lane + 1, scale * resp * (dz * dz - 1.f));
      put(3 * lane + 2, scale * (resp - pi));
    }
  }
  return ll;
}

// Subjects-with-events per term (the outer safe_weighted_avg of weighted_loss) into s_nsub_inv; TTE averages over
// all B. Called by wave 0: lane = subject (its chunk partials summed), one ballot per term; every load of a pass
// in flight together.
__device__ __forceinline__ void subjects_with_events(const int32_t* __restrict__ partial, int64_t B, int n_ch, int NT,
                                                     int lane, float* s_nsub_inv) {
  int nsub[ESGPT_MAX_TERMS];
#pragma unroll
  for (int t = 0; t < ESGPT_MAX_TERMS; ++t) nsub[t] = 0;
  for (int64_t b0 = 0; b0 < B; b0 += 64) {
    const int64_t b = b0 + lane;
    int c[ESGPT_MAX_TERMS];
#pragma unroll
    for (int t = 0; t < ESGPT_MAX_TERMS; ++t) c[t] = 0;
    for (int ch = 0; ch < n_ch; ++ch) {
      const int32_t* row = partial + (b * n_ch + ch) * (ESGPT_MAX_TERMS + 1);
#pragma unroll
      for (int t = 0; t < ESGPT_MAX_TERMS; ++t) c[t] += (t < NT && b < B) ? row[t] : 0;
    }
#pragma unroll
    for (int t = 0; t < ESGPT_MAX_TERMS; ++t) nsub[t] += __popcll(__ballot(c[t] > 0));
  }
#pragma unroll
  for (int t = 0; t < ESGPT_MAX_TERMS; ++t)
    if (lane == t && t < NT) s_nsub_inv[t] = nsub[t] > 0 ? 1.f / (float)nsub[t] : 0.f;
  if (lane == 0) s_nsub_inv[NT] = B > 0 ? 1.f / (float)B : 0.f;
}

// Subject b's counts: lane t (<= NT) returns term t's (lane NT: observed TTEs), summed over the chunk partials.
__device__ __forceinline__ int32_t subject_counts(const int32_t* __restrict__ partial, int64_t b, int n_ch, int NT,
                                                  int lane, bool active) {
  int32_t c = 0;
  if (active && lane <= NT)
    for (int ch = 0; ch < n_ch; ++ch) c += partial[(b * n_ch + ch) * (ESGPT_MAX_TERMS + 1) + lane];
  return c;
}

// The reference raises "No observed time-to-event ..." for a subject whose TTE count is 0 (model_output.py:
// 1366-1367): flagged once per subject, by the wave of its first row.
__device__ __forceinline__ void flag_no_tte(int32_t my_cnt, int NT, bool first_row, int32_t* err) {
  if (first_row && __builtin_amdgcn_readlane(my_cnt, NT) == 0 && lane_id() == 0) set_err(err, ESGPT_FLAG_TTE_NO_OBS);
}

// The wave's logit-row coordinates: w -> subject b, unshifted row r (-1: the bias row in shift mode) and content
// target position p = r + shift.
struct RowPos {
  bool active, has_content, ev;
  int64_t b, r, p;
};
__device__ __forceinline__ RowPos row_pos(const esgpt_batch& bt, int64_t w, int64_t n_rows, int shift) {
  RowPos q;
  q.active = w < n_rows;
  // 32-bit division: a 64-bit one is a long scalar instruction sequence per wave (n_rows < 2^31, host-checked)
  const uint32_t per_b = (uint32_t)(bt.L + shift), wu = (uint32_t)w;
  const uint32_t qb = wu / per_b;
  q.b = q.active ? (int64_t)qb : 0;
  q.r = q.active ? (int64_t)(wu - qb * per_b) - shift : 0;
  q.p = q.r + shift;
  q.has_content = q.active && q.p < bt.L;
  q.ev = q.has_content && bt.event_mask[q.b * bt.L + q.p] != 0;
  return q;
}

// ------------------------------------------------------------------------------------------------------------
// Generic event kernel (any row width): one wave per (subject, logit row), logits read from and gradients written
// to global memory column by column (the gradient buffers are zero-filled first).
template <typename T, bool RMW>
__global__ __launch_bounds__(256) void event_kernel(esgpt_batch bt, Terms terms, esgpt_tte_spec tte,
                                                    const T* __restrict__ zc, int64_t ldc, int64_t n_levels, int shift,
                                                    const T* __restrict__ zc_bias, const T* __restrict__ zt,
                                                    int64_t ldt, T* __restrict__ dzc, T* __restrict__ dzt,
                                                    float* __restrict__ dbias, const int32_t* __restrict__ counts, int n_ch,
                                                    float* __restrict__ contrib, int64_t n_rows,
                                                    int32_t* __restrict__ err) {
  __shared__ float s_nsub_inv[ESGPT_MAX_TERMS + 1];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: row math in SALU
  const int lane = lane_id();
  const int NT = terms.n;
  const int64_t L = bt.L, M = bt.M;
  if (wave == 0) subjects_with_events(counts, bt.B, n_ch, NT, lane, s_nsub_inv);

  const int64_t w = (int64_t)blockIdx.x * kWaves + wave;
  const RowPos q = row_pos(bt, w, n_rows, shift);
  const int64_t b = q.b, r = q.r, p = q.p;

  // the event's M entries in registers, lane m = entry m (per-term scans are ballots / readlanes, not LDS loops)
  int64_t e_idx = 0, e_meas = INT64_MIN;
  float e_val = 0.f;
  bool e_vm = false;
  if (q.has_content && lane < M) {
    const int64_t off = (b * L + p) * M + lane;
    e_idx = bt.dyn_idx[off];
    e_meas = bt.dyn_meas[off];
    e_val = bt.dyn_vals[off];
    e_vm = bt.dyn_vmask[off] != 0;
  }
  __syncthreads();  // s_nsub_inv

  // this subject's per-term counts: lane t holds term t's (one load per lane instead of one per term)
  const int32_t my_cnt = subject_counts(counts, b, n_ch, NT, lane, q.active);
  flag_no_tte(my_cnt, NT, q.active && q.r == -shift, err);
  float* my_contrib = contrib + w;  // contrib[t * n_rows + w]

  // ---------------- content terms ----------------
  for (int t = 0; t < NT; ++t) {
    const esgpt_loss_term& tm = terms.t[t];
    float c_out = 0.f;
    if (q.has_content) {
      const T* zrow;
      T* gT = nullptr;
      float* gF = nullptr;
      if (shift) {
        if (r < 0) {
          zrow = zc_bias;
          gF = dbias + b * ldc;
        } else {
          zrow = zc + (b * L + r) * ldc;
          gT = dzc + (b * L + r) * ldc;
        }
      } else {
        const int64_t row = (b * L + p) * n_levels + tm.level;
        zrow = zc + row * ldc;
        gT = dzc + row * ldc;
      }
      const bool match = e_meas == tm.meas_idx;  // this lane's entry belongs to the term
      const uint64_t mm = __ballot(match), mv = __ballot(match && e_vm);
      const bool mk = q.ev && (tm.kind == ESGPT_TERM_MULTI ||
                               (tm.kind == ESGPT_TERM_SINGLE ? mm != 0 : mv != 0));  // term_mask, restated
      const int32_t cnt = __builtin_amdgcn_readlane(my_cnt, t);
      const float scale = (mk && cnt > 0) ? s_nsub_inv[t] / (float)cnt : 0.f;
      // Gradient columns: with disjoint term columns (checked on the host) every column of a row has exactly one
      // writer, so the zero-filled buffer is stored to without a read; otherwise read-modify-write. The bias row
      // (shift mode) is this wave's own f32 row.
      const float ell = content_term(
          tm, lane, M, match, mm, mv, e_idx, e_val, e_vm, mk, scale, err,
          [&](int64_t col) { return to_f32(zrow[col]); },
          [&](int64_t col, float g) {
            if (gF) gF[col] += g;
            else if (RMW) gT[col] = from_f32<T>(to_f32(gT[col]) + g);
            else gT[col] = from_f32<T>(g);
          });
      c_out = scale * ell;
    }
    if (q.active && lane == 0) my_contrib[(int64_t)t * n_rows] = c_out;
  }

  // ---------------- time-to-event (unshifted row r) ----------------
  float c_tte = 0.f;
  if (q.active && r >= 0) {
    const int64_t e = b * L + r;
    const bool obs = (r + 1 < L) && bt.event_mask[e] && bt.event_mask[e + 1];
    const float x = obs ? bt.time_delta[e] : 1.f;
    const T* z = zt + e * ldt + tte.col;
    T* gz = dzt + e * ldt + tte.col;
    const int32_t cnt = __builtin_amdgcn_readlane(my_cnt, NT);
    const float scale = (obs && cnt > 0) ? -s_nsub_inv[NT] / (float)cnt : 0.f;  // d(-LL)/d ll
    const float ll = tte_term(
        tte, lane, x, scale, [&](int k) { return to_f32(z[k]); },
        [&](int k, float g) { gz[k] = from_f32<T>(g); });
    if (isnan(ll)) set_err(err, ESGPT_FLAG_TTE_NAN);
    c_tte = obs ? -scale * ll : 0.f;  // = obs * ll / (B * cnt): LL contribution (positive sign)
  }
  if (q.active && lane == 0) my_contrib[(int64_t)NT * n_rows] = c_tte;
}

// ------------------------------------------------------------------------------------------------------------
// Row-staged event kernel (rows that fit in LDS): each wave stages its whole logit row in LDS with 16-B loads
// issued together (the row, the event's entries and the counts in one round trip instead of one per term), the
// terms read logits from and accumulate f32 gradients into LDS, and the complete gradient row — every column,
// zeros included — is written back with 16-B stores, so the gradient buffer needs no zero-fill pass. In NA mode
// (no shift, n_levels rows per event) the wave walks its event's level rows one after another. The TTE columns
// are part of the row when zt == zc (CI); otherwise they are written to dzt directly (zero-filled).
// LDS per wave: ldp T logits + ldp f32 gradients (ldp = ldc rounded up to 16-B chunks of T).
template <typename T>
__global__ __launch_bounds__(256) void event_lds_kernel(esgpt_batch bt, Terms terms, esgpt_tte_spec tte,
                                                        const T* __restrict__ zc, int64_t ldc, int64_t n_levels,
                                                        int shift, const T* __restrict__ zc_bias,
                                                        const T* __restrict__ zt, int64_t ldt, T* __restrict__ dzc,
                                                        T* __restrict__ dzt, float* __restrict__ dbias,
                                                        const int32_t* __restrict__ counts, int n_ch, float* __restrict__ contrib,
                                                        int64_t n_rows, int tte_in_row, int32_t* __restrict__ err) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  __shared__ float s_nsub_inv[ESGPT_MAX_TERMS + 1];
  constexpr int kEl = 16 / sizeof(T);  // elements per 16-B chunk
  const int waves = blockDim.x >> 6;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: row math in SALU
  const int lane = lane_id();
  const int NT = terms.n;
  const int64_t L = bt.L, M = bt.M;
  const int64_t nch = ldc / kEl;           // 16-B chunks per row (ldc % kEl == 0, checked on the host)
  const int64_t ldp = nch * kEl;
  T* zs = reinterpret_cast<T*>(s_dyn) + (int64_t)wave * ldp;
  float* gs = reinterpret_cast<float*>(s_dyn + (size_t)waves * ldp * sizeof(T)) + (int64_t)wave * ldp;

  if (wave == 0) subjects_with_events(counts, bt.B, n_ch, NT, lane, s_nsub_inv);
  const int64_t w = (int64_t)blockIdx.x * waves + wave;
  const RowPos q = row_pos(bt, w, n_rows, shift);
  const int64_t b = q.b, r = q.r, p = q.p;

  int64_t e_idx = 0, e_meas = INT64_MIN;
  float e_val = 0.f;
  bool e_vm = false;
  if (q.has_content && lane < M) {
    const int64_t off = (b * L + p) * M + lane;
    e_idx = bt.dyn_idx[off];
    e_meas = bt.dyn_meas[off];
    e_val = bt.dyn_vals[off];
    e_vm = bt.dyn_vmask[off] != 0;
  }
  const int32_t my_cnt = subject_counts(counts, b, n_ch, NT, lane, q.active);
  flag_no_tte(my_cnt, NT, q.active && q.r == -shift, err);
  float* my_contrib = contrib + w;
  // TTE inputs (loaded with the row)
  const bool tte_row = q.active && r >= 0;
  const int64_t e = b * L + (r < 0 ? 0 : r);
  const bool obs = tte_row && (r + 1 < L) && bt.event_mask[e] && bt.event_mask[e + 1];
  const float x_tte = obs ? bt.time_delta[e] : 1.f;

  const int n_lv = shift ? 1 : (int)n_levels;
  for (int lv = 0; lv < n_lv; ++lv) {
    // ---- stage the row: logits -> zs, gradients -> 0 ----
    const T* zrow = nullptr;
    T* grow = nullptr;
    float* frow = nullptr;
    if (q.active) {
      if (shift) {
        if (r < 0) {
          zrow = zc_bias;
          frow = dbias + b * ldc;
        } else {
          zrow = zc + (b * L + r) * ldc;
          grow = dzc + (b * L + r) * ldc;
        }
      } else {
        const int64_t row = (b * L + p) * n_levels + lv;
        zrow = zc + row * ldc;
        grow = dzc + row * ldc;
      }
    }
    if (zrow) {
      constexpr int kBatch = 8;
      for (int64_t c0 = 0; c0 < nch; c0 += 64 * kBatch) {
        // unconditional loads at clamped chunk indices: all kBatch loads in flight together, in registers
        // (conditional loads were serialised one round trip each through scratch)
        uint4 v[kBatch];
#pragma unroll
        for (int i = 0; i < kBatch; ++i) {
          const int64_t c = c0 + 64 * i + lane;
          v[i] = reinterpret_cast<const uint4*>(zrow)[c < nch ? c : nch - 1];
        }
#pragma unroll
        for (int i = 0; i < kBatch; ++i) {
          const int64_t c = c0 + 64 * i + lane;
          if (c < nch) reinterpret_cast<uint4*>(zs)[c] = v[i];
        }
      }
      for (int64_t c = lane; c < ldp / 4; c += 64) reinterpret_cast<float4*>(gs)[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();  // zs / gs staged (and s_nsub_inv on the first level)

    auto zget = [&](int64_t col) { return to_f32(zs[col]); };
    auto gput = [&](int64_t col, float g) { gs[col] += g; };
    for (int t = 0; t < NT; ++t) {
      const esgpt_loss_term& tm = terms.t[t];
      if (!shift && tm.level != lv) continue;  // wave-uniform
      float c_out = 0.f;
      if (q.has_content) {
        const bool match = e_meas == tm.meas_idx;
        const uint64_t mm = __ballot(match), mv = __ballot(match && e_vm);
        const bool mk = q.ev && (tm.kind == ESGPT_TERM_MULTI || (tm.kind == ESGPT_TERM_SINGLE ? mm != 0 : mv != 0));
        const int32_t cnt = __builtin_amdgcn_readlane(my_cnt, t);
        const float scale = (mk && cnt > 0) ? s_nsub_inv[t] / (float)cnt : 0.f;
        const float ell = content_term(tm, lane, M, match, mm, mv, e_idx, e_val, e_vm, mk, scale, err, zget, gput);
        c_out = scale * ell;
      }
      if (q.active && lane == 0) my_contrib[(int64_t)t * n_rows] = c_out;
    }
    if (tte_in_row && lv == 0) {
      float c_tte = 0.f;
      if (tte_row) {
        const int32_t cnt = __builtin_amdgcn_readlane(my_cnt, NT);
        const float scale = (obs && cnt > 0) ? -s_nsub_inv[NT] / (float)cnt : 0.f;
        const float ll = tte_term(
            tte, lane, x_tte, scale, [&](int k) { return to_f32(zs[tte.col + k]); },
            [&](int k, float g) { gs[tte.col + k] += g; });
        if (isnan(ll)) set_err(err, ESGPT_FLAG_TTE_NAN);
        c_tte = obs ? -scale * ll : 0.f;
      }
      if (q.active && lane == 0) my_contrib[(int64_t)NT * n_rows] = c_tte;
    }
    __syncthreads();  // every lane's gradient columns in gs

    // ---- write the whole gradient row ----
    if (frow) {
      for (int64_t c = lane; c < ldp / 4; c += 64)
        reinterpret_cast<float4*>(frow)[c] = reinterpret_cast<const float4*>(gs)[c];
    } else if (grow) {
      for (int64_t c = lane; c < nch; c += 64) {
        uint4 o;
        if constexpr (sizeof(T) == 4) {
          o = reinterpret_cast<const uint4*>(gs)[c];
        } else {
          const float4 a0 = reinterpret_cast<const float4*>(gs)[2 * c];
          const float4 a1 = reinterpret_cast<const float4*>(gs)[2 * c + 1];
          o.x = (uint32_t)f32_to_bf16_bits(a0.x) | ((uint32_t)f32_to_bf16_bits(a0.y) << 16);
          o.y = (uint32_t)f32_to_bf16_bits(a0.z) | ((uint32_t)f32_to_bf16_bits(a0.w) << 16);
          o.z = (uint32_t)f32_to_bf16_bits(a1.x) | ((uint32_t)f32_to_bf16_bits(a1.y) << 16);
          o.w = (uint32_t)f32_to_bf16_bits(a1.z) | ((uint32_t)f32_to_bf16_bits(a1.w) << 16);
        }
        reinterpret_cast<uint4*>(grow)[c] = o;
      }
    }
    if (lv + 1 < n_lv) __syncthreads();  // zs / gs reused by the next level
  }

  // ---- time-to-event into a separate dzt (NA) ----
  if (!tte_in_row) {
    float c_tte = 0.f;
    if (tte_row) {
      const T* z = zt + e * ldt + tte.col;
      T* gz = dzt + e * ldt + tte.col;
      const int32_t cnt = __builtin_amdgcn_readlane(my_cnt, NT);
      const float scale = (obs && cnt > 0) ? -s_nsub_inv[NT] / (float)cnt : 0.f;
      const float ll = tte_term(
          tte, lane, x_tte, scale, [&](int k) { return to_f32(z[k]); },
          [&](int k, float g) { gz[k] = from_f32<T>(g); });
      if (isnan(ll)) set_err(err, ESGPT_FLAG_TTE_NAN);
      c_tte = obs ? -scale * ll : 0.f;
    }
    if (q.active && lane == 0) my_contrib[(int64_t)NT * n_rows] = c_tte;
  }
}

// ------------------------------------------------------------------------------------------------------------
// Deterministic sums of the per-row (or per-workgroup) contributions by one workgroup of NTh threads: thread i sums
// items i, i + NTh, ... of each term, then wave sums and a fixed-order sum over the waves. The next term's loads are
// issued before the current term is summed (one memory round trip per pass instead of one per term).
template <int NTh>
__device__ __forceinline__ void reduce_contrib(const float* __restrict__ contrib, int64_t n_rows, int NT,
                                               float* __restrict__ losses) {
  constexpr int NW = NTh / 64;
  __shared__ float s[NW][ESGPT_MAX_TERMS + 1];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int kU = 8;  // items per thread and pass
  for (int64_t i0 = 0; i0 < n_rows; i0 += kU * NTh) {
    float cur[kU], nxt[kU];
    auto load = [&](float (&v)[kU], int t) {
      const float* c = contrib + (int64_t)min(t, NT) * n_rows;
#pragma unroll
      for (int k = 0; k < kU; ++k) {
        const int64_t i = i0 + threadIdx.x + (int64_t)k * NTh;
        const float x = c[min(i, n_rows - 1)];
        v[k] = i < n_rows ? x : 0.f;
      }
    };
    load(cur, 0);
    for (int t = 0; t <= NT; ++t) {
      load(nxt, t + 1);  // clamped past the last term: a re-read, never used
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < kU; ++k) a += cur[k];
      const float w = wave_sum(a);
      if (lane == 0) s[wave][t] = (i0 == 0 ? 0.f : s[wave][t]) + w;
#pragma unroll
      for (int k = 0; k < kU; ++k) cur[k] = nxt[k];
    }
  }
  __syncthreads();
  // wave 0: lane t sums term t over the waves (the fixed order), then the total in term order from readlanes (no
  // serial chain of LDS reads in one thread)
  if (wave == 0) {
    float v = 0.f;
    if (lane <= NT) {
      for (int w = 0; w < NW; ++w) v += s[w][lane];
      v = (lane < NT) ? v : -v;  // last slot: -TTE_LL
      losses[lane] = v;
    }
    float total = 0.f;
    for (int t = 0; t <= NT; ++t) total += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), t));
    if (lane == 0) losses[NT + 1] = total;
  }
}

// ------------------------------------------------------------------------------------------------------------
// Streaming event kernel (the default): one wave per logit row and no whole-row staging, so occupancy is set by
// registers, not by the row width — the row-staged kernel holds ldc·(s + 4) B of LDS per wave, which at C5
// (ldc = 10,640) left ONE wave per workgroup and two per CU.
//
// Column classes of a row (host plan, per level):
//   dense   MULTI ranges [col, col+n): scale/n · (sigmoid(x) - y), y from the multi-hot labels (the event's entries)
//   narrow  the 16-B chunks touching a SINGLE slice or any is-observed / regression / (in-row) TTE column: at most
//           max_narrow<T>() chunks, staged in the wave's LDS slice (logits + f32 gradients)
//   other   0
// Pass 1 streams the row once in 16-B chunks (kEl elements per lane, 64·kEl columns per wave instruction, kB chunk
// groups in flight): dense gradients, MULTI BCE sums, zeros; chunks of the narrow set go to LDS (logits, and their
// MULTI / zero gradients) instead of HBM. Pass 2 computes the narrow terms (SINGLE softmax-CE + is-observed BCE,
// Gaussian NLLs, TTE) from LDS — no dependent global round trips — and stores the narrow chunks. Per row: ldc·s
// logits read + ldc·s gradients written, plus the event's entries. Same per-element formulas as content_term /
// tte_term: gradients are bitwise those of the other two kernels; MULTI losses are summed in another order.
constexpr int kMaxSeg = 4;       // MULTI ranges per level
constexpr int kMaxRng = 8;       // narrow chunk ranges per level
// narrow chunks per level: <= 4.5 KiB of LDS per wave (16 B of logits + kEl f32 gradients per chunk)
template <typename T>
constexpr int max_narrow() { return sizeof(T) == 4 ? 128 : 96; }
constexpr int kMaxLevels = 8;
constexpr int kMap = 1, kSkipP1 = 2, kSkipP2 = 4, kSkipSub = 8, kSkipTte = 16, kSkipStore = 32, kTot = 64;

struct StreamPlan {
  int8_t nseg[kMaxLevels];             // MULTI terms of the level, in term order
  int8_t seg[kMaxLevels][kMaxSeg];
  int8_t nrng[kMaxLevels];             // narrow chunk ranges [lo, hi) of the level; slot = base + c - lo
  int32_t lo[kMaxLevels][kMaxRng], hi[kMaxLevels][kMaxRng], base[kMaxLevels][kMaxRng];
  int32_t max_slots;                   // narrow chunks of the widest level
  // LDS element index of narrow column col = col + delta (a term's columns lie in one merged range): per term
  // (its value columns, its is-observed column) and for the in-row TTE columns
  int32_t dcol[ESGPT_MAX_TERMS], dobs[ESGPT_MAX_TERMS], dtte;
};

template <typename T>
__device__ __forceinline__ void unpack_chunk(const uint4& v, float (&x)[16 / sizeof(T)]) {
  if constexpr (sizeof(T) == 4) {
    x[0] = __uint_as_float(v.x), x[1] = __uint_as_float(v.y), x[2] = __uint_as_float(v.z), x[3] = __uint_as_float(v.w);
  } else {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[2 * i] = __uint_as_float(w[i] << 16);
      x[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
}

template <typename T>
__device__ __forceinline__ uint4 pack_chunk(const float (&o)[16 / sizeof(T)]) {
  if constexpr (sizeof(T) == 4) {
    return make_uint4(__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]), __float_as_uint(o[3]));
  } else {
    uint32_t wd[4];
#pragma unroll
    for (int h = 0; h < 4; ++h)
      wd[h] = (uint32_t)f32_to_bf16_bits(o[2 * h]) | ((uint32_t)f32_to_bf16_bits(o[2 * h + 1]) << 16);
    return make_uint4(wd[0], wd[1], wd[2], wd[3]);
  }
}

template <typename T>
// f32 logits: six waves per SIMD (80 VGPRs; measured 53.7 -> 53.0 us at C2; eight spill to scratch). bf16 logits:
// five (at six the bf16 instance spills 48 B/lane to scratch — 25 MB of scratch stores per C2 step)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 4 ? 6 : 5))) void event_stream_kernel(esgpt_batch bt, Terms terms, StreamPlan plan,
                                                           esgpt_tte_spec tte, const T* __restrict__ zc, int64_t ldc,
                                                           int64_t n_levels, int shift, const T* __restrict__ zc_bias,
                                                           const T* __restrict__ zt, int64_t ldt, T* __restrict__ dzc,
                                                           T* __restrict__ dzt, float* __restrict__ dbias,
                                                           const int32_t* __restrict__ counts, int n_ch,
                                                           float* __restrict__ contrib, int64_t n_rows, int tte_in_row,
                                                           int32_t* __restrict__ err, int flags) {
  constexpr int kEl = 16 / sizeof(T);  // elements per 16-B chunk
  constexpr int kB = 4;                // chunk groups (64 chunks each) in flight
  // Dynamic LDS: [narrow logits: 4 waves x S uint4][narrow f32 gradients: 4 x S x kEl][per-subject counts: B x (NT+1)
  // int32, kTot][chunk -> narrow slot map of every level, int16 (-1: not narrow), kMap]. The map replaces a scan of
  // the level's ranges per narrow access; the counts replace per-wave chains of loads over the count partials.
  extern __shared__ __align__(16) unsigned char s_dyn[];
  __shared__ float s_nsub_inv[ESGPT_MAX_TERMS + 1];
  const int S = plan.max_slots;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = lane_id();
  const int NT = terms.n, nt1 = NT + 1;
  const int64_t L = bt.L, M = bt.M;
  const int nch = (int)(ldc / kEl);  // < 2^31 (checked on the host)
  const bool use_map = flags & kMap, use_tot = flags & kTot;
  uint4* s_nz = reinterpret_cast<uint4*>(s_dyn) + wave * S;
  float* ng = reinterpret_cast<float*>(s_dyn + (size_t)4 * S * 16) + wave * S * kEl;
  int32_t* s_tot = reinterpret_cast<int32_t*>(s_dyn + (size_t)4 * S * 16 + (size_t)4 * S * kEl * 4);
  int16_t* s_slot = reinterpret_cast<int16_t*>(s_tot + (use_tot ? bt.B * nt1 : 0));
  const T* nzT = reinterpret_cast<const T*>(s_nz);

  const int64_t w = (int64_t)blockIdx.x * 4 + wave;
  const RowPos q = row_pos(bt, w, n_rows, shift);
  const int64_t b = q.b, r = q.r, p = q.p;
  // the logit / gradient rows of level lv
  auto rows = [&](int lv, const T*& zrow, T*& grow, float*& frow) {
    grow = nullptr, frow = nullptr;
    if (shift) {
      if (r < 0) {
        zrow = zc_bias;
        frow = dbias + b * ldc;
      } else {
        zrow = zc + (b * L + r) * ldc;
        grow = dzc + (b * L + r) * ldc;
      }
    } else {
      const int64_t row = (b * L + p) * n_levels + lv;
      zrow = zc + row * ldc;
      grow = dzc + row * ldc;
    }
  };
  // the first chunk groups of the first row, issued before the setup so their latency overlaps it
  uint4 v[kB];
  auto load_group = [&](const uint4* zv, int g0) {
#pragma unroll
    for (int i = 0; i < kB; ++i) {
      const int c = g0 + 64 * i + lane;
      v[i] = zv[c < nch ? c : nch - 1];  // unconditional: all kB loads in flight together
    }
  };
  if (q.active) {
    const T* z0;
    T* g0;
    float* f0;
    rows(0, z0, g0, f0);
    load_group(reinterpret_cast<const uint4*>(z0), 0);
  }

  // flags: kMap / kTot as above; bits 1..5 = sections skipped (tools build only, ESGPT_LOSS_SKIP: the per-section
  // instruction counts; results are then wrong)
  int64_t e_idx = 0, e_meas = INT64_MIN;
  float e_val = 0.f;
  bool e_vm = false;
  if (q.has_content && lane < M) {
    const int64_t off = (b * L + p) * M + lane;
    e_idx = bt.dyn_idx[off];
    e_meas = bt.dyn_meas[off];
    e_val = bt.dyn_vals[off];
    e_vm = bt.dyn_vmask[off] != 0;
  }
  const bool tte_row = q.active && r >= 0;
  const int64_t e = b * L + (r < 0 ? 0 : r);
  const int64_t e1 = min(e + 1, bt.B * L - 1);  // every load issued together (clamped; used only when r + 1 < L)
  const bool em0 = bt.event_mask[e] != 0, em1 = bt.event_mask[e1] != 0;
  const float td = bt.time_delta[e];
  const bool obs = tte_row && (r + 1 < L) && em0 && em1;
  const float x_tte = obs ? td : 1.f;

  if (use_tot) {  // per-subject counts: thread = (subject, term), its chunk partials summed, loads in flight together
    const int n_tot = (int)bt.B * nt1;
    for (int i = threadIdx.x; i < n_tot; i += 256) {
      const int bb = i / nt1, t = i - bb * nt1;
      const int32_t* src = counts + (int64_t)bb * n_ch * (ESGPT_MAX_TERMS + 1) + t;  // slot NT: observed TTEs
      int32_t c = 0;
#pragma unroll 8
      for (int ch = 0; ch < n_ch; ++ch) c += src[(int64_t)ch * (ESGPT_MAX_TERMS + 1)];
      s_tot[i] = c;
    }
  } else if (wave == 0 && !(flags & kSkipSub)) {
    subjects_with_events(counts, bt.B, n_ch, NT, lane, s_nsub_inv);
  }
  if (wave == 0 && (flags & kSkipSub) && lane <= NT) s_nsub_inv[lane] = 1.f;
  if (use_map) {
    const int n_lvm = shift ? 1 : (int)n_levels;
    for (int lv = 0; lv < n_lvm; ++lv)
      for (int c = threadIdx.x; c < nch; c += 256) {
        int sl = -1;
        for (int k = 0; k < plan.nrng[lv]; ++k)
          if (c >= plan.lo[lv][k] && c < plan.hi[lv][k]) sl = plan.base[lv][k] + c - plan.lo[lv][k];
        s_slot[lv * nch + c] = (int16_t)sl;
      }
  }
  __syncthreads();  // s_tot / s_nsub_inv, s_slot

  // lane t <= NT: 1 / subjects-with-events of term t (lane NT: 1 / B), and this subject's count of term t
  float nsinv;
  int32_t my_cnt = 0;
  if (use_tot) {
    int nsub = 0;
    for (int64_t b0 = 0; b0 < bt.B; b0 += 64) {
      const int64_t bb = b0 + lane;
      for (int t = 0; t < NT; ++t) {
        const int n = __popcll(__ballot(bb < bt.B && s_tot[bb * nt1 + t] > 0));
        if (lane == t) nsub += n;
      }
    }
    nsinv = lane < NT ? (nsub > 0 ? 1.f / (float)nsub : 0.f) : 1.f / (float)bt.B;
    if ((flags & kSkipSub)) nsinv = 1.f;
    if (q.active && lane <= NT) my_cnt = s_tot[b * nt1 + lane];
  } else {
    nsinv = lane <= NT ? s_nsub_inv[lane] : 0.f;
    my_cnt = subject_counts(counts, b, n_ch, NT, lane, q.active);
  }
  auto nsub_inv = [&](int t) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nsinv), t)); };
  flag_no_tte(my_cnt, NT, q.active && q.r == -shift, err);

  float cvec = 0.f;  // lane t: term t's contribution (lane NT: the TTE log-likelihood's)
  const int n_lv = !q.active ? 0 : shift ? 1 : (int)n_levels;
  for (int lv = 0; lv < n_lv; ++lv) {
    const T* zrow;
    T* grow;
    float* frow;
    rows(lv, zrow, grow, frow);
    const int nr = plan.nrng[lv];
    const int16_t* lv_slot = s_slot + lv * nch;  // narrow slot of chunk c (-1: not narrow)

    // ---------------- MULTI range parameters ----------------
    const int nseg = plan.nseg[lv];
    int labc[kMaxSeg];
    float sn[kMaxSeg], sc[kMaxSeg], acc[kMaxSeg];
#pragma unroll
    for (int k = 0; k < kMaxSeg; ++k) {
      labc[k] = -1, sn[k] = 0.f, sc[k] = 0.f, acc[k] = 0.f;
      if (k < nseg && q.has_content) {
        const int t = plan.seg[lv][k];
        const esgpt_loss_term& tm = terms.t[t];
        const int n = tm.vocab_end - tm.vocab_start;
        const bool match = e_meas == tm.meas_idx;
        const int32_t cnt = __builtin_amdgcn_readlane(my_cnt, t);
        const float scale = (q.ev && cnt > 0) ? nsub_inv(t) / (float)cnt : 0.f;
        sc[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(scale)));  // wave-uniform
        sn[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(scale / (float)n)));
        const int64_t my_lab = match ? e_idx - tm.vocab_start : -1;
        labc[k] = (my_lab >= 0 && my_lab < n) ? tm.col + (int)my_lab : -1;
      }
    }

    // ---------------- pass 1: stream the row ----------------
    const uint4* zv = reinterpret_cast<const uint4*>(zrow);
    for (int g0 = 0; g0 < nch; g0 += 64 * kB) {
      if (lv > 0 || g0 > 0) load_group(zv, g0);  // the first group was issued before the setup
#pragma unroll
      for (int i = 0; i < kB; ++i) {
        const int gb = g0 + 64 * i;  // wave-uniform
        if (gb >= nch) break;
        const int c = gb + lane;
        const int glo = gb * kEl, ghi = (gb + 64) * kEl;
        float o[kEl];
#pragma unroll
        for (int el = 0; el < kEl; ++el) o[el] = 0.f;
#pragma unroll
        for (int k = 0; k < kMaxSeg; ++k) {
          if (k >= nseg || sn[k] == 0.f || (flags & kSkipP1)) continue;  // wave-uniform
          const esgpt_loss_term& tm = terms.t[plan.seg[lv][k]];
          const int lo = tm.col, hi = tm.col + tm.vocab_end - tm.vocab_start;
          if (lo >= ghi || hi <= glo) continue;
          float x[kEl];
          unpack_chunk<T>(v[i], x);
          uint32_t ym = 0;  // this lane's label bits
          for (uint64_t bits = __ballot(labc[k] >= glo && labc[k] < ghi); bits; bits &= bits - 1) {
            const int rel = __builtin_amdgcn_readlane(labc[k], __builtin_ctzll(bits)) - glo;
            if (rel / kEl == lane) ym |= 1u << (rel % kEl);
          }
          const bool whole = lo <= glo && hi >= ghi;
          float a = 0.f;
#pragma unroll
          for (int el = 0; el < kEl; ++el) {
            const int col = c * kEl + el;
            const float xx = x[el], yf = ((ym >> el) & 1u) ? 1.f : 0.f;
            const float ex = __builtin_amdgcn_exp2f(-fabsf(xx) * 1.4426950408889634f);
            const float ope = 1.f + ex;
            const float l = fmaxf(xx, 0.f) - xx * yf + __builtin_amdgcn_logf(ope) * 0.6931471805599453f;
            const float inv = __builtin_amdgcn_rcpf(ope);
            const float g = sn[k] * ((xx >= 0.f ? inv : ex * inv) - yf);
            const bool in = whole || (col >= lo && col < hi);
            a += in ? l : 0.f;
            o[el] = in ? g : o[el];
          }
          acc[k] += a;
        }
        int slot = -1;
        if (use_map) {
          slot = c < nch ? (int)lv_slot[c] : -1;
        } else {
          for (int k = 0; k < nr; ++k)
            if (plan.lo[lv][k] < gb + 64 && plan.hi[lv][k] > gb && c >= plan.lo[lv][k] && c < plan.hi[lv][k])
              slot = plan.base[lv][k] + c - plan.lo[lv][k];
        }
        if (slot >= 0) {  // narrow chunk: logits and gradients so far to LDS, stored after pass 2
          s_nz[slot] = v[i];
#pragma unroll
          for (int el = 0; el < kEl; ++el) ng[slot * kEl + el] = o[el];
        } else if (c < nch) {
          if (frow) {
#pragma unroll
            for (int h = 0; h < kEl / 4; ++h)
              reinterpret_cast<float4*>(frow)[c * (kEl / 4) + h] =
                  make_float4(o[4 * h], o[4 * h + 1], o[4 * h + 2], o[4 * h + 3]);
          } else {
            reinterpret_cast<uint4*>(grow)[c] = pack_chunk<T>(o);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kMaxSeg; ++k) {
      if (k >= nseg) continue;
      const int t = plan.seg[lv][k];
      const int n = terms.t[t].vocab_end - terms.t[t].vocab_start;
      const float ell = wave_sum(acc[k]) / (float)n;
      if (lane == t) cvec = sc[k] * ell;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---------------- pass 2: the narrow terms, from LDS ----------------
    for (int t = 0; t < NT && q.has_content && !(flags & kSkipP2); ++t) {
      const esgpt_loss_term& tm = terms.t[t];
      if (tm.kind == ESGPT_TERM_MULTI) continue;
      if (!shift && tm.level != lv) continue;  // wave-uniform
      const bool match = e_meas == tm.meas_idx;
      const uint64_t mm = __ballot(match), mv = __ballot(match && e_vm);
      const bool mk = q.ev && (tm.kind == ESGPT_TERM_SINGLE ? mm != 0 : mv != 0);
      const int32_t cnt = __builtin_amdgcn_readlane(my_cnt, t);
      const float scale = (mk && cnt > 0) ? nsub_inv(t) / (float)cnt : 0.f;
      if (scale == 0.f) continue;  // contribution 0, gradients 0 (already in LDS)
      const int dc = plan.dcol[t], dob = plan.dobs[t], ocol = tm.obs_col;
      const float ell = content_term(
          tm, lane, M, match, mm, mv, e_idx, e_val, e_vm, mk, scale, err,
          [&](int col) { return to_f32(nzT[col + (col == ocol ? dob : dc)]); },
          [&](int col, float g) { ng[col + (col == ocol ? dob : dc)] = g; });
      if (lane == t) cvec = scale * ell;
    }
    if (tte_in_row && lv == 0 && tte_row && !(flags & kSkipTte)) {
      const int32_t cnt = __builtin_amdgcn_readlane(my_cnt, NT);
      const float scale = (obs && cnt > 0) ? -nsub_inv(NT) / (float)cnt : 0.f;
      const float ll = tte_term(
          tte, lane, x_tte, scale, [&](int k) { return to_f32(nzT[tte.col + k + plan.dtte]); },
          [&](int k, float g) { ng[tte.col + k + plan.dtte] = g; });
      if (isnan(ll)) set_err(err, ESGPT_FLAG_TTE_NAN);
      if (lane == NT) cvec = obs ? -scale * ll : 0.f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- the narrow chunks ----
    for (int k = 0; k < nr && !(flags & kSkipStore); ++k) {
      const int lo = plan.lo[lv][k], n = plan.hi[lv][k] - lo, base = plan.base[lv][k];
      for (int j = lane; j < n; j += 64) {
        float o[kEl];
#pragma unroll
        for (int el = 0; el < kEl; ++el) o[el] = ng[(base + j) * kEl + el];
        if (frow) {
#pragma unroll
          for (int h = 0; h < kEl / 4; ++h)
            reinterpret_cast<float4*>(frow)[(lo + j) * (kEl / 4) + h] =
                make_float4(o[4 * h], o[4 * h + 1], o[4 * h + 2], o[4 * h + 3]);
        } else {
          reinterpret_cast<uint4*>(grow)[lo + j] = pack_chunk<T>(o);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the LDS slice is rewritten by the next level
  }

  // ---- time-to-event into a separate dzt (NA) ----
  if (q.active && !tte_in_row && tte_row) {
    const T* z = zt + e * ldt + tte.col;
    T* gz = dzt + e * ldt + tte.col;
    const int32_t cnt = __builtin_amdgcn_readlane(my_cnt, NT);
    const float scale = (obs && cnt > 0) ? -nsub_inv(NT) / (float)cnt : 0.f;
    const float ll = tte_term(
        tte, lane, x_tte, scale, [&](int k) { return to_f32(z[k]); },
        [&](int k, float g) { gz[k] = from_f32<T>(g); });
    if (isnan(ll)) set_err(err, ESGPT_FLAG_TTE_NAN);
    if (lane == NT) cvec = obs ? -scale * ll : 0.f;
  }
  // the workgroup's contributions: rows in order, summed in a fixed order (deterministic). (Folding reduce_kernel
  // into this launch as a last-arriver sum was measured at C2 and rejected: with __threadfence releases, which
  // write back the XCD's L2 full of dirty gradient rows, 56 -> 100 us; with the write-through hand-off of common.h,
  // 53.7 + 4.5 -> 60.8 us, the last workgroup's serial sum of 2048 x 7 write-through contributions.)
  __shared__ float s_part[4][ESGPT_MAX_TERMS + 1];
  if (lane <= NT) s_part[wave][lane] = cvec;
  __syncthreads();
  if (wave == 0 && lane <= NT)
    contrib[(int64_t)lane * gridDim.x + blockIdx.x] =
        ((s_part[0][lane] + s_part[1][lane]) + s_part[2][lane]) + s_part[3][lane];
}


// The other two event kernels' contributions (per row), summed by one workgroup.
__global__ __launch_bounds__(1024) void reduce_kernel(const float* __restrict__ contrib, int64_t n_rows, int NT,
                                                      float* __restrict__ losses) {
  reduce_contrib<1024>(contrib, n_rows, NT, losses);
}

// True when no two terms write the same gradient column of one logit row (the event kernel then stores instead of
// read-modify-writing). Columns per term: SINGLE [col, col+n) + obs_col; MULTI [col, col+n); MVREG [col, col+2n);
// UVREG [col, col+2) + obs_col. Terms of different levels write different rows.
bool disjoint_columns(const esgpt_loss_term* terms, int n_terms, int shift) {
  int64_t lo[2 * ESGPT_MAX_TERMS], hi[2 * ESGPT_MAX_TERMS];
  int lvl[2 * ESGPT_MAX_TERMS], k = 0;
  for (int i = 0; i < n_terms; ++i) {
    const esgpt_loss_term& t = terms[i];
    const int64_t n = t.vocab_end - t.vocab_start;
    const int64_t w = t.kind == ESGPT_TERM_MVREG ? 2 * n : t.kind == ESGPT_TERM_UVREG ? 2 : n;
    const int level = shift ? 0 : t.level;
    lo[k] = t.col, hi[k] = t.col + w, lvl[k++] = level;
    if (t.kind == ESGPT_TERM_SINGLE || t.kind == ESGPT_TERM_UVREG) lo[k] = t.obs_col, hi[k] = t.obs_col + 1, lvl[k++] = level;
  }
  for (int a = 0; a < k; ++a)
    for (int b = a + 1; b < k; ++b)
      if (lvl[a] == lvl[b] && lo[a] < hi[b] && lo[b] < hi[a]) return false;
  return true;
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

constexpr int64_t kLdsBudget = 64 * 1024;  // row-staged event kernel: LDS bytes per block
constexpr int kCountChunk = 32;            // events per count_kernel workgroup (C2: 256 workgroups)
constexpr int kCountThreads = 256;

// The streaming kernel's plan per level: MULTI terms as dense ranges (<= kMaxSeg); the 16-B chunks touching any other
// term column (SINGLE slices, is-observed, regression, in-row TTE) as merged chunk ranges (<= kMaxRng ranges,
// <= max_narrow<T>() chunks). False when the layout does not fit it (the caller takes another kernel).
bool stream_plan(const esgpt_loss_term* terms, int n_terms, int64_t n_levels, int shift, int64_t ldc, int64_t kEl,
                 const esgpt_tte_spec& tte, bool tte_in_row, StreamPlan& plan) {
  const int64_t max_slots = kEl == 4 ? max_narrow<float>() : max_narrow<bf16>();
  const int64_t nl = shift ? 1 : n_levels;
  if (nl < 1 || nl > kMaxLevels || ldc / kEl >= (1ll << 30)) return false;
  plan = StreamPlan{};
  for (int lv = 0; lv < nl; ++lv) {
    std::vector<std::pair<int64_t, int64_t>> cols;  // narrow column ranges [a, b)
    for (int i = 0; i < n_terms; ++i) {
      const esgpt_loss_term& t = terms[i];
      if ((shift ? 0 : t.level) != lv) continue;
      const int64_t n = t.vocab_end - t.vocab_start;
      if (t.kind == ESGPT_TERM_MULTI) {
        if (plan.nseg[lv] >= kMaxSeg) return false;
        plan.seg[lv][plan.nseg[lv]++] = (int8_t)i;
        continue;
      }
      const int64_t w = t.kind == ESGPT_TERM_MVREG ? 2 * n : t.kind == ESGPT_TERM_UVREG ? 2 : n;
      cols.push_back({t.col, t.col + w});
      if (t.kind == ESGPT_TERM_SINGLE || t.kind == ESGPT_TERM_UVREG) cols.push_back({t.obs_col, t.obs_col + 1});
    }
    if (tte_in_row && lv == 0) cols.push_back({tte.col, tte.col + (tte.kind == ESGPT_TTE_EXP ? 1 : 3 * tte.K)});
    std::vector<std::pair<int64_t, int64_t>> ch;  // chunk ranges, merged
    for (auto& c : cols) {
      if (c.first < 0 || c.second > ldc || c.first >= c.second) return false;
      ch.push_back({c.first / kEl, (c.second + kEl - 1) / kEl});
    }
    std::sort(ch.begin(), ch.end());
    std::vector<std::pair<int64_t, int64_t>> merged;
    for (auto& c : ch) {
      if (!merged.empty() && c.first <= merged.back().second) merged.back().second = std::max(merged.back().second, c.second);
      else merged.push_back(c);
    }
    if ((int)merged.size() > kMaxRng) return false;
    int64_t slots = 0;
    for (size_t k = 0; k < merged.size(); ++k) {
      plan.lo[lv][k] = (int32_t)merged[k].first, plan.hi[lv][k] = (int32_t)merged[k].second;
      plan.base[lv][k] = (int32_t)slots;
      slots += merged[k].second - merged[k].first;
    }
    if (slots > max_slots) return false;
    plan.nrng[lv] = (int8_t)merged.size();
    auto delta = [&](int64_t col) -> int32_t {
      const int64_t ck = col / kEl;
      for (size_t k = 0; k < merged.size(); ++k)
        if (ck >= merged[k].first && ck < merged[k].second)
          return (int32_t)((plan.base[lv][k] - merged[k].first) * kEl);
      return 0;  // not reached: every narrow column was inserted above
    };
    for (int i = 0; i < n_terms; ++i) {
      const esgpt_loss_term& t = terms[i];
      if ((shift ? 0 : t.level) != lv || t.kind == ESGPT_TERM_MULTI) continue;
      plan.dcol[i] = delta(t.col);
      if (t.kind == ESGPT_TERM_SINGLE || t.kind == ESGPT_TERM_UVREG) plan.dobs[i] = delta(t.obs_col);
    }
    if (tte_in_row && lv == 0) plan.dtte = delta(tte.col);
    plan.max_slots = std::max<int32_t>(plan.max_slots, (int32_t)std::max<int64_t>(slots, 1));
  }
  return true;
}

}  // namespace

extern "C" {

size_t esgpt_output_loss_workspace(int64_t B, int64_t L, int n_terms) {
  const int64_t n_rows = B * (L + 1);
  return align_up(sizeof(int32_t) * B * cdiv(L, kCountChunk) * (ESGPT_MAX_TERMS + 1)) +
         align_up(sizeof(float) * n_rows * (n_terms + 1));
}

int esgpt_output_loss_ex(const esgpt_batch* batch, const void* zc, int64_t ldc, int64_t n_levels, int shift,
                         const void* zc_bias, const void* zt, int64_t ldt, int dtype, const esgpt_loss_term* terms,
                         int n_terms, const esgpt_tte_spec* tte, void* dzc, void* dzt, float* dbias, float* losses,
                         void* workspace, size_t workspace_bytes, int32_t* err, int path, void* stream) {
  ESGPT_REQUIRE(batch && zt && dzt && tte && losses && workspace);
  ESGPT_REQUIRE(n_terms >= 0 && n_terms <= ESGPT_MAX_TERMS);
  ESGPT_REQUIRE(n_terms == 0 || (zc && dzc));
  ESGPT_REQUIRE(!shift || (zc_bias && dbias && n_levels == 1));
  ESGPT_REQUIRE(batch->M <= kMaxM && (tte->kind == ESGPT_TTE_EXP || (tte->kind == ESGPT_TTE_LNM && tte->K <= kMaxK)));
  ESGPT_REQUIRE(dtype == ESGPT_F32 || dtype == ESGPT_BF16);
  ESGPT_REQUIRE(path >= ESGPT_LOSS_PATH_AUTO && path <= ESGPT_LOSS_PATH_GENERIC);
  ESGPT_REQUIRE(workspace_bytes >= esgpt_output_loss_workspace(batch->B, batch->L, n_terms));
  ESGPT_REQUIRE(batch->L <= 16384 && batch->L * batch->M < (1ll << 31));  // count_kernel: LDS word per event
  ESGPT_REQUIRE(batch->B * (batch->L + 1) < (1ll << 31));                // row_pos: 32-bit row indices
  const int64_t B = batch->B, L = batch->L;
  if (B == 0 || L == 0) return ESGPT_ERR_INVALID_ARG;
  hipStream_t st = as_stream(stream);
  Terms T{};
  T.n = n_terms;
  for (int i = 0; i < n_terms; ++i) T.t[i] = terms[i];
  const int n_ch = (int)cdiv(L, kCountChunk);
  int32_t* counts = (int32_t*)workspace;
  float* contrib = (float*)((char*)workspace + align_up(sizeof(int32_t) * B * n_ch * (ESGPT_MAX_TERMS + 1)));
  const size_t esz = dtype == ESGPT_F32 ? 4 : 2;
  const int64_t n_rows = B * (L + shift);
  // Whole-row kernels (streaming, row-staged) need 16-B aligned rows, disjoint term columns, and the TTE columns
  // either inside the content row (CI head: handled with the row) or in a separate dzt — a dzt aliasing dzc any
  // other way would race the full-row stores.
  const int64_t kEl = 16 / (int64_t)esz;
  const bool aligned = n_terms > 0 && ldc % kEl == 0 && (uintptr_t)zc % 16 == 0 && (uintptr_t)dzc % 16 == 0 &&
                       (!shift || ((uintptr_t)zc_bias % 16 == 0 && (uintptr_t)dbias % 16 == 0));
  const bool same_row = zt == zc && dzt == dzc && ldt == ldc && n_levels == 1;
  const bool whole_row = aligned && (dzt != dzc || same_row) && disjoint_columns(terms, n_terms, shift);
  StreamPlan plan;
  const bool can_stream = whole_row && stream_plan(terms, n_terms, n_levels, shift, ldc, kEl, *tte, same_row, plan);
  const int64_t per_wave = ldc * (int64_t)(esz + 4);  // row-staged: logits + f32 gradients in LDS
  const bool can_stage = aligned && per_wave <= kLdsBudget && (dzt != dzc || same_row);
  int use = path;
  if (use == ESGPT_LOSS_PATH_AUTO) use = can_stream ? ESGPT_LOSS_PATH_STREAM : can_stage ? ESGPT_LOSS_PATH_ROW_STAGED
                                                                                          : ESGPT_LOSS_PATH_GENERIC;
  if ((use == ESGPT_LOSS_PATH_STREAM && !can_stream) || (use == ESGPT_LOSS_PATH_ROW_STAGED && !can_stage))
    return ESGPT_ERR_UNSUPPORTED;
  const bool whole = use != ESGPT_LOSS_PATH_GENERIC;
  const bool tte_in_row = whole && same_row;
  if (!whole) {
    if (n_terms > 0 && zero_async(dzc, esz * B * L * n_levels * ldc, st) != hipSuccess) return ESGPT_ERR_LAUNCH;
    if (shift && zero_async(dbias, sizeof(float) * B * ldc, st) != hipSuccess) return ESGPT_ERR_LAUNCH;
  }
  if (!tte_in_row && (dzt != dzc || n_terms == 0 || whole) && zero_async(dzt, esz * B * L * ldt, st) != hipSuccess)
    return ESGPT_ERR_LAUNCH;
  count_kernel<<<dim3((unsigned)n_ch, (unsigned)B), kCountThreads, sizeof(uint32_t) * kCountChunk, st>>>(
      *batch, T, kCountChunk, counts);
  int64_t n_items = n_rows;  // contributions per term (rows, or workgroups of the streaming kernel)
  if (use == ESGPT_LOSS_PATH_STREAM) {
    const unsigned grid = (unsigned)cdiv(n_rows, 4);
    n_items = grid;
    // dynamic LDS: the narrow chunks of 4 waves, then the per-subject counts and the chunk -> slot map when they fit
    const size_t eb = 16 + sizeof(float) * kEl;  // bytes per narrow chunk: logits + f32 gradients
    const size_t narrow_bytes = 4 * (size_t)plan.max_slots * eb;
    const size_t tot_bytes = sizeof(int32_t) * (size_t)B * (n_terms + 1);
    const size_t map_bytes = sizeof(int16_t) * (size_t)(shift ? 1 : n_levels) * (size_t)(ldc / kEl);
    const bool use_tot = tot_bytes <= 8192;
    const bool use_map = narrow_bytes + (use_tot ? tot_bytes : 0) + map_bytes <= 32768;
    const size_t dyn = narrow_bytes + (use_tot ? tot_bytes : 0) + (use_map ? map_bytes : 0);
    const char* skip = tuning_env("ESGPT_LOSS_SKIP");  // tools build only
    const int flags = (use_map ? kMap : 0) | (use_tot ? kTot : 0) | (skip ? ((atoi(skip) << 1) & 62) : 0);
    if (dtype == ESGPT_F32)
      event_stream_kernel<float><<<grid, 256, dyn, st>>>(*batch, T, plan, *tte, (const float*)zc, ldc, n_levels, shift,
                                                         (const float*)zc_bias, (const float*)zt, ldt, (float*)dzc,
                                                         (float*)dzt, dbias, counts, n_ch, contrib, n_rows, tte_in_row,
                                                         err, flags);
    else
      event_stream_kernel<bf16><<<grid, 256, dyn, st>>>(*batch, T, plan, *tte, (const bf16*)zc, ldc, n_levels, shift,
                                                        (const bf16*)zc_bias, (const bf16*)zt, ldt, (bf16*)dzc,
                                                        (bf16*)dzt, dbias, counts, n_ch, contrib, n_rows, tte_in_row,
                                                        err, flags);
  } else if (use == ESGPT_LOSS_PATH_ROW_STAGED) {
    const int wpb = (int)std::min<int64_t>(kWaves, kLdsBudget / per_wave);
    const unsigned grid = (unsigned)cdiv(n_rows, wpb);
    const size_t lds = (size_t)wpb * per_wave;
    if (dtype == ESGPT_F32)
      event_lds_kernel<float><<<grid, 64 * wpb, lds, st>>>(*batch, T, *tte, (const float*)zc, ldc, n_levels, shift,
                                                          (const float*)zc_bias, (const float*)zt, ldt, (float*)dzc,
                                                          (float*)dzt, dbias, counts, n_ch, contrib, n_rows, tte_in_row,
                                                          err);
    else
      event_lds_kernel<bf16><<<grid, 64 * wpb, lds, st>>>(*batch, T, *tte, (const bf16*)zc, ldc, n_levels, shift,
                                                         (const bf16*)zc_bias, (const bf16*)zt, ldt, (bf16*)dzc,
                                                         (bf16*)dzt, dbias, counts, n_ch, contrib, n_rows, tte_in_row,
                                                         err);
  } else {
    const unsigned grid = (unsigned)cdiv(n_rows, kWaves);
    const bool rmw = !disjoint_columns(terms, n_terms, shift);
#define LAUNCH_EV(TT, RMW)                                                                                        \
  event_kernel<TT, RMW><<<grid, 256, 0, st>>>(*batch, T, *tte, (const TT*)zc, ldc, n_levels, shift,               \
                                              (const TT*)zc_bias, (const TT*)zt, ldt, (TT*)dzc, (TT*)dzt, dbias,  \
                                              counts, n_ch, contrib, n_rows, err)
    if (dtype == ESGPT_F32) {
      if (rmw) LAUNCH_EV(float, true); else LAUNCH_EV(float, false);
    } else {
      if (rmw) LAUNCH_EV(bf16, true); else LAUNCH_EV(bf16, false);
    }
#undef LAUNCH_EV
  }
  reduce_kernel<<<1, 1024, 0, st>>>(contrib, n_items, n_terms, losses);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_output_loss(const esgpt_batch* batch, const void* zc, int64_t ldc, int64_t n_levels, int shift,
                      const void* zc_bias, const void* zt, int64_t ldt, int dtype, const esgpt_loss_term* terms,
                      int n_terms, const esgpt_tte_spec* tte, void* dzc, void* dzt, float* dbias, float* losses,
                      void* workspace, size_t workspace_bytes, int32_t* err, void* stream) {
  return esgpt_output_loss_ex(batch, zc, ldc, n_levels, shift, zc_bias, zt, ldt, dtype, terms, n_terms, tte, dzc, dzt,
                              dbias, losses, workspace, workspace_bytes, err, ESGPT_LOSS_PATH_AUTO, stream);
}

}  // extern "C"
