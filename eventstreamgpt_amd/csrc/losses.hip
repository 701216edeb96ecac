// Fused generative-output losses for gfx950.
//
// Replaces GenerativeOutputLayerBase.get_classification_outputs / get_regression_outputs / get_TTE_outputs
// (EventStream/transformer/model_output.py:1311-1721), the distribution heads (generative_layers.py:6-184) and
// the weighted_loss / safe_weighted_avg reductions (utils.py:134-234) behind ONE forward pass that also emits
// d(total loss)/d(logits), so the backward of the whole output layer is two GEMMs.
//
//   pass 1  count_kernel   one block per subject: per-term masked event counts (weighted_loss denominators),
//                          observed-TTE counts (ValueError if a subject has none)
//   pass 2  event_kernel   one wave per (subject, logit row): every term's per-event loss and logit gradient,
//                          scaled by 1 / (count[b,t] * subjects_with_events[t]); per-event contributions stored
//   pass 3  reduce_kernel  one block: deterministic sums of the contributions -> per-term losses, -TTE_LL, total
//
// HBM traffic per logit row: read C logits + write C gradients (+ the event's M entries); HBM-bound.
#include "common.h"

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
__global__ __launch_bounds__(256) void count_kernel(esgpt_batch bt, Terms terms, int32_t* __restrict__ counts,
                                                    int32_t* __restrict__ err) {
  __shared__ int32_t s_cnt[ESGPT_MAX_TERMS + 1];
  const int64_t b = blockIdx.x;
  const int T = terms.n;
  if (threadIdx.x <= T) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  for (int64_t l = threadIdx.x; l < bt.L; l += blockDim.x) {
    const int64_t e = b * bt.L + l;
    const bool ev = bt.event_mask[e] != 0;
    if (ev) {
      const int64_t* ip = bt.dyn_meas + e * bt.M;
      const uint8_t* vp = bt.dyn_vmask + e * bt.M;
      for (int t = 0; t < T; ++t) {
        const esgpt_loss_term& tm = terms.t[t];
        bool mk = false;
        if (tm.kind == ESGPT_TERM_MULTI) mk = true;
        else {
          for (int64_t m = 0; m < bt.M; ++m) {
            if (ip[m] == tm.meas_idx && (tm.kind == ESGPT_TERM_SINGLE || vp[m])) {
              mk = true;
              break;
            }
          }
        }
        if (mk) atomicAdd(&s_cnt[t], 1);
      }
    }
    if (l + 1 < bt.L && ev && bt.event_mask[e + 1]) atomicAdd(&s_cnt[T], 1);
  }
  __syncthreads();
  if (threadIdx.x <= T) counts[b * (ESGPT_MAX_TERMS + 1) + threadIdx.x] = s_cnt[threadIdx.x];
  if (threadIdx.x == 0 && s_cnt[T] == 0) set_err(err, ESGPT_FLAG_TTE_NO_OBS);
}

// ------------------------------------------------------------------------------------------------------------
template <typename T, bool RMW>
__global__ __launch_bounds__(256) void event_kernel(esgpt_batch bt, Terms terms, esgpt_tte_spec tte,
                                                    const T* __restrict__ zc, int64_t ldc, int64_t n_levels, int shift,
                                                    const T* __restrict__ zc_bias, const T* __restrict__ zt,
                                                    int64_t ldt, T* __restrict__ dzc, T* __restrict__ dzt,
                                                    float* __restrict__ dbias, const int32_t* __restrict__ counts,
                                                    float* __restrict__ contrib, int64_t n_rows,
                                                    int32_t* __restrict__ err) {
  __shared__ float s_nsub_inv[ESGPT_MAX_TERMS + 1];
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int NT = terms.n;
  const int64_t B = bt.B, L = bt.L, M = bt.M;

  // subjects-with-events per term (the outer safe_weighted_avg of weighted_loss); TTE averages over all B.
  // Wave 0: lane = subject, one ballot per term (all terms' count loads in flight together).
  if (wave == 0) {
    int nsub[ESGPT_MAX_TERMS];
#pragma unroll
    for (int t = 0; t < ESGPT_MAX_TERMS; ++t) nsub[t] = 0;
    for (int64_t b0 = 0; b0 < B; b0 += 64) {
      const int64_t b = b0 + lane;
      int c[ESGPT_MAX_TERMS];
#pragma unroll
      for (int t = 0; t < ESGPT_MAX_TERMS; ++t)
        c[t] = (t < NT && b < B) ? counts[b * (ESGPT_MAX_TERMS + 1) + t] : 0;
#pragma unroll
      for (int t = 0; t < ESGPT_MAX_TERMS; ++t) nsub[t] += __popcll(__ballot(c[t] > 0));
    }
#pragma unroll
    for (int t = 0; t < ESGPT_MAX_TERMS; ++t)
      if (lane == t && t < NT) s_nsub_inv[t] = nsub[t] > 0 ? 1.f / (float)nsub[t] : 0.f;
    if (lane == 0) s_nsub_inv[NT] = B > 0 ? 1.f / (float)B : 0.f;
  }

  const int64_t w = (int64_t)blockIdx.x * kWaves + wave;
  const bool active = w < n_rows;
  const int64_t per_b = L + shift;
  const int64_t b = active ? w / per_b : 0;
  const int64_t r = active ? (w % per_b) - shift : 0;  // logit row within subject (-1: the bias row)
  const int64_t p = r + shift;                          // content target position
  const bool has_content = active && p < L;
  const bool ev = has_content && bt.event_mask[b * L + p] != 0;

  // the event's M entries in registers, lane m = entry m (per-term scans are ballots / readlanes, not LDS loops)
  int64_t e_idx = 0, e_meas = INT64_MIN;
  float e_val = 0.f;
  bool e_vm = false;
  if (has_content && lane < M) {
    const int64_t off = (b * L + p) * M + lane;
    e_idx = bt.dyn_idx[off];
    e_meas = bt.dyn_meas[off];
    e_val = bt.dyn_vals[off];
    e_vm = bt.dyn_vmask[off] != 0;
  }
  __syncthreads();  // s_nsub_inv

  // this subject's per-term counts: lane t holds term t's (one load per lane instead of one per term)
  const int32_t my_cnt = lane <= NT ? counts[b * (ESGPT_MAX_TERMS + 1) + lane] : 0;
  float* my_contrib = contrib + w;  // contrib[t * n_rows + w]

  // ---------------- content terms ----------------
  for (int t = 0; t < NT; ++t) {
    const esgpt_loss_term& tm = terms.t[t];
    float c_out = 0.f;
    if (has_content) {
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
      const bool match = e_meas == tm.meas_idx;             // this lane's entry belongs to the term
      const uint64_t mm = __ballot(match), mv = __ballot(match && e_vm);
      const bool mk = ev && (tm.kind == ESGPT_TERM_MULTI ||
                             (tm.kind == ESGPT_TERM_SINGLE ? mm != 0 : mv != 0));  // term_mask, restated
      const int32_t cnt = __builtin_amdgcn_readlane(my_cnt, t);
      const float scale = (mk && cnt > 0) ? s_nsub_inv[t] / (float)cnt : 0.f;
      // Gradient columns: with disjoint term columns (checked on the host) every column of a row has exactly one
      // writer, so the zero-filled buffer is stored to without a read; otherwise read-modify-write. The bias row
      // (shift mode) is this wave's own f32 row.
      auto put = [&](int64_t col, float g) {
        if (gF) gF[col] += g;
        else if (RMW) gT[col] = from_f32<T>(to_f32(gT[col]) + g);
        else gT[col] = from_f32<T>(g);
      };
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
        float mx = -INFINITY;
        for (int j = lane; j < n; j += 64) mx = fmaxf(mx, to_f32(zrow[tm.col + j]));
        mx = wave_max(mx);
        float se = 0.f;
        for (int j = lane; j < n; j += 64) se += expf(to_f32(zrow[tm.col + j]) - mx);
        se = wave_sum(se);
        const float lse = mx + logf(se);
        const float xl = to_f32(zrow[tm.col + lab]);
        const float zo = to_f32(zrow[tm.obs_col]);
        ell = (lse - xl) + bce_logits(zo, has ? 1.f : 0.f);
        if (scale != 0.f) {
          const float inv = 1.f / se;
          for (int j = lane; j < n; j += 64) {
            const float pj = expf(to_f32(zrow[tm.col + j]) - mx) * inv;
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
        // passes of kPass column groups: the pass's logits are loaded before any gradient is stored, so the
        // loads overlap instead of each waiting behind the previous group's store
        constexpr int kPass = 16;
        for (int j1 = 0; j1 < n; j1 += 64 * kPass) {
          float xs[kPass];
#pragma unroll
          for (int it = 0; it < kPass; ++it) {
            const int j = j1 + 64 * it + lane;
            xs[it] = j < n ? to_f32(zrow[tm.col + j]) : 0.f;
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
        bool sel = false;
        int64_t j = 0;
        float nll = 0.f, gmu = 0.f, grho = 0.f;
        {
          sel = match && e_vm;
          if (sel) {
            j = e_idx - tm.vocab_start;
            if (j < 0 || j >= n_targets) {
              set_err(err, ESGPT_FLAG_BAD_LABEL);
              j = 0;
            }
            const float mu = to_f32(zrow[tm.col + 2 * j]);
            const float rho = to_f32(zrow[tm.col + 2 * j + 1]);
            const float sd = elu1(rho);
            const float x = e_val;
            const float zz = (x - mu) / sd;
            nll = 0.5f * zz * zz + logf(sd) + kHalfLog2Pi;
            gmu = -(x - mu) / (sd * sd);
            grho = (1.f / sd - (x - mu) * (x - mu) / (sd * sd * sd)) * delu(rho);
          }
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
            const bool sm_sel = true;
            const int64_t jm = readlane64(j, m);
            const float gm = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gmu), m));
            const float gr = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(grho), m));
            if (sel && sm_sel && jm == j) {
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
        const float mu = to_f32(zrow[tm.col]);
        const float rho = to_f32(zrow[tm.col + 1]);
        const float sd = elu1(rho);
        const float zz = (x - mu) / sd;
        const float zo = to_f32(zrow[tm.obs_col]);
        ell = 0.5f * zz * zz + logf(sd) + kHalfLog2Pi + bce_logits(zo, has_meas ? 1.f : 0.f);
        if (scale != 0.f && lane == 0) {
          put(tm.col, scale * (-(x - mu) / (sd * sd)));
          put(tm.col + 1, scale * (1.f / sd - (x - mu) * (x - mu) / (sd * sd * sd)) * delu(rho));
          put(tm.obs_col, scale * (sigmoidf_(zo) - (has_meas ? 1.f : 0.f)));
        }
      }
      c_out = scale * ell;
    }
    if (active && lane == 0) my_contrib[(int64_t)t * n_rows] = c_out;
  }

  // ---------------- time-to-event (unshifted row r) ----------------
  float c_tte = 0.f;
  if (active && r >= 0) {
    const int64_t e = b * L + r;
    const bool obs = (r + 1 < L) && bt.event_mask[e] && bt.event_mask[e + 1];
    const float x = obs ? bt.time_delta[e] : 1.f;
    const T* z = zt + e * ldt + tte.col;
    T* gz = dzt + e * ldt + tte.col;
    const int32_t cnt = __builtin_amdgcn_readlane(my_cnt, NT);
    const float scale = (obs && cnt > 0) ? -s_nsub_inv[NT] / (float)cnt : 0.f;  // d(-LL)/d ll
    float ll = 0.f;
    if (tte.kind == ESGPT_TTE_EXP) {
      const float zz = to_f32(z[0]);
      const float rate = elu1(zz);
      ll = logf(rate) - rate * x;
      if (lane == 0 && scale != 0.f) gz[0] = from_f32<T>(scale * (1.f / rate - x) * delu(zz));
    } else {
      // LogNormalMixture (third-party pytorch_lognormal_mixture, restated): lanes = components.
      const int K = tte.K;
      const bool affine = !(tte.mean_log == 0.f && tte.std_log == 1.f);
      const float lx = logf(x);
      const float y = affine ? (lx - tte.mean_log) / tte.std_log : lx;
      float loc = 0.f, ls = 0.f, lw = -INFINITY, a = -INFINITY;
      if (lane < K) {
        loc = to_f32(z[3 * lane]);
        ls = to_f32(z[3 * lane + 1]);
        lw = to_f32(z[3 * lane + 2]);
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
        gz[3 * lane] = from_f32<T>(scale * resp * dz / sd);
        gz[3 * lane + 1] = from_f32<T>(scale * resp * (dz * dz - 1.f));
        gz[3 * lane + 2] = from_f32<T>(scale * (resp - pi));
      }
    }
    if (isnan(ll)) set_err(err, ESGPT_FLAG_TTE_NAN);
    c_tte = obs ? -scale * ll : 0.f;  // = obs * ll / (B * cnt): LL contribution (positive sign)
  }
  if (active && lane == 0) my_contrib[(int64_t)NT * n_rows] = c_tte;
}

// ------------------------------------------------------------------------------------------------------------
// Deterministic sums of the per-row contributions: every thread accumulates all terms over its rows, then wave
// sums and a fixed-order sum over the 16 waves.
__global__ __launch_bounds__(1024) void reduce_kernel(const float* __restrict__ contrib, int64_t n_rows, int NT,
                                                      float* __restrict__ losses) {
  __shared__ float s[16][ESGPT_MAX_TERMS + 1];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float a[ESGPT_MAX_TERMS + 1];
#pragma unroll
  for (int t = 0; t <= ESGPT_MAX_TERMS; ++t) a[t] = 0.f;
  for (int64_t i = threadIdx.x; i < n_rows; i += 1024) {
#pragma unroll
    for (int t = 0; t <= ESGPT_MAX_TERMS; ++t)
      if (t <= NT) a[t] += contrib[(int64_t)t * n_rows + i];
  }
#pragma unroll
  for (int t = 0; t <= ESGPT_MAX_TERMS; ++t) {
    if (t <= NT) {
      const float v = wave_sum(a[t]);
      if (lane == 0) s[wave][t] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float total = 0.f;
    for (int t = 0; t <= NT; ++t) {
      float v = 0.f;
      for (int w = 0; w < 16; ++w) v += s[w][t];
      v = (t < NT) ? v : -v;  // last slot: -TTE_LL
      losses[t] = v;
      total += v;
    }
    losses[NT + 1] = total;
  }
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

}  // namespace

extern "C" {

size_t esgpt_output_loss_workspace(int64_t B, int64_t L, int n_terms) {
  const int64_t n_rows = B * (L + 1);
  return align_up(sizeof(int32_t) * B * (ESGPT_MAX_TERMS + 1)) + align_up(sizeof(float) * n_rows * (n_terms + 1));
}

int esgpt_output_loss(const esgpt_batch* batch, const void* zc, int64_t ldc, int64_t n_levels, int shift,
                      const void* zc_bias, const void* zt, int64_t ldt, int dtype, const esgpt_loss_term* terms,
                      int n_terms, const esgpt_tte_spec* tte, void* dzc, void* dzt, float* dbias, float* losses,
                      void* workspace, size_t workspace_bytes, int32_t* err, void* stream) {
  ESGPT_REQUIRE(batch && zt && dzt && tte && losses && workspace);
  ESGPT_REQUIRE(n_terms >= 0 && n_terms <= ESGPT_MAX_TERMS);
  ESGPT_REQUIRE(n_terms == 0 || (zc && dzc));
  ESGPT_REQUIRE(!shift || (zc_bias && dbias && n_levels == 1));
  ESGPT_REQUIRE(batch->M <= kMaxM && (tte->kind == ESGPT_TTE_EXP || (tte->kind == ESGPT_TTE_LNM && tte->K <= kMaxK)));
  ESGPT_REQUIRE(dtype == ESGPT_F32 || dtype == ESGPT_BF16);
  ESGPT_REQUIRE(workspace_bytes >= esgpt_output_loss_workspace(batch->B, batch->L, n_terms));
  const int64_t B = batch->B, L = batch->L;
  if (B == 0 || L == 0) return ESGPT_ERR_INVALID_ARG;
  hipStream_t st = as_stream(stream);
  Terms T{};
  T.n = n_terms;
  for (int i = 0; i < n_terms; ++i) T.t[i] = terms[i];
  int32_t* counts = (int32_t*)workspace;
  float* contrib = (float*)((char*)workspace + align_up(sizeof(int32_t) * B * (ESGPT_MAX_TERMS + 1)));
  const size_t esz = dtype == ESGPT_F32 ? 4 : 2;
  if (n_terms > 0 && zero_async(dzc, esz * B * L * n_levels * ldc, st) != hipSuccess) return ESGPT_ERR_LAUNCH;
  if ((dzt != dzc || n_terms == 0) && zero_async(dzt, esz * B * L * ldt, st) != hipSuccess) return ESGPT_ERR_LAUNCH;
  if (shift && zero_async(dbias, sizeof(float) * B * ldc, st) != hipSuccess) return ESGPT_ERR_LAUNCH;
  count_kernel<<<(unsigned)B, 256, 0, st>>>(*batch, T, counts, err);
  const int64_t n_rows = B * (L + shift);
  const unsigned grid = (unsigned)cdiv(n_rows, kWaves);
  const bool rmw = !disjoint_columns(terms, n_terms, shift);
#define LAUNCH_EV(TT, RMW)                                                                                        \
  event_kernel<TT, RMW><<<grid, 256, 0, st>>>(*batch, T, *tte, (const TT*)zc, ldc, n_levels, shift,               \
                                              (const TT*)zc_bias, (const TT*)zt, ldt, (TT*)dzc, (TT*)dzt, dbias,  \
                                              counts, contrib, n_rows, err)
  if (dtype == ESGPT_F32) {
    if (rmw) LAUNCH_EV(float, true); else LAUNCH_EV(float, false);
  } else {
    if (rmw) LAUNCH_EV(bf16, true); else LAUNCH_EV(bf16, false);
  }
#undef LAUNCH_EV
  reduce_kernel<<<1, 1024, 0, st>>>(contrib, n_rows, n_terms, losses);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

}  // extern "C"
