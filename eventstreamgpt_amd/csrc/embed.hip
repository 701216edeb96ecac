// Input layer kernels for gfx950: the ragged measurement embedding-bag (JOINT / SPLIT, bucketed for NA),
// static merge, temporal position encoding and the atomic-free CSR backward.
//
// Reference semantics: EventStream/data/data_embedding_layer.py (DataEmbeddingLayer, :200-708) and
// EventStream/transformer/transformer.py (time_from_deltas :539-561, TemporalPositionEncoding :564-619,
// CI input layer :656-672, NA input layer :903-936).
//
// Layout in HBM: batch tensors as collated (int64 indices, 1-byte bools, f32 values). One wavefront owns one
// event: lanes 0..M-1 hold that event's M entries (index, measurement, value, value-mask) and compute their
// weights (bucket masks + measurement-index normalisation) in registers; the wave then streams the gathered
// table rows, VEC floats per lane, accumulating every bucket in registers. Roofline: HBM/L2 gather-bound,
// algorithmic bytes per event = nnz_e * D * 4 (rows, per occurrence) + M * 18 (index/meas/value/mask) + G*D*4.
#include <algorithm>

#include "common.h"

using namespace esgpt;

namespace {

constexpr int kMaxM = 64;      // entries per event handled by one wave (lanes)
constexpr int kMaxG = 8;       // dependency-graph buckets
constexpr int kWavesPerBlock = 4;

struct Buckets {
  int G;
  bool bucketed;
  uint64_t cat_bits[kMaxG];
  uint64_t num_bits[kMaxG];
};

__device__ __forceinline__ bool has_bit(uint64_t bits, int64_t meas) {
  return meas >= 0 && meas < 64 && ((bits >> meas) & 1ull);
}

// Per-lane entry state for one event (lane m < M).
struct Entry {
  int64_t idx;
  int64_t meas;
  float val;
  bool vmask;
  float norm;  // measurement-index normalisation (1 when disabled)
};

// Loads lane m's entry of event e and computes its normalisation weight
// (get_measurement_index_normalziation, data_embedding_layer.py:314-349).
__device__ __forceinline__ Entry load_entry(const esgpt_batch& bt, int64_t e, int lane, bool normalize,
                                            int64_t V, int32_t* err) {
  Entry en{0, 0, 0.f, false, 1.f};
  const int64_t M = bt.M;
  if (lane < M) {
    const int64_t off = e * M + lane;
    en.idx = bt.dyn_idx[off];
    en.meas = bt.dyn_meas[off];
    en.val = bt.dyn_vals[off];
    en.vmask = bt.dyn_vmask[off] != 0;
    if (en.idx < 0 || en.idx >= V) {
      set_bad_index(err, en.idx);
      en.idx = 0;
    }
  }
  if (normalize) {
    int cnt = 0;
    for (int j = 0; j < M; ++j) {
      const int64_t mj = __shfl(en.meas, j, 64);
      cnt += (mj == en.meas) ? 1 : 0;
    }
    float nv = (lane < M && en.meas != 0) ? 1.0f / (float)cnt : 0.0f;
    // Sequential (index-order) row sum, as the reference's CPU reduction does for rows of <= M elements.
    float s = 0.f;
    for (int j = 0; j < M; ++j) s += __shfl(nv, j, 64);
    if (s == 0.f) s = 1.f;
    en.norm = nv / s;
  }
  return en;
}

// Bucket weight of an entry (JOINT: values_mask ? value : 1; CAT: cat-bucket ? 1 : 0; NUM: num&mask ? value : 0),
// times the normalisation. This is the per_sample_weights of the reference's EmbeddingBag calls.
__device__ __forceinline__ float entry_weight(const Entry& en, const Buckets& bk, int g, int selector) {
  const bool in_num = bk.bucketed ? has_bit(bk.num_bits[g], en.meas) : true;
  const bool in_cat = bk.bucketed ? has_bit(bk.cat_bits[g], en.meas) : true;
  float w;
  if (selector == ESGPT_BAG_JOINT) {
    w = (en.vmask && in_num) ? en.val : 1.0f;
  } else if (selector == ESGPT_BAG_CAT) {
    w = in_cat ? 1.0f : 0.0f;
  } else {
    w = (en.vmask && in_num) ? en.val : 0.0f;
  }
  return w * en.norm;
}

// Static entries: lane s < S. Weight = normalisation (or 1).
__device__ __forceinline__ void load_static(const esgpt_batch& bt, int64_t b, int lane, bool normalize,
                                            int64_t V, int32_t* err, int64_t& sidx, float& sw) {
  const int64_t S = bt.S;
  int64_t meas = 0;
  sidx = 0;
  if (lane < S) {
    sidx = bt.st_idx[b * S + lane];
    meas = bt.st_meas[b * S + lane];
    if (sidx < 0 || sidx >= V) {
      set_bad_index(err, sidx);
      sidx = 0;
    }
  }
  sw = 1.0f;
  if (normalize) {
    int cnt = 0;
    for (int j = 0; j < S; ++j) cnt += (__shfl(meas, j, 64) == meas) ? 1 : 0;
    float nv = (lane < S && meas != 0) ? 1.0f / (float)cnt : 0.0f;
    float s = 0.f;
    for (int j = 0; j < S; ++j) s += __shfl(nv, j, 64);
    if (s == 0.f) s = 1.f;
    sw = nv / s;
  }
}

// Exclusive cumsum of masked deltas up to event l of subject b, accumulated in double (the reference's CPU
// cumsum accumulates f32 in double, so this reproduces its values) and rounded to f32.
__device__ __forceinline__ float event_time(const esgpt_batch& bt, int64_t b, int64_t l, int lane, bool abs_time) {
  if (abs_time) return bt.time_abs[b * bt.L + l];
  double acc = 0.0;
  for (int64_t j = lane; j < l; j += 64) {
    const float d = bt.event_mask[b * bt.L + j] ? bt.time_delta[b * bt.L + j] : 0.0f;
    acc += (double)d;
  }
  acc = wave_sum_d(acc);
  return (float)acc;
}

__device__ __forceinline__ float time_enc(float t, int64_t d, const float* sin_div, const float* cos_div) {
  return (d & 1) ? cosf(t * cos_div[d >> 1]) : sinf(t * sin_div[d >> 1]);
}

Buckets make_buckets(const esgpt_buckets* b) {
  Buckets k{};
  if (b == nullptr) {
    k.G = 1;
    k.bucketed = false;
  } else {
    k.G = (int)b->G;
    k.bucketed = true;
    for (int g = 0; g < kMaxG; ++g) {
      k.cat_bits[g] = b->cat_bits[g];
      k.num_bits[g] = b->num_bits[g];
    }
  }
  return k;
}

// ------------------------------------------------------------------------------------------------------------
// JOINT forward: one wave per event.
// ------------------------------------------------------------------------------------------------------------
template <int VEC, int GMAX>
__global__ __launch_bounds__(256) void embed_joint_fwd_kernel(esgpt_batch bt, Buckets bk, const float* __restrict__ table,
                                                              int64_t V, int64_t D, const float* __restrict__ sin_div,
                                                              const float* __restrict__ cos_div, int flags, float sw,
                                                              float dw, float* __restrict__ out, int32_t* err) {
  __shared__ float s_w[kWavesPerBlock][GMAX][kMaxM];
  __shared__ int64_t s_idx[kWavesPerBlock][kMaxM];
  __shared__ float s_sw[kWavesPerBlock][kMaxM];
  __shared__ int64_t s_sidx[kWavesPerBlock][kMaxM];

  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int64_t e_raw = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const bool active = e_raw < bt.B * bt.L;  // no early return: the block barrier below must see every wave
  const int64_t e = active ? e_raw : 0;
  const int64_t b = e / bt.L, l = e % bt.L;
  const int G = bk.G;
  const bool normalize = flags & ESGPT_EMB_NORMALIZE;
  const bool use_static = (flags & ESGPT_EMB_STATIC) && bt.S > 0;
  const bool valid = active && bt.event_mask[e] != 0;

  const Entry en = load_entry(bt, e, lane, normalize, V, err);
  if (lane < bt.M) {
    s_idx[wave][lane] = en.idx;
    for (int g = 0; g < G; ++g) s_w[wave][g][lane] = entry_weight(en, bk, g, ESGPT_BAG_JOINT);
  }
  if (use_static) {
    int64_t sidx;
    float swt;
    load_static(bt, b, lane, normalize, V, err, sidx, swt);
    if (lane < bt.S) {
      s_sidx[wave][lane] = sidx;
      s_sw[wave][lane] = swt;
    }
  }
  float t = 0.f;
  if (flags & ESGPT_EMB_TIME) t = event_time(bt, b, l, lane, flags & ESGPT_EMB_TIME_ABS);
  __syncthreads();

  const int64_t n_chunks = (D + 64 * VEC - 1) / (64 * VEC);
  for (int64_t c = 0; c < n_chunks; ++c) {
    const int64_t d0 = c * 64 * VEC + lane * VEC;
    float acc[GMAX][VEC];
#pragma unroll
    for (int g = 0; g < GMAX; ++g)
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[g][v] = 0.f;
    if (valid) {
      for (int m = 0; m < bt.M; ++m) {
        const int64_t i = s_idx[wave][m];
        if (i == 0) continue;  // padding_idx=0 contributes nothing
        float r[VEC];
        if (VEC == 4 && d0 + 3 < D) {
          const float4 x = *reinterpret_cast<const float4*>(table + i * D + d0);
          r[0] = x.x; r[1] = x.y; r[2] = x.z; r[3] = x.w;
        } else {
#pragma unroll
          for (int v = 0; v < VEC; ++v) r[v] = (d0 + v < D) ? table[i * D + d0 + v] : 0.f;
        }
#pragma unroll
        for (int g = 0; g < GMAX; ++g) {
          if (g < G) {
            const float w = s_w[wave][g][m];
#pragma unroll
            for (int v = 0; v < VEC; ++v) acc[g][v] = fmaf(w, r[v], acc[g][v]);
          }
        }
      }
    }
    float st[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) st[v] = 0.f;
    if (use_static && valid) {
      for (int s = 0; s < bt.S; ++s) {
        const int64_t i = s_sidx[wave][s];
        if (i == 0) continue;
        const float w = s_sw[wave][s];
#pragma unroll
        for (int v = 0; v < VEC; ++v)
          if (d0 + v < D) st[v] = fmaf(w, table[i * D + d0 + v], st[v]);
      }
    }
    double run[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) run[v] = 0.0;
#pragma unroll
    for (int g = 0; g < GMAX; ++g) {
      if (g >= G) break;
      float o[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        float x = acc[g][v];
        if (use_static) x = dw * x + sw * st[v];
        if ((flags & ESGPT_EMB_TIME) && g == 0 && d0 + v < D) x = x + time_enc(t, d0 + v, sin_div, cos_div);
        if (flags & ESGPT_EMB_CUMSUM) {
          run[v] += (double)x;
          x = (float)run[v];
        }
        o[v] = valid ? x : 0.f;
      }
      if (!active) continue;
      float* dst = out + (e * G + g) * D + d0;
      if (VEC == 4 && d0 + 3 < D) {
        *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
      } else {
#pragma unroll
        for (int v = 0; v < VEC; ++v)
          if (d0 + v < D) dst[v] = o[v];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// SPLIT forward: bag sums for both tables, scaled, static added to the categorical half.
// ------------------------------------------------------------------------------------------------------------
template <int GMAX>
__global__ __launch_bounds__(256) void embed_split_bags_kernel(esgpt_batch bt, Buckets bk, const float* __restrict__ ct,
                                                               int64_t Dc, const float* __restrict__ nt, int64_t Dn,
                                                               int64_t V, int flags, float cat_scale, float num_scale,
                                                               float static_scale, float* __restrict__ x,
                                                               int32_t* err) {
  __shared__ float s_wc[kWavesPerBlock][GMAX][kMaxM];
  __shared__ float s_wn[kWavesPerBlock][GMAX][kMaxM];
  __shared__ int64_t s_idx[kWavesPerBlock][kMaxM];
  __shared__ float s_sw[kWavesPerBlock][kMaxM];
  __shared__ int64_t s_sidx[kWavesPerBlock][kMaxM];

  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int64_t e_raw = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const bool active = e_raw < bt.B * bt.L;
  const int64_t e = active ? e_raw : 0;
  const int64_t b = e / bt.L;
  const int G = bk.G;
  const bool normalize = flags & ESGPT_EMB_NORMALIZE;
  const bool use_static = (flags & ESGPT_EMB_STATIC) && bt.S > 0;
  const bool valid = active && bt.event_mask[e] != 0;
  const Entry en = load_entry(bt, e, lane, normalize, V, err);
  if (lane < bt.M) {
    s_idx[wave][lane] = en.idx;
    for (int g = 0; g < G; ++g) {
      s_wc[wave][g][lane] = entry_weight(en, bk, g, ESGPT_BAG_CAT);
      s_wn[wave][g][lane] = entry_weight(en, bk, g, ESGPT_BAG_NUM);
    }
  }
  if (use_static) {
    int64_t sidx;
    float swt;
    load_static(bt, b, lane, normalize, V, err, sidx, swt);
    if (lane < bt.S) {
      s_sidx[wave][lane] = sidx;
      s_sw[wave][lane] = swt;
    }
  }
  __syncthreads();
  const int64_t Dx = Dc + Dn;
  for (int64_t d = lane; d < Dx; d += 64) {
    const bool is_cat = d < Dc;
    const float* tb = is_cat ? ct : nt;
    const int64_t DD = is_cat ? Dc : Dn;
    const int64_t dd = is_cat ? d : d - Dc;
    float acc[GMAX];
#pragma unroll
    for (int g = 0; g < GMAX; ++g) acc[g] = 0.f;
    if (valid) {
      for (int m = 0; m < bt.M; ++m) {
        const int64_t i = s_idx[wave][m];
        if (i == 0) continue;
        const float r = tb[i * DD + dd];
#pragma unroll
        for (int g = 0; g < GMAX; ++g)
          if (g < G) acc[g] = fmaf(is_cat ? s_wc[wave][g][m] : s_wn[wave][g][m], r, acc[g]);
      }
    }
    float st = 0.f;
    if (use_static && is_cat && valid) {
      for (int s = 0; s < bt.S; ++s) {
        const int64_t i = s_sidx[wave][s];
        if (i == 0) continue;
        st = fmaf(s_sw[wave][s], ct[i * Dc + dd], st);
      }
    }
#pragma unroll
    for (int g = 0; g < GMAX; ++g) {
      if (g >= G) break;
      float v = (is_cat ? cat_scale : num_scale) * acc[g];
      if (is_cat && use_static) v = v + static_scale * st;
      if (active) x[(e * G + g) * Dx + d] = valid ? v : 0.f;
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// Epilogue (split mode): time at level 0, cumsum over levels, event mask. One wave per event.
// ------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void embed_epilogue_fwd_kernel(esgpt_batch bt, int64_t G, int64_t D,
                                                                 const float* __restrict__ y,
                                                                 const float* __restrict__ sin_div,
                                                                 const float* __restrict__ cos_div, int flags,
                                                                 float* __restrict__ out) {
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int64_t e = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  if (e >= bt.B * bt.L) return;
  const int64_t b = e / bt.L, l = e % bt.L;
  const bool valid = bt.event_mask[e] != 0;
  float t = 0.f;
  if (flags & ESGPT_EMB_TIME) t = event_time(bt, b, l, lane, flags & ESGPT_EMB_TIME_ABS);
  for (int64_t d = lane; d < D; d += 64) {
    double run = 0.0;
    for (int64_t g = 0; g < G; ++g) {
      float x = y[(e * G + g) * D + d];
      if ((flags & ESGPT_EMB_TIME) && g == 0) x = x + time_enc(t, d, sin_div, cos_div);
      if (flags & ESGPT_EMB_CUMSUM) {
        run += (double)x;
        x = (float)run;
      }
      out[(e * G + g) * D + d] = valid ? x : 0.f;
    }
  }
}

__global__ __launch_bounds__(256) void embed_epilogue_bwd_kernel(esgpt_batch bt, int64_t G, int64_t D,
                                                                 const float* __restrict__ dout, int flags,
                                                                 float* __restrict__ dy) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = bt.B * bt.L * D;
  if (i >= n) return;
  const int64_t e = i / D, d = i % D;
  const bool valid = bt.event_mask[e] != 0;
  if (flags & ESGPT_EMB_CUMSUM) {
    float run = 0.f;  // reverse cumsum in f32 (autograd of cumsum = flip-cumsum-flip in f32)
    for (int64_t g = G - 1; g >= 0; --g) {
      run += dout[(e * G + g) * D + d];
      dy[(e * G + g) * D + d] = valid ? run : 0.f;
    }
  } else {
    for (int64_t g = 0; g < G; ++g) dy[(e * G + g) * D + d] = valid ? dout[(e * G + g) * D + d] : 0.f;
  }
}

// ------------------------------------------------------------------------------------------------------------
// Bag backward: CSR (vocab-row -> entries) built with integer counters, then a chunked segmented reduction.
//   slots: dynamic (e, g, m) in [0, B*L*G*M) then static (b, s) in [0, B*S).
//   src row of a dynamic slot = e*G + g (dsrc); of a static slot = b (subject sums, workspace).
// ------------------------------------------------------------------------------------------------------------
struct BagBwdArgs {
  esgpt_batch bt;
  Buckets bk;
  int selector;
  int flags;
  float dyn_scale;
  float static_scale;
  int64_t V;
};

// Returns true and fills (v, w, src) if the slot contributes. Recomputes the slot's weight like the forward.
__device__ __forceinline__ bool bag_slot(const BagBwdArgs& a, int64_t slot, int64_t& v, float& w, int64_t& src) {
  const esgpt_batch& bt = a.bt;
  const int64_t G = a.bk.G;
  const int64_t n_dyn = bt.B * bt.L * G * bt.M;
  const bool normalize = a.flags & ESGPT_EMB_NORMALIZE;
  if (slot < n_dyn) {
    const int64_t m = slot % bt.M;
    const int64_t eg = slot / bt.M;
    const int64_t g = eg % G, e = eg / G;
    if (!bt.event_mask[e]) return false;
    const int64_t* ip = bt.dyn_idx + e * bt.M;
    const int64_t* mp = bt.dyn_meas + e * bt.M;
    v = ip[m];
    if (v <= 0 || v >= a.V) return false;
    Entry en;
    en.idx = v;
    en.meas = mp[m];
    en.val = bt.dyn_vals[e * bt.M + m];
    en.vmask = bt.dyn_vmask[e * bt.M + m] != 0;
    en.norm = 1.f;
    if (normalize) {
      int cnt = 0;
      float s = 0.f;
      // sum_j 1/cnt_j over j with meas != 0, in index order (matches the forward's normaliser bit-for-bit).
      for (int64_t j = 0; j < bt.M; ++j) {
        const int64_t mj = mp[j];
        if (mj == en.meas) ++cnt;
        int cj = 0;
        for (int64_t k = 0; k < bt.M; ++k) cj += (mp[k] == mj) ? 1 : 0;
        s += (mj != 0) ? 1.0f / (float)cj : 0.0f;
      }
      if (s == 0.f) s = 1.f;
      en.norm = (en.meas != 0 ? 1.0f / (float)cnt : 0.0f) / s;
    }
    w = entry_weight(en, a.bk, (int)g, a.selector) * a.dyn_scale;
    if (a.selector != ESGPT_BAG_JOINT && w == 0.f) {
      // CAT/NUM: entries outside the bucket have weight exactly 0; skipping them is exact for finite grads.
      const bool in = (a.selector == ESGPT_BAG_CAT)
                          ? (a.bk.bucketed ? has_bit(a.bk.cat_bits[g], en.meas) : true)
                          : (en.vmask && (a.bk.bucketed ? has_bit(a.bk.num_bits[g], en.meas) : true));
      if (!in) return false;
    }
    src = eg;
    return true;
  }
  if (!(a.flags & ESGPT_EMB_STATIC) || a.selector == ESGPT_BAG_NUM) return false;
  const int64_t ss = slot - n_dyn;
  if (ss >= bt.B * bt.S) return false;
  const int64_t b = ss / bt.S, s = ss % bt.S;
  v = bt.st_idx[ss];
  if (v <= 0 || v >= a.V) return false;
  float sw = 1.f;
  if (normalize) {
    const int64_t* mp = bt.st_meas + b * bt.S;
    const int64_t me = mp[s];
    int cnt = 0;
    float sum = 0.f;
    for (int64_t j = 0; j < bt.S; ++j) {
      const int64_t mj = mp[j];
      if (mj == me) ++cnt;
      int cj = 0;
      for (int64_t k = 0; k < bt.S; ++k) cj += (mp[k] == mj) ? 1 : 0;
      sum += (mj != 0) ? 1.0f / (float)cj : 0.0f;
    }
    if (sum == 0.f) sum = 1.f;
    sw = (me != 0 ? 1.0f / (float)cnt : 0.0f) / sum;
  }
  w = sw * a.static_scale;
  src = -1 - b;  // negative: subject-sum row b
  return true;
}

// Slot ranges: block i owns the contiguous slots [i*per, (i+1)*per) in both the count and the fill pass.
constexpr int kBagBlocks = 256;
constexpr int kLdsBins = 16384;  // vocabularies up to this size are histogrammed in LDS (2 x 64 KiB)

// Per-block LDS histogram, then one global add per non-empty bin (hot rows such as event types would otherwise
// serialise thousands of same-address atomics).
template <bool LDS>
__global__ __launch_bounds__(256) void bag_count_kernel(BagBwdArgs a, int64_t n_slots, int64_t per,
                                                        int32_t* __restrict__ count) {
  extern __shared__ int32_t s_hist[];
  const int64_t lo = (int64_t)blockIdx.x * per, hi = min(n_slots, lo + per);
  if (LDS) {
    for (int64_t i = threadIdx.x; i < a.V; i += blockDim.x) s_hist[i] = 0;
    __syncthreads();
  }
  for (int64_t slot = lo + threadIdx.x; slot < hi; slot += blockDim.x) {
    int64_t v, src;
    float w;
    if (bag_slot(a, slot, v, w, src)) {
      if (LDS) atomicAdd(s_hist + v, 1);
      else atomicAdd(count + v, 1);
    }
  }
  if (LDS) {
    __syncthreads();
    for (int64_t i = threadIdx.x; i < a.V; i += blockDim.x)
      if (s_hist[i]) atomicAdd(count + i, s_hist[i]);
  }
}

// Exclusive scan of count[0..V) into rowptr[0..V]; single workgroup of 1024 threads. Also zeroes cursor.
__global__ __launch_bounds__(1024) void bag_scan_kernel(const int32_t* __restrict__ count, int64_t V,
                                                        int32_t* __restrict__ rowptr, int32_t* __restrict__ cursor) {
  __shared__ int32_t s_part[1024];
  const int tid = threadIdx.x;
  const int64_t per = (V + 1023) / 1024;
  const int64_t lo = tid * per, hi = min(V, lo + per);
  int32_t sum = 0;
  for (int64_t i = lo; i < hi; ++i) sum += count[i];
  s_part[tid] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    int32_t add = (tid >= o) ? s_part[tid - o] : 0;
    __syncthreads();
    s_part[tid] += add;
    __syncthreads();
  }
  int32_t run = s_part[tid] - sum;
  for (int64_t i = lo; i < hi; ++i) {
    rowptr[i] = run;
    cursor[i] = 0;
    run += count[i];
  }
  if (tid == 1023) rowptr[V] = s_part[1023];
}

// Scatter into CSR order. LDS variant: block-local counts, one global cursor reservation per (block, bin), then
// in-block ranks from LDS atomics.
template <bool LDS>
__global__ __launch_bounds__(256) void bag_fill_kernel(BagBwdArgs a, int64_t n_slots, int64_t per,
                                                       const int32_t* __restrict__ rowptr,
                                                       int32_t* __restrict__ cursor, int64_t* __restrict__ ent_src,
                                                       float* __restrict__ ent_w, int32_t* __restrict__ ent_v) {
  extern __shared__ int32_t s_mem[];
  int32_t* s_cnt = s_mem;
  int32_t* s_base = s_mem + a.V;
  const int64_t lo = (int64_t)blockIdx.x * per, hi = min(n_slots, lo + per);
  if (LDS) {
    for (int64_t i = threadIdx.x; i < a.V; i += blockDim.x) s_cnt[i] = 0;
    __syncthreads();
    for (int64_t slot = lo + threadIdx.x; slot < hi; slot += blockDim.x) {
      int64_t v, src;
      float w;
      if (bag_slot(a, slot, v, w, src)) atomicAdd(s_cnt + v, 1);
    }
    __syncthreads();
    for (int64_t i = threadIdx.x; i < a.V; i += blockDim.x) {
      const int32_t c = s_cnt[i];
      s_base[i] = c ? rowptr[i] + atomicAdd(cursor + i, c) : 0;
      s_cnt[i] = 0;
    }
    __syncthreads();
  }
  for (int64_t slot = lo + threadIdx.x; slot < hi; slot += blockDim.x) {
    int64_t v, src;
    float w;
    if (!bag_slot(a, slot, v, w, src)) continue;
    const int32_t pos = LDS ? s_base[v] + atomicAdd(s_cnt + v, 1) : rowptr[v] + atomicAdd(cursor + v, 1);
    ent_src[pos] = src;
    ent_w[pos] = w;
    ent_v[pos] = (int32_t)v;
  }
}

// Subject sums of dsrc over valid events and all levels: sub[b, d] (zeroed beforehand). Block (b, c) sums the
// event chunk c of subject b for every column and adds it in.
constexpr int kSubChunks = 8;
__global__ __launch_bounds__(256) void bag_subject_sum_kernel(esgpt_batch bt, int64_t G, const float* __restrict__ dsrc,
                                                              int64_t ld, int64_t D, float* __restrict__ sub) {
  const int64_t b = blockIdx.x;
  const int64_t per = (bt.L + kSubChunks - 1) / kSubChunks;
  const int64_t l0 = blockIdx.y * per, l1 = min(bt.L, l0 + per);
  for (int64_t d = threadIdx.x; d < D; d += blockDim.x) {
    float acc = 0.f;
    for (int64_t l = l0; l < l1; ++l) {
      const int64_t e = b * bt.L + l;
      if (!bt.event_mask[e]) continue;
      for (int64_t g = 0; g < G; ++g) acc += dsrc[(e * G + g) * ld + d];
    }
    if (l1 > l0) atomicAdd(sub + b * D + d, acc);
  }
}

// One wave per chunk of kChunk sorted entries. Lane l loads entries l and 64 + l of the chunk (coalesced); the wave
// then walks them in groups of kGroup with the group's gathered gradient rows in flight together (the entry fields
// are wave-uniform via readlane). Rows fully inside the chunk are stored; a row that continues into a neighbouring
// chunk (at most the first and the last run) is added with f32 atomics — long chunks keep the number of atomic
// adds per address low for the very frequent rows (a univariate measurement's row gets ~20k entries per batch).
// dtable is zeroed beforehand.
constexpr int kChunk = 128;
constexpr int kGroup = 8;

__device__ __forceinline__ int64_t readlane64(int64_t x, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)x, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)x >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

template <int VEC>
__global__ __launch_bounds__(256) void bag_reduce_kernel(int64_t V, const int32_t* __restrict__ rowptr,
                                                         const int64_t* __restrict__ ent_src,
                                                         const float* __restrict__ ent_w,
                                                         const int32_t* __restrict__ ent_v,
                                                         const float* __restrict__ dsrc, int64_t ld,
                                                         const float* __restrict__ sub, int64_t D,
                                                         float* __restrict__ dtable) {
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int64_t chunk = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const int64_t lo = chunk * kChunk;
  const int64_t n_ent = rowptr[V];
  if (lo >= n_ent) return;
  const int n = (int)min<int64_t>(kChunk, n_ent - lo);
  int32_t my_v[2] = {-1, -1};
  int64_t my_s[2] = {0, 0};
  float my_w[2] = {0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int p = 64 * u + lane;
    if (p < n) {
      my_v[u] = ent_v[lo + p];
      my_s[u] = ent_src[lo + p];
      my_w[u] = ent_w[lo + p];
    }
  }
  // the chunk's first / last run continues into the previous / next chunk when those entries share its row
  const int32_t prev_v = lo > 0 ? ent_v[lo - 1] : -1;
  const int32_t next_v = lo + n < n_ent ? ent_v[lo + n] : -1;
  for (int64_t base = 0; base < D; base += 64 * VEC) {
    const int64_t d0 = base + (int64_t)lane * VEC;
    const bool dok = d0 < D;  // VEC == 4 only when D % 4 == 0
    float acc[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
    int32_t cur = __builtin_amdgcn_readlane(my_v[0], 0);
    bool head = true;  // the current run starts at the chunk's first entry
    auto flush = [&](bool tail) {
      const bool shared = (head && prev_v == cur) || (tail && next_v == cur);
      float* dst = dtable + (int64_t)cur * D + d0;
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        if (dok && (VEC == 4 || d0 + k < D)) {
          if (shared) atomicAdd(dst + k, acc[k]);
          else dst[k] = acc[k];
        }
        acc[k] = 0.f;
      }
    };
    for (int p0 = 0; p0 < n; p0 += kGroup) {
      // the group's entries live in register half u = p0 / 64 (groups never straddle it): uniform selects
      const bool up = p0 >= 64;
      const int32_t gv = up ? my_v[1] : my_v[0];
      const int64_t gs = up ? my_s[1] : my_s[0];
      const float gw = up ? my_w[1] : my_w[0];
      float x[kGroup][VEC];
#pragma unroll
      for (int j = 0; j < kGroup; ++j) {
        const int p = min(p0 + j, n - 1);
        const int64_t s = readlane64(gs, p & 63);
        const float* row = s >= 0 ? dsrc + s * ld : sub + (-1 - s) * D;
        if (VEC == 4) {
          float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
          if (dok) t = *reinterpret_cast<const float4*>(row + d0);
          x[j][0] = t.x;
          x[j][1] = t.y;
          x[j][2] = t.z;
          x[j][3] = t.w;
        } else {
#pragma unroll
          for (int k = 0; k < VEC; ++k) x[j][k] = (d0 + k < D) ? row[d0 + k] : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < kGroup; ++j) {
        const int p = p0 + j;
        if (p < n) {
          const int32_t v = __builtin_amdgcn_readlane(gv, p & 63);
          if (v != cur) {
            flush(false);
            cur = v;
            head = false;
          }
          const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gw), p & 63));
#pragma unroll
          for (int k = 0; k < VEC; ++k) acc[k] = fmaf(w, x[j][k], acc[k]);
        }
      }
    }
    flush(true);
  }
}

struct BagWs {
  int32_t* count;
  int32_t* rowptr;
  int32_t* cursor;
  int32_t* n_ent_dummy;
  int64_t* ent_src;
  float* ent_w;
  int32_t* ent_v;
  float* sub;
  size_t bytes;
};

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

static BagWs carve(void* base, const esgpt_batch* bt, int64_t G, int64_t V, int64_t D) {
  BagWs w{};
  const int64_t n_slots = bt->B * bt->L * G * bt->M + bt->B * bt->S;
  char* p = (char*)base;
  size_t off = 0;
  auto take = [&](size_t n) {
    char* r = p ? p + off : nullptr;
    off += align_up(n);
    return r;
  };
  w.count = (int32_t*)take(sizeof(int32_t) * (V + 1));
  w.rowptr = (int32_t*)take(sizeof(int32_t) * (V + 1));
  w.cursor = (int32_t*)take(sizeof(int32_t) * (V + 1));
  w.ent_src = (int64_t*)take(sizeof(int64_t) * n_slots);
  w.ent_w = (float*)take(sizeof(float) * n_slots);
  w.ent_v = (int32_t*)take(sizeof(int32_t) * n_slots);
  w.sub = (float*)take(sizeof(float) * bt->B * D);
  w.bytes = off;
  return w;
}

}  // namespace

extern "C" {

int esgpt_embed_joint_fwd(const esgpt_batch* batch, const esgpt_buckets* buckets, const float* table, int64_t V,
                          int64_t D, const float* sin_div, const float* cos_div, int flags, float static_w,
                          float dynamic_w, float* out, int32_t* err, void* stream) {
  ESGPT_REQUIRE(batch && table && out && D > 0 && V > 0);
  ESGPT_REQUIRE(batch->M <= kMaxM && batch->S <= kMaxM);
  ESGPT_REQUIRE(!(flags & ESGPT_EMB_TIME) || (sin_div && cos_div));
  const Buckets bk = make_buckets(buckets);
  ESGPT_REQUIRE(bk.G >= 1 && bk.G <= kMaxG);
  const int64_t n_ev = batch->B * batch->L;
  if (n_ev == 0) return ESGPT_OK;
  dim3 grid((unsigned)cdiv(n_ev, kWavesPerBlock)), block(256);
  hipStream_t st = as_stream(stream);
  const bool vec4 = (D % 4 == 0) && D >= 256;
#define LAUNCH_J(VEC, GM)                                                                                 \
  embed_joint_fwd_kernel<VEC, GM><<<grid, block, 0, st>>>(*batch, bk, table, V, D, sin_div, cos_div, flags, \
                                                          static_w, dynamic_w, out, err)
  if (bk.G == 1) {
    if (vec4) LAUNCH_J(4, 1); else LAUNCH_J(1, 1);
  } else if (bk.G <= 4) {
    if (vec4) LAUNCH_J(4, 4); else LAUNCH_J(1, 4);
  } else {
    if (vec4) LAUNCH_J(4, 8); else LAUNCH_J(1, 8);
  }
#undef LAUNCH_J
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_embed_split_bags_fwd(const esgpt_batch* batch, const esgpt_buckets* buckets, const float* cat_table,
                               int64_t Dc, const float* num_table, int64_t Dn, int64_t V, int flags, float cat_scale,
                               float num_scale, float static_scale, float* x, int32_t* err, void* stream) {
  ESGPT_REQUIRE(batch && cat_table && num_table && x && Dc > 0 && Dn > 0);
  ESGPT_REQUIRE(batch->M <= kMaxM && batch->S <= kMaxM);
  const Buckets bk = make_buckets(buckets);
  ESGPT_REQUIRE(bk.G >= 1 && bk.G <= kMaxG);
  const int64_t n_ev = batch->B * batch->L;
  if (n_ev == 0) return ESGPT_OK;
  dim3 grid((unsigned)cdiv(n_ev, kWavesPerBlock)), block(256);
  hipStream_t st = as_stream(stream);
  if (bk.G == 1)
    embed_split_bags_kernel<1><<<grid, block, 0, st>>>(*batch, bk, cat_table, Dc, num_table, Dn, V, flags, cat_scale,
                                                       num_scale, static_scale, x, err);
  else if (bk.G <= 4)
    embed_split_bags_kernel<4><<<grid, block, 0, st>>>(*batch, bk, cat_table, Dc, num_table, Dn, V, flags, cat_scale,
                                                       num_scale, static_scale, x, err);
  else
    embed_split_bags_kernel<8><<<grid, block, 0, st>>>(*batch, bk, cat_table, Dc, num_table, Dn, V, flags, cat_scale,
                                                       num_scale, static_scale, x, err);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_embed_epilogue_fwd(const esgpt_batch* batch, int64_t G, int64_t D, const float* y, const float* sin_div,
                             const float* cos_div, int flags, float* out, void* stream) {
  ESGPT_REQUIRE(batch && y && out && G >= 1 && D > 0);
  ESGPT_REQUIRE(!(flags & ESGPT_EMB_TIME) || (sin_div && cos_div));
  const int64_t n_ev = batch->B * batch->L;
  if (n_ev == 0) return ESGPT_OK;
  embed_epilogue_fwd_kernel<<<dim3((unsigned)cdiv(n_ev, kWavesPerBlock)), dim3(256), 0, as_stream(stream)>>>(
      *batch, G, D, y, sin_div, cos_div, flags, out);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_embed_epilogue_bwd(const esgpt_batch* batch, int64_t G, int64_t D, const float* dout, int flags, float* dy,
                             void* stream) {
  ESGPT_REQUIRE(batch && dout && dy && G >= 1 && D > 0);
  const int64_t n = batch->B * batch->L * D;
  if (n == 0) return ESGPT_OK;
  embed_epilogue_bwd_kernel<<<dim3((unsigned)cdiv(n, 256)), dim3(256), 0, as_stream(stream)>>>(*batch, G, D, dout,
                                                                                               flags, dy);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

size_t esgpt_embed_bag_bwd_workspace(const esgpt_batch* batch, int64_t G, int64_t V, int64_t D) {
  if (!batch) return 0;
  return carve(nullptr, batch, G, V, D).bytes;
}

int esgpt_embed_bag_bwd(const esgpt_batch* batch, const esgpt_buckets* buckets, int selector, int flags,
                        float dyn_scale, float static_scale, const float* dsrc, int64_t ld, int64_t D, int64_t V,
                        float* dtable, void* workspace, size_t workspace_bytes, void* stream) {
  ESGPT_REQUIRE(batch && dsrc && dtable && D > 0 && V > 0 && V < (1ll << 31));
  const Buckets bk = make_buckets(buckets);
  ESGPT_REQUIRE(bk.G >= 1 && bk.G <= kMaxG);
  BagWs w = carve(workspace, batch, bk.G, V, D);
  ESGPT_REQUIRE(workspace && workspace_bytes >= w.bytes);
  hipStream_t st = as_stream(stream);
  BagBwdArgs a{*batch, bk, selector, flags, dyn_scale, static_scale, V};
  const int64_t n_slots = batch->B * batch->L * bk.G * batch->M + batch->B * batch->S;
  if (zero_async(dtable, sizeof(float) * V * D, st) != hipSuccess) return ESGPT_ERR_LAUNCH;
  if (zero_async(w.count, sizeof(int32_t) * (V + 1), st) != hipSuccess) return ESGPT_ERR_LAUNCH;
  if (n_slots == 0) return ESGPT_OK;
  const int64_t nblk = std::min<int64_t>(kBagBlocks, cdiv(n_slots, 256));
  const int64_t per = cdiv(n_slots, nblk);
  // Dynamic LDS stays within the 64 KiB default: count needs 4 B/bin, fill 8 B/bin.
  const bool lds = V <= kLdsBins;
  const bool lds_fill = V <= kLdsBins / 2;
  if (lds) {
    bag_count_kernel<true><<<(unsigned)nblk, 256, sizeof(int32_t) * V, st>>>(a, n_slots, per, w.count);
  } else {
    bag_count_kernel<false><<<(unsigned)nblk, 256, 0, st>>>(a, n_slots, per, w.count);
  }
  bag_scan_kernel<<<1, 1024, 0, st>>>(w.count, V, w.rowptr, w.cursor);
  if (lds_fill) {
    bag_fill_kernel<true><<<(unsigned)nblk, 256, 2 * sizeof(int32_t) * V, st>>>(a, n_slots, per, w.rowptr, w.cursor,
                                                                               w.ent_src, w.ent_w, w.ent_v);
  } else {
    bag_fill_kernel<false><<<(unsigned)nblk, 256, 0, st>>>(a, n_slots, per, w.rowptr, w.cursor, w.ent_src, w.ent_w,
                                                          w.ent_v);
  }
  if ((flags & ESGPT_EMB_STATIC) && batch->S > 0 && selector != ESGPT_BAG_NUM) {
    if (zero_async(w.sub, sizeof(float) * batch->B * D, st) != hipSuccess) return ESGPT_ERR_LAUNCH;
    bag_subject_sum_kernel<<<dim3((unsigned)batch->B, kSubChunks), 256, 0, st>>>(*batch, bk.G, dsrc, ld, D, w.sub);
  }
  ESGPT_LAUNCH_CHECK();
  // The number of entries is data-dependent (not known on the host without a sync): launch for the upper bound;
  // chunks past rowptr[V] exit immediately.
  const int64_t n_chunks = cdiv(n_slots, kChunk);
  const unsigned g_red = (unsigned)cdiv(n_chunks, kWavesPerBlock);
  if (D % 4 == 0 && D >= 256 && ld % 4 == 0 && ((uintptr_t)dsrc % 16) == 0)
    bag_reduce_kernel<4><<<g_red, 256, 0, st>>>(V, w.rowptr, w.ent_src, w.ent_w, w.ent_v, dsrc, ld, w.sub, D,
                                                dtable);
  else
    bag_reduce_kernel<1><<<g_red, 256, 0, st>>>(V, w.rowptr, w.ent_src, w.ent_w, w.ent_v, dsrc, ld, w.sub, D,
                                                dtable);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

}  // extern "C"
