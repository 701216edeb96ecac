// Input layer kernels for gfx950: the ragged measurement embedding-bag (JOINT / SPLIT, bucketed for NA),
// static merge, temporal position encoding and the deterministic, atomic-free sorted-CSR backward.
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

#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/block/block_scan.hpp>

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
// Loads are issued kTU per lane at a time from clamped addresses (selected away past l), so a long prefix costs one
// memory round trip per 64·kTU events instead of one per 64; each lane still adds its deltas in ascending order.
__device__ __forceinline__ float event_time(const esgpt_batch& bt, int64_t b, int64_t l, int lane, bool abs_time) {
  if (abs_time) return bt.time_abs[b * bt.L + l];
  constexpr int kTU = 4;
  const uint8_t* em = bt.event_mask + b * bt.L;
  const float* td = bt.time_delta + b * bt.L;
  double acc = 0.0;
  for (int64_t j0 = 0; j0 < l; j0 += 64 * kTU) {
    uint8_t m[kTU];
    float d[kTU];
#pragma unroll
    for (int u = 0; u < kTU; ++u) {
      const int64_t j = min(j0 + 64 * u + lane, l > 0 ? l - 1 : 0);
      m[u] = em[j];
      d[u] = td[j];
    }
#pragma unroll
    for (int u = 0; u < kTU; ++u)
      if (j0 + 64 * u + lane < l) acc += (double)(m[u] ? d[u] : 0.0f);
  }
  acc = wave_sum_d(acc);
  return (float)acc;
}

__device__ __forceinline__ float time_enc(float t, int64_t d, const float* sin_div, const float* cos_div) {
  return (d & 1) ? cosf(t * cos_div[d >> 1]) : sinf(t * sin_div[d >> 1]);
}

// The encodings of dims d0 .. d0+VEC-1 (d0 even): the sine and cosine of one frequency share one sincosf (one
// argument reduction, the same results as sinf / cosf) when the two divisor tables agree there (they are one tensor
// in the reference, TemporalPositionEncoding); the libm argument reductions of t·w at large event times were 40 us
// of the 2 GiB-table microbench (C5 shape).
template <int VEC>
__device__ __forceinline__ void time_enc_vec(float t, int64_t d0, int64_t D, const float* sin_div, const float* cos_div,
                                             float (&te)[VEC]) {
  if ((VEC & 1) == 0 && (d0 & 1) == 0 && d0 + VEC <= D) {
#pragma unroll
    for (int v = 0; v < VEC; v += 2) {
      const int64_t k = (d0 + v) >> 1;
      const float ws = sin_div[k], wc = cos_div[k];
      if (ws == wc) {
        sincosf(t * ws, &te[v], &te[v + 1]);
      } else {
        te[v] = sinf(t * ws);
        te[v + 1] = cosf(t * wc);
      }
    }
    return;
  }
#pragma unroll
  for (int v = 0; v < VEC; ++v) te[v] = d0 + v < D ? time_enc(t, d0 + v, sin_div, cos_div) : 0.f;
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
// Table row segment (VEC consecutive elements, f32 or bf16 storage) as f32.
template <int VEC, typename TT>
__device__ __forceinline__ void load_row(const TT* __restrict__ table, int64_t i, int64_t D, int64_t d0, float (&r)[VEC]) {
  if constexpr (sizeof(TT) == 4) {
    if (VEC == 4 && d0 + 3 < D) {
      const float4 x = *reinterpret_cast<const float4*>(table + i * D + d0);
      r[0] = x.x; r[1] = x.y; r[2] = x.z; r[3] = x.w;
      return;
    }
  } else {
    if (VEC == 4 && d0 + 3 < D) {  // 8-B load of 4 bf16
      const uint2 x = *reinterpret_cast<const uint2*>(table + i * D + d0);
      r[0] = __uint_as_float(x.x << 16), r[1] = __uint_as_float(x.x & 0xffff0000u);
      r[2] = __uint_as_float(x.y << 16), r[3] = __uint_as_float(x.y & 0xffff0000u);
      return;
    }
  }
#pragma unroll
  for (int v = 0; v < VEC; ++v) r[v] = (d0 + v < D) ? to_f32(table[i * D + d0 + v]) : 0.f;
}

template <int VEC, int GMAX, typename TT = float>
__global__ __launch_bounds__(256) void embed_joint_fwd_kernel(esgpt_batch bt, Buckets bk, const TT* __restrict__ table,
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

  // The event's non-padding entries are compacted to the front of the wave's LDS lists in entry order (ballot +
  // prefix popcount), so the gathers below walk only real rows: the same f32 sums in the same order.
  const Entry en = load_entry(bt, e, lane, normalize, V, err);
  const uint64_t below = (1ull << lane) - 1ull;
  const uint64_t live = __ballot(lane < bt.M && en.idx != 0);
  const int n_live = __popcll(live);
  if ((live >> lane) & 1ull) {
    const int pos = __popcll(live & below);
    s_idx[wave][pos] = en.idx;
    for (int g = 0; g < G; ++g) s_w[wave][g][pos] = entry_weight(en, bk, g, ESGPT_BAG_JOINT);
  }
  int n_slive = 0;
  if (use_static) {
    int64_t sidx;
    float swt;
    load_static(bt, b, lane, normalize, V, err, sidx, swt);
    const uint64_t slive = __ballot(lane < bt.S && sidx != 0);
    n_slive = __popcll(slive);
    if ((slive >> lane) & 1ull) {
      const int pos = __popcll(slive & below);
      s_sidx[wave][pos] = sidx;
      s_sw[wave][pos] = swt;
    }
  }
  // each wave reads back only its own LDS lists: a wave-level barrier (LDS accesses of one wave complete in order),
  // not a workgroup one — the four events of a workgroup no longer wait for the slowest one's entry loads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  const int64_t n_chunks = (D + 64 * VEC - 1) / (64 * VEC);
  float t = 0.f;
  bool t_done = !(flags & ESGPT_EMB_TIME);
  for (int64_t c = 0; c < n_chunks; ++c) {
    const int64_t d0 = c * 64 * VEC + lane * VEC;
    float acc[GMAX][VEC];
#pragma unroll
    for (int g = 0; g < GMAX; ++g)
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[g][v] = 0.f;
    // Rows are gathered kGU at a time, every load of a group in flight before the first FMA (one dependent
    // memory round trip per group instead of per row: a gather from a table beyond the caches is latency-bound
    // otherwise). Padding entries (index 0, padding_idx) load row 0 harmlessly and are skipped in the sums, which
    // keep the entry order (the same f32 results bit for bit).
    constexpr int kGU = sizeof(TT) == 4 ? 4 : 8;  // bf16 (large tables beyond the caches): more rows in flight
    float st[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) st[v] = 0.f;
    // whole chunks (D a multiple of 64·VEC, every lane in range): unconditional vector loads in a branch-free loop,
    // so the compiler keeps each group's loads in flight together (a per-lane bounds branch around each load makes
    // it wait for every load in turn: one row per memory round trip)
    auto gather_all = [&](auto whole_c) {
      constexpr bool WHOLE = decltype(whole_c)::value;
      auto gather = [&](float (&r)[VEC], int64_t i) {
        if constexpr (WHOLE && sizeof(TT) == 4) {
          const float4 x = *reinterpret_cast<const float4*>(table + i * D + d0);
          r[0] = x.x; r[1] = x.y; r[2] = x.z; r[3] = x.w;
        } else if constexpr (WHOLE) {
          const uint2 x = *reinterpret_cast<const uint2*>(table + i * D + d0);
          r[0] = __uint_as_float(x.x << 16), r[1] = __uint_as_float(x.x & 0xffff0000u);
          r[2] = __uint_as_float(x.y << 16), r[3] = __uint_as_float(x.y & 0xffff0000u);
        } else {
          load_row<VEC>(table, i, D, d0, r);
        }
      };
      if (valid) {
        for (int m0 = 0; m0 < n_live; m0 += kGU) {
          float r[kGU][VEC];
          int64_t iu[kGU];
#pragma unroll
          for (int u = 0; u < kGU; ++u) iu[u] = s_idx[wave][min(m0 + u, kMaxM - 1)] * (m0 + u < n_live ? 1 : 0);
#pragma unroll
          for (int u = 0; u < kGU; ++u) gather(r[u], iu[u]);
#pragma unroll
          for (int u = 0; u < kGU; ++u) {
            if (iu[u] == 0) continue;  // padding_idx=0 contributes nothing (wave-uniform)
#pragma unroll
            for (int g = 0; g < GMAX; ++g) {
              if (g < G) {
                const float w = s_w[wave][g][m0 + u];
#pragma unroll
                for (int v = 0; v < VEC; ++v) acc[g][v] = fmaf(w, r[u][v], acc[g][v]);
              }
            }
          }
        }
      }
      if (use_static && valid) {
        for (int s0 = 0; s0 < n_slive; s0 += kGU) {
          float r[kGU][VEC];
          int64_t iu[kGU];
#pragma unroll
          for (int u = 0; u < kGU; ++u) iu[u] = s_sidx[wave][min(s0 + u, kMaxM - 1)] * (s0 + u < n_slive ? 1 : 0);
#pragma unroll
          for (int u = 0; u < kGU; ++u) gather(r[u], iu[u]);
#pragma unroll
          for (int u = 0; u < kGU; ++u) {
            if (iu[u] == 0) continue;
            const float w = s_sw[wave][s0 + u];
#pragma unroll
            for (int v = 0; v < VEC; ++v)
              if (d0 + v < D) st[v] = fmaf(w, r[u][v], st[v]);
          }
        }
      }
    };
    if (VEC == 4 && D % (64 * VEC) == 0) gather_all(std::true_type{});
    else gather_all(std::false_type{});
    if (!t_done) {  // the event's time (a prefix sum over the subject's deltas) after the gathers are in flight
      t = event_time(bt, b, l, lane, flags & ESGPT_EMB_TIME_ABS);
      t_done = true;
    }
    double run[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) run[v] = 0.0;
    float te[VEC];
    if (flags & ESGPT_EMB_TIME) time_enc_vec<VEC>(t, d0, D, sin_div, cos_div, te);
#pragma unroll
    for (int g = 0; g < GMAX; ++g) {
      if (g >= G) break;
      float o[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        float x = acc[g][v];
        if (use_static) x = dw * x + sw * st[v];
        if ((flags & ESGPT_EMB_TIME) && g == 0 && d0 + v < D) x = x + te[v];
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
// Event times (esgpt_event_times): t[b][l] = Σ_{j<l} mask[b][j] · Δt[b][j], the reference's time_from_deltas
// (transformer.py:305-313), once per subject instead of once per event inside the input-layer kernels (an O(L)
// prefix per event: 22 % of the C5 microbench at L = 1024). One workgroup per subject: each thread sums a contiguous
// run of events in double, the run totals are scanned in double through LDS, and each event's exclusive prefix is
// rounded to f32 (f32 deltas summed in double, as the event_time prefix: the same values).
// ------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void event_times_kernel(esgpt_batch bt, float* __restrict__ times) {
  __shared__ double s_tot[256];
  const int64_t b = blockIdx.x, L = bt.L;
  const int tid = threadIdx.x;
  const int64_t per = (L + 255) / 256, j0 = tid * per, j1 = min(L, j0 + per);
  const uint8_t* em = bt.event_mask + b * L;
  const float* td = bt.time_delta + b * L;
  double run = 0.0;
  for (int64_t j = j0; j < j1; ++j) run += (double)(em[j] ? td[j] : 0.0f);
  s_tot[tid] = run;
  __syncthreads();
  // inclusive scan of the 256 run totals (Hillis-Steele, double)
  for (int o = 1; o < 256; o <<= 1) {
    const double v = tid >= o ? s_tot[tid - o] : 0.0;
    __syncthreads();
    s_tot[tid] += v;
    __syncthreads();
  }
  double acc = tid > 0 ? s_tot[tid - 1] : 0.0;
  for (int64_t j = j0; j < j1; ++j) {
    times[b * L + j] = (float)acc;
    acc += (double)(em[j] ? td[j] : 0.0f);
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
  // wave-local LDS lists: a wave-level barrier suffices (see embed_joint_fwd_kernel)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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

// dy in OT: f32, or bf16 when it feeds the SPLIT projection's bf16 backward GEMM directly (no separate cast pass)
template <typename OT>
__global__ __launch_bounds__(256) void embed_epilogue_bwd_kernel(esgpt_batch bt, int64_t G, int64_t D,
                                                                 const float* __restrict__ dout, int flags,
                                                                 OT* __restrict__ dy) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = bt.B * bt.L * D;
  if (i >= n) return;
  const int64_t e = i / D, d = i % D;
  const bool valid = bt.event_mask[e] != 0;
  if (flags & ESGPT_EMB_CUMSUM) {
    float run = 0.f;  // reverse cumsum in f32 (autograd of cumsum = flip-cumsum-flip in f32)
    for (int64_t g = G - 1; g >= 0; --g) {
      run += dout[(e * G + g) * D + d];
      dy[(e * G + g) * D + d] = from_f32<OT>(valid ? run : 0.f);
    }
  } else {
    for (int64_t g = 0; g < G; ++g) dy[(e * G + g) * D + d] = from_f32<OT>(valid ? dout[(e * G + g) * D + d] : 0.f);
  }
}

// ------------------------------------------------------------------------------------------------------------
// SPLIT projection operands (data_embedding_layer.py:390-450: cat_proj(cat bags) + num_proj(num bags) as ONE GEMM
// over the concatenated bag columns). prep: W = [cat_w | num_w] in the GEMM dtype (column concatenation),
// bias = a_c·cat_b + a_n·num_b (f32, no fused multiply-add: PyTorch's scalar-times-tensor then add), and the bag
// matrix in the GEMM dtype (bf16; the f32 form reads the bags as they are). post: the grouped backward's dW columns
// back to the two weights, d bias = a·db for each, and dx to f32 for the bag backward.
// ------------------------------------------------------------------------------------------------------------
template <typename LT>
__global__ __launch_bounds__(256) void split_proj_prep_kernel(const float* __restrict__ x, int64_t nx4,
                                                              LT* __restrict__ x_lp, const float* __restrict__ wc,
                                                              const float* __restrict__ wn, int64_t D, int64_t Dc,
                                                              int64_t Dn, const float* __restrict__ bc,
                                                              const float* __restrict__ bn, float a_c, float a_n,
                                                              LT* __restrict__ w_lp, float* __restrict__ bias,
                                                              int64_t nw_blocks) {
  const int64_t Dx = Dc + Dn;
  if ((int64_t)blockIdx.x < nw_blocks) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < D * Dx) {
      const int64_t r = i / Dx, c = i % Dx;
      w_lp[i] = from_f32<LT>(c < Dc ? wc[r * Dc + c] : wn[r * Dn + (c - Dc)]);
    } else if (i < D * Dx + D) {
      const int64_t r = i - D * Dx;
      bias[r] = __fadd_rn(__fmul_rn(a_c, bc[r]), __fmul_rn(a_n, bn[r]));
    }
    return;
  }
  const int64_t j = ((int64_t)blockIdx.x - nw_blocks) * 256 + threadIdx.x;  // 4 bag values per thread
  if (j >= nx4) return;
  const float4 v = reinterpret_cast<const float4*>(x)[j];
  if constexpr (sizeof(LT) == 2) {
    uint2 o;
    o.x = (uint32_t)f32_to_bf16_bits(v.x) | ((uint32_t)f32_to_bf16_bits(v.y) << 16);
    o.y = (uint32_t)f32_to_bf16_bits(v.z) | ((uint32_t)f32_to_bf16_bits(v.w) << 16);
    reinterpret_cast<uint2*>(x_lp)[j] = o;
  }
}

template <typename LT>
__global__ __launch_bounds__(256) void split_proj_post_kernel(const LT* __restrict__ dx_lp, int64_t ndx4,
                                                              float* __restrict__ dx, const float* __restrict__ dw,
                                                              const float* __restrict__ db, int64_t D, int64_t Dc,
                                                              int64_t Dn, float a_c, float a_n, float* __restrict__ dwc,
                                                              float* __restrict__ dwn, float* __restrict__ dbc,
                                                              float* __restrict__ dbn, int64_t nw_blocks) {
  const int64_t Dx = Dc + Dn;
  if ((int64_t)blockIdx.x < nw_blocks) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < D * Dx) {
      const int64_t r = i / Dx, c = i % Dx;
      if (c < Dc) dwc[r * Dc + c] = dw[i];
      else dwn[r * Dn + (c - Dc)] = dw[i];
    } else if (i < D * Dx + D) {
      const int64_t r = i - D * Dx;
      if (dbc) dbc[r] = __fmul_rn(db[r], a_c);
      if (dbn) dbn[r] = __fmul_rn(db[r], a_n);
    }
    return;
  }
  const int64_t j = ((int64_t)blockIdx.x - nw_blocks) * 256 + threadIdx.x;
  if (j >= ndx4) return;
  if constexpr (sizeof(LT) == 2) {
    const uint2 t = reinterpret_cast<const uint2*>(dx_lp)[j];
    reinterpret_cast<float4*>(dx)[j] = make_float4(__uint_as_float(t.x << 16), __uint_as_float(t.x & 0xffff0000u),
                                                   __uint_as_float(t.y << 16), __uint_as_float(t.y & 0xffff0000u));
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

// ------------------------------------------------------------------------------------------------------------
// Deterministic, atomic-free bag backward: a stable counting sort of the slots by vocabulary row, then a segmented
// reduction in slot order (every sum runs in a fixed order: table gradients are bitwise repeatable).
//   K1 bag_block_sort   per block of 1,024 or 4,096 slots: a stable radix sort of the slots by row (slot order within a
//                       row), the block's per-row counts (counts[blk][V]) and every valid slot's (row, rank within
//                       the block's run) in block-sorted order; extra workgroups of the same launch compute the static
//                       SUM_ALL subject sums of dsrc (fixed order)
//   K2 bag_col_prefix   per row: exclusive prefix of counts over blocks (in place) and the row total; the last-arriving
//                       workgroup scans the row totals -> rowptr[0..V] and the list of rows spanning several chunks
//   K3 bag_scatter      (row, block, rank) -> CSR position rowptr[row] + prefix[blk][row] + rank: (row, src, w)
//   K4 bag_reduce       one wave per kChunk CSR entries: rows complete in the chunk are stored; a row continuing
//                       into the previous / next chunk is stored as that chunk's head / tail partial
//   K5 bag_combine      rows spanning chunks (compact lists): tail(c0) + the heads of c0+1 .. c1 in a fixed order —
//                       one wave per short row, 256-head segments of the long rows on 16-wave workgroups summed by
//                       the last-arriving segment; rows without entries stay zero-filled
// ------------------------------------------------------------------------------------------------------------
constexpr int kSortItems = 4;
// Slots per sort block: 256 threads x 4 (1,024) by default; 1,024 x 4 (4,096) when the per-block count rows would be
// large (blocks x V > kBigCounts ints: 21 MB of count rows at C5 -> 5 MB), i.e. a large vocabulary over many slots.
constexpr int64_t kBigCounts = 1 << 21;
static int64_t sort_threads(int64_t n_slots, int64_t V) {
  return cdiv(n_slots, 256 * kSortItems) * V > kBigCounts ? 1024 : 256;
}

// K1: a stable LSD radix sort of the block's (row, local slot) pairs (rocPRIM block_radix_sort: bit-stable, no
// atomics; invalid slots carry the sentinel row V and sort last), run starts by a block max-scan of the positions
// where the row changes, then per valid slot (row, rank within the block's run | local slot << 12) in sorted order
// and, at every run end, the run length into counts[blk][row] (the block zeroes its counts row first; the barriers
// of the sort order those stores before the run-end stores).
// Subject sums of the static SUM_ALL rows (sub[b] = Σ over valid events and levels of dsrc), in two fixed-order
// levels that ride in the sort and prefix launches as extra workgroups (independent of the sort; only the reduce
// reads them):
//   part (sort launch): workgroup (b, chunk of kSubWaveEv events per wave); wave w sums its kSubWaveEv events over
//        every level in (event, level) order, 8 row loads in flight (float4 per lane when D % 4 == 0), every
//        256-column block in turn; wave 0 adds the wave partials in wave order -> sub_part[b][chunk][D];
//   final (prefix launch): workgroup (b, 256-column block) adds the chunk partials in chunk order -> sub[b].
constexpr int kSubWaveEv = 16;
struct SubjArgs {
  const float* dsrc;
  int64_t ld, D, G;
  float* sub;       // [B][D]
  float* sub_part;  // [B][n_sub][D]
  int64_t n_sub;    // chunks per subject
  int64_t nblk;     // workgroups of the launch's main part (sort blocks / prefix blocks)
  int64_t sub_jobs; // B x 256-column blocks (final level)
};

__device__ __forceinline__ bool subj_vec(const SubjArgs& s) {
  return (s.D % 4 == 0) && (s.ld % 4 == 0) && (((uintptr_t)s.dsrc % 16) == 0);
}

__device__ __forceinline__ float4 load_cols4(const float* p, int64_t d0, int64_t D, bool vec) {
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (vec) {
    if (d0 < D) t = *reinterpret_cast<const float4*>(p + d0);
  } else {
    if (d0 < D) t.x = p[d0];
    if (d0 + 1 < D) t.y = p[d0 + 1];
    if (d0 + 2 < D) t.z = p[d0 + 2];
    if (d0 + 3 < D) t.w = p[d0 + 3];
  }
  return t;
}

__device__ __forceinline__ void store_cols4(float* p, int64_t d0, int64_t D, bool vec, float4 r) {
  if (vec) {
    if (d0 < D) *reinterpret_cast<float4*>(p + d0) = r;
  } else {
    if (d0 < D) p[d0] = r.x;
    if (d0 + 1 < D) p[d0 + 1] = r.y;
    if (d0 + 2 < D) p[d0 + 2] = r.z;
    if (d0 + 3 < D) p[d0 + 3] = r.w;
  }
}

template <int kWaves>
__device__ __forceinline__ void subject_part_block(const esgpt_batch& bt, const SubjArgs& s, int64_t job,
                                                   float4* __restrict__ s_part) {
  constexpr int U = 8;
  const int wave = threadIdx.x >> 6, lane = lane_id();
  const int64_t b = job / s.n_sub, c = job % s.n_sub;
  const int64_t l0 = (c * kWaves + wave) * kSubWaveEv, l1 = min<int64_t>(bt.L, l0 + kSubWaveEv);
  const int64_t nrow = l1 > l0 ? (l1 - l0) * s.G : 0;
  const bool vec = subj_vec(s);
  for (int64_t db = 0; db * 256 < s.D; ++db) {
    const int64_t d0 = db * 256 + (int64_t)lane * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t r0 = 0; r0 < nrow; r0 += U) {
      float4 x[U];
      bool on[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // every load issued (clamped row), the masked ones dropped after it
        const int64_t r = min(r0 + u, nrow - 1);
        const int64_t e = b * bt.L + l0 + r / s.G, g = r % s.G;
        on[u] = r0 + u < nrow && bt.event_mask[e];
        x[u] = load_cols4(s.dsrc + (e * s.G + g) * s.ld, d0, s.D, vec);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (on[u]) acc.x += x[u].x, acc.y += x[u].y, acc.z += x[u].z, acc.w += x[u].w;
    }
    s_part[wave * 64 + lane] = acc;
    __syncthreads();
    if (wave == 0) {
      float4 r = s_part[lane];
#pragma unroll
      for (int w = 1; w < kWaves; ++w) {
        const float4 q = s_part[w * 64 + lane];
        r.x += q.x, r.y += q.y, r.z += q.z, r.w += q.w;
      }
      store_cols4(s.sub_part + (b * s.n_sub + c) * s.D, d0, s.D, s.D % 4 == 0, r);
    }
    __syncthreads();  // s_part is rewritten for the next column block
  }
}

// sub[b][cols] = Σ_c sub_part[b][c][cols] in chunk order (one wave per (b, 256-column block))
__device__ __forceinline__ void subject_final_wave(const SubjArgs& s, int64_t job) {
  const int lane = lane_id();
  const int64_t ncb = (s.D + 255) / 256;
  const int64_t b = job / ncb, d0 = (job % ncb) * 256 + (int64_t)lane * 4;
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t c0 = 0; c0 < s.n_sub; c0 += 8) {
    float4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      x[u] = load_cols4(s.sub_part + (b * s.n_sub + min(c0 + u, s.n_sub - 1)) * s.D, d0, s.D, s.D % 4 == 0);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (c0 + u < s.n_sub) r.x += x[u].x, r.y += x[u].y, r.z += x[u].z, r.w += x[u].w;
  }
  store_cols4(s.sub + b * s.D, d0, s.D, s.D % 4 == 0, r);
}

template <int kSortThreads>
__global__ __launch_bounds__(kSortThreads) void bag_block_sort_kernel(BagBwdArgs a, int64_t n_slots, int end_bit,
                                                                      int32_t* __restrict__ counts,
                                                                      int2* __restrict__ sorted,
                                                                      int32_t* __restrict__ n_valid, SubjArgs sj,
                                                                      int32_t* __restrict__ ticket) {
  constexpr int kSortCh = kSortThreads * kSortItems;
  using Sort = rocprim::block_radix_sort<uint32_t, kSortThreads, kSortItems, uint32_t>;
  using Scan = rocprim::block_scan<int, kSortThreads>;
  __shared__ union {
    typename Sort::storage_type sort;
    typename Scan::storage_type scan;
  } tmp;
  // the sort's row keys; in a subject-sum workgroup the wave partials (kSortThreads x 16 B: the same bytes)
  __shared__ __attribute__((aligned(16))) uint32_t s_row[kSortCh];
  __shared__ int s_nv;
  if (blockIdx.x >= sj.nblk) {
    subject_part_block<kSortThreads / 64>(a.bt, sj, blockIdx.x - sj.nblk, reinterpret_cast<float4*>(s_row));
    return;
  }
  const int t = threadIdx.x;
  if (blockIdx.x == 0 && t == 0) *ticket = 0;  // bag_col_prefix's last-arriver ticket (the kernel boundary orders it)
  const int64_t base = (int64_t)blockIdx.x * kSortCh;
  const uint32_t sentinel = (uint32_t)a.V;
  uint32_t key[kSortItems], val[kSortItems];
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const int pos = t * kSortItems + i;  // blocked arrangement: the input order is slot order (stable sort)
    int64_t v = 0, src = 0;
    float w = 0.f;
    key[i] = (base + pos < n_slots && bag_slot(a, base + pos, v, w, src)) ? (uint32_t)v : sentinel;
    val[i] = (uint32_t)pos;
  }
  if (t == 0) s_nv = 0;
  int32_t* col = counts + (int64_t)blockIdx.x * a.V;
  for (int64_t v = t; v < a.V; v += kSortThreads) col[v] = 0;  // this block's counts row (run ends written below)
  Sort().sort(key, val, tmp.sort, 0, end_bit);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) s_row[t * kSortItems + i] = key[i];
  __syncthreads();
  int start[kSortItems];
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const int pos = t * kSortItems + i;
    start[i] = (pos == 0 || s_row[pos - 1] != key[i]) ? pos : 0;
  }
  Scan().inclusive_scan(start, start, tmp.scan, rocprim::maximum<int>());
  int2* out = sorted + base;
#pragma unroll
  for (int i = 0; i < kSortItems; ++i) {
    const int pos = t * kSortItems + i;
    if (key[i] >= sentinel) continue;
    const int rank = pos - start[i];
    out[pos] = make_int2((int)key[i], rank | ((int)val[i] << 12));
    const bool run_end = pos + 1 == kSortCh || s_row[pos + 1] != key[i];
    if (run_end) col[key[i]] = rank + 1;
    if (pos + 1 == kSortCh || s_row[pos + 1] >= sentinel) s_nv = pos + 1;
  }
  __syncthreads();
  if (t == 0) n_valid[blockIdx.x] = s_nv;
}

// counts[blk][v] -> exclusive prefix over blocks (in place); total[v]. Workgroup = 64 rows (lanes) x 16 waves; wave
// w owns the contiguous block segment [w*S, (w+1)*S): segment sums, their exclusive prefix over waves (LDS), then
// the segment rewritten as running prefixes. Loads of a segment are issued 16 at a time.
// The workgroup whose ticket add comes last then runs the row scan (bag_row_scan) over every row total: the totals
// are stored write-through and read back with agent-scope loads (the last-arriver recipe of common.h), so the scan
// needs no launch of its own.
constexpr int kPrefWaves = 16;
constexpr int kCombWaves = 16;
__device__ __forceinline__ void row_scan_body(const int32_t* __restrict__ total, int64_t V, int32_t* __restrict__ rowptr,
                                              int32_t* __restrict__ multi, int32_t* __restrict__ heavy, int chunk);
__global__ __launch_bounds__(1024) void bag_col_prefix_kernel(int32_t* __restrict__ counts, int nblk, int64_t V,
                                                              int32_t* __restrict__ total, float* __restrict__ dtable,
                                                              int64_t D, int32_t* __restrict__ rowptr,
                                                              int32_t* __restrict__ multi, int32_t* __restrict__ heavy,
                                                              int chunk, int32_t* __restrict__ ticket, SubjArgs sj) {
  __shared__ int32_t s_seg[kPrefWaves][64];
  __shared__ int32_t s_tot[64];
  __shared__ int s_last;
  if (blockIdx.x >= sj.nblk) {  // subject sums, second level: one wave per (b, 256-column block)
    const int64_t job = (int64_t)(blockIdx.x - sj.nblk) * kPrefWaves + (threadIdx.x >> 6);
    if (job < sj.sub_jobs) subject_final_wave(sj, job);
    return;
  }
  const int wave = threadIdx.x >> 6, lane = lane_id();
  const int64_t v = (int64_t)blockIdx.x * 64 + lane;
  const bool ok = v < V;
  const int S = (nblk + kPrefWaves - 1) / kPrefWaves;
  const int b0 = wave * S, b1 = min(nblk, b0 + S);
  int32_t sum = 0;
  for (int bb = b0; bb < b1; bb += 16) {
    int32_t c[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) c[u] = (ok && bb + u < b1) ? counts[(int64_t)(bb + u) * V + v] : 0;
#pragma unroll
    for (int u = 0; u < 16; ++u) sum += c[u];
  }
  s_seg[wave][lane] = sum;
  __syncthreads();
  int32_t run = 0;
  for (int w = 0; w < wave; ++w) run += s_seg[w][lane];
  if (wave == kPrefWaves - 1) {
    if (ok) __hip_atomic_store(total + v, run + sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // write-through
    s_tot[lane] = ok ? run + sum : 1;
  }
  __syncthreads();
  // gradient rows of this block's vocabulary rows without entries: zero (the reduce writes every other row)
  const int64_t v0 = (int64_t)blockIdx.x * 64;
  if ((D & 3) == 0) {
    const int64_t q = D / 4;
    for (int64_t i = threadIdx.x; i < 64 * q; i += 1024) {
      const int rr = (int)(i / q);
      if (s_tot[rr] == 0) reinterpret_cast<float4*>(dtable + (v0 + rr) * D)[i % q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  } else {
    for (int64_t i = threadIdx.x; i < 64 * D; i += 1024) {
      const int rr = (int)(i / D);
      if (s_tot[rr] == 0) dtable[(v0 + rr) * D + i % D] = 0.f;
    }
  }
  for (int bb = b0; bb < b1; bb += 16) {
    int32_t c[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) c[u] = (ok && bb + u < b1) ? counts[(int64_t)(bb + u) * V + v] : 0;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (ok && bb + u < b1) counts[(int64_t)(bb + u) * V + v] = run;
      run += c[u];
    }
  }
  if (last_arrival(ticket, (int)sj.nblk, &s_last)) row_scan_body(total, V, rowptr, multi, heavy, chunk);
}

// rowptr[0..V] = exclusive scan of total[0..V) (the 1,024 threads of the last bag_col_prefix workgroup; per-thread
// contiguous segments, fixed order; block scans by rocPRIM), and the compact list of rows whose entries span more
// than one reduce chunk (multi[1 + j], count in multi[0]) and its subset spanning more than kCombWaves + 1 chunks
// (heavy[1 + k], count in heavy[0]). total is read with sc1 loads (written through by other workgroups of the launch).
__device__ __forceinline__ void row_scan_body(const int32_t* __restrict__ total, int64_t V, int32_t* __restrict__ rowptr,
                                              int32_t* __restrict__ multi, int32_t* __restrict__ heavy, int chunk) {
  using Scan = rocprim::block_scan<int, 1024>;
  __shared__ typename Scan::storage_type s_scan;
  constexpr int kReg = 16;  // row totals held in registers per thread (V <= 16,384); larger V re-reads them
  const int tid = threadIdx.x;
  const int64_t per = (V + 1023) / 1024;
  const int64_t lo = tid * per, hi = min(V, lo + per);
  // sc1 buffer loads (write-through data of other XCDs), all issued before any is used
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(total), (short)0, 0x7fffffff, 0x00020000);
  constexpr int kSC1 = 16;
  auto tot = [&](int64_t i) { return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4 * i), 0, kSC1); };
  int32_t t[kReg];
  const bool in_reg = per <= kReg;
  if (in_reg) {
#pragma unroll
    for (int k = 0; k < kReg; ++k) t[k] = lo + k < hi ? tot(lo + k) : 0;
  }
  auto get = [&](int64_t i) { return in_reg ? t[i - lo] : tot(i); };
  int32_t sum = 0, nm = 0, nh = 0;
  if (in_reg) {
#pragma unroll
    for (int k = 0; k < kReg; ++k) sum += t[k];
  } else {
    for (int64_t i = lo; i < hi; ++i) sum += tot(i);
  }
  int32_t base = 0, all = 0;
  Scan().exclusive_scan(sum, base, 0, all, s_scan);
  int32_t run = base;
  for (int64_t i = lo; i < hi; ++i) {
    rowptr[i] = run;
    const int32_t e = run + get(i);
    if (e > run && run / chunk != (e - 1) / chunk) ++nm;
    if (e > run && (e - 1) / chunk - run / chunk > kCombWaves) ++nh;
    run = e;
  }
  if (tid == 1023) rowptr[V] = all;
  __syncthreads();  // s_scan is reused
  int32_t j = 0, n_multi = 0;
  Scan().exclusive_scan(nm, j, 0, n_multi, s_scan);
  __syncthreads();
  int32_t k = 0, n_heavy = 0;
  Scan().exclusive_scan(nh, k, 0, n_heavy, s_scan);
  run = base;
  for (int64_t i = lo; i < hi; ++i) {
    const int32_t e = run + get(i);
    if (e > run && run / chunk != (e - 1) / chunk) multi[1 + j++] = (int32_t)i;
    if (e > run && (e - 1) / chunk - run / chunk > kCombWaves) heavy[1 + k++] = (int32_t)i;
    run = e;
  }
  if (tid == 1023) multi[0] = n_multi, heavy[0] = n_heavy;
}

// CSR entry: (row, src, weight bits, 0); src < 0 = subject-sum row (-1 - b)
__global__ __launch_bounds__(256) void bag_scatter_kernel(BagBwdArgs a, const int2* __restrict__ sorted,
                                                          const int32_t* __restrict__ n_valid,
                                                          const int32_t* __restrict__ prefix,
                                                          const int32_t* __restrict__ rowptr, int4* __restrict__ ent,
                                                          int64_t sort_ch) {
  const int blk = blockIdx.y;
  const int nv = n_valid[blk];
  const int64_t base = (int64_t)blk * sort_ch;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += gridDim.x * blockDim.x) {
    const int2 e = sorted[base + i];
    const int row = e.x, rank = e.y & 4095, slot = e.y >> 12;
    int64_t v, src;
    float w;
    bag_slot(a, base + slot, v, w, src);  // valid by construction: recompute its weight and source row
    const int64_t pos = (int64_t)rowptr[row] + prefix[(int64_t)blk * a.V + row] + rank;
    ent[pos] = make_int4(row, (int)src, __float_as_int(w), 0);
  }
}

// One wave per chunk of kChunk = 64 CSR entries (lane l holds entry l); the wave walks them in groups of kGroup with
// the group's gathered gradient rows in flight together (entry fields wave-uniform via readlane). A run (the entries
// of one row) that starts before / continues after the chunk is written to the chunk's head / tail partial instead
// of the table (a run shared with both sides: the head partial).
constexpr int kChunk = 64;
constexpr int kGroup = 16;

template <int VEC>
__global__ __launch_bounds__(256) void bag_reduce_kernel(const int32_t* __restrict__ rowptr, int64_t V,
                                                         const int4* __restrict__ ent, const float* __restrict__ dsrc,
                                                         int64_t ld, const float* __restrict__ sub, int64_t D,
                                                         float* __restrict__ dtable, float* __restrict__ part_head,
                                                         float* __restrict__ part_tail, int32_t* __restrict__ comb_ticket) {
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int64_t chunk = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const int64_t lo = chunk * kChunk;
  const int64_t n_ent = rowptr[V];
  if (lo >= n_ent) return;
  const int64_t dblocks = (D + 255) / 256;
  if (lane < dblocks) comb_ticket[chunk * dblocks + lane] = 0;  // bag_combine's tickets of the rows starting here
  const int n = (int)min<int64_t>(kChunk, n_ent - lo);
  int32_t my_v = -1, my_s = 0;
  float my_w = 0.f;
  if (lane < n) {
    const int4 x = ent[lo + lane];
    my_v = x.x;
    my_s = x.y;
    my_w = __int_as_float(x.z);
  }
  const int32_t prev_v = lo > 0 ? ent[lo - 1].x : -1;
  const int32_t next_v = lo + n < n_ent ? ent[lo + n].x : -1;
  for (int64_t base = 0; base < D; base += 64 * VEC) {
    const int64_t d0 = base + (int64_t)lane * VEC;
    const bool dok = d0 < D;  // VEC == 4 only when D % 4 == 0
    float acc[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
    int32_t cur = __builtin_amdgcn_readlane(my_v, 0);
    bool head = true;  // the current run starts at the chunk's first entry
    auto flush = [&](bool tail) {
      float* dst;
      if (head && prev_v == cur) dst = part_head + chunk * D;
      else if (tail && next_v == cur) dst = part_tail + chunk * D;
      else dst = dtable + (int64_t)cur * D;
      if (VEC == 4) {
        if (dok) *reinterpret_cast<float4*>(dst + d0) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k)
          if (d0 + k < D) dst[d0 + k] = acc[k];
      }
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
    };
    for (int p0 = 0; p0 < n; p0 += kGroup) {
      float x[kGroup][VEC];
#pragma unroll
      for (int j = 0; j < kGroup; ++j) {
        const int p = min(p0 + j, n - 1);
        const int32_t s = __builtin_amdgcn_readlane(my_s, p);
        const float* row = s >= 0 ? dsrc + (int64_t)s * ld : sub + (int64_t)(-1 - s) * D;
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
          const int32_t v = __builtin_amdgcn_readlane(my_v, p);
          if (v != cur) {
            flush(false);
            cur = v;
            head = false;
          }
          const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_w), p));
#pragma unroll
          for (int k = 0; k < VEC; ++k) acc[k] = fmaf(w, x[j][k], acc[k]);
        }
      }
    }
    flush(true);
  }
}

// Rows spanning several chunks (the compact list of bag_row_scan). Persistent 1024-thread workgroups; per (row,
// 256-column block): wave w sums the row's head partials of chunks c0 + 1 + w, c0 + 17 + w, ... (8 independent
// loads in flight), then wave 0 adds tail(c0) and the 16 wave sums in a fixed order (deterministic whatever the
// row's length: a univariate measurement's row spans ~300 chunks of a C2 batch). Empty rows stay as zero-filled.
// Rows spanning at most kCombWaves + 1 chunks (most of them: 2-3 chunks) are summed by ONE wave each: tail(c0) then
// head(c0 + 1) .. head(c1) in order. Longer rows ("heavy", their own list) are cut into segments of kSeg heads, one
// workgroup per (row, segment, 256-column block) (rows of at most 2·kSeg heads: one segment): wave w sums heads
// first + w, first + w + 16, … of the segment,
// then wave 0 adds the 16 wave sums in wave order. A one-segment row adds them onto its tail and stores the row
// (the same additions in the same order as a short row whose wave w holds at most one head); a longer row stores the
// segment sum write-through over head(first), and the segment whose ticket add comes last (per row and column
// block; tickets zeroed by bag_reduce) adds tail + the segment sums in segment order. Every order is fixed: bitwise
// repeatable. (A C5 batch has one measurement in 31 % of all entries: 1,250 chunks.)
constexpr int kSeg = 256;
constexpr int kCombBlocks = 256;
__global__ __launch_bounds__(1024) void bag_combine_kernel(const int32_t* __restrict__ rowptr,
                                                          const int32_t* __restrict__ multi,
                                                          const int32_t* __restrict__ heavy, int64_t seg_bound,
                                                          int64_t D, float* __restrict__ part_head,
                                                          const float* __restrict__ part_tail,
                                                          int32_t* __restrict__ comb_ticket, float* __restrict__ dtable) {
  __shared__ float4 s_acc[kCombWaves][64];
  const int wave = threadIdx.x >> 6, lane = lane_id();
  const int n_multi = multi[0], n_heavy = heavy[0];
  const int64_t dblocks = (D + 255) / 256;
  const bool vec = (D % 4 == 0);
  auto span = [&](int64_t v, int64_t& c0, int64_t& c1) {
    const int64_t s = rowptr[v], e = rowptr[v + 1];
    c0 = s / kChunk;
    c1 = (e - 1) / kChunk;
  };
  auto add4 = [](float4& r, const float4& h) { r.x += h.x, r.y += h.y, r.z += h.z, r.w += h.w; };
  // short rows: one wave each
  const int64_t nwaves = (int64_t)gridDim.x * kCombWaves;
  for (int64_t j = (int64_t)blockIdx.x * kCombWaves + wave; j < n_multi; j += nwaves) {
    const int64_t v = multi[1 + j];
    int64_t c0, c1;
    span(v, c0, c1);
    if (c1 - c0 > kCombWaves) continue;
    for (int64_t db = 0; db < dblocks; ++db) {
      const int64_t d0 = db * 256 + lane * 4;
      float4 r = load_cols4(part_tail + c0 * D, d0, D, vec);
      for (int64_t u0 = 0; u0 < c1 - c0; u0 += 4) {  // 4 heads in flight (clamped loads, ordered adds)
        float4 h[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) h[u] = load_cols4(part_head + min(c0 + 1 + u0 + u, c1) * D, d0, D, vec);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (c0 + 1 + u0 + u <= c1) add4(r, h[u]);
      }
      store_cols4(dtable + v * D, d0, D, vec, r);
    }
  }
  // heavy rows: one workgroup per (row, segment, 256-column block)
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  constexpr int kSC1 = 16;  // buffer cache policy sc1: write-through stores, L1-bypassing loads
  const __amdgpu_buffer_rsrc_t rs_head = __builtin_amdgcn_make_buffer_rsrc(part_head, (short)0, 0x7fffffff, 0x00020000);
  const int64_t per_row = seg_bound * dblocks;
  // (dealt from the last workgroup down: the short rows of phase 1 sit on the first workgroups)
  for (int64_t job = gridDim.x - 1 - blockIdx.x; job < (int64_t)n_heavy * per_row; job += gridDim.x) {
    const int64_t kk = job / per_row, si = (job % per_row) / dblocks, db = job % dblocks;
    const int64_t v = heavy[1 + kk];
    int64_t c0, c1;
    span(v, c0, c1);
    // up to 2·kSeg heads in one segment (the single-job form: no hand-off), longer rows in kSeg-head segments
    const int64_t nseg = c1 - c0 <= 2 * kSeg ? 1 : (c1 - c0 + kSeg - 1) / kSeg;
    if (si >= nseg) continue;  // workgroup-uniform
    const int64_t first = c0 + 1 + si * kSeg, last = nseg == 1 ? c1 : min(c1, first + kSeg - 1);
    const int64_t d0 = db * 256 + lane * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    constexpr int U = 8;
    for (int64_t cb = first + wave; cb <= last; cb += (int64_t)kCombWaves * U) {
      float4 t[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t c = min(cb + (int64_t)kCombWaves * u, last);
        t[u] = load_cols4(part_head + c * D, d0, D, vec);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (cb + (int64_t)kCombWaves * u <= last) add4(acc, t[u]);
    }
    s_acc[wave][lane] = acc;
    __syncthreads();
    if (wave == 0) {
      if (nseg == 1) {
        float4 r = load_cols4(part_tail + c0 * D, d0, D, vec);
#pragma unroll
        for (int w = 0; w < kCombWaves; ++w) add4(r, s_acc[w][lane]);
        store_cols4(dtable + v * D, d0, D, vec, r);
      } else {
        float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int w = 0; w < kCombWaves; ++w) add4(p, s_acc[w][lane]);
        // segment sum over head(first) (this workgroup's read of it is behind the barrier), write-through
        const int64_t off = first * D + d0;
        if (d0 < D) {
          if (vec) {
            const u32x4 w4 = {__float_as_uint(p.x), __float_as_uint(p.y), __float_as_uint(p.z), __float_as_uint(p.w)};
            __builtin_amdgcn_raw_buffer_store_b128(w4, rs_head, (int)(4 * off), 0, kSC1);
          } else {
            const float pv[4] = {p.x, p.y, p.z, p.w};
            for (int q = 0; q < 4 && d0 + q < D; ++q)
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(pv[q]), rs_head, (int)(4 * (off + q)), 0, kSC1);
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int t = 0;
        if (lane == 0)
          t = __hip_atomic_fetch_add(comb_ticket + c0 * dblocks + db, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = __shfl(t, 0, 64);
        if (t == nseg - 1) {  // last segment of this row and column block: tail + segment sums in segment order
          float4 r = load_cols4(part_tail + c0 * D, d0, D, vec);
          for (int64_t s0 = 0; s0 < nseg; s0 += 4) {
            float4 h[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int64_t o = (c0 + 1 + min(s0 + u, nseg - 1) * kSeg) * D + d0;
              h[u] = make_float4(0.f, 0.f, 0.f, 0.f);
              if (d0 < D) {
                if (vec) {
                  const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs_head, (int)(4 * o), 0, kSC1);
                  h[u] = make_float4(__uint_as_float(x[0]), __uint_as_float(x[1]), __uint_as_float(x[2]),
                                     __uint_as_float(x[3]));
                } else {
                  float hv[4] = {0.f, 0.f, 0.f, 0.f};
                  for (int q = 0; q < 4 && d0 + q < D; ++q)
                    hv[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_head, (int)(4 * (o + q)), 0, kSC1));
                  h[u] = make_float4(hv[0], hv[1], hv[2], hv[3]);
                }
              }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (s0 + u < nseg) add4(r, h[u]);
          }
          store_cols4(dtable + v * D, d0, D, vec, r);
        }
      }
    }
    __syncthreads();  // s_acc is rewritten by the next job
  }
}

struct BagWs {
  int32_t* counts;   // [nblk][V]: block counts, then in-place prefixes over blocks
  int32_t* total;    // [V]
  int32_t* rowptr;   // [V + 1]
  int32_t* multi;    // [1 + V]: count, then the rows spanning several reduce chunks
  int32_t* heavy;    // [1 + V]: count, then the rows spanning more than kCombWaves + 1 chunks
  int32_t* comb_ticket;  // [n_chunks][D / 256]: bag_combine's per-(row, column block) tickets (zeroed by bag_reduce)
  int32_t* n_valid;  // [nblk]
  int2* sorted;      // [nblk * kSortCh]
  int4* ent;         // [n_slots]
  float* part_head;  // [n_chunks][D]
  float* part_tail;  // [n_chunks][D]
  float* sub;        // [B][D]
  float* sub_part;   // [B][n_sub][D]
  int32_t* ticket;   // bag_col_prefix's last-arriver ticket (zeroed by the sort launch)
  int64_t nblk, n_slots, n_chunks, sort_threads, sort_ch;
  size_t bytes;
};

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

static BagWs carve(void* base, const esgpt_batch* bt, int64_t G, int64_t V, int64_t D) {
  BagWs w{};
  w.n_slots = bt->B * bt->L * G * bt->M + bt->B * bt->S;
  w.sort_threads = sort_threads(w.n_slots, V);
  w.sort_ch = w.sort_threads * kSortItems;
  w.nblk = std::max<int64_t>(1, cdiv(w.n_slots, w.sort_ch));
  w.n_chunks = std::max<int64_t>(1, cdiv(w.n_slots, kChunk));
  char* p = (char*)base;
  size_t off = 0;
  auto take = [&](size_t n) {
    char* r = p ? p + off : nullptr;
    off += align_up(n);
    return r;
  };
  w.counts = (int32_t*)take(sizeof(int32_t) * w.nblk * V);
  w.total = (int32_t*)take(sizeof(int32_t) * V);
  w.rowptr = (int32_t*)take(sizeof(int32_t) * (V + 1));
  w.multi = (int32_t*)take(sizeof(int32_t) * (V + 1));
  w.heavy = (int32_t*)take(sizeof(int32_t) * (V + 1));
  w.n_valid = (int32_t*)take(sizeof(int32_t) * w.nblk);
  w.sorted = (int2*)take(sizeof(int2) * w.nblk * w.sort_ch);
  w.ent = (int4*)take(sizeof(int4) * w.n_slots);
  w.part_head = (float*)take(sizeof(float) * w.n_chunks * D);
  w.part_tail = (float*)take(sizeof(float) * w.n_chunks * D);
  w.comb_ticket = (int32_t*)take(sizeof(int32_t) * w.n_chunks * cdiv(D, 256));
  w.sub = (float*)take(sizeof(float) * bt->B * D);
  w.sub_part = (float*)take(sizeof(float) * bt->B * cdiv(bt->L, (w.sort_threads / 64) * kSubWaveEv) * D);
  w.ticket = (int32_t*)take(sizeof(int32_t));
  w.bytes = off;
  return w;
}

}  // namespace

extern "C" {

int esgpt_embed_joint_fwd(const esgpt_batch* batch, const esgpt_buckets* buckets, const float* table, int64_t V,
                          int64_t D, const float* sin_div, const float* cos_div, int flags, float static_w,
                          float dynamic_w, float* out, int32_t* err, void* stream) {
  return esgpt_embed_joint_fwd_ex(batch, buckets, table, ESGPT_F32, V, D, sin_div, cos_div, flags, static_w, dynamic_w,
                                  out, err, stream);
}

int esgpt_event_times(const esgpt_batch* batch, float* times, void* stream) {
  ESGPT_REQUIRE(batch && times && batch->event_mask && batch->time_delta && batch->B >= 0 && batch->L >= 0);
  if (batch->B * batch->L == 0) return ESGPT_OK;
  event_times_kernel<<<(unsigned)batch->B, 256, 0, as_stream(stream)>>>(*batch, times);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_embed_joint_fwd_ex(const esgpt_batch* batch, const esgpt_buckets* buckets, const void* table,
                             int table_dtype, int64_t V, int64_t D, const float* sin_div, const float* cos_div,
                             int flags, float static_w, float dynamic_w, float* out, int32_t* err, void* stream) {
  ESGPT_REQUIRE(batch && table && out && D > 0 && V > 0);
  ESGPT_REQUIRE(table_dtype == ESGPT_F32 || table_dtype == ESGPT_BF16);
  ESGPT_REQUIRE(batch->M <= kMaxM && batch->S <= kMaxM);
  ESGPT_REQUIRE(!(flags & ESGPT_EMB_TIME) || (sin_div && cos_div));
  const Buckets bk = make_buckets(buckets);
  ESGPT_REQUIRE(bk.G >= 1 && bk.G <= kMaxG);
  const int64_t n_ev = batch->B * batch->L;
  if (n_ev == 0) return ESGPT_OK;
  dim3 grid((unsigned)cdiv(n_ev, kWavesPerBlock)), block(256);
  hipStream_t st = as_stream(stream);
  const bool vec4 = (D % 4 == 0) && D >= 256;
#define LAUNCH_J(VEC, GM)                                                                                    \
  do {                                                                                                       \
    if (table_dtype == ESGPT_F32)                                                                            \
      embed_joint_fwd_kernel<VEC, GM, float><<<grid, block, 0, st>>>(*batch, bk, (const float*)table, V, D,   \
                                                                     sin_div, cos_div, flags, static_w,       \
                                                                     dynamic_w, out, err);                    \
    else                                                                                                     \
      embed_joint_fwd_kernel<VEC, GM, bf16><<<grid, block, 0, st>>>(*batch, bk, (const bf16*)table, V, D,     \
                                                                    sin_div, cos_div, flags, static_w,        \
                                                                    dynamic_w, out, err);                     \
  } while (0)
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
  return esgpt_embed_epilogue_bwd_ex(batch, G, D, dout, flags, dy, ESGPT_F32, stream);
}

int esgpt_embed_epilogue_bwd_ex(const esgpt_batch* batch, int64_t G, int64_t D, const float* dout, int flags, void* dy,
                                int dy_dtype, void* stream) {
  ESGPT_REQUIRE(batch && dout && dy && G >= 1 && D > 0 && (dy_dtype == ESGPT_F32 || dy_dtype == ESGPT_BF16));
  const int64_t n = batch->B * batch->L * D;
  if (n == 0) return ESGPT_OK;
  const dim3 grid((unsigned)cdiv(n, 256)), block(256);
  if (dy_dtype == ESGPT_BF16)
    embed_epilogue_bwd_kernel<bf16><<<grid, block, 0, as_stream(stream)>>>(*batch, G, D, dout, flags, (bf16*)dy);
  else
    embed_epilogue_bwd_kernel<float><<<grid, block, 0, as_stream(stream)>>>(*batch, G, D, dout, flags, (float*)dy);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_split_proj_prep(const float* x, int64_t N, void* x_lp, const float* cat_w, const float* num_w, int64_t D,
                          int64_t Dc, int64_t Dn, const float* cat_b, const float* num_b, float a_c, float a_n,
                          void* w_lp, float* bias, int dtype, void* stream) {
  ESGPT_REQUIRE(cat_w && num_w && cat_b && num_b && w_lp && bias && D > 0 && Dc > 0 && Dn > 0 && N >= 0);
  ESGPT_REQUIRE(dtype == ESGPT_F32 || dtype == ESGPT_BF16);
  const int64_t Dx = Dc + Dn;
  const bool conv = dtype == ESGPT_BF16;
  ESGPT_REQUIRE(!conv || (x && x_lp && Dx % 4 == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)x_lp % 8) == 0));
  const int64_t nw = cdiv(D * Dx + D, 256), nx4 = conv ? N * Dx / 4 : 0;
  const dim3 grid((unsigned)(nw + cdiv(nx4, 256))), block(256);
  hipStream_t st = as_stream(stream);
  if (conv)
    split_proj_prep_kernel<bf16><<<grid, block, 0, st>>>(x, nx4, (bf16*)x_lp, cat_w, num_w, D, Dc, Dn, cat_b, num_b,
                                                         a_c, a_n, (bf16*)w_lp, bias, nw);
  else
    split_proj_prep_kernel<float><<<grid, block, 0, st>>>(x, 0, nullptr, cat_w, num_w, D, Dc, Dn, cat_b, num_b, a_c,
                                                          a_n, (float*)w_lp, bias, nw);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_split_proj_post(const void* dx_lp, int64_t N, float* dx, const float* dw, const float* db, int64_t D,
                          int64_t Dc, int64_t Dn, float a_c, float a_n, float* cat_dw, float* num_dw, float* cat_db,
                          float* num_db, int dtype, void* stream) {
  ESGPT_REQUIRE(dw && db && cat_dw && num_dw && D > 0 && Dc > 0 && Dn > 0 && N >= 0);
  ESGPT_REQUIRE(dtype == ESGPT_F32 || dtype == ESGPT_BF16);
  const int64_t Dx = Dc + Dn;
  const bool conv = dtype == ESGPT_BF16 && dx_lp;
  ESGPT_REQUIRE(!conv || (dx && Dx % 4 == 0 && ((uintptr_t)dx % 16) == 0 && ((uintptr_t)dx_lp % 8) == 0));
  const int64_t nw = cdiv(D * Dx + D, 256), ndx4 = conv ? N * Dx / 4 : 0;
  const dim3 grid((unsigned)(nw + cdiv(ndx4, 256))), block(256);
  hipStream_t st = as_stream(stream);
  if (conv)
    split_proj_post_kernel<bf16><<<grid, block, 0, st>>>((const bf16*)dx_lp, ndx4, dx, dw, db, D, Dc, Dn, a_c, a_n,
                                                         cat_dw, num_dw, cat_db, num_db, nw);
  else
    split_proj_post_kernel<float><<<grid, block, 0, st>>>(nullptr, 0, nullptr, dw, db, D, Dc, Dn, a_c, a_n, cat_dw,
                                                          num_dw, cat_db, num_db, nw);
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
  ESGPT_REQUIRE(batch && dsrc && dtable && D > 0 && V > 0 && V < (1ll << 31) - 1);
  const Buckets bk = make_buckets(buckets);
  ESGPT_REQUIRE(bk.G >= 1 && bk.G <= kMaxG);
  BagWs w = carve(workspace, batch, bk.G, V, D);
  ESGPT_REQUIRE(workspace && workspace_bytes >= w.bytes);
  ESGPT_REQUIRE(w.n_slots < (1ll << 31) && batch->B * batch->L * bk.G < (1ll << 31));  // int32 CSR fields
  hipStream_t st = as_stream(stream);
  BagBwdArgs a{*batch, bk, selector, flags, dyn_scale, static_scale, V};
  // the subject sums (static SUM_ALL) ride in the sort and prefix launches as extra workgroups
  const bool subj = (flags & ESGPT_EMB_STATIC) && batch->S > 0 && selector != ESGPT_BAG_NUM && batch->B > 0;
  const int64_t n_sub = cdiv(batch->L, (w.sort_threads / 64) * kSubWaveEv);
  SubjArgs sj{dsrc, ld, D, bk.G, w.sub, w.sub_part, n_sub, w.nblk, batch->B * cdiv(D, 256)};
  const int64_t n_part = subj ? batch->B * n_sub : 0;
  // (no zero-fill launches: the sort blocks zero their counts rows, bag_col_prefix the table rows without entries)
  int end_bit = 1;
  while (end_bit < 32 && (V >> end_bit) != 0) ++end_bit;  // keys 0 .. V (the sentinel) fit in end_bit bits
  const unsigned g_sort = (unsigned)(w.nblk + n_part);
  if (w.sort_threads == 1024)
    bag_block_sort_kernel<1024><<<g_sort, 1024, 0, st>>>(a, w.n_slots, end_bit, w.counts, w.sorted, w.n_valid, sj,
                                                         w.ticket);
  else
    bag_block_sort_kernel<256><<<g_sort, 256, 0, st>>>(a, w.n_slots, end_bit, w.counts, w.sorted, w.n_valid, sj,
                                                       w.ticket);
  // column prefixes, then (last-arriving workgroup) the row scan; extra workgroups finish the subject sums
  SubjArgs sp = sj;
  sp.nblk = cdiv(V, 64);
  const int64_t n_fin = subj ? cdiv(sj.sub_jobs, kPrefWaves) : 0;
  bag_col_prefix_kernel<<<(unsigned)(sp.nblk + n_fin), 1024, 0, st>>>(w.counts, (int)w.nblk, V, w.total, dtable, D,
                                                                      w.rowptr, w.multi, w.heavy, kChunk, w.ticket, sp);
  bag_scatter_kernel<<<dim3(4, (unsigned)w.nblk), 256, 0, st>>>(a, w.sorted, w.n_valid, w.counts, w.rowptr, w.ent,
                                                                 w.sort_ch);
  // The number of entries is data-dependent (not known on the host without a sync): launch for the upper bound;
  // chunks past rowptr[V] exit immediately.
  const unsigned g_red = (unsigned)cdiv(w.n_chunks, kWavesPerBlock);
  if (D % 4 == 0 && D >= 256 && ld % 4 == 0 && ((uintptr_t)dsrc % 16) == 0 && ((uintptr_t)dtable % 16) == 0)
    bag_reduce_kernel<4><<<g_red, 256, 0, st>>>(w.rowptr, V, w.ent, dsrc, ld, w.sub, D, dtable, w.part_head,
                                                w.part_tail, w.comb_ticket);
  else
    bag_reduce_kernel<1><<<g_red, 256, 0, st>>>(w.rowptr, V, w.ent, dsrc, ld, w.sub, D, dtable, w.part_head,
                                                w.part_tail, w.comb_ticket);
  bag_combine_kernel<<<kCombBlocks, 1024, 0, st>>>(w.rowptr, w.multi, w.heavy, cdiv(w.n_chunks, kSeg) + 1, D,
                                                   w.part_head, w.part_tail, w.comb_ticket, dtable);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

}  // extern "C"
