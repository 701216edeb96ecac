// Host-side batch producer for the training step: PytorchDataset.collate (EventStream/data/pytorch_dataset.py:
// 527-701) restated over flat ragged arrays — the DL_reps parquet columns as Arrow buffers, zero copy — into
// caller-allocated (pinned) host buffers that one asynchronous copy moves to HBM.
//
// Subject b of the batch owns events ev_start[b] .. ev_start[b] + ev_count[b] - 1 of the flat event arrays (a
// window: subsequence sampling needs no copy), event e owns elements el_off[e] .. el_off[e+1] - 1 of the flat
// element arrays, and static elements st_start[b] .. st_start[b] + st_count[b] - 1.
// Semantics of the reference collate, restated:
//   * L = max events, M = max elements per event over the batch (no element at all: the reference's ValueError),
//     S = max static elements;
//   * time_delta NaN <=> padded event (the reference derives event_mask from its NaN padding), stored as 0;
//   * values f64 -> f32, dynamic_values_mask = !isnan(value), masked values stored as 0;
//   * padded slots: index 0, measurement 0, value 0, mask false; sequence padding right or left, static on the right.
// Indices are copied as int64 exactly (the reference round-trips them through float32, exact below 2^24).
// Subjects are split over n_threads host threads.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/esgpt_amd.h"

namespace {

struct Args {
  int64_t B, L, M, S;
  const int64_t* ev_start;
  const int64_t* ev_count;
  const double* time_delta;
  const int64_t* el_off;
  const int64_t* idx;
  const int64_t* meas;
  const double* vals;
  const int64_t* st_start;
  const int64_t* st_count;
  const int64_t* st_idx;
  const int64_t* st_meas;
  int left;
  uint8_t* event_mask;
  float* td;
  int64_t* dyn_idx;
  int64_t* dyn_meas;
  float* dyn_vals;
  uint8_t* dyn_vmask;
  int64_t* st_idx_out;
  int64_t* st_meas_out;
};

void collate_subjects(const Args& a, int64_t b0, int64_t b1) {
  const int64_t L = a.L, M = a.M, S = a.S;
  for (int64_t b = b0; b < b1; ++b) {
    std::memset(a.event_mask + b * L, 0, L);
    std::memset(a.td + b * L, 0, sizeof(float) * L);
    std::memset(a.dyn_idx + b * L * M, 0, sizeof(int64_t) * L * M);
    std::memset(a.dyn_meas + b * L * M, 0, sizeof(int64_t) * L * M);
    std::memset(a.dyn_vals + b * L * M, 0, sizeof(float) * L * M);
    std::memset(a.dyn_vmask + b * L * M, 0, L * M);
    const int64_t n = a.ev_count[b];
    const int64_t pos0 = a.left ? L - n : 0;
    for (int64_t j = 0; j < n; ++j) {
      const int64_t e = a.ev_start[b] + j, l = pos0 + j;
      const float t = (float)a.time_delta[e];
      const bool ev = !std::isnan(t);
      a.event_mask[b * L + l] = ev;
      a.td[b * L + l] = ev ? t : 0.f;
      const int64_t k0 = a.el_off[e], nk = a.el_off[e + 1] - k0;
      const int64_t o = (b * L + l) * M;
      std::memcpy(a.dyn_idx + o, a.idx + k0, sizeof(int64_t) * nk);
      std::memcpy(a.dyn_meas + o, a.meas + k0, sizeof(int64_t) * nk);
      for (int64_t k = 0; k < nk; ++k) {
        const float v = (float)a.vals[k0 + k];
        const bool ok = !std::isnan(v);
        a.dyn_vals[o + k] = ok ? v : 0.f;
        a.dyn_vmask[o + k] = ok;
      }
    }
    if (S > 0) {
      std::memset(a.st_idx_out + b * S, 0, sizeof(int64_t) * S);
      std::memset(a.st_meas_out + b * S, 0, sizeof(int64_t) * S);
      const int64_t ns = a.st_count ? a.st_count[b] : 0;
      if (ns > 0) {
        std::memcpy(a.st_idx_out + b * S, a.st_idx + a.st_start[b], sizeof(int64_t) * ns);
        std::memcpy(a.st_meas_out + b * S, a.st_meas + a.st_start[b], sizeof(int64_t) * ns);
      }
    }
  }
}

}  // namespace

extern "C" {

int esgpt_collate_shape(int64_t B, const int64_t* ev_start, const int64_t* ev_count, const int64_t* el_off,
                        const int64_t* st_count, int64_t* L, int64_t* M, int64_t* S) {
  if (B < 0 || (B > 0 && !(ev_start && ev_count && el_off)) || !L || !M || !S) return ESGPT_ERR_INVALID_ARG;
  int64_t l = 0, m = 0, s = 0;
  for (int64_t b = 0; b < B; ++b) {
    if (ev_count[b] < 0 || ev_start[b] < 0) return ESGPT_ERR_INVALID_ARG;
    l = std::max(l, ev_count[b]);
    for (int64_t e = ev_start[b]; e < ev_start[b] + ev_count[b]; ++e) m = std::max(m, el_off[e + 1] - el_off[e]);
    if (st_count) s = std::max(s, st_count[b]);
  }
  *L = l;
  *M = m;
  *S = s;
  return m > 0 ? ESGPT_OK : ESGPT_ERR_INVALID_ARG;  // "Batch has no dynamic measurements!"
}

int esgpt_collate(int64_t B, const int64_t* ev_start, const int64_t* ev_count, const double* time_delta,
                  const int64_t* el_off, const int64_t* idx, const int64_t* meas, const double* vals,
                  const int64_t* st_start, const int64_t* st_count, const int64_t* st_idx, const int64_t* st_meas,
                  int64_t L, int64_t M, int64_t S, int padding_left, uint8_t* event_mask, float* time_delta_out,
                  int64_t* dyn_idx, int64_t* dyn_meas, float* dyn_vals, uint8_t* dyn_vmask, int64_t* st_idx_out,
                  int64_t* st_meas_out, int n_threads) {
  if (B < 0 || L < 0 || M < 0 || S < 0) return ESGPT_ERR_INVALID_ARG;
  if (B == 0) return ESGPT_OK;
  if (!(ev_start && ev_count && time_delta && el_off && idx && meas && vals && event_mask && time_delta_out &&
        dyn_idx && dyn_meas && dyn_vals && dyn_vmask))
    return ESGPT_ERR_INVALID_ARG;
  if (S > 0 && !(st_idx_out && st_meas_out && (!st_count || (st_start && st_idx && st_meas))))
    return ESGPT_ERR_INVALID_ARG;
  for (int64_t b = 0; b < B; ++b) {  // every subject fits the output shape
    if (ev_count[b] < 0 || ev_count[b] > L || (st_count && st_count[b] > S)) return ESGPT_ERR_INVALID_ARG;
    for (int64_t e = ev_start[b]; e < ev_start[b] + ev_count[b]; ++e)
      if (el_off[e + 1] - el_off[e] > M || el_off[e + 1] < el_off[e]) return ESGPT_ERR_INVALID_ARG;
  }
  const Args a{B,        L,       M,           S,        ev_start,       ev_count,   time_delta, el_off,
               idx,      meas,    vals,        st_start, st_count,       st_idx,     st_meas,    padding_left,
               event_mask, time_delta_out, dyn_idx, dyn_meas, dyn_vals, dyn_vmask, st_idx_out, st_meas_out};
  const int64_t nt = std::max<int64_t>(1, std::min<int64_t>(n_threads, B));
  const int64_t per = (B + nt - 1) / nt;
  std::vector<std::thread> pool;
  for (int64_t t = 1; t < nt; ++t) {
    const int64_t b0 = t * per, b1 = std::min(B, b0 + per);
    if (b0 < b1) pool.emplace_back(collate_subjects, std::cref(a), b0, b1);
  }
  collate_subjects(a, 0, std::min(B, per));
  for (auto& th : pool) th.join();
  return ESGPT_OK;
}

}  // extern "C"
