// Version / device probes of the C ABI, the zero-fill helper and the fused AdamW step.
#include <math.h>
#include <string.h>

#include "common.h"

namespace esgpt {

namespace {
// 16-byte stores over the 16-B aligned body, byte stores for the unaligned head / tail.
__global__ __launch_bounds__(256) void zero_kernel(uint8_t* __restrict__ p, size_t head, size_t n16, size_t tail) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t j = i; j < head; j += stride) p[j] = 0;
  uint4* body = reinterpret_cast<uint4*>(p + head);
  for (size_t j = i; j < n16; j += stride) body[j] = make_uint4(0u, 0u, 0u, 0u);
  uint8_t* t = p + head + 16 * n16;
  for (size_t j = i; j < tail; j += stride) t[j] = 0;
}
// AdamW (torch.optim.AdamW, decoupled weight decay) over a table of tensors. Block b updates elements
// [start, start + kAdamChunk) of tensor (blocks[b] >> 40) where start = blocks[b] & (2^40 - 1).
constexpr int kAdamChunk = 4096;

__global__ __launch_bounds__(256) void adamw_kernel(const esgpt_adam_tensor* __restrict__ table,
                                                    const int64_t* __restrict__ blocks, float lr, float beta1,
                                                    float beta2, float eps, float wd, float step_size_all,
                                                    float bc2_sqrt_all, const float* __restrict__ per_tensor,
                                                    const int32_t* __restrict__ err, const float* __restrict__ lr_dev) {
  // A data-dependent error raised by this step's forward (bad embedding index, NaN TTE log-likelihood, subject
  // without an observed TTE) leaves the parameters untouched: the reference raises before its optimizer step. The
  // gate also holds while an EARLIER step's flags are pending in the sticky word (err[1], set by the next step's
  // first launch until the host has read and cleared the block): a step queued behind a failed one is discarded.
  if (err != nullptr && (err[0] | err[1]) != 0) return;
  const int64_t e = blocks[blockIdx.x];
  const int64_t ti = e >> 40;
  const esgpt_adam_tensor t = table[ti];
  // per-parameter step counts (torch keeps one `step` per parameter): (lr / bc1, sqrt(bc2)) per tensor
  const float step_size = per_tensor ? per_tensor[2 * ti] : step_size_all;
  const float bc2_sqrt = per_tensor ? per_tensor[2 * ti + 1] : bc2_sqrt_all;
  const int64_t start = e & ((1ll << 40) - 1);
  const int64_t end = start + kAdamChunk < t.n ? start + kAdamChunk : t.n;
  const float decay = 1.f - (lr_dev ? *lr_dev : lr) * wd;
  auto upd = [&](float& p, float g, float& m, float& v) {
    p *= decay;
    m = beta1 * m + (1.f - beta1) * g;
    v = beta2 * v + (1.f - beta2) * g * g;
    p -= step_size * m / (sqrtf(v) / bc2_sqrt + eps);
  };
  const bool vec = ((reinterpret_cast<uintptr_t>(t.p) | reinterpret_cast<uintptr_t>(t.g) |
                     reinterpret_cast<uintptr_t>(t.m) | reinterpret_cast<uintptr_t>(t.v)) & 15) == 0;
  if (vec) {
    const int64_t n4 = (end - start) / 4;
    for (int64_t j = threadIdx.x; j < n4; j += blockDim.x) {
      const int64_t i = start + 4 * j;
      float4 p = *reinterpret_cast<float4*>(t.p + i);
      const float4 g = *reinterpret_cast<const float4*>(t.g + i);
      float4 m = *reinterpret_cast<float4*>(t.m + i);
      float4 v = *reinterpret_cast<float4*>(t.v + i);
      upd(p.x, g.x, m.x, v.x);
      upd(p.y, g.y, m.y, v.y);
      upd(p.z, g.z, m.z, v.z);
      upd(p.w, g.w, m.w, v.w);
      *reinterpret_cast<float4*>(t.p + i) = p;
      *reinterpret_cast<float4*>(t.m + i) = m;
      *reinterpret_cast<float4*>(t.v + i) = v;
    }
    for (int64_t i = start + 4 * n4 + threadIdx.x; i < end; i += blockDim.x) upd(t.p[i], t.g[i], t.m[i], t.v[i]);
  } else {
    for (int64_t i = start + threadIdx.x; i < end; i += blockDim.x) upd(t.p[i], t.g[i], t.m[i], t.v[i]);
  }
}

// The step's learning rate and per-tensor bias corrections on the device (esgpt_adamw_prepare), so that the
// optimizer step needs no host arguments and replays inside a HIP graph. One workgroup: counters[t] (the 1-based
// step of parameter t after this step) for the active tensors, counters[n_params] = the schedule's step; gated by
// the same error condition as the update, so a failed (or discarded) step advances nothing.
__global__ __launch_bounds__(256) void adamw_prepare_kernel(int64_t* __restrict__ counters,
                                                            const int32_t* __restrict__ active, int n_active,
                                                            int n_params, esgpt_lr_schedule sc, double beta1,
                                                            double beta2, float* __restrict__ per_tensor,
                                                            float* __restrict__ lr_out,
                                                            const int32_t* __restrict__ err,
                                                            const float* __restrict__ copy_src, int n_copy,
                                                            float* __restrict__ ring,
                                                            float* const* __restrict__ ring_tab,
                                                            int64_t* __restrict__ ring_ctr, int64_t ring_len,
                                                            int32_t* __restrict__ host_words) {
  // The step's hand-off entry riding in this launch, whatever the error state: copy_src (the replayed step's loss,
  // which the next replay overwrites) and the error block's four words, into ring entry ring_ctr % ring_len (stride
  // round_up(n_copy, 4) + 4 floats; the error words 16-B aligned at round_up(n_copy, 4)); the counter then advances.
  // With ring_tab the entries are separate allocations reached through a device table of ring_len pointers (the
  // caller may swap an entry's allocation between launches: a returned loss the caller still holds is never
  // overwritten). host_words (coherent, mapped host memory, ring_len x 4 words): the error words also land there,
  // so the host reads them after the step's event without a D2H copy launch.
  if (ring != nullptr || ring_tab != nullptr) {
    const int body = (n_copy + 3) & ~3;
    const int64_t slot = ring_ctr ? *ring_ctr % ring_len : 0;
    float* e = ring_tab ? ring_tab[slot] : ring + slot * (int64_t)(body + 4);
    for (int i = threadIdx.x; i < n_copy; i += blockDim.x) e[i] = copy_src[i];
    if (threadIdx.x < 4) {
      int32_t* ew = reinterpret_cast<int32_t*>(e + body);
      const int32_t v = err ? err[threadIdx.x] : 0;
      ew[threadIdx.x] = v;
      if (host_words) host_words[slot * 4 + threadIdx.x] = v;
    }
    __syncthreads();  // every thread has read the counter before it advances
    if (ring_ctr && threadIdx.x == 0) *ring_ctr += 1;
  }
  if (err != nullptr && (err[0] | err[1]) != 0) return;
  const int64_t s = counters[n_params];  // LambdaLR: the k-th optimizer step uses lambda(k - 1)
  double f = 1.0;
  if (sc.kind == 1) {  // transformers.get_polynomial_decay_schedule_with_warmup (train.poly_decay_lambda)
    if (s < sc.warmup) f = (double)s / (double)(sc.warmup > 1 ? sc.warmup : 1);
    else if (s > sc.total) f = sc.end_lr / sc.init_lr;
    else if (sc.total == sc.warmup) f = sc.end_lr / sc.init_lr;  // s == total == warmup: the reference's lambda
                                                                   // divides 0 / 0 there (the host raises first)
    else f = ((sc.init_lr - sc.end_lr) * pow(1.0 - (double)(s - sc.warmup) / (double)(sc.total - sc.warmup), sc.power) +
              sc.end_lr) / sc.init_lr;
  }
  const double lr = sc.init_lr * f;
  for (int t = threadIdx.x; t < n_active; t += blockDim.x) {
    const int i = active[t];
    const int64_t c = counters[i] + 1;
    counters[i] = c;
    per_tensor[2 * t] = (float)(lr / (1.0 - pow(beta1, (double)c)));
    per_tensor[2 * t + 1] = (float)sqrt(1.0 - pow(beta2, (double)c));
  }
  __syncthreads();  // every wave has read counters[n_params] before it advances
  if (threadIdx.x == 0) {
    counters[n_params] = s + 1;
    *lr_out = (float)lr;
  }
}

// Parameter packing (esgpt_pack): one workgroup per kPackChunk elements of one segment; segment descriptors and
// their first-chunk prefix are kernel arguments (kPackSegs per launch).
constexpr int kPackSegs = 48;
constexpr int kPackChunk = 2048;  // 256 threads x 8 elements
struct PackArgs {
  esgpt_pack_seg s[kPackSegs];
  int64_t c0[kPackSegs + 1];
  int n;
};

__global__ __launch_bounds__(256) void pack_kernel(const PackArgs a) {
  const int64_t blk = blockIdx.x;
  int s = 0;
  while (s + 1 < a.n && a.c0[s + 1] <= blk) ++s;  // workgroup-uniform
  const esgpt_pack_seg g = a.s[s];
  const int64_t e0 = (blk - a.c0[s]) * kPackChunk + 8 * (int64_t)threadIdx.x;
  if (e0 >= g.n_pad) return;
  float v[8];
  if (g.src && e0 + 8 <= g.n && (reinterpret_cast<uintptr_t>(g.src) & 15) == 0) {
    const float4 x = *reinterpret_cast<const float4*>(g.src + e0), y = *reinterpret_cast<const float4*>(g.src + e0 + 4);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (g.src && e0 + j < g.n) ? g.src[e0 + j] : 0.f;
  }
  const bool whole = e0 + 8 <= g.n_pad;
  if (g.dst_dtype == ESGPT_BF16) {
    uint16_t* d = reinterpret_cast<uint16_t*>(g.dst) + e0;
    if (whole && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
      uint4 w;
      w.x = (uint32_t)f32_to_bf16_bits(v[0]) | ((uint32_t)f32_to_bf16_bits(v[1]) << 16);
      w.y = (uint32_t)f32_to_bf16_bits(v[2]) | ((uint32_t)f32_to_bf16_bits(v[3]) << 16);
      w.z = (uint32_t)f32_to_bf16_bits(v[4]) | ((uint32_t)f32_to_bf16_bits(v[5]) << 16);
      w.w = (uint32_t)f32_to_bf16_bits(v[6]) | ((uint32_t)f32_to_bf16_bits(v[7]) << 16);
      *reinterpret_cast<uint4*>(d) = w;
    } else {
      for (int j = 0; j < 8 && e0 + j < g.n_pad; ++j) d[j] = f32_to_bf16_bits(v[j]);
    }
  } else {
    float* d = reinterpret_cast<float*>(g.dst) + e0;
    if (whole && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
      *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      for (int j = 0; j < 8 && e0 + j < g.n_pad; ++j) d[j] = v[j];
    }
  }
}
}  // namespace

hipError_t zero_async(void* p, size_t bytes, hipStream_t st) {
  if (bytes == 0) return hipSuccess;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  size_t head = (16 - (a & 15)) & 15;
  if (head > bytes) head = bytes;
  const size_t n16 = (bytes - head) / 16, tail = bytes - head - 16 * n16;
  const size_t work = n16 > head + tail ? n16 : head + tail;
  const unsigned grid = (unsigned)(work / 256 + 1 < 2048 ? work / 256 + 1 : 2048);
  zero_kernel<<<grid, 256, 0, st>>>(reinterpret_cast<uint8_t*>(p), head, n16, tail);
  return hipGetLastError();
}

// bank[i] = counter + i (i < slots), then counter += slots: one block (every thread reads the counter before the
// barrier; thread 0 advances it after).
// With `err` (the step's error block, 16 bytes: int32 flags, int32 sticky word, int64 max bad index) the same launch
// starts the step's own flags: the previous step's flags are OR-ed into the sticky word (which keeps every later
// AdamW a no-op until the host has read and cleared the block), then the flags are zeroed (and the max bad index,
// unless an error is pending: it belongs to that error's message).
__global__ __launch_bounds__(256) void seed_bank_kernel(int64_t* __restrict__ counter, int64_t* __restrict__ bank,
                                                        int64_t slots, int32_t* __restrict__ err) {
  const int64_t c = *counter;
  for (int64_t i = threadIdx.x; i < slots; i += blockDim.x) bank[i] = c + i;
  if (err && threadIdx.x == 0) {
    const int32_t sticky = err[1] | err[0];
    err[1] = sticky;
    err[0] = 0;
    if (sticky == 0) *reinterpret_cast<int64_t*>(err + 2) = 0;  // kept while an error is pending (its message)
  }
  __syncthreads();
  if (threadIdx.x == 0) *counter = c + slots;
}

}  // namespace esgpt

extern "C" {

int esgpt_seed_bank(int64_t* counter, int64_t* bank, int64_t slots, void* stream) {
  return esgpt_step_begin(counter, bank, slots, nullptr, stream);
}

int esgpt_step_begin(int64_t* counter, int64_t* bank, int64_t slots, int32_t* err, void* stream) {
  ESGPT_REQUIRE(counter && bank && slots > 0 && (uintptr_t)err % 8 == 0);
  esgpt::seed_bank_kernel<<<1, 256, 0, esgpt::as_stream(stream)>>>(counter, bank, slots, err);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

const char* esgpt_version(void) { return "eventstreamgpt_amd 0.1.0 (gfx950)"; }

int64_t esgpt_adamw_chunk(void) { return esgpt::kAdamChunk; }

int esgpt_adamw(const esgpt_adam_tensor* table, const int64_t* blocks, int64_t n_blocks, float lr, float beta1,
                float beta2, float eps, float weight_decay, int64_t step, const float* per_tensor,
                const int32_t* err, void* stream) {
  ESGPT_REQUIRE(table && blocks && n_blocks >= 0 && (step >= 1 || per_tensor != nullptr));
  if (n_blocks == 0) return ESGPT_OK;
  const double s = step >= 1 ? (double)step : 1.0;
  const double bc1 = 1.0 - pow((double)beta1, s), bc2 = 1.0 - pow((double)beta2, s);
  esgpt::adamw_kernel<<<(unsigned)n_blocks, 256, 0, esgpt::as_stream(stream)>>>(table, blocks, lr, beta1, beta2, eps,
                                                                   weight_decay, (float)(lr / bc1),
                                                                   (float)sqrt(bc2), per_tensor, err, nullptr);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_adamw_prepare(int64_t* counters, const int32_t* active, int n_active, int n_params,
                        const esgpt_lr_schedule* sched, double beta1, double beta2, float* per_tensor, float* lr_out,
                        const int32_t* err, void* stream) {
  return esgpt_adamw_prepare_ex(counters, active, n_active, n_params, sched, beta1, beta2, per_tensor, lr_out, err,
                                nullptr, 0, nullptr, nullptr, 1, stream);
}

static int adamw_prepare_impl(int64_t* counters, const int32_t* active, int n_active, int n_params,
                              const esgpt_lr_schedule* sched, double beta1, double beta2, float* per_tensor,
                              float* lr_out, const int32_t* err, const float* copy_src, int64_t n_copy, float* ring,
                              float* const* ring_tab, int64_t* ring_ctr, int64_t ring_len, int32_t* host_words,
                              void* stream) {
  ESGPT_REQUIRE(counters && sched && per_tensor && lr_out && n_active >= 0 && n_params >= 0);
  ESGPT_REQUIRE(n_active == 0 || active);
  ESGPT_REQUIRE(!(ring && ring_tab));
  ESGPT_REQUIRE(n_copy >= 0 && n_copy <= 1024 && ring_len >= 1 && (n_copy == 0 || (copy_src && (ring || ring_tab))) &&
                (ring || ring_tab || !ring_ctr) && (reinterpret_cast<uintptr_t>(ring) & 15) == 0 &&
                (reinterpret_cast<uintptr_t>(ring_tab) & 7) == 0 && (!host_words || ring_ctr));
  ESGPT_REQUIRE(sched->kind == 0 || (sched->kind == 1 && sched->init_lr > sched->end_lr && sched->total >= sched->warmup));
  esgpt::adamw_prepare_kernel<<<1, 256, 0, esgpt::as_stream(stream)>>>(counters, active, n_active, n_params, *sched,
                                                                       beta1, beta2, per_tensor, lr_out, err,
                                                                       copy_src, (int)n_copy, ring, ring_tab,
                                                                       ring_ctr, ring_len, host_words);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_adamw_prepare_ex(int64_t* counters, const int32_t* active, int n_active, int n_params,
                           const esgpt_lr_schedule* sched, double beta1, double beta2, float* per_tensor,
                           float* lr_out, const int32_t* err, const float* copy_src, int64_t n_copy, float* ring,
                           int64_t* ring_ctr, int64_t ring_len, void* stream) {
  return adamw_prepare_impl(counters, active, n_active, n_params, sched, beta1, beta2, per_tensor, lr_out, err,
                            copy_src, n_copy, ring, nullptr, ring_ctr, ring_len, nullptr, stream);
}

int esgpt_adamw_prepare_tab(int64_t* counters, const int32_t* active, int n_active, int n_params,
                            const esgpt_lr_schedule* sched, double beta1, double beta2, float* per_tensor,
                            float* lr_out, const int32_t* err, const float* copy_src, int64_t n_copy,
                            float* const* ring_tab, int64_t* ring_ctr, int64_t ring_len, int32_t* host_words,
                            void* stream) {
  ESGPT_REQUIRE(ring_tab != nullptr);
  return adamw_prepare_impl(counters, active, n_active, n_params, sched, beta1, beta2, per_tensor, lr_out, err,
                            copy_src, n_copy, nullptr, ring_tab, ring_ctr, ring_len, host_words, stream);
}

// Coherent, device-mapped host memory for esgpt_adamw_prepare_tab's host_words (GPU stores reach host memory
// without a cache flush or a copy launch; the host reads them once the step's event has completed).
int esgpt_host_words_alloc(int64_t bytes, void** host, void** dev) {
  ESGPT_REQUIRE(bytes > 0 && host && dev);
  void* p = nullptr;
  if (hipHostMalloc(&p, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess || !p)
    return ESGPT_ERR_LAUNCH;
  memset(p, 0, (size_t)bytes);
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || !d) {
    (void)hipHostFree(p);
    return ESGPT_ERR_LAUNCH;
  }
  *host = p;
  *dev = d;
  return ESGPT_OK;
}

int esgpt_host_words_free(void* host) {
  if (host == nullptr) return ESGPT_OK;
  return hipHostFree(host) == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
}

int esgpt_adamw_dev(const esgpt_adam_tensor* table, const int64_t* blocks, int64_t n_blocks, const float* lr_dev,
                    float beta1, float beta2, float eps, float weight_decay, const float* per_tensor,
                    const int32_t* err, void* stream) {
  ESGPT_REQUIRE(table && blocks && n_blocks >= 0 && lr_dev && per_tensor);
  if (n_blocks == 0) return ESGPT_OK;
  esgpt::adamw_kernel<<<(unsigned)n_blocks, 256, 0, esgpt::as_stream(stream)>>>(table, blocks, 0.f, beta1, beta2, eps,
                                                                   weight_decay, 0.f, 1.f, per_tensor, err, lr_dev);
  ESGPT_LAUNCH_CHECK();
  return ESGPT_OK;
}

int esgpt_pack(const esgpt_pack_seg* segs, int64_t n_segs, void* stream) {
  ESGPT_REQUIRE(n_segs >= 0 && (n_segs == 0 || segs != nullptr));
  for (int64_t i = 0; i < n_segs; ++i)
    ESGPT_REQUIRE(segs[i].n >= 0 && segs[i].n_pad >= segs[i].n && (segs[i].n == 0 || segs[i].src != nullptr) &&
                  (segs[i].n_pad == 0 || segs[i].dst != nullptr) &&
                  (segs[i].dst_dtype == ESGPT_F32 || segs[i].dst_dtype == ESGPT_BF16));
  for (int64_t b = 0; b < n_segs; b += esgpt::kPackSegs) {
    esgpt::PackArgs a{};
    a.n = (int)(n_segs - b < esgpt::kPackSegs ? n_segs - b : esgpt::kPackSegs);
    a.c0[0] = 0;
    for (int i = 0; i < a.n; ++i) {
      a.s[i] = segs[b + i];
      a.c0[i + 1] = a.c0[i] + esgpt::cdiv(a.s[i].n_pad, esgpt::kPackChunk);
    }
    if (a.c0[a.n] == 0) continue;
    esgpt::pack_kernel<<<(unsigned)a.c0[a.n], 256, 0, esgpt::as_stream(stream)>>>(a);
    ESGPT_LAUNCH_CHECK();
  }
  return ESGPT_OK;
}

// `waiter` waits (on the device) for every piece of work queued on `signaller` so far: one event from a per-device
// ring (an event may be re-recorded as soon as the wait on it has been enqueued; under HIP-graph capture each record
// / wait pair becomes a graph edge, so this forks and joins captured streams).
int esgpt_stream_wait(void* waiter, void* signaller) {
  constexpr int kRing = 64, kDevs = 16;
  static hipEvent_t ring[kDevs][kRing] = {};
  static int next[kDevs] = {};
  ESGPT_REQUIRE(waiter != signaller);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kDevs) return ESGPT_ERR_LAUNCH;
  hipEvent_t& ev = ring[dev][next[dev]];
  next[dev] = (next[dev] + 1) % kRing;
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return ESGPT_ERR_LAUNCH;
  if (hipEventRecord(ev, esgpt::as_stream(signaller)) != hipSuccess) return ESGPT_ERR_LAUNCH;
  return hipStreamWaitEvent(esgpt::as_stream(waiter), ev, 0) == hipSuccess ? ESGPT_OK : ESGPT_ERR_LAUNCH;
}

int esgpt_device_arch_ok(void) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 0;
  return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

}  // extern "C"
