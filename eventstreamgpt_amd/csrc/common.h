// Shared helpers for the gfx950 kernels of eventstreamgpt_amd.
// Wave = 64 lanes on CDNA4; every wave-level idiom below assumes that.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "../../include/esgpt_amd.h"

#define ESGPT_WAVE 64

#define ESGPT_LAUNCH_CHECK()                                   \
  do {                                                         \
    hipError_t _e = hipGetLastError();                         \
    if (_e != hipSuccess) return ESGPT_ERR_LAUNCH;             \
  } while (0)

#define ESGPT_REQUIRE(cond)                                    \
  do {                                                         \
    if (!(cond)) return ESGPT_ERR_INVALID_ARG;                 \
  } while (0)

namespace esgpt {

typedef __hip_bfloat16 bf16;

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return __bfloat162float(x); }

template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return __float2bfloat16(x); }

__device__ __forceinline__ float bf16_bits_to_f32(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

// Round-to-nearest-even f32 -> bf16 bits (finite inputs; NaN stays NaN through the plain cast path).
__device__ __forceinline__ uint16_t f32_to_bf16_bits(float f) {
  bf16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

// Wave reductions in registers: DPP butterflies within each 16-lane row (quad_perm xor 1, xor 2, then the half-row
// and row mirrors), v_permlane16_swap across row pairs and v_permlane32_swap across the halves — 8 VALU
// instructions, no LDS crossbar (ds_bpermute) round trips. Every lane ends with the same bits (each step combines
// the same two operands in every lane of a pair).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));
  v = fmaxf(v, dpp_mov<0x140>(v));
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ void set_err(int32_t* err, int code) {
  if (err) atomicOr(err, code);
}

// Out-of-range embedding index: the flag plus the largest offending index in the error block's int64 slot
// (bytes 8..15), so the host can raise the reference's "Invalid embedding! {max} >= {V}".
__device__ __forceinline__ void set_bad_index(int32_t* err, int64_t idx) {
  if (err) {
    atomicOr(err, ESGPT_FLAG_BAD_INDEX);
    atomicMax(reinterpret_cast<long long*>(err + 2), (long long)idx);
  }
}

// XCD-aware workgroup order: the dispatcher deals consecutive workgroup ids round-robin over the 8 XCDs (each with
// its own L2), so id -> (xcd = id % 8, slot = id / 8) is remapped (bijectively) to a linear index that gives every
// XCD a contiguous run: workgroups with neighbouring linear indices (the query blocks of one (batch, head), the two
// halves of a key block) share an L2.
__device__ __forceinline__ int xcd_linear(int id, int nwg) {
  const int q = nwg >> 3, rr = nwg & 7, xcd = id & 7, slot = id >> 3;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + slot;
}

// Activations of the GEMM / bias epilogues (act: 0 erf-GELU, 1 tanh-GELU, 2 ReLU) and their derivatives.
// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7 for the CDF): one reciprocal and one exp2, the exp2 shared
// with the normal density of the derivative; tanh as 1 - 2 / (1 + e^{2u}). The library erff / tanhf (branchy
// polynomials) made the c_fc epilogue VALU-bound: 8.4 M activations per C2 layer.
__device__ __forceinline__ void normal_cdf_pdf(float z, float& cdf, float& pdf) {
  const float u = fabsf(z) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, u, 1.f));
  const float e = __builtin_amdgcn_exp2f(z * z * -0.72134752044448170368f);  // exp(-z^2 / 2)
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  const float q = 0.5f * poly * e;  // (1 - erf(|z| / sqrt 2)) / 2
  cdf = z >= 0.f ? 1.f - q : q;
  pdf = 0.39894228040143267794f * e;
}

__device__ __forceinline__ float fast_tanh(float u) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u * 2.88539008177792681472f));
}

__device__ __forceinline__ float act_fwd(float z, int act) {
  if (act == 0) {
    float cdf, pdf;
    normal_cdf_pdf(z, cdf, pdf);
    return z * cdf;
  }
  if (act == 1) {
    const float k = 0.79788456080286535588f;  // sqrt(2/pi)
    return 0.5f * z * (1.f + fast_tanh(k * (z + 0.044715f * z * z * z)));
  }
  return z > 0.f ? z : 0.f;
}

__device__ __forceinline__ float act_grad(float z, int act) {
  if (act == 0) {
    float cdf, pdf;
    normal_cdf_pdf(z, cdf, pdf);
    return cdf + z * pdf;
  }
  if (act == 1) {
    const float k = 0.79788456080286535588f;
    const float t = fast_tanh(k * (z + 0.044715f * z * z * z));
    return 0.5f * (1.f + t) + 0.5f * z * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * z * z);
  }
  return z > 0.f ? 1.f : 0.f;
}

// act(z) and act'(z) together (one normal-density / tanh evaluation for both): the c_fc epilogue under
// ESGPT_ACT_DERIV, which stores the derivative for the backward in place of the pre-activation.
__device__ __forceinline__ void act_fwd_grad(float z, int act, float& y, float& g) {
  if (act == 0) {
    float cdf, pdf;
    normal_cdf_pdf(z, cdf, pdf);
    y = z * cdf;
    g = cdf + z * pdf;
    return;
  }
  if (act == 1) {
    const float k = 0.79788456080286535588f;
    const float t = fast_tanh(k * (z + 0.044715f * z * z * z));
    y = 0.5f * z * (1.f + t);
    g = 0.5f * (1.f + t) + 0.5f * z * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * z * z);
    return;
  }
  y = z > 0.f ? z : 0.f;
  g = z > 0.f ? 1.f : 0.f;
}
// the backward's factor at one element: the stored derivative (ESGPT_ACT_DERIV), or act'(pre)
__device__ __forceinline__ float act_factor(float aux, int act) {
  return (act & ESGPT_ACT_DERIV) ? aux : act_grad(aux, act & 7);
}

// Dropout (attention probabilities, residual / input): a counter-based hash of (seed, element index), so the
// forward and backward regenerate the same keep-mask without storing it. One hash per PAIR of elements: element idx
// takes the 16-bit half (idx & 1) of h = mix32(pair_lo ^ key ^ pair_hi * 0x9E3779B9), pair = idx >> 1 ("lowbias32"
// finaliser; key = mix32(seed_lo ^ mix32(seed_hi ^ 0x9E3779B9)) once per kernel); keep <=> half >= thresh =
// round(p * 2^16) (drop probability quantised to 2^-16; kept values scaled by 1 / (1 - p)). Two integer multiplies
// (quarter-rate on CDNA) per two elements; the hot loops take both halves of one hash (dropout_mult2).
struct DropoutSpec {
  float p;          // drop probability (0 = off)
  float scale;      // 1 / (1 - p)
  uint32_t thresh;  // round(p * 2^16)
  uint32_t key;
};

__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__host__ __device__ __forceinline__ uint32_t dropout_key(uint64_t seed) {
  return mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) ^ 0x9E3779B9u));
}

// 32 random bits for the element pair (2 * pair, 2 * pair + 1)
__host__ __device__ __forceinline__ uint32_t dropout_hash(uint32_t key, uint64_t pair) {
  return mix32((uint32_t)pair ^ key ^ ((uint32_t)(pair >> 32) * 0x9E3779B9u));
}

__device__ __forceinline__ float dropout_mult(const DropoutSpec& d, uint64_t idx) {
  const uint32_t hh = dropout_hash(d.key, idx >> 1);
  const uint32_t half = (idx & 1) ? (hh >> 16) : (hh & 0xffffu);
  return half >= d.thresh ? d.scale : 0.f;
}

// Both elements of the pair starting at the EVEN index idx: m0 for idx, m1 for idx + 1.
__device__ __forceinline__ void dropout_mult2(const DropoutSpec& d, uint64_t idx, float& m0, float& m1) {
  const uint32_t hh = dropout_hash(d.key, idx >> 1);
  m0 = (hh & 0xffffu) >= d.thresh ? d.scale : 0.f;
  m1 = (hh >> 16) >= d.thresh ? d.scale : 0.f;
}

// 32-bit index forms (the launch's element indices all fit 32 bits, so the high word of every pair index is 0):
// the same bits as dropout_mult / dropout_mult2 without 64-bit index arithmetic or the high-word multiply.
__device__ __forceinline__ float dropout_mult_32(const DropoutSpec& d, uint32_t idx) {
  const uint32_t hh = mix32((idx >> 1) ^ d.key);
  const uint32_t half = (idx & 1) ? (hh >> 16) : (hh & 0xffffu);
  return half >= d.thresh ? d.scale : 0.f;
}
__device__ __forceinline__ void dropout_mult2_32(const DropoutSpec& d, uint32_t idx, float& m0, float& m1) {
  const uint32_t hh = mix32((idx >> 1) ^ d.key);
  m0 = (hh & 0xffffu) >= d.thresh ? d.scale : 0.f;
  m1 = (hh >> 16) >= d.thresh ? d.scale : 0.f;
}

// Both multipliers of the element pair at the EVEN index row·D + col, in the 32-bit form when every element index of
// the launch fits 32 bits (`i32`, wave-uniform): the same bits as dropout_mult2 without 64-bit index products.
__device__ __forceinline__ void dropout_pair_rc(const DropoutSpec& d, bool i32, int64_t row, int64_t D, int64_t col,
                                                float& m0, float& m1) {
  if (i32) dropout_mult2_32(d, (uint32_t)row * (uint32_t)D + (uint32_t)col, m0, m1);
  else dropout_mult2(d, (uint64_t)(row * D + col), m0, m1);
}

__device__ __forceinline__ DropoutSpec make_dropout(float p, const uint64_t* seed_ptr) {
  DropoutSpec d;
  d.p = p;
  d.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  d.thresh = p > 0.f ? (uint32_t)fminf(rintf(p * 65536.f), 65536.f) : 0u;
  d.key = dropout_key((p > 0.f && seed_ptr) ? *seed_ptr : 0ull);
  return d;
}

// In-launch last-arriver ticket, write-through form (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms):
// the handed-off bytes are stored with sc1 stores (st_wt) and read back with sc1 loads (ld_wt); every thread calls
// this after its stores; each wave drains them, the workgroup barrier orders them before ONE agent-scope ticket add,
// and the workgroup whose add comes last — of the `expected` ones sharing `counter` — gets true and resets the
// counter for the next launch. No L2 write-back fence (buffer_wbl2 would write back every dirty line of the XCD's
// L2, which the streaming kernels around it keep full). `flag`: one int of the caller's LDS.
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool last_arrival(int32_t* counter, int expected, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == expected - 1;
    if (last) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Kernel-selection tuning hooks (ESGPT_GEMM_*, ESGPT_ATTN_*, ESGPT_LN_*): read from the environment only in a tools
// build (`make TUNING=1`, -DESGPT_TUNING_HOOKS, used by tools/env_sweep.sh); the product library never consults the
// caller's environment, so its kernel choices and numerics are a function of the arguments alone.
static inline const char* tuning_env(const char* name) {
#ifdef ESGPT_TUNING_HOOKS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Zero-fills `bytes` bytes at `p` on `st` with a kernel (misc.hip). Used instead of hipMemsetAsync so that every
// reset is an ordinary kernel node when the caller captures the stream into a HIP graph (memset nodes captured
// from this library were observed not to re-run on graph replay). Returns hipSuccess or the launch error.
hipError_t zero_async(void* p, size_t bytes, hipStream_t st);

}  // namespace esgpt
