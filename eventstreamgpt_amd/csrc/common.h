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

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ void set_err(int32_t* err, int code) {
  if (err) atomicOr(err, code);
}

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace esgpt
