// Version / device probes of the C ABI.
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

}  // namespace esgpt

extern "C" {

const char* esgpt_version(void) { return "eventstreamgpt_amd 0.1.0 (gfx950)"; }

int esgpt_device_arch_ok(void) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 0;
  return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

}  // extern "C"
