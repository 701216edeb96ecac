// Version / device probes of the C ABI.
#include <string.h>

#include "common.h"

extern "C" {

const char* esgpt_version(void) { return "eventstreamgpt_amd 0.1.0 (gfx950)"; }

int esgpt_device_arch_ok(void) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 0;
  return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

}  // extern "C"
