#!/bin/bash
# libesgpt_amd_stamps.so: the kernel library with the attention backward's s_memtime stamps (tools/attn_stamps.py)
set -e
cd "$(dirname "$0")/../eventstreamgpt_amd/csrc"
mkdir -p build_stamps
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -DESGPT_STAMPS -c attention_bwd.hip \
  -o build_stamps/attention_bwd.o
objs=$(ls build/*.o | grep -v attention_bwd.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o ../libesgpt_amd_stamps.so $objs build_stamps/attention_bwd.o
