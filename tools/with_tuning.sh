#!/bin/bash
# Runs a command against the tools build (`make TUNING=1` in eventstreamgpt_amd/csrc: eventstreamgpt_amd/tuning/),
# whose kernel-selection defaults the ESGPT_* tuning variables may override; the product libraries stay untouched.
#   bash tools/with_tuning.sh bash tools/bwd_sweep.sh
D="$(cd "$(dirname "$0")/.." && pwd)/eventstreamgpt_amd/tuning"
export ESGPT_AMD_LIB="$D/libesgpt_amd.so" ESGPT_AMD_TORCH_LIB="$D/libesgpt_torch.so"
exec "$@"
