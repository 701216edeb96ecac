#!/bin/bash
# Step profile of the C2 bench under forced dW split counts: tools/split_sweep.sh 2 4 8 16
for s in "$@"; do
  ESGPT_GEMM_SPLITS=$s timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ss$s -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ss$s.log 2>&1 || exit 1
  echo "== splits $s: $(grep -o 'ms_per_step[^,]*' gpurun_out/ss$s.log)"
  python tools/pair_shapes.py gpurun_out/ss$s/run_kernel_trace.csv | grep pair
done
