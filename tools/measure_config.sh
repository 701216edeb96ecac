#!/bin/bash
# One configuration's measurement set on the GPU box, every step under its own time limit, stopping at the first
# failure: its PMC traffic passes (marker-attributed, tools/pmc_traffic.py --entries), the bench line (reading that
# traffic), and a rocprofv3 kernel-stats profile of the training step.
#   tools/measure_config.sh C2 [steps]
# Outputs: gpurun_out/pmc_traffic_<C>.json (also copied to profiles/ on the box for the bench), gpurun_out/bench_<C>.json,
# gpurun_out/step_<C>/ (rocprofv3 stats).
set -o pipefail
C=${1:-C2}
STEPS=${2:-20}
export TMPDIR=/tmp
mkdir -p gpurun_out
E=gpurun_out/entries_$C.json
timeout -k 10 180 python bench.py --config $C --roofline-only --pmc-pass $E > gpurun_out/pmcnames_$C.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF_$C -o run -- \
    python bench.py --config $C --roofline-only --pmc-pass $E > gpurun_out/pmcF_$C.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW_$C -o run -- \
    python bench.py --config $C --roofline-only --pmc-pass $E > gpurun_out/pmcW_$C.log 2>&1 &&
python tools/pmc_traffic.py --entries $E gpurun_out/pmcF_$C gpurun_out/pmcW_$C gpurun_out/pmc_traffic_$C.json \
    > /dev/null &&
cp gpurun_out/pmc_traffic_$C.json profiles/pmc_traffic_$C.json &&
rm -rf gpurun_out/pmcF_$C gpurun_out/pmcW_$C &&
timeout -k 10 300 python bench.py --config $C --steps $STEPS --warmup 5 > gpurun_out/bench_$C.log 2>&1 &&
grep '^{' gpurun_out/bench_$C.log > gpurun_out/bench_$C.json &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/step_$C -o run -- \
    python bench.py --config $C --steps $STEPS --warmup 3 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/step_$C.log 2>&1
rc=$?
echo "measure_config $C rc=$rc"
exit $rc
