# C3 step kernel trace (rocprofv3) for per-shape launch times.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 250 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/step_C3_r06 -o run -- \
    python bench.py --config C3 --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/step_C3_r06.log 2>&1
rc=$?; tail -1 gpurun_out/step_C3_r06.log | cut -c1-200; exit $rc
