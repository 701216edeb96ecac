set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_train_paths.py -m gpu -x -q --timeout 120 --timeout-method thread -k "derivative or linear_bwd or linear_fwd_act or gemm_big or golden or width or train" > gpurun_out/r06e_tests.log 2>&1 &&
bash tools/gpu_bigbench.sh rule &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r06e_bench_c2.log 2>&1 &&
timeout -k 10 300 python bench.py --config C3 --steps 10 --no-cpu-baseline --no-roofline > gpurun_out/r06e_bench_c3.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/r06e_tests.log
for f in c2 c3; do tail -1 gpurun_out/r06e_bench_$f.log | cut -c1-300; echo; done
exit $rc
