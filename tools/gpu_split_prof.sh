# C5 step kernel stats with the split attention backward (product rule, tools build) and with the fused one forced.
set -o pipefail
export TMPDIR=/tmp
D="$(pwd)/eventstreamgpt_amd/tuning"
export ESGPT_AMD_LIB="$D/libesgpt_amd.so" ESGPT_AMD_TORCH_LIB="$D/libesgpt_torch.so"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5_split -o run -- python bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/c5_split.log 2>&1 || exit 1
export ESGPT_ATTN_BWD_SPLIT2=0
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5_fused -o run -- python bench.py --config C5 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-hbm-line > gpurun_out/c5_fused.log 2>&1 || exit 1
echo done
