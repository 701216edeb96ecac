# rocprofv3 kernel stats of the C4 bench step (graph replay): bash tools/c4_profile.sh <outdir> [extra bench args]
out=${1:-gpurun_out/c4p}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python bench.py --config C4 \
  --steps 20 --warmup 3 --no-cpu-baseline --no-roofline "$@" > $out.log 2>&1 || exit 1
f=$(ls $out/*/run_kernel_stats.csv 2>/dev/null | head -1)
[ -z "$f" ] && f=$(find $out -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" - 45
