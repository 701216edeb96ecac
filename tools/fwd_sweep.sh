run() { echo "== $*"; env ESGPT_GEMM_PANEL=0 "$@" timeout -k 10 100 python tools/fwd_gemm_time.py 2>&1 | grep -v amdgpu || exit 1; }
run X=0
run ESGPT_GEMM_FWD_NB=2
run ESGPT_GEMM_FWD_NS=4
run ESGPT_GEMM_DBG=1
run ESGPT_GEMM_DBG=2
run ESGPT_GEMM_DBG=3
run ESGPT_GEMM_PERSIST=2
run ESGPT_GEMM_TILE_FWD=21
run ESGPT_GEMM_TILE_FWD=12
run ESGPT_GEMM_TILE_FWD=22
