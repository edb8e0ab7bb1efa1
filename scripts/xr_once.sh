set -u
# (record: the MAP / XR knobs this script sets were measured and removed; see DESIGN.md §4, profiles/r02_xr_bench_ab.txt)
# The XR rule (dispatch-order tiles for WS star grids of >= 3 rounds) against the always-remap order (XR=0).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-xr}"
run() { timeout -k 10 300 python scripts/tune_march.py --workload $1 --shape $2 --rounds 5 --configs "$3" > gpurun_out/${TAG}_$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; grep -E "^tune" gpurun_out/${TAG}_$1_$2.log; }
C="default;XR=0;default;XR=0"
run diffusion7 1024,1024,1024 "$C"
run diffusion7 768,768,768 "$C"
run diffusion7 128,1024,1024 "$C"
run diffusion7 512,512,512 "$C"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit $?
cut -c1-400 gpurun_out/bench_${TAG}.json
