set -u
# New defaults (fp16 star 256x32 tiles, WS star chunks down to 8 planes) against the previous ones, and the
# parity suites that exercise the march/WS schedules.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-dchk}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rows_f.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
run() { timeout -k 10 300 python scripts/tune_march.py --workload $1 --shape $2 --rounds 4 --configs "$3" > gpurun_out/${TAG}_$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; grep -E "^tune" gpurun_out/${TAG}_$1_$2.log; }
run diffusion7 1024,1024,1024 "default;ZMIN=32;default"
run diffusion7 128,1024,1024 "default;ZMIN=32;default"
run diffusion7 256,256,256 "default;ZMIN=32;default"
run diffusion7 128,128,128 "default;ZMIN=32;default"
run diffusion7_f16 768,768,768 "default;NR=4;default"
