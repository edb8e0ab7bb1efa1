set -u
# (record: the MAP / XR knobs this script sets were measured and removed; see DESIGN.md §4, profiles/r02_xr_bench_ab.txt)
# Workgroup -> tile mapping: XCD-aware remap with x-fastest tiles (default) vs no remap vs y-fastest tiles.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-map}"
run() { timeout -k 10 300 python scripts/tune_march.py --workload $1 --shape $2 --rounds 4 --configs "$3" > gpurun_out/${TAG}_$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; grep -E "^tune" gpurun_out/${TAG}_$1_$2.log; }
C="default;MAP=1;MAP=2;default"
run stencil27 768,768,768 "$C"
run diffusion7 768,768,768 "$C"
run diffusion7 1024,1024,1024 "$C"
