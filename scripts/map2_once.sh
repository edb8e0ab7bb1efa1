set -u
# (record: the MAP / XR knobs this script sets were measured and removed; see DESIGN.md §4, profiles/r02_xr_bench_ab.txt)
# No XCD remap (MAP=1) vs the XCD-aware remap across the WS star shapes, the 27-point and 2-D.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-map2}"
run() { timeout -k 10 300 python scripts/tune_march.py --workload $1 --shape $2 --rounds 5 --configs "$3" > gpurun_out/${TAG}_$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; grep -E "^tune" gpurun_out/${TAG}_$1_$2.log; }
C="default;MAP=1;default;MAP=1"
run diffusion7 1024,1024,1024 "$C"
run diffusion7 512,512,512 "$C"
run diffusion7 128,1024,1024 "$C"
run diffusion7 256,1024,1024 "$C"
run diffusion7 384,384,384 "$C"
run diffusion7 640,640,640 "$C"
run diffusion7_f64 512,512,512 "$C"
run diffusion7_f16 1024,1024,1024 "$C"
run stencil27 96,768,768 "$C"
run veclap3 384,384,384 "$C"
