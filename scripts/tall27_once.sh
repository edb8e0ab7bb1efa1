set -u
# Taller tiles (more bytes per plane and workgroup) for the 27-point half ring and the 768^3 fp32 7-point.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-tall}"
run() { timeout -k 10 300 python scripts/tune_march.py --workload $1 --shape $2 --rounds 4 --configs "$3" > gpurun_out/${TAG}_$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; grep -E "^tune" gpurun_out/${TAG}_$1_$2.log; }
run stencil27 768,768,768 "default;NR=4,ZC=24;NR=6,ZC=24;NR=8,ZC=24;NR=8,ZC=48;NR=8,D=2,ZC=24;default"
run stencil27 1024,1024,1024 "default;NR=8,ZC=24;NR=8,ZC=32;default"
run diffusion7 768,768,768 "default;NR=8;NR=8,D=3;CX=2,NR=8;default"
