set -u
# Small / odd 3-D shapes, WS star schedule: chunk length (ZC) against the ZMIN=32 floor of the chunk model;
# plus the fp16 256x32-tile default on the shapes of the earlier odd-size sweep.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-small}"
run() { timeout -k 10 300 python scripts/tune_march.py --workload $1 --shape $2 --rounds 4 --configs "$3" > gpurun_out/${TAG}_$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; grep -E "^tune|torch.mul" gpurun_out/${TAG}_$1_$2.log; }
C="default;ZC=4;ZC=8;ZC=16;ZMIN=8;ZMIN=4;default"
run diffusion7 200,300,260 "$C"
run diffusion7 256,256,256 "$C"
run diffusion7 128,128,128 "$C"
run diffusion7 384,384,384 "$C"
run diffusion7_f16 200,300,260 "$C"
run diffusion7_f16 384,384,384 "$C"
