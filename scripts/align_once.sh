set -u
# Rows whose byte pitch is not a multiple of 16 (X*esize % 16 != 0): the LDS-DMA loader's 16-byte pieces
# are then misaligned. WS vs the register-prefetch schedule (WS=0) on aligned / misaligned extents.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-align}"
run() { timeout -k 10 300 python scripts/tune_march.py --workload $1 --shape $2 --rounds 4 --configs "$3" > gpurun_out/${TAG}_$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; grep -E "^tune|torch.mul" gpurun_out/${TAG}_$1_$2.log; }
C="default;WS=0;WS=0,CX=2;default"
run diffusion7 128,300,260 "$C"
run diffusion7 128,300,261 "$C"
run diffusion7 128,300,262 "$C"
run diffusion7_f16 128,300,264 "$C"
run diffusion7_f16 128,300,260 "$C"
run diffusion7_f16 128,300,261 "$C"
run stencil27 128,300,264 "$C"
run stencil27 128,300,260 "$C"
