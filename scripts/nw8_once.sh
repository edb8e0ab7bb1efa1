set -u
# Warp-specialised schedules with 8 compute waves (+ the loader wave, 576 threads) — measured, not kept: the
# knob (NW=8 allowed with WS, block 64*(NW+1), loader = wave NW) was removed; logs profiles/r02_tune_nw8_*.log
# bytes per plane and workgroup without more registers per lane.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-nw8}"
run() { timeout -k 10 300 python scripts/tune_march.py --workload $1 --n $2 --rounds 4 --configs "$3" > gpurun_out/${TAG}_$1_$2.log 2>&1 || exit $?; echo "== $1 $2"; grep -E "^tune|torch.mul" gpurun_out/${TAG}_$1_$2.log; }
run stencil27 768 "default;NW=8,NR=1;NW=8,NR=2;NW=8,NR=2,D=2;NW=8,NR=2,ZC=48;NW=8,NR=1,ZC=48;default"
run stencil27 1024 "default;NW=8,NR=1;NW=8,NR=2;NW=8,NR=2,ZC=48;default"
run diffusion7 1024 "default;NW=8,NR=2;NW=8,NR=4;default"
run diffusion7_f16 1024 "default;NR=8;NW=8,NR=4;default"
