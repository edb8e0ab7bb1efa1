set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
timeout -k 10 200 python scripts/tune_march.py --n 512 --rounds 5 --configs "default;CX=2;CX=2,ZC=64;D=3;D=3,ZC=64;ZC=64;NR=2;CX=2,NR=8,D=2;default" 2>&1 | grep -E "^tune|torch.mul"
