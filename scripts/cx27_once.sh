set -u
# 27-point fp16 half ring: row-segment length per tile (CX = x-adjacent cells per lane, TX = 64*CX).
# 768^3 full-row tiles (CX=12, TX=768) against the 256-wide default; 1024^3 CX=8 (1 KB rows) vs CX=4.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-cx27}"
C768="default;CX=12,WX=1,NR=1,ZC=24;CX=12,WX=1,NR=1,ZC=48;CX=12,WX=1,NR=2,ZC=24;CX=12,WX=1,NR=1,D=2,ZC=24;CX=12,WX=1,NR=1,ZC=12;CX=12,WX=1,NR=1,DPP=0,ZC=24;default"
C1024="default;CX=8,WX=1,NR=2,ZC=32;CX=8,WX=1,NR=1,ZC=32;CX=4,WX=1,NR=2,ZC=32;default"
timeout -k 10 300 python scripts/tune_march.py --workload stencil27 --n 768 --rounds 5 --configs "$C768" > gpurun_out/${TAG}_768.log 2>&1 && \
timeout -k 10 300 python scripts/tune_march.py --workload stencil27 --n 1024 --rounds 5 --configs "$C1024" > gpurun_out/${TAG}_1024.log 2>&1
cat gpurun_out/${TAG}_768.log gpurun_out/${TAG}_1024.log | grep -v amdgpu.ids
