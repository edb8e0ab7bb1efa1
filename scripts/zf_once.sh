set -u
# chunk-fastest block order (ZF knob, measured slower everywhere and removed; the knob was two lines in
# _march_prelude: chunk = lb % (nb / nt), tile = lb / (nb / nt)). Logs: profiles/r02_tune_zf_*.log
# so the halo planes two chunks share meet in L2; short chunks then approach a one-pass sweep.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
python -m pystencils_autodiff_amd.build > /dev/null || exit 3
TAG="${TAG:-zf}"
C27="default;ZF=1;ZF=1,ZC=12;ZF=1,ZC=8;ZF=1,ZC=4;ZC=8;ZF=1,ZC=48;default"
C7="default;ZF=1;ZF=1,ZC=32;ZF=1,ZC=16;ZF=1,ZC=8;ZC=32;default"
timeout -k 10 300 python scripts/tune_march.py --workload stencil27 --n 768 --rounds 5 --configs "$C27" > gpurun_out/${TAG}_27_768.log 2>&1 && \
timeout -k 10 200 python scripts/tune_march.py --workload stencil27 --shape 96,768,768 --rounds 5 --configs "$C27" > gpurun_out/${TAG}_27_slab8.log 2>&1 && \
timeout -k 10 400 python scripts/tune_march.py --workload diffusion7 --n 1024 --rounds 5 --configs "$C7" > gpurun_out/${TAG}_7_1024.log 2>&1
grep -hv amdgpu.ids gpurun_out/${TAG}_27_768.log gpurun_out/${TAG}_27_slab8.log gpurun_out/${TAG}_7_1024.log
