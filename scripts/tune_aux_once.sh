export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 300 python -u scripts/tune_march.py --workload diffusion7_f64 --n 512 --rounds 3 --configs "default;CX=2,NR=4,D=4;CX=2,NR=8,D=2;CX=2,NR=2,D=4;CX=4,NR=2,D=2;CX=1,NR=8,D=4;CX=2,NR=4,D=3,ZC=64;CX=2,NR=4,D=4,ZC=32;default" > gpurun_out/tune_f64.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/tune_march.py --workload veclap3 --n 384 --rounds 3 --configs "default;CX=1,NR=2;CX=1,NR=8;CX=1,NR=4,D=3;CX=1,NR=4,D=2;CX=1,WX=2,NR=4;CX=1,NR=4,WS=0;CX=1,NR=4,ZC=48;default" > gpurun_out/tune_veclap.log 2>&1 || exit $?
