set -u
# round 4: LBM link tables cached per boundary change -- LBM GPU tests, the four LBM configs
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
timeout -k 10 600 python -u -m pytest tests/test_lbm.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r04_pytest11.log 2>&1 || { grep -B2 -A12 "^E " gpurun_out/r04_pytest11.log | head -40; tail -3 gpurun_out/r04_pytest11.log; exit 1; }
tail -2 gpurun_out/r04_pytest11.log
timeout -k 10 400 python -u scripts/bench_configs.py lbm_d2q9_f32_2048^2 lbm_d3q19_f32_192^3 lbm_d2q9_f32_2048^2_channel lbm_d3q19_f32_192^3_channel > gpurun_out/r04_lbm_configs.jsonl 2> gpurun_out/r04_lbm_configs.err || { tail -20 gpurun_out/r04_lbm_configs.err; exit 1; }
cut -c1-400 gpurun_out/r04_lbm_configs.jsonl
