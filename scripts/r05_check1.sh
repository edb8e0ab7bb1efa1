set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_band.py -m gpu > gpurun_out/r05_band_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_band_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r05_bench1.json 2> gpurun_out/r05_bench1.err && tail -c 3000 gpurun_out/r05_bench1.json && \
timeout -k 10 400 python -u scripts/bench_configs.py laplace5_f32_4096^2 stencil27_f16_768^3 diffusion7_f16_768^3 slab8_stencil27_f16_96x768^2 pitch_stencil27_f16_511^3 pitch_stencil27_f16_512^3 pitch_stencil27_f16_255^3 pitch_stencil27_f16_256^3 2>&1 | tee gpurun_out/r05_cfg3.jsonl
