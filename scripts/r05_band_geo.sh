set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_distributed.py::test_zslab_native_plan_on_two_streams "tests/test_lbm.py::test_lbm_density_weighted_ubb_gpu" \
  > gpurun_out/r05_tests3.log 2>&1
rc=$?; tail -3 gpurun_out/r05_tests3.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u scripts/probes/op_band_ab.py s27:768::BTY=16,BAND=2,D=2:BTY=16,BAND=2,D=1:BTY=8,BAND=2,D=2:BTY=8,BAND=2,D=3:BTY=16,BAND=2,D=2,ZMIN=32,ZMAX=32:BTY=16,BAND=2,D=2,BABL=1 2>&1 | tee gpurun_out/r05_band_geo1.log && \
timeout -k 10 400 python -u scripts/probes/op_band_ab.py s27:1024::BTY=8,BAND=2,D=2:BTY=8,BAND=2,D=3:BTY=8,BAND=4,D=2 s27:512::BTY=16,BAND=2,D=2:BTY=8,BAND=2,D=2 h7:768::BTY=16,BAND=2,D=2:BTY=16,BAND=2,D=1 2>&1 | tee gpurun_out/r05_band_geo2.log && \
timeout -k 10 300 python -u scripts/probes/lbm_force_ab.py field 2>&1 | tee gpurun_out/r05_lbm_force_field.jsonl && \
timeout -k 10 200 python -u scripts/bench_configs.py laplace5_f32_4096^2 readme_op_f32_20x30 --repeat=3 2>&1 | tee gpurun_out/r05_cfg2.jsonl && \
PSAD_BENCH_ADDR=1 timeout -k 10 200 python bench.py --secondary none --no-cpu-baseline > gpurun_out/r05_addr1.json 2> gpurun_out/r05_addr1.err && \
PSAD_BENCH_ADDR=1 timeout -k 10 200 python bench.py --secondary none --no-cpu-baseline > gpurun_out/r05_addr2.json 2> gpurun_out/r05_addr2.err
