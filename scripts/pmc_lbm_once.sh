export TMPDIR=/tmp PSAD_CACHE_DIR=/tmp/psad_cache
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_lbm_fetch -o pmc -- python $R/scripts/bench_configs.py "lbm_d3q19_f32_192^3" > $R/gpurun_out/pmc_lbm_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_lbm_write -o pmc -- python $R/scripts/bench_configs.py "lbm_d3q19_f32_192^3" > $R/gpurun_out/pmc_lbm_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $R/gpurun_out/pmc_lbm_sq -o pmc -- python $R/scripts/bench_configs.py "lbm_d3q19_f32_192^3" > $R/gpurun_out/pmc_lbm_sq.log 2>&1 || exit $?
