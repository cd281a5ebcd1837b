set -e
# Round-3 measurement pass B: the C5-shape hair frame (10M tris, 16 spp,
# 8 bounces) and its PMC passes: HBM bytes (FETCH_SIZE / WRITE_SIZE) and the
# L1 / L2 / TD counters behind the "algorithmic frac > 1" reading.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
H="--scene hair --spp 16 --steps 1 --warmup 0 --no-cpu --no-roofline-frame"
timeout -k 10 500 python -u bench.py --scene hair --spp 16 --no-cpu > gpurun_out/bench_hair.json 2> gpurun_out/bench_hair.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/hpmc_fetch -o f -- python3 bench.py $H > gpurun_out/hpmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/hpmc_write -o w -- python3 bench.py $H > gpurun_out/hpmc_write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/hpmc_cache -o c -- python3 bench.py $H > gpurun_out/hpmc_cache.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -s -q --timeout 250 --timeout-method thread -k "c2_config" > gpurun_out/c2test.log 2>&1
