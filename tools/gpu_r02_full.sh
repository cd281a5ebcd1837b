set -e
# Round-2 full measurement: parity tests, headline bench (+ rocprof stats and
# PMC HBM passes), C2 Cornell, photon mapping, and the C5-shape hair frame.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pt -o pt -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_pt.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_write.log 2>&1
timeout -k 10 300 python -u bench.py --scene cornell --width 1024 --height 1024 --spp 64 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
timeout -k 10 400 python -u bench.py --integrator photon --spp 16 > gpurun_out/bench_pm.json 2> gpurun_out/bench_pm.err
timeout -k 10 900 python -u bench.py --scene hair --spp 16 --no-cpu > gpurun_out/bench_hair.json 2> gpurun_out/bench_hair.err
