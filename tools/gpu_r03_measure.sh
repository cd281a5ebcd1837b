set -e
# Round-3 measurement pass A: headline bench, rocprofv3 kernel stats of the
# serialised frame (YK_PIPES=1, the frame bench.py's roofline is timed on),
# the two HBM PMC passes, C2 Cornell and photon mapping. Each GPU step under
# its own time limit; set -e stops at the first failure.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_p1 -o p1 -- python3 bench.py --pipes 1 --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_p1.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-roofline-frame > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-roofline-frame > gpurun_out/pmc_write.log 2>&1
timeout -k 10 300 python -u bench.py --scene cornell --width 1024 --height 1024 --spp 64 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
timeout -k 10 400 python -u bench.py --integrator photon --spp 16 > gpurun_out/bench_pm.json 2> gpurun_out/bench_pm.err
