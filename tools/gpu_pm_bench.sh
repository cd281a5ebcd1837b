set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --integrator photon --spp 16 --steps 2 --warmup 1 > gpurun_out/bench_pm.json 2> gpurun_out/bench_pm.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pm -o pm -- python3 bench.py --integrator photon --spp 16 --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_pm.log 2>&1
