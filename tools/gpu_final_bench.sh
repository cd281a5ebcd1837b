set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pt -o pt -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_pt.log 2>&1
timeout -k 10 400 python -u bench.py --integrator photon --spp 16 > gpurun_out/bench_pm.json 2> gpurun_out/bench_pm.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pm -o pm -- python3 bench.py --integrator photon --spp 16 --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_pm.log 2>&1
timeout -k 10 300 python -u bench.py --scene cornell --width 1024 --height 1024 --spp 64 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
timeout -k 10 900 python -u bench.py --scene hair --spp 16 --no-cpu > gpurun_out/bench_hair.json 2> gpurun_out/bench_hair.err
