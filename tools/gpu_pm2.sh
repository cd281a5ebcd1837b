set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_photon_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_pm.log 2>&1
timeout -k 10 400 python -u bench.py --integrator photon --spp 16 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_pm.json 2> gpurun_out/bench_pm.err
