set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench.json 2>/dev/null
timeout -k 10 300 python -u bench.py --no-cpu --integrator photon --spp 16 > gpurun_out/bench_pm.json 2>/dev/null
