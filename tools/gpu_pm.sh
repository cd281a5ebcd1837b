set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_photon_gpu.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_pm.log 2>&1
