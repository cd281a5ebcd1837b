set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_transparent_shadows.py tests/test_gpu_parity.py tests/test_photon_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_ts.log 2>&1
