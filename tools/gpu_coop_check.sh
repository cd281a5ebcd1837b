#!/bin/bash
# parity of the traversal kernels on the default build, then an A/B of tuning builds
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kdtree.py tests/test_photon_gpu.py tests/test_curves.py tests/test_transparent_shadows.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_coop.log 2>&1 || { tail -30 gpurun_out/pytest_coop.log; exit 1; }
tail -2 gpurun_out/pytest_coop.log
bash tools/gpu_ab.sh "${1:-old base}"
