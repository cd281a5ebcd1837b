#!/bin/bash
# parity of tuning builds (traversal tests through YK_LIB), then A/B
set -e
cd $GRAFT_REPO_ROOT
for v in $1; do
  YK_LIB=$PWD/tune/libyk_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kdtree.py tests/test_curves.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1 || { echo "PARITY FAIL $v"; tail -30 gpurun_out/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"
done
bash tools/gpu_ab.sh "base $1"
