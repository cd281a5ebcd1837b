#!/bin/bash
# Parity of a tuning build on the GPU render / traversal tests, then the
# headline + C2 A/B against other builds:
#   tools/gpu_ab_par.sh VARIANT "base VARIANT ..." [pytest -k expression]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$1
YK_LIB=$PWD/tune/libyk_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread ${3:+-k "$3"} > gpurun_out/par_$V.log 2>&1
tail -2 gpurun_out/par_$V.log
bash tools/gpu_ab_c2.sh "$2"
