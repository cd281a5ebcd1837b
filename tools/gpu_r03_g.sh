#!/bin/bash
# GPU suite on the candidate build (bfl), then A/B of several tuning builds
# on headline + C2, and the crowded-leaf kernel on the hair frame.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
YK_LIB=$PWD/tune/libyk_bfl.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gputest_bfl.log 2>&1
tail -1 gpurun_out/gputest_bfl.log
bash tools/gpu_ab_c2.sh "bf2 sseg pc4 ntw sw6 sw6c6"
bash tools/gpu_ab_hair.sh "bf2 bfl"
