#!/bin/bash
# GPU suite on the committed build, then headline + C2 A/B of tuning builds.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gputest_h.log 2>&1
tail -1 gpurun_out/gputest_h.log
bash tools/gpu_ab_c2.sh "nt sseg nt2 nt2s"
