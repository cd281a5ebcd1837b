#!/bin/bash
# End-of-round check: the GPU suite on the committed build, then the final
# measurement pass (tools/gpu_r03_final.sh).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gputest_k.log 2>&1
tail -1 gpurun_out/gputest_k.log
bash tools/gpu_r03_final.sh
