#!/bin/bash
# GPU suite on the plane-layout build (cur), then: headline / C2 with the
# runtime hand-out shift (cur) against compile-time chunks (stc), and the hair
# frame with the crowded-leaf plane layout (cur) against 48-B records (nopl).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
YK_LIB=$PWD/tune/libyk_cur.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gputest_j.log 2>&1
tail -1 gpurun_out/gputest_j.log
bash tools/gpu_ab_c2.sh "cur stc"
bash tools/gpu_ab_hair.sh "nopl cur"
