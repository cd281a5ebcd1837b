#!/bin/bash
# GPU suite on one tuning build, then headline / C2 / hair / photon-mapping A/B.
#   tools/gpu_r03_f.sh VARIANT "base VARIANT ..."
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$1
YK_LIB=$PWD/tune/libyk_$V.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gputest_$V.log 2>&1
tail -1 gpurun_out/gputest_$V.log
bash tools/gpu_ab_c2.sh "$2"
bash tools/gpu_ab_hair.sh "$2"
for rep in 1 2; do
  for v in $2; do
    L=$PWD/tune/libyk_$v.so
    p=$(YK_LIB=$L timeout -k 10 300 python -u bench.py --integrator photon --spp 16 --no-cpu --no-roofline-frame --steps 2 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
    echo "$v rep$rep pm $p"
  done
done
