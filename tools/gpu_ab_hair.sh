#!/bin/bash
# A/B of tuning builds on the C5-shape hair frame (10M tris, 16 spp):
#   tools/gpu_ab_hair.sh "base v1 ..."
set -e
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in $1; do
    if [ $v = base ]; then L=$PWD/core_amd/libyk.so; else L=$PWD/tune/libyk_$v.so; fi
    h=$(YK_LIB=$L timeout -k 10 300 python -u bench.py --scene hair --spp 16 --no-cpu --no-roofline-frame --steps 2 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
    echo "$v rep$rep hair $h"
  done
done
