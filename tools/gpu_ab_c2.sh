#!/bin/bash
# A/B of tuning builds on the headline frame and on C2 (Cornell 1024^2 64 spp):
#   tools/gpu_ab_c2.sh "base v1 ..."
set -e
cd $GRAFT_REPO_ROOT
for rep in $(seq 1 ${REPS:-2}); do
  for v in $1; do
    if [ $v = base ]; then L=$PWD/core_amd/libyk.so; else L=$PWD/tune/libyk_$v.so; fi
    a=$(YK_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu --no-roofline-frame --steps 2 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
    c=$(YK_LIB=$L timeout -k 10 200 python -u bench.py --scene cornell --width 1024 --height 1024 --spp 64 --no-cpu --no-roofline-frame --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
    echo "$v rep$rep headline $a c2 $c"
  done
done
