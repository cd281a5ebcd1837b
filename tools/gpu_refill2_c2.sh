#!/bin/bash
# C2 against separate refill thresholds for the closest-hit / any-hit kernels:
#   tools/gpu_refill2_c2.sh "40:40 32:48 ..."   (YK_REFILL:YK_REFILL_SHADOW)
set -e
cd $GRAFT_REPO_ROOT
for rep in $(seq 1 ${REPS:-2}); do
  for v in $1; do
    c=$(YK_REFILL=${v%%:*} YK_REFILL_SHADOW=${v##*:} timeout -k 10 200 python -u bench.py --scene cornell --width 1024 --height 1024 --spp 64 --no-cpu --no-roofline-frame --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
    echo "refill $v rep$rep c2 $c"
  done
done
