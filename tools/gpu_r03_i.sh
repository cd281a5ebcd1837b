#!/bin/bash
# A/B: non-temporal hit stores (nt3) against the committed build (nt), and
# the any-hit kernel's refill threshold alone (YK_REFILL_S) on the rf build.
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_c2.sh "nt pb bb ab nt3"
for rep in 1 2; do
  for r in 24 16 32; do
    a=$(YK_LIB=$PWD/tune/libyk_rf.so YK_REFILL_S=$r timeout -k 10 200 python -u bench.py --no-cpu --no-roofline-frame --steps 2 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
    c=$(YK_LIB=$PWD/tune/libyk_rf.so YK_REFILL_S=$r timeout -k 10 200 python -u bench.py --scene cornell --width 1024 --height 1024 --spp 64 --no-cpu --no-roofline-frame --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
    echo "refill_s $r rep$rep headline $a c2 $c"
  done
done
