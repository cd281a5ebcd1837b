#!/bin/bash
# Headline frame (bumpy 1M tris) under environment settings, one per argument
# word (VAR=value, or "-" for none):  tools/gpu_env_headline.sh "- YK_PIPES=3"
set -e
cd $GRAFT_REPO_ROOT
for rep in $(seq 1 ${REPS:-2}); do
  for v in $1; do
    if [ "$v" = - ]; then E=""; else E="$v"; fi
    c=$(env $E timeout -k 10 200 python -u bench.py --no-cpu --no-roofline-frame --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
    echo "$v rep$rep headline $c"
  done
done
