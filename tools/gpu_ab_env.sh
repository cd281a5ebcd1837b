#!/bin/bash
# A/B of runtime knobs on the default build: tools/gpu_ab_env.sh "VAR=a VAR=b ..." [bench args]
# ("-" = no override; "A=1,B=2" sets several). Runs the headline bench for each setting, twice, interleaved.
set -e
cd $GRAFT_REPO_ROOT
VS="$1"
shift
BARGS="${@:---no-cpu --steps 2 --warmup 1}"
for rep in 1 2; do
  for v in $VS; do
    if [ "$v" = "-" ]; then E=""; else E="${v//,/ }"; fi
    env $E timeout -k 10 200 python -u bench.py $BARGS > gpurun_out/abe_${rep}.json 2>/dev/null
    echo "$v rep$rep bench $(python3 -c "import json;print(json.load(open('gpurun_out/abe_${rep}.json'))['value'])")"
  done
done
