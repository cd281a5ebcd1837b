#!/bin/bash
# A/B of tuning builds: tools/gpu_ab.sh "v1 v2 ..." [bench args]
# (v = base for core_amd/libyk.so, else tune/libyk_v.so). Runs the traversal
# microbenchmark and the headline bench for each, twice, interleaved.
set -e
cd $GRAFT_REPO_ROOT
VS="$1"
shift
BARGS="${@:---no-cpu --steps 2 --warmup 1}"
for rep in 1 2; do
  for v in $VS; do
    if [ $v = base ]; then L=$PWD/core_amd/libyk.so; else L=$PWD/tune/libyk_$v.so; fi
    YK_LIB=$L timeout -k 10 120 python -u tools/trav_bench.py --spp 4 > gpurun_out/ab_tb_${v}_$rep.json 2>/dev/null
    YK_LIB=$L timeout -k 10 200 python -u bench.py $BARGS > gpurun_out/ab_b_${v}_$rep.json 2>/dev/null
    echo "$v rep$rep tb $(python3 -c "import json;d=json.load(open('gpurun_out/ab_tb_${v}_$rep.json'));print(d['total_Mrays_s'], [d[k]['Mrays_s'] for k in ('camera','bounce','shadow1','shadow2')])") bench $(python3 -c "import json;print(json.load(open('gpurun_out/ab_b_${v}_$rep.json'))['value'])")"
  done
done
