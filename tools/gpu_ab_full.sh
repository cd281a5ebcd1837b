#!/bin/bash
# Parity (GPU parity tests) of one tuning build, then for each build the
# traversal microbenchmark, the headline frame and C2, two interleaved reps:
#   tools/gpu_ab_full.sh VARIANT "base VARIANT ..." [pytest -k expression]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$1
YK_LIB=$PWD/tune/libyk_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread ${3:+-k "$3"} > gpurun_out/par_$V.log 2>&1
tail -1 gpurun_out/par_$V.log
for rep in 1 2; do
  for v in $2; do
    if [ $v = base ]; then L=$PWD/core_amd/libyk.so; else L=$PWD/tune/libyk_$v.so; fi
    YK_LIB=$L timeout -k 10 120 python -u tools/trav_bench.py --spp 4 > gpurun_out/ab_tb_${v}_$rep.json 2>/dev/null
    t=$(python3 -c "import json;d=json.load(open('gpurun_out/ab_tb_${v}_$rep.json'));print(d['total_Mrays_s'], [d[k]['Mrays_s'] for k in ('camera','bounce','shadow1','shadow2')])")
    a=$(YK_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu --no-roofline-frame --steps 2 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
    c=$(YK_LIB=$L timeout -k 10 200 python -u bench.py --scene cornell --width 1024 --height 1024 --spp 64 --no-cpu --no-roofline-frame --steps 3 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
    echo "$v rep$rep tb $t headline $a c2 $c"
  done
done
