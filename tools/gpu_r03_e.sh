#!/bin/bash
# Traversal statistics (YK_TRAV_STATS build) of the current kernels on the
# traversal microbenchmark, and a refill-threshold sweep on the headline.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
YK_LIB=$PWD/tune/libyk_stats.so timeout -k 10 120 python -u tools/trav_bench.py --spp 4 --reps 1 > gpurun_out/tb_stats.json 2> gpurun_out/tb_stats.err
grep trav-stats gpurun_out/tb_stats.err
for r in 16 24 32; do
  a=$(YK_REFILL=$r timeout -k 10 200 python -u bench.py --no-cpu --no-roofline-frame --steps 2 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
  echo "refill $r headline $a"
done
bash tools/gpu_ab_par.sh sh1 "cur sh1"
