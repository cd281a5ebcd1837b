#!/bin/bash
# refill-threshold sweep (YK_REFILL) on the traversal microbenchmark + stats build
set -e
cd $GRAFT_REPO_ROOT
for r in 8 16 24 32 40; do
  YK_REFILL=$r timeout -k 10 120 python -u tools/trav_bench.py --spp 4 > gpurun_out/rf_$r.json 2>/dev/null
  echo "refill $r: $(cat gpurun_out/rf_$r.json)"
done
YK_LIB=$PWD/tune/libyk_stats.so timeout -k 10 120 python -u tools/trav_bench.py --spp 4 --reps 1 > gpurun_out/tb_stats2.json 2> gpurun_out/tb_stats2.err
grep trav-stats gpurun_out/tb_stats2.err
