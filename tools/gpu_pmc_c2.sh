#!/bin/bash
# PMC passes over one serialised C2 frame (Cornell PT 1024^2 64 spp, one pipe):
# kernel times, HBM bytes and the issue / wait / cache counters of every kernel
# (the shading kernels are what bounds C2).  bash tools/gpu_pmc_c2.sh [tag]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-c2}
O=gpurun_out/pmc_$TAG
mkdir -p $O
C2="--scene cornell --width 1024 --height 1024 --spp 64 --pipes 1 --steps 1 --warmup 0 --no-cpu --no-roofline-frame"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $C2 > $O/kt.log 2>&1
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_LEVEL_WAVES" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/p$i -o p$i -- python3 bench.py $C2 > $O/p$i.log 2>&1
  echo "pass $i done"
done
python3 tools/pmc_dump.py $O "k_" > $O/summary.txt
