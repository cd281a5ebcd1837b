#!/bin/bash
# PMC counters of the traversal kernels, kernels serialised (one pipe), for the
# traversal-efficiency analysis in DESIGN.md. Usage on the GPU box:
#   bash tools/gpu_pmc_trav.sh [lib] [tag]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LIB=${1:-$PWD/tune/libyk_p1.so}
TAG=${2:-p1}
ARGS=${PMC_ARGS:-"--steps 1 --warmup 0 --no-cpu --spp 64"}
O=gpurun_out/pmc_$TAG
mkdir -p $O
YK_LIB=$LIB timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py $ARGS > $O/kt.log 2>&1
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
         "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum"; do
  i=$((i+1))
  YK_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/p$i -o p$i -- python3 bench.py $ARGS > $O/p$i.log 2>&1
  echo "pass $i done"
done
