#!/bin/bash
# One parametrised GPU measurement script (run under gpurun):
#   tools/gpu.sh OUTDIR STEP [STEP ...]
# Every step runs under its own time limit; set -e stops at the first failure,
# so nothing else touches the GPU after a fault, abort or timeout.
# Steps (VARIANT = base for core_amd/libyk.so, else tune/libyk_VARIANT.so; VARIANT@NAME=VALUE
# adds one environment setting, e.g. base@YK_SMALL=0):
#   test                 pytest -m gpu (one process, per-test timeout)
#   testv:VARIANT        the traversal / render parity files with a tuning variant's library
#   smoke                __graft_entry__.smoke()
#   bench                headline bench.py (1M tris, 1080p, 256 spp)
#   c2 | pm | hair       BASELINE configs[1] Cornell / photon mapping / C5 hair benches
#   prof                 rocprofv3 --kernel-trace --stats of the one-pipe headline frame
#   prof4                kernel trace of one 4-pipe headline frame (overlap analysis)
#   prof1:V / prof1c2:V  the same (headline / Cornell) with a variant's library (VARIANT[@ENV])
#   pmcw1:V / pmcw1c2:V  WRITE_SIZE of the one-pipe headline / Cornell frame with a variant's library
#   prof_c2 | prof_hair | prof_pm  the same for the Cornell / hair / photon-mapping frames
#   pmc                  FETCH_SIZE and WRITE_SIZE passes of the one-pipe headline frame
#   pmc_c2 | pmc_hair    the same for Cornell / hair
#   tb:VARIANT           traversal microbenchmark (tools/trav_bench.py)
#   tbs:VARIANT          the same with launch time against ray count (prefixes; intercept = per-launch cost)
#   ab:V1,V2,...         A/B: trav bench + headline bench per variant, two interleaved reps
#   abc2:V1,V2,...       A/B on the Cornell (C2) bench
#   abpm:V1,V2,...       A/B on the photon-mapping bench
#   abhair:V1,V2,...     A/B on the C5 hair bench
#   tbab:V1,V2,...       A/B of the traversal microbenchmark only, three interleaved reps
#   coh:VARIANT          primary-shadow ray-order experiment (tools/coherence_bench.py)
#   pmctb:VARIANT        PMC counter passes over the traversal microbenchmark (tools/pmc_dump.py summary)
#   multi                tests/test_multi_device.py + tests/test_0_multi_process.py
#   shard                projected strong scaling (rank 0's share of the headline frame, N = 1/2/4/8)
#   pmcw:VARIANT         WRITE_SIZE passes (one-pipe headline frame, traversal microbenchmark)
#   pmcb:c2|head|hair    the pmctb counter sets over a one-pipe frame, every kernel
#   mallocs              hipMalloc count of 1 vs 3 yk_render_multi calls (rocprofv3 --hip-trace)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
# VARIANT[@NAME=VALUE]: the library plus one environment setting (env A/B)
lib() { local v=${1%%@*}; if [ "$v" = base ]; then echo $PWD/core_amd/libyk.so; else echo $PWD/tune/libyk_$v.so; fi; }
envv() { case $1 in *@*) echo "${1#*@}" ;; *) echo "YK_AB=1" ;; esac; }
C2="--scene cornell --width 1024 --height 1024 --spp 64"
HAIR="--scene hair --spp 16"
PM="--integrator photon --spp 16"
P1="--pipes 1 --steps 1 --warmup 0 --no-cpu --no-roofline-frame"
for s in "$@"; do
  case $s in
  test)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1
    tail -3 $O/gputest.txt ;;
  testv:*)
    # the parity files against a tuning variant's library (bit-exactness of an A/B build)
    v=${s#testv:}
    YK_LIB=$(lib $v) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_big_leaf.py tests/test_universal.py tests/test_transparent_shadows.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/testv_$v.txt 2>&1
    tail -2 $O/testv_$v.txt ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
    tail -1 $O/smoke.txt ;;
  bench)
    timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
    head -c 400 $O/bench.json; echo ;;
  c2)
    timeout -k 10 300 python -u bench.py $C2 > $O/bench_c2.json 2> $O/bench_c2.err
    head -c 300 $O/bench_c2.json; echo ;;
  pm)
    timeout -k 10 400 python -u bench.py $PM > $O/bench_pm.json 2> $O/bench_pm.err
    head -c 300 $O/bench_pm.json; echo ;;
  hair)
    timeout -k 10 500 python -u bench.py $HAIR --no-cpu > $O/bench_hair.json 2> $O/bench_hair.err
    head -c 300 $O/bench_hair.json; echo ;;
  prof|prof_c2|prof_hair|prof_pm)
    A=""; [ $s = prof_c2 ] && A="$C2"; [ $s = prof_hair ] && A="$HAIR"; [ $s = prof_pm ] && A="$PM"
    timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$s -o p1 -- python3 bench.py $A $P1 > $O/$s.log 2>&1
    echo "$s done" ;;
  prof1:*)
    # one-pipe headline frame, rocprofv3 --kernel-trace --stats, with VARIANT[@ENV]
    v=${s#prof1:}
    env $(envv $v) YK_LIB=$(lib $v) timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1_${v//[@=]/_} -o p1 -- python3 bench.py $P1 > $O/prof1_${v//[@=]/_}.log 2>&1
    echo "prof1 $v done" ;;
  prof4)
    # kernel trace of one 4-pipe headline frame (pipeline overlap / idle analysis)
    timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof4 -o p4 -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-roofline-frame > $O/prof4.log 2>&1
    echo "prof4 done" ;;
  prof1c2:*)
    # one-pipe Cornell (C2) frame, rocprofv3 --kernel-trace --stats, with VARIANT[@ENV]
    v=${s#prof1c2:}
    env $(envv $v) YK_LIB=$(lib $v) timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1c2_${v//[@=]/_} -o p1 -- python3 bench.py $C2 $P1 > $O/prof1c2_${v//[@=]/_}.log 2>&1
    echo "prof1c2 $v done" ;;
  pmcw1c2:*)
    # WRITE_SIZE of the one-pipe Cornell frame, library VARIANT
    v=${s#pmcw1c2:}
    YK_LIB=$(lib $v) timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw1c2_${v}_frame -o w -- python3 bench.py $C2 $P1 > $O/pmcw1c2_${v}_frame.log 2>&1
    echo "pmcw1c2 $v done" ;;
  pmc|pmc_c2|pmc_hair)
    A=""; [ $s = pmc_c2 ] && A="$C2"; [ $s = pmc_hair ] && A="$HAIR"
    timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${s}_fetch -o f -- python3 bench.py $A $P1 > $O/${s}_fetch.log 2>&1
    timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${s}_write -o w -- python3 bench.py $A $P1 > $O/${s}_write.log 2>&1
    echo "$s done" ;;
  tbs:*)
    # launch time against ray count (prefixes of each population)
    v=${s#tbs:}
    YK_LIB=$(lib $v) timeout -k 10 300 python -u tools/trav_bench.py --spp 4 --sizes > $O/tbs_$v.json 2> $O/tbs_$v.err
    cat $O/tbs_$v.json ;;
  tb:*)
    v=${s#tb:}
    env $(envv $v) YK_VERBOSE=1 YK_LIB=$(lib $v) timeout -k 10 200 python -u tools/trav_bench.py --spp 4 > $O/tb_$v.json 2> $O/tb_$v.err
    grep libyk $O/tb_$v.err || true
    cat $O/tb_$v.json ;;
  ab:*|abc2:*|abpm:*|abhair:*)
    VS=$(echo ${s#*:} | tr , ' ')
    BA="--no-cpu --steps 2 --warmup 1 --no-roofline-frame"; [ ${s%%:*} = abc2 ] && BA="$BA $C2"; [ ${s%%:*} = abpm ] && BA="$BA $PM"
    [ ${s%%:*} = abhair ] && BA="--no-cpu --steps 1 --warmup 1 --no-roofline-frame $HAIR"
    for rep in 1 2; do
      for v in $VS; do
        L=$(lib $v)
        if [ ${s%%:*} = ab ]; then
          env $(envv $v) YK_LIB=$L timeout -k 10 200 python -u tools/trav_bench.py --spp 4 > $O/ab_tb_${v}_$rep.json 2> $O/ab_tb_${v}_$rep.err
        fi
        env $(envv $v) YK_LIB=$L timeout -k 10 300 python -u bench.py $BA > $O/${s%%:*}_b_${v}_$rep.json 2> $O/${s%%:*}_b_${v}_$rep.err
        python3 - $O ${s%%:*} $v $rep <<'EOF'
import json, os, sys
o, kind, v, rep = sys.argv[1:]
b = json.load(open(f"{o}/{kind}_b_{v}_{rep}.json"))
line = f"{v} rep{rep} bench {b['value']}"
tb = f"{o}/ab_tb_{v}_{rep}.json"
if kind == "ab" and os.path.exists(tb):
    d = json.load(open(tb))
    line += f" tb {d['total_Mrays_s']} " + str([d[k]['Mrays_s'] for k in ('camera', 'bounce', 'shadow1', 'shadow2')])
print(line)
EOF
      done
    done ;;
  tbab:*)
    VS=$(echo ${s#*:} | tr , ' ')
    for rep in 1 2 3; do
      for v in $VS; do
        env $(envv $v) YK_LIB=$(lib $v) timeout -k 10 200 python -u tools/trav_bench.py --spp 4 > $O/tbab_${v}_$rep.json 2> $O/tbab_${v}_$rep.err
        python3 -c "import json;d=json.load(open('$O/tbab_${v}_$rep.json'));print('$v rep$rep', d['total_Mrays_s'], [d[k]['Mrays_s'] for k in ('camera','bounce','shadow1','shadow2')])"
      done
    done ;;
  coh:*)
    v=${s#coh:}
    YK_LIB=$(lib $v) timeout -k 10 300 python -u tools/coherence_bench.py > $O/coh_$v.json 2> $O/coh_$v.err
    cat $O/coh_$v.json
    YK_LIB=$(lib $v) timeout -k 10 300 python -u tools/coherence_bench.py --bounce > $O/cohb_$v.json 2> $O/cohb_$v.err
    cat $O/cohb_$v.json ;;
  pmctb:*)
    # issue / wait / LDS / L1-TA-TD / L2 counters of the traversal kernels over
    # the traversal microbenchmark, one rocprofv3 pass per counter set
    v=${s#pmctb:}
    P=$O/pmctb_$v
    mkdir -p $P
    YK_LIB=$(lib $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o kt -- python3 tools/trav_bench.py --reps 1 > $P/kt.log 2>&1
    i=0
    for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" \
             "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
             "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LEVEL_WAVES TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
             "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS_ATOMIC SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VSKIPPED"; do
      i=$((i+1))
      YK_LIB=$(lib $v) timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $P/p$i -o p$i -- python3 tools/trav_bench.py --reps 1 > $P/p$i.log 2>&1
    done
    python3 tools/pmc_dump.py $P > $P/summary.txt
    echo "pmctb $v done" ;;
  pmcw1:*)
    # WRITE_SIZE of the one-pipe headline frame only, library VARIANT (write attribution)
    v=${s#pmcw1:}
    YK_LIB=$(lib $v) timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw1_${v}_frame -o w -- python3 bench.py $P1 > $O/pmcw1_${v}_frame.log 2>&1
    echo "pmcw1 $v done" ;;
  pmcw:*)
    # WRITE_SIZE of the one-pipe headline frame and of the traversal
    # microbenchmark with library VARIANT (write-traffic attribution)
    v=${s#pmcw:}
    YK_LIB=$(lib $v) timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_${v}_frame -o w -- python3 bench.py $P1 > $O/pmcw_${v}_frame.log 2>&1
    YK_LIB=$(lib $v) timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_${v}_tb -o w -- python3 tools/trav_bench.py --reps 1 > $O/pmcw_${v}_tb.log 2>&1
    echo "pmcw $v done" ;;
  pmcb:*)
    # the pmctb counter sets over a one-pipe frame (c2 | head), all kernels
    sc=${s#pmcb:}
    A=""; [ $sc = c2 ] && A="$C2"; [ $sc = hair ] && A="$HAIR"
    P=$O/pmcb_$sc
    mkdir -p $P
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o kt -- python3 bench.py $A $P1 > $P/kt.log 2>&1
    i=0
    for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" \
             "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
             "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_LEVEL_WAVES SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_WAVES TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
      i=$((i+1))
      timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $P/p$i -o p$i -- python3 bench.py $A $P1 > $P/p$i.log 2>&1
    done
    python3 tools/pmc_dump.py $P "shade|trace|resolve" > $P/summary.txt
    echo "pmcb $sc done" ;;
  mallocs)
    for k in 1 3; do
      timeout -k 10 300 rocprofv3 --hip-trace --output-format csv -d $O/mallocs_$k -o m -- python3 tools/multi_malloc_trace.py --calls $k > $O/mallocs_$k.log 2>&1
      python3 - $O/mallocs_$k $k <<'PY'
import csv, glob, sys
n = 0
for f in glob.glob(sys.argv[1] + "/**/*hip_api_trace.csv", recursive=True):
    n += sum(1 for r in csv.DictReader(open(f)) if "Malloc" in r.get("Function", ""))
print(f"{sys.argv[2]} render_multi call(s): {n} hipMalloc* calls")
PY
    done ;;
  shard)
    # projected strong scaling: rank 0's share of the headline frame for N = 1, 2, 4, 8 (tools/exp_shard.py)
    timeout -k 10 300 python -u tools/exp_shard.py > $O/shard.txt 2> $O/shard.err
    cat $O/shard.txt ;;
  multi)
    timeout -k 10 600 python -u -m pytest tests/test_multi_device.py tests/test_0_multi_process.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/multi.txt 2>&1
    tail -3 $O/multi.txt ;;
  *)
    echo "unknown step $s"; exit 2 ;;
  esac
done
