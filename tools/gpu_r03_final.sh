#!/bin/bash
# Round-3 final measurement pass: headline bench, rocprofv3 kernel stats of
# the serialised frame (YK_PIPES=1, the frame bench.py's roofline is timed
# on), the two HBM PMC passes (headline and hair), C2, photon mapping and the
# C5-shape hair frame. Each GPU step under its own time limit; set -e stops
# at the first failure.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/final
O=gpurun_out/final
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench $(cat $O/bench.json | head -c 120)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p1 -o p1 -- python3 bench.py --pipes 1 --steps 1 --warmup 0 --no-cpu > $O/prof_p1.log 2>&1
echo "prof done"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o f -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-roofline-frame > $O/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o w -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-roofline-frame > $O/pmc_write.log 2>&1
echo "pmc done"
timeout -k 10 300 python -u bench.py --scene cornell --width 1024 --height 1024 --spp 64 > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 400 python -u bench.py --integrator photon --spp 16 > $O/bench_pm.json 2> $O/bench_pm.err
echo "c2/pm done"
H="--scene hair --spp 16 --steps 1 --warmup 0 --no-cpu --no-roofline-frame"
timeout -k 10 500 python -u bench.py --scene hair --spp 16 --no-cpu > $O/bench_hair.json 2> $O/bench_hair.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/hpmc_fetch -o f -- python3 bench.py $H > $O/hpmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/hpmc_write -o w -- python3 bench.py $H > $O/hpmc_write.log 2>&1
echo "hair done"
