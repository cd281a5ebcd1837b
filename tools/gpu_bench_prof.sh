set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pt -o pt -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_pt.log 2>&1
