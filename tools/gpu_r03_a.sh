set -e
# GPU suite (new cases) + traversal phase profile (diagnostic build).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "not fullsize and not multi_process and not big_leaf and not kdtree" > gpurun_out/gputest.log 2>&1
YK_LIB=$PWD/tune/libyk_stats.so timeout -k 10 200 python -u tools/trav_bench.py --reps 1 > gpurun_out/tb_stats.json 2> gpurun_out/tb_stats.err
timeout -k 10 200 python -u tools/trav_bench.py > gpurun_out/tb_base.json 2> gpurun_out/tb_base.err
