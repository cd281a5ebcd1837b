set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/trav_bench.py > gpurun_out/tb_base.json 2> gpurun_out/tb_base.err
YK_LIB=$PWD/tune/libyk_stats.so timeout -k 10 200 python -u tools/trav_bench.py --reps 1 > gpurun_out/tb_stats.json 2> gpurun_out/tb_stats.err
