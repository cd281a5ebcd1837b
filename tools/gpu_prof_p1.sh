set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
YK_LIB=$PWD/tune/libyk_p1.so timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_p1 -o p1 -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_p1.log 2>&1
