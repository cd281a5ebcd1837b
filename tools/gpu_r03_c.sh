set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/trav_bench.py --reps 2 > gpurun_out/tb.json 2> gpurun_out/tb.err
timeout -k 10 200 python -u bench.py --scene cornell --width 1024 --height 1024 --spp 64 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
bash tools/gpu_pmc_c2.sh c2
