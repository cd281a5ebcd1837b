set -e
cd $GRAFT_REPO_ROOT
for c in 256 4096 100000000; do
  YK_KD_CLIP_PRIMS=$c timeout -k 10 300 python -u bench.py --no-cpu --gpu-tree > gpurun_out/bench_clip_$c.json 2> gpurun_out/bench_clip_$c.err
done
