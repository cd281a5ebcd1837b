set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "universal or dof or fw or abort or big_leaf" > gpurun_out/gputest.log 2>&1
bash tools/gpu_ab.sh "base nseg8" --no-cpu --no-roofline-frame --steps 2 --warmup 1
