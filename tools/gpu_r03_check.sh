set -e
# Round 3: GPU parity suite (resumable with a -k expression in $1) + headline bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
sel=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ${sel:+-k "$sel"} > gpurun_out/gputest.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
