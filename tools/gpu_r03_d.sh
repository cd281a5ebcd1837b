set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
YK_LIB=$PWD/tune/libyk_pw.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gputest_pw.log 2>&1
tail -1 gpurun_out/gputest_pw.log
for rep in 1 2; do
  for v in h2 pw pwpm; do
    L=$PWD/tune/libyk_$v.so
    p=$(YK_LIB=$L timeout -k 10 300 python -u bench.py --integrator photon --spp 16 --no-cpu --no-roofline-frame --steps 2 --warmup 1 2>/dev/null | python3 -c "import json,sys;print(json.load(sys.stdin)['value'])")
    echo "$v rep$rep pm $p"
  done
done
bash tools/gpu_ab_c2.sh "h2 pw"
