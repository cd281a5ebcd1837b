set -e
cd $GRAFT_REPO_ROOT
for v in base e1 e4 base e1 e4; do
  if [ $v = base ]; then L=core_amd/libyk.so; else L=tune/libyk_$v.so; fi
  YK_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/tune_$v.json 2>/dev/null
  echo "$v PT $(python3 -c "import json;print(json.load(open('gpurun_out/tune_$v.json'))['value'])")"
done
