set -e
cd $GRAFT_REPO_ROOT
for v in base s8w7 s8w6 c7 c5 base; do
  if [ $v = base ]; then L=core_amd/libyk.so; else L=tune/libyk_$v.so; fi
  YK_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/tune_$v.json 2>/dev/null
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/tune_$v.json'));print(d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['roofline']['other_kernel'])")"
done
