set -e
cd $GRAFT_REPO_ROOT
for v in base nseg8 base nseg8; do
  if [ $v = base ]; then L=$PWD/core_amd/libyk.so; else L=$PWD/tune/libyk_$v.so; fi
  YK_LIB=$L timeout -k 10 200 python -u tools/exp_coherence.py --spp 16 > gpurun_out/coh_$v.json 2>/dev/null
  echo "$v $(cat gpurun_out/coh_$v.json)"
done
