#!/bin/bash
# GPU kd-tree clip-threshold sweep (YK_KD_CLIP_PRIMS): the headline frame
# traced on the device-built tree at three settings. Outputs are copied to
# profiles/<round>_kd_clip_<setting>.json.
set -e
cd $GRAFT_REPO_ROOT
for c in 256 4096 100000000; do
  YK_KD_CLIP_PRIMS=$c timeout -k 10 300 python -u bench.py --no-cpu --gpu-tree > gpurun_out/kd_clip_$c.json 2> gpurun_out/kd_clip_$c.err
done
