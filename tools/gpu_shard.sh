set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/exp_shard.py > gpurun_out/exp_shard.log 2>&1
YK_BATCH_SAMPLES=8388608 timeout -k 10 300 python -u tools/exp_shard.py >> gpurun_out/exp_shard.log 2>&1
YK_BATCH_SAMPLES=16777216 timeout -k 10 300 python -u tools/exp_shard.py >> gpurun_out/exp_shard.log 2>&1
