#!/bin/bash
# Rehearse the N>1 bench path on a one-GPU box: 2 ranks on device 0, gloo collectives
# (RCCL refuses two ranks on one device). Correctness of the protocol is covered by
# tests/test_shard_*.py; this checks that bench.py's distributed leg runs end to end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} \
  --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus ${NPROC:-2} --steps 3 --warmup 1 \
  --dist-backend gloo --packets ${SHARD_N:-4194304} --config4-packets ${SHARD_N:-4194304} \
  > gpurun_out/shard_bench.log 2>&1
rc=$?
echo "shard bench rc=$rc"
tail -3 gpurun_out/shard_bench.log | cut -c1-1500
exit $rc
