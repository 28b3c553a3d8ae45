# Multi-rank rehearsal on one GPU after this round's changes: bench.py --gpus 2 over gloo
# (self-launched ranks, the global-batch check against the sharded oracle).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --legs "" --no-cpu-baseline > gpurun_out/r04ah_gloo2.log 2>&1
rc=$?; echo rc=$rc
python3 -c "import json;d=json.loads(open('gpurun_out/r04ah_gloo2.log').read().strip().splitlines()[-1]);print(d['n_gpus'],d['value'],d['ms_per_step'],json.dumps(d.get('check'))[:300])"
exit $rc
