# The heavy sources' carried-state check moved to the tail start (k_hmode_state): GPU suite,
# then the previous batch's tail before the parse (FSX_TAIL_AT=-1) against after it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ab_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/r04ab_pytest.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=20 bash scripts/ab_env.sh "" "FSX_TAIL_AT=-1" "" "FSX_TAIL_AT=-1" > gpurun_out/ab_r04ab.txt 2>&1 || exit $?
cut -c1-60 gpurun_out/ab_r04ab.txt
FSX_TAIL_AT=-1 timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --legs "" --no-cpu-baseline > gpurun_out/r04ab_check.log 2>&1 || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/r04ab_check.log').read().strip().splitlines()[-1]);print('tail_at=-1 checked',d['ms_per_step'],json.dumps(d.get('check'))[:200])"
