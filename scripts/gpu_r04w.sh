# k_pass0h payload words from the parse's light masks: GPU suite, a checked headline run,
# then the same-box A/B against the gather build (libfsx_hip.gath.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04w_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/r04w_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --legs "" --no-cpu-baseline > gpurun_out/r04w_check.log 2>&1 || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/r04w_check.log').read().strip().splitlines()[-1]);print(d['ms_per_step'],json.dumps(d.get('check'))[:300])"
AB_STEPS=20 bash scripts/ab.sh "" gath "" gath > gpurun_out/ab_r04w.txt 2>&1 || exit $?
cut -c1-400 gpurun_out/ab_r04w.txt
