# Flood walkers take a new source's family and key from its first packet's record: GPU
# suite, config 5 checked, then config 5 against the previous build (libfsx_hip.pre.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ae_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/r04ae_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 1 --warmup 1 --legs config5 --no-cpu-baseline > gpurun_out/r04ae_check.log 2>&1 || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/r04ae_check.log').read().strip().splitlines()[-1]);v=d['config5'];print('config5',v['ms_per_step'],json.dumps(v.get('check'))[:200],v.get('oracle_check'))"
for v in pre "" pre ""; do
  FSX_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --legs config5 --no-check \
    --no-config5-oracle --no-cpu-baseline > gpurun_out/r04ae_ab_$v.log 2>&1 || exit $?
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r04ae_ab_$v.log').read().strip().splitlines()[-1]);print('${v:-cur}','config5',d['config5']['ms_per_step'])"
done
