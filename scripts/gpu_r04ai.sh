# The insert mark (kFreshBit) on the unsorted-heavy path too (light words; config 4's and the
# cold leg's first batches): GPU suite, headline + cold + config 4 checked at full size, then
# config 4 and the cold leg against the previous build (libfsx_hip.pre.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ai_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/r04ai_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 10 --warmup 2 --legs cold,config4 --no-cpu-baseline > gpurun_out/r04ai_check.log 2>&1 || exit $?
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r04ai_check.log").read().strip().splitlines()[-1])
print("headline", d["ms_per_step"], d["check"]["verdicts_equal"], d["check"]["maps_equal"], d["check"].get("flows_last_batch"))
for k in ("cold", "config4"):
    v = d[k]; print(k, v["ms_per_step"], json.dumps(v.get("check"))[:240])
PY
for v in pre "" pre ""; do
  FSX_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --legs cold,config4 --leg-steps 6 --no-check \
    --no-cpu-baseline > gpurun_out/r04ai_ab_$v.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/r04ai_ab_$v.log').read().strip().splitlines()[-1]);print('${v:-cur}','cold',d['cold']['ms_per_step'],'config4',d['config4']['ms_per_step'])"
done
