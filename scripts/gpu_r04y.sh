# Flood-batch walkers (kFreshBit) and the identity segment order: GPU suite, the config-4 /
# config-5 legs checked at full size, then config 4 / 5 against the previous build
# (libfsx_hip.pre.so) on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04y_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/r04y_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --steps 2 --warmup 1 --legs config4,config5 --no-cpu-baseline > gpurun_out/r04y_check.log 2>&1 || exit $?
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r04y_check.log").read().strip().splitlines()[-1])
for k in ("config4", "config5"):
    v = d[k]; print(k, v["ms_per_step"], json.dumps(v.get("check"))[:300], json.dumps(v.get("oracle_check")))
PY
for v in pre "" pre ""; do
  FSX_LIB_VARIANT=$v timeout -k 10 400 python3 bench.py --steps 1 --warmup 1 --legs config4,config5 --no-check \
    --no-config5-oracle --no-cpu-baseline > gpurun_out/r04y_ab_$v.log 2>&1 || exit $?
  python3 - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r04y_ab_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[1] or "cur", "config4", d["config4"]["ms_per_step"], "config5", d["config5"]["ms_per_step"])
PY
done
