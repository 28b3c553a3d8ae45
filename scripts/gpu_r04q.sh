# Owner warm-record debug, then headline and config-5 A/B of the whole-line slot access.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/dbg_owner_warm.py > gpurun_out/r04q_owner_warm.log 2>&1
rc=$?; echo owner_rc=$rc; tail -6 gpurun_out/r04q_owner_warm.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_scale.py -k "not wide" > gpurun_out/r04q_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -2 gpurun_out/r04q_pytest.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=20 bash scripts/ab_env.sh "" "FSX_EAGER_SLOTS=1" "" "FSX_EAGER_SLOTS=1" > gpurun_out/ab_r04q.txt 2>&1 || exit $?
cut -c1-60 gpurun_out/ab_r04q.txt
for v in "" "FSX_EAGER_SLOTS=1"; do
  env $v timeout -k 10 400 python bench.py --steps 3 --warmup 1 --legs config5 --leg-steps 3 --leg-timing --no-check \
     --no-cpu-baseline > gpurun_out/r04q_c5_$([ -z "$v" ] && echo lazy || echo eager).json 2>&1 || exit $?
done
python3 - <<'PY'
import json
for tag in ("lazy", "eager"):
    d = json.loads(open(f"gpurun_out/r04q_c5_{tag}.json").read().strip().splitlines()[-1])
    c5 = d["config5"]
    print(tag, c5["ms_per_step"], [(k["name"], k["ms_per_step"]) for k in (c5.get("timing") or {}).get("kernels", [])])
PY
