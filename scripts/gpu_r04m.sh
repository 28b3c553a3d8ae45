# Flow tests, headline A/B of the lazy slots / direct DROPs, config 4 / 5 legs A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "flow" > gpurun_out/r04m_pytest.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -2 gpurun_out/r04m_pytest.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=20 bash scripts/ab_env.sh "" "FSX_EAGER_SLOTS=1" "FSX_DROP_LISTS=1" "" > gpurun_out/ab_r04m.txt 2>&1 || exit $?
cut -c1-60 gpurun_out/ab_r04m.txt
for v in "" "FSX_EAGER_SLOTS=1 FSX_DROP_LISTS=1"; do
  env $v timeout -k 10 500 python bench.py --steps 3 --warmup 1 --legs config4,config5 --leg-steps 3 --leg-timing \
     --no-check --no-cpu-baseline > gpurun_out/r04m_legs_$([ -z "$v" ] && echo new || echo old).json 2>&1 || exit $?
done
python3 - <<'PY'
import json
for tag in ("new", "old"):
    d = json.loads(open(f"gpurun_out/r04m_legs_{tag}.json").read().strip().splitlines()[-1])
    for leg in ("config4", "config5"):
        v = d[leg]
        print(tag, leg, v["ms_per_step"], [(k["name"], k["ms_per_step"]) for k in v.get("kernels", [])][:40])
PY
