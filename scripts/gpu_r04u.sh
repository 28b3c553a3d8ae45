# Same-box A/B of the current library against the r04i-era build (libfsx_hip.r04i.so):
# headline, token bucket.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=20 bash scripts/ab.sh "" r04i "" r04i > gpurun_out/ab_r04u.txt 2>&1 || exit $?
cut -c1-70 gpurun_out/ab_r04u.txt
AB_ARGS="--limiter token" AB_STEPS=20 bash scripts/ab.sh "" r04i > gpurun_out/ab_r04u_token.txt 2>&1 || exit $?
cut -c1-70 gpurun_out/ab_r04u_token.txt
python3 - <<'PY'
import json
for v in ("", "r04i"):
    d = json.loads(open(f"gpurun_out/ab_{v}.json").read().strip().splitlines()[-1])
    print(v or "cur", d["ms_per_step"], {k["name"]: k["ms_per_step"] for k in d["kernels"]})
PY
