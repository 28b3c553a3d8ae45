#!/bin/bash
# One parametrised GPU session (replaces the per-experiment gpu_r04*.sh drivers).
#   bash scripts/gpu_run.sh TAG STEP [STEP ...]
# Steps, run in order, each under its own time limit; the session stops at the first step
# that fails (a GPU test *failure* included), so nothing runs after a fault, abort or timeout:
#   tests[=EXPR]   pytest -m gpu (optionally -k EXPR), one process, per-test thread timeouts
#   smoke          __graft_entry__.smoke()
#   bench          python bench.py $BENCH_ARGS                      -> TAG_bench.json.log
#   prof           rocprofv3 kernel trace + stats of a short bench   -> prof_TAG/
#   timeline       kernel timeline of 3 steps                         -> timeline_TAG.txt
#   pmc            PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) + summary  -> pmc_TAG/
#   ab=V1,V2,..    A/B of library variants (scripts/ab.sh)           -> TAG_ab.txt
#   leg=LEG        A/B of one bench leg under env settings $LEG_ENVS (";"-separated, scripts/ab_leg.sh)
#   abenv          A/B of the headline under env settings $AB_ENVS (";"-separated, scripts/ab_env.sh)
# Env: BENCH_ARGS (bench / prof / pmc / timeline / ab), PROF_LEGS, LEG (prof: a bench leg
# run as the headline: config4 / config5 / config3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; shift
run() {   # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "== $name rc=$rc"
  return $rc
}
for s in "$@"; do
  case "$s" in
    tests|tests=*)
      k=()
      [ "$s" != tests ] && k=(-k "${s#tests=}")
      run tests 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 \
          --timeout-method thread "${k[@]}" > "gpurun_out/${TAG}_pytest.log" 2>&1
      rc=$?; tail -3 "gpurun_out/${TAG}_pytest.log"; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/${TAG}_smoke.log" 2>&1 || exit $? ;;
    bench)
      run bench 900 python -u bench.py ${BENCH_ARGS:-} > "gpurun_out/${TAG}_bench.json.log" 2> "gpurun_out/${TAG}_bench.err" || exit $?
      tail -c 400 "gpurun_out/${TAG}_bench.json.log"; echo ;;
    prof)
      if [ -n "${LEG:-}" ]; then
        PROF_TAG=$TAG run prof 700 bash scripts/gpu_legs_profile.sh || exit $?
      else
        PROF_TAG=$TAG run prof 700 bash scripts/gpu_profile.sh || exit $?
      fi ;;
    timeline)
      TL_TAG=$TAG run timeline 400 bash scripts/gpu_timeline.sh > "gpurun_out/timeline_${TAG}.txt" || exit $? ;;
    pmc)
      PROF_TAG=$TAG PMC_MORE=${PMC_MORE:-0} run pmc 1000 bash scripts/gpu_pmc.sh || exit $?
      python3 scripts/pmc_summary.py "gpurun_out/pmc_$TAG" > "gpurun_out/pmc_${TAG}_summary.json" \
          2> "gpurun_out/pmc_${TAG}_summary.err" || true ;;
    ab=*)
      IFS=, read -r -a vs <<< "${s#ab=}"
      AB_ARGS="${BENCH_ARGS:-}" run ab 900 bash scripts/ab.sh "${vs[@]}" > "gpurun_out/${TAG}_ab.txt" 2>&1 || exit $?
      cat "gpurun_out/${TAG}_ab.txt" ;;
    leg=*)
      IFS=';' read -r -a es <<< "${LEG_ENVS:-}"
      [ ${#es[@]} -eq 0 ] && es=("")
      run leg 1000 bash scripts/ab_leg.sh "${s#leg=}" "${es[@]}" > "gpurun_out/${TAG}_leg.txt" 2>&1 || exit $?
      cat "gpurun_out/${TAG}_leg.txt" ;;
    abenv)
      IFS=';' read -r -a es <<< "${AB_ENVS:-}"
      [ ${#es[@]} -eq 0 ] && es=("")
      run abenv 1000 bash scripts/ab_env.sh "${es[@]}" > "gpurun_out/${TAG}_abenv.txt" 2>&1 || exit $?
      cut -c1-400 "gpurun_out/${TAG}_abenv.txt" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
