# PMC passes (FETCH_SIZE, WRITE_SIZE; kernel trace only) of the config-4 and config-5 legs,
# the headline reduced to one step.
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$REPO/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for c in 4 5; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    OUT="$REPO/gpurun_out/pmc_r04af_c$c/$ctr"
    mkdir -p "$OUT"
    timeout -s KILL 400 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$OUT" -o run -- \
      python3 "$REPO/bench.py" --steps 1 --warmup 0 --legs config$c --leg-steps 2 --no-check --no-cpu-baseline \
      --no-config5-oracle --kernel-timing-steps 0 > "$OUT.log" 2>&1
    rc=$?; echo "config $c $ctr rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
