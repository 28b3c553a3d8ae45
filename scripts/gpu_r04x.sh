# Kernel traces of the config-4 and config-5 legs (rocprofv3 kernel trace + stats; the
# headline reduced to one step, no checks).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in 4 5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r04x_c$c" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --legs config$c --leg-steps 2 --no-check --no-cpu-baseline \
    --no-config5-oracle --kernel-timing-steps 0 > "$R/gpurun_out/prof_r04x_c$c.log" 2>&1 || exit $?
  echo "config $c rc=0"
done
