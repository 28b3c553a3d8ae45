# Short-segment bound 512 and short-walker grid 4096 against the product (headline, config 4).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=20 bash scripts/ab.sh "" ss512 wsb4k "" ss512 wsb4k > gpurun_out/ab_r04ak.txt 2>&1 || exit $?
cut -c1-40 gpurun_out/ab_r04ak.txt
for v in "" ss512 wsb4k; do
  FSX_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --legs config4 --leg-steps 4 --no-check \
    --no-cpu-baseline > gpurun_out/r04ak_c4_$v.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/r04ak_c4_$v.log').read().strip().splitlines()[-1]);print('${v:-cur}','config4',d['config4']['ms_per_step'])"
done
