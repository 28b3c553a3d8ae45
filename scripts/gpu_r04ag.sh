# k_parse's deferred-probe list of 64 instead of 128 per wave (CAS inserts closer to their
# probe reads): config 5 and the headline against the product build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "" dc64 "" dc64; do
  FSX_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --legs config4,config5 --no-check \
    --no-config5-oracle --no-cpu-baseline > gpurun_out/r04ag_$v.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/r04ag_$v.log').read().strip().splitlines()[-1]);print('${v:-cur}','config4',d['config4']['ms_per_step'],'config5',d['config5']['ms_per_step'])"
done
AB_STEPS=20 bash scripts/ab.sh "" dc64 "" dc64 > gpurun_out/ab_r04ag.txt 2>&1 || exit $?
cut -c1-60 gpurun_out/ab_r04ag.txt
