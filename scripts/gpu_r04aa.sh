# Tuning A/B on top of scatter MINB 3 + flow-tile grid 1024: flow-tile grid 512, parse at 3
# waves/SIMD, long-walker grid 1024, k_pass0h at 4 waves/SIMD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=20 bash scripts/ab.sh "" ftb512 parse3 wlb1k p0h4 "" ftb512 parse3 wlb1k p0h4 > gpurun_out/ab_r04aa.txt 2>&1 || exit $?
cut -c1-60 gpurun_out/ab_r04aa.txt
