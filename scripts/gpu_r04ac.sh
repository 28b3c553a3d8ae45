# k_parse's persistent grid (1024 blocks = every VGPR slot) against 896 / 768 / 512, which
# leave room for the previous tail beside the parse.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_STEPS=20 bash scripts/ab.sh "" pg896 pg768 pg512 "" pg896 pg768 pg512 > gpurun_out/ab_r04ac.txt 2>&1 || exit $?
cut -c1-60 gpurun_out/ab_r04ac.txt
