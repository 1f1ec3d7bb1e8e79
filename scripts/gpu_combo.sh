# a batch of round-6 measurements in one GPU call: A/B specs, then projections
#   scripts/gpu_combo.sh "AB_SPECS" "PROJ_SPECS"   (space-separated spec lists; either may be "")
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "$1" ]; then bash scripts/gpu.sh abopt $1 || exit $?; fi
if [ -n "$2" ]; then bash scripts/gpu_proj.sh $2 || exit $?; fi
