# GPU suite (scripts/gpu_suite.sh) and then an interleaved A/B of variant packages.
#   scripts/gpu_suite_ab.sh VARIANT [VARIANT ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_suite.sh || exit $?
bash scripts/variant_bench.sh "$@"
