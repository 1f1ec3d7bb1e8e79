# Build copies of the package with extra compile flags for A/B runs on the GPU box:
#   build_variants.sh NAME "FLAGS" [NAME "FLAGS" ...] -> gpurun_var/NAME/{bench.py,sparsecholesky_amd,profiles}
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=gpurun_var/$name
  rm -rf "$d"; mkdir -p "$d/profiles/r03" "$d/oracle"
  cp bench.py "$d/"; mkdir -p "$d/scripts"; cp scripts/panel_breakdown.py "$d/scripts/"
  cp profiles/r03/pmc_summary.json profiles/r03/mfma_util.json "$d/profiles/r03/"
  mkdir -p "$d/sparsecholesky_amd"
  cp sparsecholesky_amd/__init__.py "$d/sparsecholesky_amd/"
  make -s -j8 -C sparsecholesky_amd/csrc OBJDIR=build_$name OUT="$PWD/$d/sparsecholesky_amd/libsparsecholesky_amd.so" OPT="-O3 $flags"
done
