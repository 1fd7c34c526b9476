# Build flag variants of the current tree's library into abl/ (travels to the
# GPU box; git-ignored):  bash tools/build_variants.sh name:"-DFLAG=1 -DOTHER" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p abl
for v in "$@"; do
  n=${v%%:*}; f=${v#*:}
  ORPCD_EXTRA_FLAGS="$f" ORPCD_BUILD_LIB=abl/$n.so python3 multi-scale-pointcloud-registration_amd/build_native.py | tail -1
done
