# Build liborpcd_hip.so of a given commit into ab_libs/<name>.so for A/B runs
# against the working tree:   bash tools/build_ab.sh <commit> <name>
set -e
C=$1; NAME=$2
REPO=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/orpcd_ab_$NAME
rm -rf "$W"; git -C "$REPO" worktree prune
git -C "$REPO" worktree add -f --detach "$W" "$C" > /dev/null
mkdir -p "$REPO/ab_libs"
ORPCD_BUILD_LIB="$REPO/ab_libs/$NAME.so" python3 "$W/multi-scale-pointcloud-registration_amd/build_native.py" --force
git -C "$REPO" worktree remove --force "$W"
