# A/B: build the library of a git revision (default HEAD) as exp/base and the
# working tree as exp/new, then time both on the GPU box with
#   VARIANTS="base new" gpurun ... bash scripts/gpu_exp.sh
# usage: bash scripts/ab.sh [REV]
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$ROOT/exp/base" "$ROOT/exp/new" /tmp/airs_ab
mkdir -p "$ROOT/exp/base" "$ROOT/exp/new"
git -C "$ROOT" worktree remove --force /tmp/airs_ab 2>/dev/null || true
git -C "$ROOT" worktree add --detach /tmp/airs_ab "$REV" >/dev/null
make -s -j8 -C /tmp/airs_ab/airs-compression_amd >/dev/null
cp /tmp/airs_ab/airs-compression_amd/lib/libairscmp.so "$ROOT/exp/base/"
git -C "$ROOT" worktree remove --force /tmp/airs_ab
make -s -j8 -C "$ROOT/airs-compression_amd" >/dev/null
cp "$ROOT/airs-compression_amd/lib/libairscmp.so" "$ROOT/exp/new/"
ls -la "$ROOT"/exp/*/libairscmp.so
