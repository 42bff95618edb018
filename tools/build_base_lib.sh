# usage: bash tools/build_base_lib.sh [rev] [overlay files...] — libfedhip.so of git revision
# rev (default HEAD), with the named working-tree files (paths relative to the repo) copied
# over it, into ab_lib/base/ (git-ignored) for interleaved A/B runs against the tree's library
set -e
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
PKG=federated-learning-for-privacy-preserving-image-classification_amd
T=$(mktemp -d)
git -C $R archive $REV $PKG/csrc include | tar -x -C $T
shift || true
for f in "$@"; do cp $R/$f $T/$f; done
OUT=${OUT:-base}
mkdir -p $R/ab_lib/$OUT
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -munsafe-fp-atomics -I$T/include -Wno-unused-result"
for s in $T/$PKG/csrc/*.hip; do /opt/rocm/bin/hipcc $F -c $s -o ${s%.hip}.o & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $T/$PKG/csrc/*.o -o $R/ab_lib/$OUT/libfedhip.so
rm -rf $T
echo "built ab_lib/$OUT/libfedhip.so from $REV"
