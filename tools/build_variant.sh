# Build libflacmi_<name>.so from the kernel sources at git revision <rev> (default: the
# working tree), with extra compiler flags, for same-box A/B runs (tools/gpu_libab.sh).
# Usage: bash tools/build_variant.sh <name> [rev] [extra HIPFLAGS...]
set -e
NAME=$1; REV=${2:-WORKTREE}; shift 2 || true
REPO=$(cd "$(dirname "$0")/.." && pwd)
D=/tmp/flacmi_variant_$NAME
rm -rf $D && mkdir -p $D/csrc $D/include
cp $REPO/flac-py_amd/csrc/* $D/csrc/ 2>/dev/null || true
cp $REPO/include/* $D/include/
if [ "$REV" != WORKTREE ]; then
  for f in $(cd $REPO && git ls-tree --name-only $REV flac-py_amd/csrc/); do git -C $REPO show $REV:$f > $D/csrc/$(basename $f); done
  for f in $(cd $REPO && git ls-tree --name-only $REV include/); do git -C $REPO show $REV:$f > $D/include/$(basename $f); done
fi
mkdir -p $D/x && ln -sfn $D/include $D/x/include 2>/dev/null || true
# the Makefile refers to ../../include/flacmi.h: lay the tree out the same way
mkdir -p $D/tree/flac-py_amd && mv $D/csrc $D/tree/flac-py_amd/csrc && mv $D/include $D/tree/include
make -s -C $D/tree/flac-py_amd/csrc -j8 OUT=$REPO/flac-py_amd/libflacmi_$NAME.so HIPFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 $*" > /dev/null
echo built $REPO/flac-py_amd/libflacmi_$NAME.so
