#!/bin/bash
# Build an A/B library variant into variants/NAME/libpdivgnn_hip.so (see tools/ab.sh).
#   usage: tools/mkvariant.sh NAME [REV|-] [extra hipcc flags...]
#   REV "-" (default) builds the working tree's csrc; a git revision builds that revision's.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=${2:--}; shift 2 || shift $#
SRC=$R/p-div-gnn_amd/csrc
if [ "$REV" != "-" ]; then
  T=$(mktemp -d)
  git -C "$R" archive "$REV" p-div-gnn_amd/csrc include | tar -x -C "$T"
  SRC=$T/p-div-gnn_amd/csrc
fi
mkdir -p "$R/variants/$NAME"
PDG_CSRC=$SRC PDG_OUT=$R/variants/$NAME/libpdivgnn_hip.so PDG_BUILD_DIR=$R/variants/$NAME/build \
  PDG_EXTRA_FLAGS="$*" python "$R/p-div-gnn_amd/build.py" --force > /dev/null
rm -rf "$R/variants/$NAME/build"
echo "variants/$NAME ($REV $*)"
