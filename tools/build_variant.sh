#!/bin/bash
# Build the library from a git revision (or the working tree: "wt") into build/variants/NAME/.
# usage: [EXTRA="-DKNOB=V"] tools/build_variant.sh NAME [REV]
set -e
NAME=$1; REV=${2:-wt}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
DST=$ROOT/build/variants/$NAME
rm -rf $DST && mkdir -p $DST/src
if [ "$REV" = wt ]; then cp -r $ROOT/transformer-lm_amd/csrc $DST/src/csrc; mkdir -p $DST/src/include; cp $ROOT/include/*.h $DST/src/include/;
else (cd $ROOT && git archive $REV transformer-lm_amd/csrc include) | tar -x -C $DST/src && mv $DST/src/transformer-lm_amd/csrc $DST/src/csrc; fi
mkdir -p $DST/src/x && mv $DST/src/csrc $DST/src/x/csrc && mv $DST/src/include $DST/src/include 2>/dev/null || true
make -s -j8 -C $DST/src/x/csrc OUT=$DST OBJ=$DST/obj CXXFLAGS_EXTRA="$EXTRA" >/dev/null
ls -la $DST/libbpe355.so
