#!/bin/bash
# Build a libgwa variant for tools/ab.py: copy the package to /tmp, apply a python patch script to
# its csrc/, build there, copy the library back as genome-weaver-align_amd/libgwa_<name>.so.
#   tools/build_variant.sh NAME PATCH.py
set -e
NAME=$1; PATCH=$2
REPO=$(cd "$(dirname $0)/.." && pwd)
D=/tmp/gwa_variant_$NAME
rm -rf $D && mkdir -p $D && cp -r $REPO/genome-weaver-align_amd/csrc $REPO/genome-weaver-align_amd/Makefile $D/
mkdir -p $D/../include_$NAME && cp $REPO/include/gwa.h $D/../include_$NAME/
sed -i "s#../../include/gwa.h#$REPO/include/gwa.h#" $D/csrc/*.cpp $D/csrc/*.h $D/csrc/*.hip 2>/dev/null || true
(cd $D/csrc && python3 $PATCH)
make -s -j${VJ:-8} -C $D HDR="$(echo $D/csrc/*.h) $REPO/include/gwa.h" libgwa.so
cp $D/libgwa.so $REPO/genome-weaver-align_amd/libgwa_$NAME.so
echo built $REPO/genome-weaver-align_amd/libgwa_$NAME.so
