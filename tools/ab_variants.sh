#!/bin/bash
# Builds kernel variants of librr.so (same sources, -D switches) into
# ab_builds/<name>/librr.so (objects in <pkg>/build/ab_<name>/, which does not
# travel) for A/B timing on the GPU box with RR_LIB_PATH.
#   tools/ab_variants.sh name1 "-DFOO=1" name2 "-DFOO=0" ...
# AB_MAKE_ARGS: extra make variables for every variant (e.g. TILES_TUFLAGS=...)
set -e
PKG=diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
    d=$ROOT/ab_builds/$1
    o=$ROOT/$PKG/build/ab_$1
    mkdir -p $d $o
    make -s -j8 -C $ROOT/$PKG/csrc OUT=$d OBJ=$o EXTRA="$2" ${AB_MAKE_ARGS:-} $d/librr.so
    echo "built $d/librr.so ($2)"
    shift 2
done
