#!/bin/bash
# Build the engine library of git revision REV (WT: the working tree) into
# foundationdb_amd/variants/libfdbcs_<NAME>.so (same-box A/B of kernel changes: bench.py loads it with
# FDBCS_LIB=...), with EXTRA compiler flags (e.g. EXTRA=-DFDBCS_RUN_PROBES=7).  Usage:
#   [EXTRA=...] bash scripts/build_variant.sh <rev> <name>
set -eu
cd "$(dirname "$0")/.."
REV=$1; NAME=$2
TMP=$(mktemp -d)
mkdir -p $TMP/foundationdb_amd/csrc $TMP/include foundationdb_amd/variants
for f in foundationdb_amd/csrc/engine.cpp foundationdb_amd/csrc/kernels.hip foundationdb_amd/csrc/engine.h \
         foundationdb_amd/csrc/scan.h foundationdb_amd/csrc/launch.h foundationdb_amd/csrc/dkey.h foundationdb_amd/csrc/lane_xor.h include/fdb_conflict_set.h; do
  if [ "$REV" = "WT" ]; then cp $f $TMP/$f; else git show $REV:$f > $TMP/$f 2>/dev/null || : > $TMP/$f; fi
done
H=/opt/rocm/bin/hipcc
$H -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -disable-promote-alloca-to-lds ${EXTRA:-} \
  -c $TMP/foundationdb_amd/csrc/kernels.hip -o $TMP/kernels.o
$H -O3 -std=c++17 -fPIC -Wall ${EXTRA:-} -c $TMP/foundationdb_amd/csrc/engine.cpp -o $TMP/engine.o
$H --offload-arch=gfx950 -shared -fPIC -o foundationdb_amd/variants/libfdbcs_$NAME.so $TMP/engine.o $TMP/kernels.o
rm -rf $TMP
echo foundationdb_amd/variants/libfdbcs_$NAME.so
