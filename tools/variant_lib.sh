#!/bin/bash
# Build a variant of libbrd_hip.so with extra compile flags (developer A/B tool):
#   bash tools/variant_lib.sh NAME "-DFOO=1 -DBAR=2" [source.hip ...]
# Recompiles the listed sources (default: brd_stage2.hip) with the flags, links
# them with the main build's other objects into tools/ablib/NAME.so.  Select
# it at run time with BRD_LIB=tools/ablib/NAME.so.
set -e
name=$1; flags=$2; shift 2
srcs=${*:-brd_stage2.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/svdsolver_amd
make -s -C $C >/dev/null
out=$ROOT/tools/ablib/build_$name; mkdir -p $out
objs=""
for o in $C/build/*.o; do
  base=$(basename $o .o)            # e.g. brd_stage2.hip
  if [[ " $srcs " == *" $base "* ]]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include -I$C/csrc -w $flags \
      -c $C/csrc/$base -o $out/$base.o
    objs="$objs $out/$base.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $ROOT/tools/ablib/$name.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built tools/ablib/$name.so ($flags)"
