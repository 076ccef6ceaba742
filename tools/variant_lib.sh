#!/bin/bash
# Build a variant of libbrd_hip.so with extra compile flags (developer A/B tool):
#   bash tools/variant_lib.sh NAME "-DFOO=1 -DBAR=2" [source.hip ...]
# Recompiles the listed sources (default: brd_stage2.hip) with the flags, links
# them with the main build's other objects into tools/ablib/NAME.so.  Select
# it at run time with BRD_LIB=tools/ablib/NAME.so.
# Diagnostic builds (results wrong by construction, never in the product
# sources): VARIANT_SED='sed script' is applied to a copy of each listed
# source first, e.g. VARIANT_SED='s/dma16(rs, off/if (0) dma16(rs, off/'.
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
    src=$C/csrc/$base
    if [ -n "$VARIANT_SED" ]; then sed -e "$VARIANT_SED" $src > $out/$base; src=$out/$base; cmp -s $src $C/csrc/$base && { echo "VARIANT_SED changed nothing in $base"; exit 1; }; fi
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$ROOT/include -I$C/csrc -w $flags \
      -c $src -o $out/$base.o
    objs="$objs $out/$base.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $ROOT/tools/ablib/$name.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built tools/ablib/$name.so ($flags)"
