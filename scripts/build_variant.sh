#!/bin/bash
# A/B variant of the library: the LDS-DMA engine's units recompiled with extra flags, linked with
# the product objects of build/ -> tmrnet_amd/libtmr_<name>.so (run with TMR_LIB_PATH).
#   scripts/build_variant.sh <name> "<flags>" [units...]   (default units: the dgrad views)
set -e
NAME=$1; FLAGS=$2; shift 2
UNITS=${*:-"gemm16_dgrad_bf16 gemm16_dgrad_f32 gemm16_dpar_bf16 gemm16_dpar_f32"}
D=build_var/$NAME
mkdir -p $D
CF="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Itmrnet_amd/csrc -munsafe-fp-atomics -DTMR_PROLOGUES=0"
pids=()
for u in $UNITS; do
  /opt/rocm/bin/hipcc $CF $FLAGS -c tmrnet_amd/csrc/$u.hip -o $D/$u.hip.o -Rpass-analysis=kernel-resource-usage \
    2> $D/$u.res &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
objs=""
for o in build/*.o; do
  b=$(basename $o .hip.o)
  if [[ " $UNITS " == *" $b "* ]]; then objs="$objs $D/$b.hip.o"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tmrnet_amd/libtmr_$NAME.so $objs
echo "built tmrnet_amd/libtmr_$NAME.so"
