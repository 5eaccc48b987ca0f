#!/bin/bash
# A/B builds: recompile ONE source of the engine with extra defines and link it with the other objects of the
# current build into siddhi_amd/_lib/var_<name>/libsiddhi_amd.so (load it with SDG_LIB=<that path>).
# usage: scripts/build_variant.sh <name> <sources, comma-separated: chain,kernels,seq3,order,engine> [-DFOO=1 ...]
set -eu
cd "$(dirname "$0")/../siddhi_amd"
NAME=$1; SRC=$2; shift 2
make -s -j8 _lib/libsiddhi_amd.so
D=_lib/var_$NAME
mkdir -p $D
FLAGS="-std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-result -Wno-unused-function"
for S in ${SRC//,/ }; do
    case $S in
        engine) IN=csrc/engine/engine.cpp; X="-x hip" ;;
        *) IN=csrc/kernels/$S.hip; X="" ;;
    esac
    /opt/rocm/bin/hipcc $FLAGS $X "$@" -Rpass-analysis=kernel-resource-usage -c $IN -o $D/$S.o 2> $D/$S.resource.txt &
done
wait
OBJS=""
for o in engine compile sched kernels chain order keytab ingest seq3 merge; do
    if [[ ",$SRC," == *",$o,"* ]]; then OBJS="$OBJS $D/$o.o"; else OBJS="$OBJS _lib/$o.o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,--no-undefined -o $D/libsiddhi_amd.so $OBJS -pthread
echo "built $D/libsiddhi_amd.so"
