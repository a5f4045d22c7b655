#!/bin/bash
# Build an A/B variant of libdtgpu.so in diamond-types_amd/<dir>/: every object from lib/ except
# the one rebuilt from the given source file (e.g. a replay kernel variant), then the .so.
#   bash tools/variant.sh lib_base /tmp/dt_replay_base.hip dt_replay [extra hipcc flags]
set -e
DIR=$1; SRC=$2; OBJ=$3; shift 3
cd "$(dirname "$0")/../diamond-types_amd"
mkdir -p "$DIR"
for o in lib/*.o; do [[ $(basename $o .o) == $OBJ ]] || cp "$o" "$DIR/"; done
/opt/rocm/bin/hipcc -O3 -g -fPIC -std=c++17 -Wall -Wno-unused-function --offload-arch=gfx950 -munsafe-fp-atomics -mllvm -structurizecfg-skip-uniform-regions=true -mllvm -amdgpu-atomic-optimizer-strategy=None \
  -Icsrc "$@" -c "$SRC" -o "$DIR/$OBJ.o"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$DIR/libdtgpu.so" "$DIR"/*.o -lpthread
rm -f "$DIR"/*.o
echo "built $DIR/libdtgpu.so"
