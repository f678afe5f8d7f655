#!/bin/bash
# Build a variant of libscflow_hip.so with extra -D flags for one source file (tuning A/B).
# usage: tools/build_variant.sh NAME FILE.hip "-DFOO=1 -DBAR=2"  → scflow_amd/lib/ab/NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; SRC=$2; DEFS=$3
OBJ=$R/scflow_amd/lib/obj; OUT=$R/scflow_amd/lib/ab; mkdir -p $OUT/$NAME
python -m scflow_amd.build > /dev/null
objs=""
for o in $OBJ/*.o; do
  if [ "$(basename $o)" = "$SRC.o" ]; then
    /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -fvisibility=hidden -I $R/include $DEFS \
      -c $R/scflow_amd/csrc/$SRC -o $OUT/$NAME/$SRC.o
    objs="$objs $OUT/$NAME/$SRC.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/$NAME.so $objs
echo $OUT/$NAME.so
