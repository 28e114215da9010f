#!/bin/bash
# Experiment library built from every source with extra compile flags (for changes that span
# translation units, e.g. a record layout): lib/libfourc_gpu_<name>.so (FCG_LIB=<name> selects it).
# usage: tools/exp_full.sh name [-Dflags...]
set -e
cd "$(dirname "$0")/../4c_amd"
name=$1; shift
X="$*"
make -s OBJ=build/x_$name OUT=build/x_$name/lib \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc -Wall -Wno-unused-result $X" \
  HOSTFLAGS="-O3 -std=c++17 -fPIC -I../include -Icsrc -Wall $X" -j8 build/x_$name/lib/libfourc_gpu.so
cp build/x_$name/lib/libfourc_gpu.so lib/libfourc_gpu_$name.so
echo "built lib/libfourc_gpu_$name.so"
