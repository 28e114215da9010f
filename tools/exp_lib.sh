#!/bin/bash
# Experiment library for same-box A/B timing: builds lib/libfourc_gpu_<name>.so from the default
# objects with fcg_sweep.o (OBJ=<object stem> for another one) replaced by <source> compiled with
# <extra hipcc flags> (FCG_LIB=<name> selects it in 4c_amd/fcg.py).
# usage: [OBJ=fcg_hex27] tools/exp_lib.sh name source.hip [flags...]
set -e
cd "$(dirname "$0")/../4c_amd"
name=$1; src=$2; shift 2
make -s all
obj=${OBJ:-fcg_sweep}
objs=$(ls build/*.o | grep -v -e _diag.o -e "$obj.o" -e '_exp_')
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc "$@" -c -o build/${obj}_exp_$name.o "$src"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/libfourc_gpu_$name.so build/${obj}_exp_$name.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -lpthread
echo "built lib/libfourc_gpu_$name.so"
