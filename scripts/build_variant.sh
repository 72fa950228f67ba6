#!/bin/bash
# build_variant.sh NAME [extra hipcc flags for mstep.hip] -> igm_amd/lib/ab/libigmhip_NAME.so (tuning A/B only)
# SRC=path: build that mstep.hip instead (e.g. one saved from git show HEAD:igm_amd/csrc/mstep.hip)
set -e
cd "$(dirname "$0")/.."
python -m igm_amd.build --lib >/dev/null
name=$1; shift
mkdir -p igm_amd/lib/ab build/ab
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics \
  -Iinclude -Iigm_amd/csrc -fno-hip-fp32-correctly-rounded-divide-sqrt "$@" -c ${SRC:-igm_amd/csrc/mstep.hip} -o build/ab/mstep_$name.o
objs=$(ls build/obj/*.o | grep -v '/mstep.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o igm_amd/lib/ab/libigmhip_$name.so build/ab/mstep_$name.o $objs -lz
echo built igm_amd/lib/ab/libigmhip_$name.so
