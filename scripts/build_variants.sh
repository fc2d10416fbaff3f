#!/bin/bash
# Build librhmc.so variants with extra -D flags for A/B runs on the GPU box:
#   build_variants.sh name1="-DFOO=1" name2="-DBAR=2" ...
# -> build/variants/lib_<name>.so (select at run time with RHMC_LIB=...)
cd "$(dirname "$0")/../hmc-stellar-toy-model_amd" || exit 1
mkdir -p ../build/variants
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc $flags \
      -c -o ../build/variants/$name.o csrc/rhmc_kernels.hip &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../build/variants/lib_$name.so ../build/variants/$name.o &&
    rm -f ../build/variants/$name.o && echo "built $name" ) &
done
wait
