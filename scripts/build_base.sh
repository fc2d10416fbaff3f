#!/bin/bash
# Build the library of a git revision (default HEAD) as build/variants/lib_<name>.so
# for A/B runs against the working tree (scripts/ab_lib.sh <name>).
#   build_base.sh [REV] [NAME]
REV=${1:-HEAD}; NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/rhmc_base.XXXX)
git -C "$ROOT" archive "$REV" hmc-stellar-toy-model_amd/csrc include | tar -x -C "$T" || exit 1
mkdir -p "$ROOT/build/variants"
cd "$T/hmc-stellar-toy-model_amd" &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I../include -Icsrc \
  -c -o base.o csrc/rhmc_kernels.hip &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/build/variants/lib_$NAME.so" base.o &&
echo "built lib_$NAME.so from $REV"
rm -rf "$T"
