#!/bin/bash
# Builds the shipping library with sha256_kernel.hip compiled under other
# AMDGPU machine-scheduler strategies (lab A/B of the SHA-256 chain's
# instruction order; tools/sha_ldg_ab.py --libs):
#   maxio_amd/lib/libmaxio_ec_sched_<strategy>.so
set -e
cd "$(dirname "$0")/../maxio_amd/csrc"
make -j8 >/dev/null
O=../../build/obj
for st in "$@"; do
  mkdir -p ../../build/obj_sched_$st
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter --offload-arch=gfx950 -x hip \
    -mllvm -amdgpu-sched-strategy=$st -c sha256_kernel.hip -o ../../build/obj_sched_$st/sha256_kernel.hip.o
  objs=$(ls $O/*.o | grep -v sha256_kernel)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,--version-script=maxio_ec.map -Wl,--no-undefined \
    -o ../lib/libmaxio_ec_sched_$st.so $objs ../../build/obj_sched_$st/sha256_kernel.hip.o
  echo "built ../lib/libmaxio_ec_sched_$st.so"
done
