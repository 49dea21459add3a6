#!/bin/bash
# Build librsac variants for scripts/mf_ab.py into build/ab/librsac_<name>.so: each argument is
# name=FLAGS, rsac_kernels.hip compiled with FLAGS (e.g. -DSOME_SWITCH=1; empty = the tree as
# is), the other objects shared.  Prints each variant's k_pnp_score_mf register use.
#   scripts/build_ab.sh base= trial=-DMY_TRIAL=1
set -e
cd "$(dirname "$0")/../code-reproduction-ransac_amd/csrc"
make -s
mkdir -p ../../build/ab
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
 -fhip-fp32-correctly-rounded-divide-sqrt -fvisibility=hidden -mllvm -amdgpu-atomic-optimizer-strategy=None"
for arg in "$@"; do
  name="${arg%%=*}"; extra="${arg#*=}"
  (
  /opt/rocm/bin/hipcc $FLAGS $extra -c rsac_kernels.hip -o ../../build/ab/k_$name.o \
     -Rpass-analysis=kernel-resource-usage 2> ../../build/ab/res_$name.txt
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o ../../build/ab/librsac_$name.so \
     ../../build/ab/k_$name.o build/rsac_host.o build/rsac_api.o
  echo "$name: $(grep -A 8 'k_pnp_score_mf' ../../build/ab/res_$name.txt | grep -E 'VGPRs:|Scratch|Occupancy' \
     | sed 's/.*remark: *//; s/ \[-Rpass.*//' | tr '\n' ' ')"
  rm -f ../../build/ab/k_$name.o ../../build/ab/res_$name.txt
  ) &
done
wait
