#!/bin/bash
# Build librsac variants for scripts/mf_ab.py: one .so per RSAC_MF_V value given
# (rsac_kernels.hip compiled with -DRSAC_MF_V=v, the other objects shared), into build/ab/.
# Prints each variant's k_pnp_score_mf register use.
set -e
cd "$(dirname "$0")/../code-reproduction-ransac_amd/csrc"
make -s
mkdir -p ../../build/ab
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
 -fhip-fp32-correctly-rounded-divide-sqrt -fvisibility=hidden -mllvm -amdgpu-atomic-optimizer-strategy=None"
for v in "$@"; do
  (
  /opt/rocm/bin/hipcc $FLAGS -DRSAC_MF_V=$v -c rsac_kernels.hip -o ../../build/ab/k_$v.o \
     -Rpass-analysis=kernel-resource-usage 2> ../../build/ab/res_$v.txt
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o ../../build/ab/librsac_v$v.so \
     ../../build/ab/k_$v.o build/rsac_host.o build/rsac_api.o
  echo "v$v: $(grep -A 8 'k_pnp_score_mf' ../../build/ab/res_$v.txt | grep -E 'VGPRs:|AGPRs:|Scratch|Occupancy' | sed 's/.*remark: *//' | tr '\n' ' ')"
  ) &
done
wait
