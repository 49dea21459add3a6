#!/bin/bash
# Register / LDS / scratch metadata of the library's kernels (device assembly of rsac_kernels.hip,
# same flags as the Makefile): bash scripts/kregs.sh [name-filter]
cd "$(dirname "$0")/../code-reproduction-ransac_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
  -fhip-fp32-correctly-rounded-divide-sqrt -mllvm -amdgpu-atomic-optimizer-strategy=None $EXTRA_FLAGS \
  --cuda-device-only -S rsac_kernels.hip -o /tmp/rsac_kernels_gfx950.s 2>/dev/null || exit 1
python3 ../../scripts/kmeta.py /tmp/rsac_kernels_gfx950.s "$1"
