#!/bin/bash
# Build scripts/ubench/mf_mix.hip into build/ubench/mf_mix with each mode's VALU instructions per
# wave-iteration (MFMA included) counted from the ISA of its loop.
set -e
cd "$(dirname "$0")/../.."
mkdir -p build/ubench
F="--offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math"
/opt/rocm/bin/hipcc $F -DVALU0=1 -DVALU1=1 -DVALU2=1 -DVALU3=1 -DVALU4=1 --cuda-device-only -S scripts/ubench/mf_mix.hip \
    -o build/ubench/mf_mix.s
D=""
for m in 0 1 2 3 4; do
  sym=$(grep -o "^_Z1kILi${m}EEvPfif:" build/ubench/mf_mix.s | head -1)
  n=$(awk -v s="$sym" 'index($0, s) == 1 {f = 1} f && /Loop Header/ {l = 1} l && /^[ \t]*v_[a-z]/ {c++} l && /s_cbranch_scc/ {print c; exit}' \
      build/ubench/mf_mix.s)
  echo "mode $m: $n VALU per wave-iteration"
  D="$D -DVALU$m=$n"
done
/opt/rocm/bin/hipcc $F $D scripts/ubench/mf_mix.hip -o build/ubench/mf_mix
