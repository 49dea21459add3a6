#!/bin/bash
# In-kernel shader clock of the scoring kernel (MI355X_MICROARCH.md "DVFS give-back" item 6): builds
# a copy of librsac.so with -DRSAC_MF_CLOCK in /tmp (every 97th block of k_pnp_score_mf printfs its
# lifetime in s_memtime cycles and s_memrealtime 100 MHz ticks) and runs the C2 workload on it
# after >= 2 s of back-to-back launches.  clock = cycles / ticks x 100 MHz.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=/tmp/rsac_clock
rm -rf $T && mkdir -p $T && cp -r code-reproduction-ransac_amd include $T/ && rm -rf $T/code-reproduction-ransac_amd/csrc/build
make -C $T/code-reproduction-ransac_amd/csrc -j16 EXTRA_FLAGS=-DRSAC_MF_CLOCK > /dev/null
PYTHONPATH=$T/code-reproduction-ransac_amd timeout -k 10 120 python3 scripts/workload_prof.py ${1:-c2} ${2:-400}
