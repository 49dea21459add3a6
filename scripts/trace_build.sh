#!/bin/bash
# Phase timing of device code: builds a copy of librsac.so with -DRSAC_TRACE in /tmp (block 0
# printfs s_memrealtime stamps, 100 MHz, at RSAC_TRACE_MARK points) and runs $1 (a python file) on it.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=/tmp/rsac_trace
rm -rf $T && mkdir -p $T && cp -r code-reproduction-ransac_amd include $T/ && rm -rf $T/code-reproduction-ransac_amd/csrc/build
make -C $T/code-reproduction-ransac_amd/csrc -j16 EXTRA_FLAGS=-DRSAC_TRACE > /dev/null
PYTHONPATH=$T/code-reproduction-ransac_amd timeout -k 10 120 python3 "$1"
