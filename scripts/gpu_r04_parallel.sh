#!/bin/bash
# r04: first-round mode + sharded loop GPU tests, then a 2-rank gloo rehearsal of bench's N>1 legs
# on the one GPU (ranks share it).  Each GPU step has its own limit; a failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "first_round or parallel_driver or scan_device or hypothesis_rows" > gpurun_out/r04_par_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r04_par_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --no-cpu \
    > gpurun_out/r04_rehearsal.json 2> gpurun_out/r04_rehearsal.err
rc=$?; tail -3 gpurun_out/r04_rehearsal.err; exit $rc
