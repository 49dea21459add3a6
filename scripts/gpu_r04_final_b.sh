#!/bin/bash
# r04 final pass, part B: the whole GPU suite + smoke + bench line (gpu_check.sh), then the 2-rank
# gloo rehearsal of bench's N>1 legs on the one GPU (scripts/gpu_r04_parallel.sh's second step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh || exit $?
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --no-cpu \
    > gpurun_out/r04_rehearsal.json 2> gpurun_out/r04_rehearsal.err
rc=$?; tail -3 gpurun_out/r04_rehearsal.err; tail -c 1500 gpurun_out/r04_rehearsal.json; exit $rc
