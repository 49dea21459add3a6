cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1
rc=$?; tail -1 gpurun_out/smoke_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
rc=$?; tail -c 600 gpurun_out/bench_final.json; exit $rc
