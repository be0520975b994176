cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/tr_pytest.log 2>&1; rc=$?
tail -30 gpurun_out/tr_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --train > gpurun_out/tr_bench.json 2> gpurun_out/tr_bench.err || { tail -20 gpurun_out/tr_bench.err; exit 1; }
cat gpurun_out/tr_bench.json
