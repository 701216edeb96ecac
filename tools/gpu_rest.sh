cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_train_paths.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/suite_tp.log 2>&1
rc=$?; tail -4 gpurun_out/suite_tp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect tests/test_train_paths.py > gpurun_out/suite.log 2>&1
rc=$?; tail -4 gpurun_out/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -2 gpurun_out/bench.log; exit $rc
