timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gt_r3d.log 2>&1; rc=$?; tail -5 gpurun_out/gt_r3d.log; grep -E "FAILED|Error" gpurun_out/gt_r3d.log | head; [ $rc -eq 0 ] || exit $rc
bash tools/latency_trace.sh b
