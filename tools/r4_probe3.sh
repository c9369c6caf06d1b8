#!/bin/bash
# Round 4: the drop-in tests (device-resident samples, evaluateMT pattern, reference main), walk phases, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu -s \
  tests/test_cpp_shim.py tests/test_reference_main.py > gpurun_out/r4c_tests.log 2>&1
rc=$?; grep -E 'PASS|FAIL|timings|Error' gpurun_out/r4c_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
FFD_LIBRARY=$PWD/build/t3/libffd.so timeout -k 10 240 python tools/trav_stats.py --phases --out gpurun_out/trav_phases_t3.json > gpurun_out/trav_phases_t3.log 2>&1 || { tail -20 gpurun_out/trav_phases_t3.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/trav_phases_t3.json'))
for k in ('headpose','ffd'): print(k, 'ms=%.2f'%d['stage_ms'][k+'_traverse'][0], {a: round(b) for a,b in d[k].items()})
"
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4c_bench.log 2>&1 || { tail -5 gpurun_out/r4c_bench.log; exit 1; }
tail -1 gpurun_out/r4c_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'host_incl', d.get('host_inclusive',{}).get('value'), 'evaluate_mt', d.get('evaluate_mt_path'))"
