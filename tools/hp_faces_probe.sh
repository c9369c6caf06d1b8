#!/bin/bash
# k_hp_pose faces per workgroup (FFD_HP_FACES) at C2: the head-pose reduction stage time per setting
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for nf in 4 8 16; do
  FFD_HP_FACES=$nf timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/bench_hpf$nf.log 2>&1 || exit 1
  echo "nf=$nf $(tail -1 gpurun_out/bench_hpf$nf.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step']['headpose_reduce_select'])")"
done
