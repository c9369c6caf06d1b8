#!/bin/bash
# Round 4 traversal diagnosis: walk statistics (stats builds) and the timing probes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in stats s4 s6 s2 s7; do
  FFD_LIBRARY=$PWD/build/$v/libffd.so timeout -k 10 240 python tools/trav_stats.py --out gpurun_out/trav_stats_r4a_$v.json > gpurun_out/trav_stats_r4a_$v.log 2>&1 || { tail -20 gpurun_out/trav_stats_r4a_$v.log; exit 1; }
  echo "== $v"; python3 -c "
import json,sys; d=json.load(open('gpurun_out/trav_stats_r4a_$v.json'))
for k in ('headpose','ffd'):
  x=d[k]; print(k, 'ms=%.2f'%d['stage_ms'][k+'_traverse'][0], 'period=%.0f'%x['block_period_cycles_mean'], 'busy=%.0f'%x['walker_wave_busy_cycles_mean'], 'step=%.0f'%x['cycles_per_wave_step_mean'], 'act=%.2f'%x['lane_activity_mean'], 'commit=%.0f'%x['stager_commit_cycles_mean'], 'len=%.1f/%.1f'%(x['walk_len_mean'],x['walk_len_block_max_mean']))
"
done
STAGES=headpose_traverse,ffd_traverse STEPS=3 tools/lib_variant_probe.sh build/p1/libffd.so build/p2/libffd.so build/p3/libffd.so build/p4/libffd.so build/p6/libffd.so build/p7/libffd.so
