#!/bin/bash
# Round 6, first lease: (a) the traversal drift -- round-2 HEAD (92fc7c9, abtree/r2g) and today's HEAD benched on one
# box; (b) A/B of the window staging loads bypassing L1 (ablib/libffd_{nt,sc1}.so); (c) PMC passes
# (tools/pmc_groups_r6.txt: TCP hit / miss, UTCL1 translation, TA / TD stalls) on HEAD, the walk-only probe
# (ablib/libffd_walkonly.so: one window per workgroup, no staging) and nt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), 'ms', s['meanshift'])" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p1_head_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p1_head_$rep.log head
  (cd abtree/r2g && timeout -k 10 300 python3 bench.py $BA > $R/gpurun_out/r6/p1_r2g_$rep.log 2>&1) || exit $?
  summ gpurun_out/r6/p1_r2g_$rep.log r2g
  for tag in nt sc1; do
    FFD_LIBRARY=$R/ablib/libffd_$tag.so timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p1_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p1_${tag}_$rep.log $tag
  done
done
export PMC_GROUPS=$R/tools/pmc_groups_r6.txt BENCH_ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-host-paths"
bash tools/pmc.sh r6_head || exit $?
python3 tools/pmc_table.py gpurun_out/pmc_r6_head traverse > gpurun_out/r6/pmc_head.txt
for tag in walkonly nt; do
  FFD_LIBRARY=$R/ablib/libffd_$tag.so bash tools/pmc.sh r6_$tag || exit $?
  python3 tools/pmc_table.py gpurun_out/pmc_r6_$tag traverse > gpurun_out/r6/pmc_$tag.txt
done
echo done
