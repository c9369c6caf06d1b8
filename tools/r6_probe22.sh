#!/bin/bash
# Round 6: 9x9 Gabor in the 2-column instances — 512-thread 8-row bands (ablib/libffd_m14.so, FFD_GS_CPT2_MASK=14)
# and 256-thread 4-row bands (ablib/libffd_s18.so, FFD_GS_CPT2S_MASK=18) — against the 4-column default; C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), {k[6:]: v for k, v in s.items() if k.startswith('gabor')}, 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  for tag in def m14 s18; do
    L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
    FFD_LIBRARY=$L timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p22_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p22_${tag}_$rep.log c2_$tag
  done
done
# the per-patch evaluateMT pattern (examples/evaluate_mt, face 0 of C2) with a FFD block's trees over up to 8
# workgroups in a one-face grid (ablib/tg8/libffd.so, FFD_TRAV_TG_FFD=8) against 4 (ablib/def/libffd.so)
for rep in 1 2 3; do
  for tag in def tg8; do
    LD_LIBRARY_PATH=$R/ablib/$tag timeout -k 10 120 python3 tools/emt_once.py > gpurun_out/r6/p22_emt_${tag}_$rep.log 2>&1 || { cat gpurun_out/r6/p22_emt_${tag}_$rep.log; exit 1; }
    echo "emt $tag $(tail -1 gpurun_out/r6/p22_emt_${tag}_$rep.log)"
  done
done
