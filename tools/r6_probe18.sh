#!/bin/bash
# Round 6: plain vs packed f32 VALU rate (tools/valu_rate), then the 7x7 Gabor as plain v_mul_f32 / v_add_f32
# (ablib/libffd_g7p.so: FFD_G7_PLAIN=1, -fno-slp-vectorize) and the whole kernel file without SLP packing
# (ablib/libffd_nslp.so) against the default, C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
timeout -k 10 120 ./tools/valu_rate > gpurun_out/r6/valu_rate.log 2>&1 || exit $?
cat gpurun_out/r6/valu_rate.log
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'ms', s['meanshift'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), {k[6:]: v for k, v in s.items() if k.startswith('gabor')}, 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  for tag in def g7p nslp; do
    L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
    FFD_LIBRARY=$L timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p18_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p18_${tag}_$rep.log c2_$tag
  done
done
