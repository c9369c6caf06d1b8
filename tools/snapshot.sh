#!/bin/bash
# Copy one profile round (tools/profile_round.sh TAG + tools/bench_configs.sh TAG) from gpurun_out/
# into profiles/TAG/: bench.json, kernel_stats.csv, traffic.json, configs/*.json, source_digest.txt, the GPU suite's
# log (gpurun_out/r6/snap_tests_TAG.log, when present), the compiler's per-kernel registers / occupancy
# (kernel_resources.json) and the per-scale Gabor table (gabor_scales.json).
set -eu
cd "$(dirname "$0")/.."
TAG=$1
D=profiles/$TAG
mkdir -p $D/configs
tail -1 gpurun_out/round_$TAG/bench.log > $D/bench.json
cp "$(find gpurun_out/round_$TAG/trace -name '*kernel_stats.csv' | head -1)" $D/kernel_stats.csv
cp gpurun_out/round_$TAG/traffic.json $D/traffic.json
for f in gpurun_out/configs_$TAG/*.json; do cp "$f" $D/configs/; done
cp gpurun_out/round_$TAG/source_digest.txt $D/source_digest.txt
[ -f gpurun_out/r6/snap_tests_$TAG.log ] && cp gpurun_out/r6/snap_tests_$TAG.log $D/gpu_tests.log
python3 tools/kernel_resources.py $D/kernel_resources.json k_ > /dev/null
python3 tools/gabor_table.py $D
cat $D/source_digest.txt
