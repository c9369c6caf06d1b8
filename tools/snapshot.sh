#!/bin/bash
# Copy one profile round (tools/profile_round.sh TAG + tools/bench_configs.sh TAG) from gpurun_out/
# into profiles/TAG/: bench.json, kernel_stats.csv, traffic.json, configs/*.json.
set -eu
cd "$(dirname "$0")/.."
TAG=$1
D=profiles/$TAG
mkdir -p $D/configs
tail -1 gpurun_out/round_$TAG/bench.log > $D/bench.json
cp "$(find gpurun_out/round_$TAG/trace -name '*kernel_stats.csv' | head -1)" $D/kernel_stats.csv
cp gpurun_out/round_$TAG/traffic.json $D/traffic.json
for f in gpurun_out/configs_$TAG/*.json; do cp "$f" $D/configs/; done
cat gpurun_out/round_$TAG/source_digest.txt
