#!/bin/bash
# Round 4: blocked pair layout (build/blk, host encoding + kernel) against the in-tree build: leaves on every C2
# face and 512 C4 faces (far offsets), stage times, walk phases (build/blkph).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VARIANTS="${VARIANTS:-blk}" PHASES="${PHASES:-blkph}" tools/r4_probe7.sh
