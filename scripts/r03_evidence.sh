#!/bin/bash
# Round-3 evidence at HEAD: GPU tests + smoke + storm line, trace and PMC passes; the 1M-peer gossip
# line, trace and PMC passes; then the default bench line as the driver runs it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
TESTS=1 SHAPES=storm scripts/round_evidence.sh || exit 1
scripts/round_evidence_gossip.sh || exit 1
mkdir -p gpurun_out/final
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail gpurun_out/final/bench.err; exit 1; }
tail -c 600 gpurun_out/final/bench.json
