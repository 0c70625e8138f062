#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, no tracing domains) + a kernel-trace/stats pass of the same
# bench command. Usage on the GPU box: bash tools/pmc_passes.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r1}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 2 --cpu-seconds 0 --no-parity --no-extras --step-marker $*"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/fetch.json" 2> "$OUT/fetch.err" && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/write.json" 2> "$OUT/write.err" && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/hit" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/hit.json" 2> "$OUT/hit.err" && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/trace.json" 2> "$OUT/trace.err"
rc=$?
echo "exit $rc"
find "$OUT" -name '*.csv' | head -20
exit $rc
