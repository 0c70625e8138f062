#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace. Every GPU step is time-limited and
# the chain stops at the first failure. Usage (on the GPU box): bash tools/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-r1}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
echo "== gpu tests" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 && \
echo "== smoke" && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && \
echo "== bench" && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" && \
echo "== rocprof" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err"
rc=$?
echo "exit $rc"
tail -3 "$OUT/gpu_tests.log" 2>/dev/null
cat "$OUT/bench.json" 2>/dev/null
exit $rc
