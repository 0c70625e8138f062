#!/bin/bash
# One GPU session: the GPU test suite (every test, failures reported, not fatal), smoke, the default bench, a
# rocprofv3 kernel-trace of it, then the measurement set of tools/gpu_perf.sh. A step that faults, aborts or times out
# (status > 1 for pytest, any non-zero status otherwise) ends the session: nothing more runs on the GPU.
# Usage (on the GPU box): bash tools/gpu_round.sh <tag> [perf]
set -o pipefail
TAG=${1:-r3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
trc=$?
tail -4 "$OUT/gpu_tests.log"
grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head -20
if [ $trc -gt 1 ]; then echo "tests ended with status $trc: stopping"; exit $trc; fi
echo "== smoke" && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" && \
echo "== bench" && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" && \
echo "== rocprof" && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err")
rc=$?
python3 -c "
import json
d=json.load(open('$OUT/bench.json'));r=d['roofline']
print('bench', round(d['value']/1e9,2), 'G/s', round(d['ms_per_step'],3), 'ms', d['parity'], 'frac', r['frac'], 'cpu', d.get('cpu_baseline',{}).get('value'))
print({k: round(v['ms_per_step'],3) for k,v in r['kernels'].items()})" 2>/dev/null
if [ $rc -ne 0 ]; then echo "exit $rc"; exit $rc; fi
if [ "$2" = "perf" ]; then bash tools/gpu_perf.sh "$TAG"; rc=$?; fi
echo "exit $rc"
[ $trc -eq 0 ] || exit 1
exit $rc
