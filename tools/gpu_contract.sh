#!/bin/bash
# The library built without FP contraction: A/B of the kernel times against
# the previous (contracting) build (tools/_ab/librmsf_old.so), the fold and
# Chan merge bit for bit against RMSF.py:36-41's arithmetic, then the whole
# GPU suite, smoke() and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/contract
mkdir -p $O
set -o pipefail
timeout -k 10 300 python -u tools/ab_fold.py > $O/ab_fold.txt 2>&1 || { tail -20 $O/ab_fold.txt; exit 1; }
grep -v "coord\|segments\|orders\|partials" $O/ab_fold.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_reference_vectors.py -k "reference_chan_merge or chan_merge_vs_reference" -v --timeout 200 --timeout-method thread > $O/exact.txt 2>&1 || { tail -40 $O/exact.txt; exit 1; }
grep -E "PASS|FAIL" $O/exact.txt | cut -c1-120
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], d['roofline']['frac'], {k: (v.get('ms_per_step') if isinstance(v, dict) else v) for k, v in d.get('modes', {}).items()})"
