#!/bin/bash
# Round 6: new tests (exact aligned / compaction / merge reuse), then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact_aligned.py tests/test_reduce_order.py tests/test_gpu_multirank.py \
    -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 \
    || { grep -E "FAILED|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
grep -E "literal shape" $O/tests.log || true
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])
for k,v in d.get('modes',{}).items():
    if isinstance(v, dict) and 'compacted' in v:
        print(k, 'compacted', round(v['compacted']['ms_per_step'],3), 'regathered', round(v['regathered']['ms_per_step'],3), 'speedup', round(v['speedup_compacted'],3), 'frac', round(v['compacted']['frac_of_single_read_roofline'],3), 'same_bits', v['same_bits'], 'sanity', v['sanity']['ok'])
    elif isinstance(v, dict) and 'ms_per_step' in v:
        print(k, 'ms', round(v['ms_per_step'],3))
"
