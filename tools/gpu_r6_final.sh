#!/bin/bash
# Round 6, last tree: the whole GPU suite in the driver's form and smoke(), then the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/tests.log 2>&1 || { grep -E "FAILED|ERROR|Error" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'])
for k,v in d.get('modes',{}).items():
    if isinstance(v, dict) and 'compacted' in v:
        print(k, 'compacted', round(v['compacted']['ms_per_step'],3), 'regathered', round(v['regathered']['ms_per_step'],3), 'speedup', round(v['speedup_compacted'],3), 'same_bits', v['same_bits'])
    elif isinstance(v, dict) and 'ms_per_step' in v:
        print(k, 'ms', round(v['ms_per_step'],3))
    elif isinstance(v, dict) and 'gpu_ms_eager' in v:
        print(k, {kk: vv for kk, vv in v.items() if kk != 'sanity'})
"
