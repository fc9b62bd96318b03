#!/bin/bash
# Round-4 validation on one GPU: randomised parity sweeps over the new
# context / merge code, and C4's configuration in the one-process form
# (8 contexts x 30 GB on device 0, atom slabs, reduce to context 0) against
# the unsharded 1M x 20k run.  Each step has its own time limit; the script
# stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4_validate
mkdir -p $O
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi_step.py tests/test_gpu_context_fuzz.py -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 400 python -u tools/fuzz_parity.py 150 > $O/fuzz_parity_150.txt 2>&1 || { tail -5 $O/fuzz_parity_150.txt; exit 1; }
tail -1 $O/fuzz_parity_150.txt
timeout -k 10 500 python -u tools/fuzz_multirank.py 30 --root --planes --scatter > $O/fuzz_multirank_30.txt 2>&1 || { tail -5 $O/fuzz_multirank_30.txt; exit 1; }
tail -1 $O/fuzz_multirank_30.txt
timeout -k 10 300 python -u bench.py --workload c4 --frames 20000 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4_unsharded_one_gpu.json 2> $O/c4_unsharded_one_gpu.err || exit $?
timeout -k 10 300 python -u bench.py --workload c4 --gpus 8 --rehearse --steps 2 --warmup 1 --no-cpu-baseline > $O/c4_one_process_8_contexts.json 2> $O/c4_one_process_8_contexts.err || exit $?
python - <<'PY'
import json
a = json.loads(open("gpurun_out/r4_validate/c4_unsharded_one_gpu.json").read().strip().splitlines()[-1])
b = json.loads(open("gpurun_out/r4_validate/c4_one_process_8_contexts.json").read().strip().splitlines()[-1])
print("unsharded", a["ms_per_step"], repr(a["rmsf_checksum"]), "| 8 contexts", b["ms_per_step"], repr(b["rmsf_checksum"]),
      "| rel", abs(a["rmsf_checksum"] - b["rmsf_checksum"]) / abs(a["rmsf_checksum"]), "| launches", b["roofline"]["launches"])
PY
