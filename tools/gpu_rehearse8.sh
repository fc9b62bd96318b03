#!/bin/bash
# The driver's torchrun bench form at N = 2, 4 and 8 rehearsed with gloo ranks
# sharing the one GPU (C2, strong scaling: 20k frames split over the ranks),
# then N = 1: every line's rmsf_checksum must match the 1-GPU run's (the
# merge's summation order differs with N: within 1e-12 relative).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1
port() { python3 -c "import socket;s=socket.socket();s.bind(('127.0.0.1',0));print(s.getsockname()[1])"; }
for n in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $(port) bench.py --gpus $n --backend gloo --steps 3 --warmup 1 \
      > gpurun_out/rehearse${n}_c2.json 2> gpurun_out/rehearse${n}_c2.err
  rc=$?; echo "N=$n rc=$rc"; if [ $rc -ne 0 ]; then tail -20 gpurun_out/rehearse${n}_c2.err; exit $rc; fi
done
timeout -k 10 300 python bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-modes \
    > gpurun_out/rehearse1_c2.json 2> gpurun_out/rehearse1_c2.err
rc=$?; echo "N=1 rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python3 - <<'PY'
import json
v = {n: json.loads(open(f"gpurun_out/rehearse{n}_c2.json").read().strip().splitlines()[-1]) for n in (1, 2, 4, 8)}
for n, d in v.items():
    r = d["roofline"]
    print(f"N={n}: checksum {d['rmsf_checksum']!r} value {d['value']:.4g} ms/step {d['ms_per_step']:.3f} "
          f"ranks {r.get('ranks')} per_device_gbs {[round(x) for x in r.get('per_device_gbs', [])]}")
c1 = v[1]["rmsf_checksum"]
worst = max(abs(d["rmsf_checksum"] - c1) / abs(c1) for d in v.values())
print(f"worst relative checksum difference to the 1-GPU run: {worst:.3e}")
assert worst < 1e-12, "a rank count changes the merged RMSF"
PY
