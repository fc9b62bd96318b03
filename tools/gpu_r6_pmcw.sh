#!/bin/bash
# Round 6: where the dense copy's writes cost time -- the C3 1-in-10 covariance
# pass compacted (c1) vs re-gathered (c0), L2 write path, TCP and SQ counters,
# one counter group per rocprofv3 pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
O=gpurun_out/${1:-r6pmcw}
mkdir -p $O
run() {  # name, counters, command...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/$name -o run -- "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$name.log; exit $rc; }
  return 0
}
for c in 1 0; do
  run w1_c$c "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum GRBM_GUI_ACTIVE" python3 tools/sparse_once.py 10 frame0 $c 1
  run w2_c$c "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_DRAM_sum" python3 tools/sparse_once.py 10 frame0 $c 1
  run w3_c$c "TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum" python3 tools/sparse_once.py 10 frame0 $c 1
  run w4_c$c "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM" python3 tools/sparse_once.py 10 frame0 $c 1
done
echo done
