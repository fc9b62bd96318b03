#!/bin/bash
# Round 6 PMC: (1) L2->memory read requests by size and WRITE_SIZE of the sparse aligned
# modes, compacted vs re-gathered (verdict item 2); (2) C4 share vs same-bytes headline
# shape: UTCL1 translation hits/misses and TA busy (verdict item 4).  One counter group
# per rocprofv3 pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
O=gpurun_out/${1:-r6pmc}
mkdir -p $O
run() {  # name, counters, command...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/$name -o run -- "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/$name.log; exit $rc; }
  return 0
}
for c in 1 0; do
  run sp_rd_c$c "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" python3 tools/sparse_once.py 10 frame0 $c 1
  run sp_wr_c$c "WRITE_SIZE" python3 tools/sparse_once.py 10 frame0 $c 1
  run spa_rd_c$c "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" python3 tools/sparse_once.py 10 average $c 1
done
run c4_tlb "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum GRBM_GUI_ACTIVE" python3 tools/c4_once.py 2
run c4_ta "TA_BUSY_avr TCP_TCP_TA_DATA_STALL_CYCLES_sum" python3 tools/c4_once.py 2
run c4_rd "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" python3 tools/c4_once.py 2
echo done
