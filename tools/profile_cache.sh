#!/bin/bash
# Cache / memory-issue counters of the recon kernels (dev tool, GPU box), one pass per pair.
set -u
OUT=gpurun_out/profk_$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$name -o $name -- python3 tools/launch_breakdown.py --gops 32 > $OUT/$name.log 2>&1
  echo "$name rc=$?"
}
run k1 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
run k2 TCC_HIT_sum TCC_MISS_sum
run k3 SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL
run k4 TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr
run k5 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum
run k6 SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM
run k7 GRBM_GUI_ACTIVE SQ_WAIT_ANY
