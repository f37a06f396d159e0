#!/bin/bash
# rocprofv3 evidence of the ONE-STREAM bench batch (tools/onestream.py: one launch shape per
# kernel): a kernel-trace --stats pass, then one --kernel-trace --pmc pass per counter group
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in passes of their own; at most 4 TCC / 4 TCP /
# 8 SQ / 2 TA counters per pass).  Summary: tools/pmc5_summary.py gpurun_out/pmc5_<tag>.
#   CFG=c2 [GOPS=n] REPS=2 [PMC_GROUPS="<counters>\n<counters>"] [MP2VG_LIB=<variant .so>] tools/pmc5.sh <tag>
set -u
TAG=$1
CFG=${CFG:-c2}
REPS=${REPS:-2}
OUT=gpurun_out/pmc5_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o ktrace -- \
  python3 tools/onestream.py --config $CFG ${GOPS:+--gops $GOPS} --reps 5 > $OUT/ktrace.log 2>&1
rc=$?; echo "ktrace rc=$rc $(tail -c 400 $OUT/ktrace.log)"; [ $rc = 0 ] || exit 1
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- \
    python3 tools/onestream.py --config $CFG ${GOPS:+--gops $GOPS} --reps $REPS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc ($grp)"; [ $rc = 0 ] || exit 1
done <<GROUPS
${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum
TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_PENDING_STALL_CYCLES_sum
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES
TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_REQ_sum TCC_STREAMING_REQ_sum TCC_NORMAL_EVICT_sum TCC_EA0_RDREQ_DRAM_sum}
GROUPS
python3 tools/pmc5_summary.py $OUT > $OUT/summary.md && cat $OUT/summary.md
