#!/bin/bash
# round-4 session-2 GPU experiments: 2-D luma tap variants (parity, then c2/c3 A/B), pool
# placement (c3), tiled-anchor ablation (c2).  Logs in gpurun_out/r4b/.
#   VS="l2d1 l2d2" QUICK=1 tools/r4_session2.sh
set -o pipefail
mkdir -p gpurun_out/r4b
VS=${VS:-l2d1 l2d2}
for V in $VS; do
  MP2VG_LIB=tiny_mp2v_dec_amd/_var/$V/libmp2vg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b/parity_$V.log 2>&1
  rc=$?; echo "parity $V rc=$rc $(tail -1 gpurun_out/r4b/parity_$V.log)"; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4b/parity_$V.log | head; exit 1; }
done
tools/ab_cfg_env.sh "c2" 3 "--steps 8" base $VS > gpurun_out/r4b/ab_c2.log 2>&1 || { cat gpurun_out/r4b/ab_c2.log; exit 1; }
cat gpurun_out/r4b/ab_c2.log
[ "${QUICK:-0}" = 1 ] && exit 0
tools/ab_cfg_env.sh "c3" 2 "--steps 8" base $VS > gpurun_out/r4b/ab_c3.log 2>&1 || { cat gpurun_out/r4b/ab_c3.log; exit 1; }
cat gpurun_out/r4b/ab_c3.log
timeout -k 10 240 python -u tools/pool_var.py c3 2 > gpurun_out/r4b/pool_var_default.log 2>&1 || exit 1
MP2VG_POOL_ALLOC=1 timeout -k 10 240 python -u tools/pool_var.py c3 2 > gpurun_out/r4b/pool_var_contig.log 2>&1 || exit 1
tools/ab_abl_values.sh dev "--config c2 --steps 8" 2 32768 1024 16384 17408 > gpurun_out/r4b/abl_tiled.log 2>&1 || exit 1
