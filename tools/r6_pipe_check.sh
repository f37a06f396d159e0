#!/bin/bash
# Round-6: GPU parity of the cross-group IDCT pipeline variant, then a same-box A/B (gpurun)
set -o pipefail
mkdir -p gpurun_out
MP2VG_LIB=tiny_mp2v_dec_amd/_var/pipe/libmp2vg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_parity_pipe.log 2>&1 || { tail -30 gpurun_out/gpu_parity_pipe.log; exit 1; }
tail -2 gpurun_out/gpu_parity_pipe.log
CFG=c2 timeout -k 10 900 tools/ab5.sh 2 base head pipe > gpurun_out/ab_r6e.txt 2>&1 || exit 1
cat gpurun_out/ab_r6e.txt
