#!/bin/bash
# Round-3 evidence for the current build, one GPU call: GPU tests, smoke, bench lines c2 (with the
# CPU baseline and the drop-in e2e), c1, c3, c4, c5 (tools/r3_final.sh), then the rocprofv3 kernel
# trace + PMC passes of the default two-stream c2 bench command (profiles/traffic_c2_g64.json,
# the roofline.traffic of the bench line) and of the single-stream one (per-kernel launch times).
#   tools/r3_evidence.sh <tag>
set -u
TAG=$1
bash tools/r3_final.sh $TAG || exit 1
tools/profile.sh ${TAG}_s2 --steps 10 --warmup 2 --no-e2e > gpurun_out/r3f_$TAG/profile_s2.log 2>&1 || { tail -5 gpurun_out/r3f_$TAG/profile_s2.log; exit 1; }
echo "profile (2 streams) ok"
MP2VG_STREAMS=1 tools/profile.sh ${TAG}_s1 --steps 10 --warmup 2 --no-e2e > gpurun_out/r3f_$TAG/profile_s1.log 2>&1 || { tail -5 gpurun_out/r3f_$TAG/profile_s1.log; exit 1; }
echo "profile (1 stream) ok"
