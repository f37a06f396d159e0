#!/bin/bash
# Round-end evidence on the GPU box: default bench line (with CPU baseline), the rocprofv3 profile
# of the same configuration, and bench lines for configs c3/c4/c5.  Logs in gpurun_out/rb_<tag>/.
set -u
TAG=$1
OUT=gpurun_out/rb_$TAG
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
echo "c2: $(tail -1 $OUT/bench_c2.json | head -c 300)"
tools/profile.sh $TAG > $OUT/profile.log 2>&1 || { cat $OUT/profile.log; exit 1; }
echo "profile ok"
for c in c3 c4 c5; do
  G=64; [ $c = c4 ] && G=16
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --gops $G > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
  echo "$c: $(tail -1 $OUT/bench_$c.json | head -c 200)"
done
