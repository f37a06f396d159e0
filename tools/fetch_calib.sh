#!/bin/bash
# rocprofv3 passes over tools/fetch_calib.bin (one counter group per pass); summary per kernel.
#   tools/fetch_calib.sh <tag>
set -u
OUT=gpurun_out/fcal_$1
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- tools/fetch_calib.bin > $OUT/p$i.log 2>&1
  echo "pass $i ($grp) rc=$?"
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(k, {c: f"{x:.4g}" for c, x in sorted(v.items())})
PY
