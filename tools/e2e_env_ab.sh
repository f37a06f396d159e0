#!/bin/bash
# drop-in end-to-end A/B of one environment switch (interleaved rounds, c2 bench stream, 64 GOPs):
#   tools/e2e_env_ab.sh <rounds> VAR=value      (base = the variable unset)
R=$1; KV=$2
for r in $(seq 1 $R); do
  echo "base $(timeout -k 10 200 python tools/e2e_bench.py --gops 64 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["dropin_fps"])')" || exit 1
  echo "$KV $(env $KV timeout -k 10 200 python tools/e2e_bench.py --gops 64 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["dropin_fps"])')" || exit 1
done
