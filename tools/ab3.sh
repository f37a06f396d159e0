#!/bin/bash
# Interleaved A/B of the in-tree build against variant libraries (tools/variant.sh) on one box:
#   CFGS="c2 c3" tools/ab3.sh <rounds> <variant>...     (prints frames/s, ms/step, frac, digest)
R=$1; shift
python -c "import json,sys; sys.path.insert(0,'.'); from tiny_mp2v_dec_amd import build as B; print('provenance:', json.dumps(B.provenance()))"
for cfg in ${CFGS:-c2}; do
  tools/ab_lib.sh "--config $cfg --steps ${STEPS:-10} --no-e2e" $R "$@" | sed "s/^/$cfg /" || exit 1
done
