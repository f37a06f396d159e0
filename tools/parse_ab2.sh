set -e
for r in 1 2; do
  for L in "" tiny_mp2v_dec_amd/_var/pold/libmp2vg.so; do
    echo "${L:-new}: $(MP2VG_LIB=$L timeout -k 10 120 python tools/parse_bench.py --gops 16 --threads 1 14)"
  done
done
for r in 1 2; do
  for L in "" tiny_mp2v_dec_amd/_var/pold/libmp2vg.so; do
    echo "${L:-new} e2e: $(MP2VG_LIB=$L timeout -k 10 200 python tools/e2e_bench.py --gops 64 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["dropin_fps"], d["parse_fps"])')"
  done
done
