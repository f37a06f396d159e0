# per-level times of the fused kernel under ablations (MP2VG_ABLATE; wrong output, timing only)
export MP2VG_LIB=${MP2VG_LIB:-tiny_mp2v_dec_amd/_var/dev/libmp2vg.so}  # tools/dev_build.sh
set -e
mkdir -p gpurun_out/fabl
for a in ${ABLS:-0 8 32}; do
  MP2VG_ABLATE=$a timeout -k 10 200 python tools/launch_breakdown.py --gops 32 > gpurun_out/fabl/$a.txt 2>&1
  echo "abl=$a $(grep -E '^launch [0-9]' gpurun_out/fabl/$a.txt | awk '{printf "%s ", $3}') span $(grep 'batch span' gpurun_out/fabl/$a.txt | awk '{print $3}')"
done
