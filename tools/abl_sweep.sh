export MP2VG_LIB=${MP2VG_LIB:-tiny_mp2v_dec_amd/_var/dev/libmp2vg.so}  # tools/dev_build.sh
for v in base v8; do
  if [ $v = base ]; then L=""; else L=tiny_mp2v_dec_amd/_var/$v/libmp2vg.so; fi
  for a in 0 1 2 4 8 32 64; do
    r=$(MP2VG_LIB=$L MP2VG_ABLATE=$a timeout -k 10 100 python tools/launch_breakdown.py --gops 32 | awk '/^launch [0-7]:/{t[$2]=$3} END{printf "I %.4f P %.4f B %.4f", t["0:"], (t["1:"]+t["3:"]+t["5:"])/3, (t["4:"]+t["6:"]+t["7:"])/3}') || exit 1
    echo "$v abl=$a $r"
  done
done
