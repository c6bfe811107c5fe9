set -e
G="4,1,2;64,0,8;64,0,16"
for r in 1 2; do
for v in cur wpe5 wpe6; do
  if [ $v = cur ]; then L=libxudp_amd/libxcsum.so; else L=libxudp_amd/variants/$v/libxcsum.so; fi
  XCSUM_LIB=$L timeout -k 10 120 python tools/sweep.py --config 3 --geoms "$G" --bpc 0,3,4,5 --rounds 3 > gpurun_out/r02e/sw_${v}_$r.log 2>&1
done
done
