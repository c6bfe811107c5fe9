set -e
for spec in cur=cur wpe7=libxudp_amd/variants/wpe7/libxcsum.so wpe8=libxudp_amd/variants/wpe8/libxcsum.so; do
  name="${spec%%=*}"; lib="${spec#*=}"
  if [ "$lib" = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=$lib; fi
  tools/gpu_run.sh e8_3_${name} 200 python tools/sweep.py --config 3 --rounds 5 --geoms "4,1,2;4,2,2" --bpc 0,6,7,8
done
