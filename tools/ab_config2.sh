set -e
for i in 1 2; do
for spec in grid=cur hyb=libxudp_amd/variants/hyb/libxcsum.so head=libxudp_amd/variants/head/libxcsum.so; do
  name="${spec%%=*}"; lib="${spec#*=}"
  if [ "$lib" = cur ]; then unset XCSUM_LIB; else export XCSUM_LIB=$lib; fi
  tools/gpu_run.sh e6_2_${name}_$i 200 python tools/sweep.py --config 2 --rounds 6 --geoms "16,1,6;16,2,6" --bpc 3
done
done
