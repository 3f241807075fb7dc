mkdir -p gpurun_out
for k in "" "narrow_kmax=64" "sb_afp=1" "stream1x1_f32=0" "narrow_kmax=64 sb_afp=1"; do
  n=$(echo "$k" | tr ' =' '__'); [ -z "$n" ] && n=default
  timeout -k 10 200 python -u tools/gemm32bench.py $k > gpurun_out/sw_$n.log 2>&1 || exit 1
done
