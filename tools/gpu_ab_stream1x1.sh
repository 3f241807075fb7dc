# A/B of the fp32 streaming 1x1 kernel (res2 conv3 / conv1) against k_conv_sb
# with the direct epilogue, interleaved, driver bench command without
# secondaries.  Usage: bash tools/gpu_ab_stream1x1.sh
O=gpurun_out
mkdir -p $O
B="--no-cpu-baseline --no-secondary"
for r in 1 2; do
  timeout -k 10 200 python3 -u bench.py $B > $O/ab_s1_$r.json 2>&1 || exit 1
  timeout -k 10 200 python3 -u bench.py $B --set mdx_conv_set_stream1x1_f32=0 > $O/ab_s0_$r.json 2>&1 || exit 1
done
