# Winograd GEMMs on the fp32 LDS-DMA kernel: tests, then bench A/B over the tile threshold
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread -k "winograd" > $O/twd.log 2>&1 || { echo "EXIT tests $?" >> $O/twd.log; exit 1; }
echo "EXIT 0" >> $O/twd.log
bash tools/gpu_benchvar.sh wd '--set mdx_conv_set_winograd_dma=1,4096|--set mdx_conv_set_winograd_dma=1,16384|--set mdx_conv_set_winograd_dma=0,8192'
