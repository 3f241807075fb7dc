# RPN / mask-selection GPU tests, then two independent fp32 bench processes on
# the one GPU (the configuration that faulted before the scratch-free kernels)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_instances.py tests/test_mask_nms_golden.py -x -q --timeout 120 --timeout-method thread -k "rpn or select or nms" > $O/tchk.log 2>&1 || { echo "TESTS FAILED" >> $O/two.log; exit 1; }
bash tools/gpu_two_proc.sh
