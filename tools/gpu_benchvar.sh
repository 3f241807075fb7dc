# fp32 bench lines for a list of extra-argument variants ("|"-separated)
set -o pipefail
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
mkdir -p $O
IFS='|' read -ra VARS <<< "$2"
i=0
for v in "${VARS[@]}"; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-secondary $v --dump-convs $O/convsv$T-$i.json > $O/benchv$T-$i.json 2> $O/benchv$T-$i.err || { echo "EXIT $? variant $i" >> $O/benchv$T.log; exit 1; }
  echo "$i: $v -> $(python3 -c "import json; d=json.load(open('$O/benchv$T-$i.json')); print(d['value'], d['roofline']['all_conv']['ms_per_step'])")" >> $O/benchv$T.log
  i=$((i+1))
done
echo EXIT 0 >> $O/benchv$T.log
