#!/bin/bash
# A/B timing of two builds of libfri_amd.so in one GPU session, interleaved:
#   tools/ab.sh A.so B.so [rounds=4] [steps=20]
# prints ms_per_step of each run (bench.py, no profiling, no CPU baseline).
A=$1; B=$2; R=${3:-4}; S=${4:-20}
for i in $(seq 1 $R); do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    ms=$(FRI_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --steps $S --warmup 3 --no-cpu-baseline --no-profile --no-extras \
         | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['ms_per_step'])") || exit 1
    echo "$v $ms"
  done
done
