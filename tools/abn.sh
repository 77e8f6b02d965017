#!/bin/bash
# N-way interleaved timing of builds of libfri_amd.so in one GPU session:
#   tools/abn.sh ROUNDS STEPS A.so B.so [C.so ...]   -> "<lib> <ms_per_step>" lines
R=$1; S=$2; shift 2
for i in $(seq 1 $R); do
  for lib in "$@"; do
    ms=$(FRI_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --steps $S --warmup 3 --no-cpu-baseline --no-profile --no-extras \
         | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['ms_per_step'])") || exit 1
    echo "$(basename $lib) $ms"
  done
done
