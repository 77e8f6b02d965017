# two-pass 2^24 NTT (NTT_WIDE24 build): parity, A/B against the 8+8+8 build, LDE traffic
set -o pipefail
mkdir -p gpurun_out
FRI_AMD_LIB=libfri_amd_w24.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "lde or interpolate_roundtrip or 2p24 or commit_matches" > gpurun_out/r03_w24_parity.log 2>&1 || exit 1
for i in 1 2 3 4; do for lib in libfri_amd.so libfri_amd_w24.so; do
  echo "$lib $(FRI_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras | python3 -c "import json,sys; j=json.loads(sys.stdin.readline()); print(j['ms_per_step'], j['breakdown_ms_per_step']['lde'], j['oracle_verified'])")" >> gpurun_out/r03_ab_w24.txt || exit 2
done; done
FRI_AMD_LIB=libfri_amd_w24.so bash tools/pmc_lde.sh 24 gpurun_out/r03_pmc_lde_2p24_w24.json
