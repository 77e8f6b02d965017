# A/B of the XCD-aware tile order in the wide first NTT pass: LDE time and input fetch at 2^28 / 2^25
set -o pipefail
mkdir -p gpurun_out
for L in 28 25; do for i in 1 2; do for lib in libfri_amd_noxcd.so libfri_amd.so; do
  echo "$L $lib $(FRI_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --log-n $L --steps 5 --warmup 1 --no-cpu-baseline --no-extras | python3 -c "import json,sys; j=json.loads(sys.stdin.readline()); print(j['ms_per_step'], j['breakdown_ms_per_step']['lde'], j['oracle_verified'])")" >> gpurun_out/r03_ab_xcd.txt || exit 1
done; done; done
FRI_AMD_LIB=libfri_amd.so bash tools/pmc_lde.sh 28 gpurun_out/r03_pmc_lde_2p28_xcd.json
