# parity of the channel micro-changes, then interleaved A/B against the committed build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_prover.py -m gpu -k "golden or commit_matches or 2p24 or decommit or tiny or plan_reuse or stale or error or fuzz or prover or fibsq or trace" > gpurun_out/r03_parity5.log 2>&1 || exit 1
for L in 24 20; do for i in 1 2 3 4; do for lib in libfri_amd_base.so libfri_amd.so; do
  ms=$(FRI_AMD_LIB=$lib timeout -k 10 120 python3 bench.py --log-n $L --steps 20 --warmup 3 --no-cpu-baseline --no-extras --no-profile | python3 -c "import json,sys; print(json.loads(sys.stdin.readline())['ms_per_step'])") || exit 2
  echo "$L $lib $ms" >> gpurun_out/r03_ab_chan.txt
done; done; done
