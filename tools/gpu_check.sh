set -e
mkdir -p gpurun_out
FRI_AMD_LIB=libfri_amd_stamps.so timeout -k 10 120 python3 -u stark-prover_amd/bench/stamps.py 24 > gpurun_out/r05t_stamps6.txt 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "commit or tiny or merkle or trace" --timeout 300 --timeout-method thread > gpurun_out/r05t_uni_parity.log 2>&1
bash tools/abn.sh 5 40 libfri_amd_prev.so libfri_amd.so 2>/dev/null > gpurun_out/r05_ab_uniform_job.txt
