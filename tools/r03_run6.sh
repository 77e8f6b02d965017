# per-kernel A/B (rocprofv3 kernel trace) of the channel micro-changes
set -e
bash tools/kt_ab.sh 2 libfri_amd_base.so libfri_amd_beta.so libfri_amd.so
python3 tools/kt_summary.py gpurun_out libfri_amd_base libfri_amd_beta libfri_amd > gpurun_out/r03_kt_chan.txt
