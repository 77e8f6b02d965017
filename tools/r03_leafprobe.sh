set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/leafprobe -o run -- python3 $R/tools/leaf_probe.py > $R/gpurun_out/leafprobe.txt 2>&1
