# round-3 final evidence with the final library: collection (bench lines,
# kernel stats, PMC traffic, LDE passes), then a plain bench line
set -e
bash tools/r03_collect.sh
timeout -k 10 300 python3 bench.py > gpurun_out/prof_r03/bench_final.json 2>> gpurun_out/prof_r03/bench.err
