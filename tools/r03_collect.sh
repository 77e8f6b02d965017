# round-3 evidence: bench lines, kernel stats, PMC traffic at 2^24 and the
# LDE passes at 2^28 (each step under its own time limit; first failure ends it)
set -e
bash tools/collect_profiles.sh r03
bash tools/pmc_lde.sh 28 gpurun_out/prof_r03/pmc_lde_2p28.json
bash tools/pmc_lde.sh 24 gpurun_out/prof_r03/pmc_lde_2p24.json
