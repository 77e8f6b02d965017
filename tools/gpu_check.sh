set -e
mkdir -p gpurun_out
bash tools/pmc_icache.sh libfri_amd.so > gpurun_out/r05_pmc_icache.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_ic_libfri_amd k_tree_top k_tree_tail k_tree_mid8 k_layer_leaf_wide > gpurun_out/r05_pmc_icache_summary.txt
