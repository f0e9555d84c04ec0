set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
bash tools/pmc_probe.sh conv_fwd_64_56_64_3_1 conv_fwd_256_14_256_3_1 conv_fwd_64_56_256_1_1 conv_fwd_512_7_512_3_1 || exit 1
for op in conv_fwd_64_56_64_3_1 conv_fwd_256_14_256_3_1 conv_fwd_64_56_256_1_1 conv_fwd_512_7_512_3_1; do
  echo "#### $op"
  python3 tools/pmc_table.py $(ls gpurun_out/pmc_$op/p1/*counter_collection.csv gpurun_out/pmc_$op/p2/*counter_collection.csv) | grep -v "^## zero\|weight_transpose" 
done
