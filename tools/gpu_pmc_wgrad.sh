set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
R=$(pwd)
OPS="conv_wgrad_64_56_64_3_1 conv_wgrad_128_28_128_3_1 conv_wgrad_256_56_64_1_1"
bash tools/pmc_probe.sh $OPS || exit 1
cd /tmp && export TMPDIR=/tmp
for op in $OPS; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_$op/p3 -o x -- python3 $R/tools/probe_kernels.py $op > $R/gpurun_out/pmc_${op}_3.log 2>&1 || exit 1
done
cd $R
for op in $OPS; do
  echo "#### $op"
  python3 tools/pmc_table.py $(ls gpurun_out/pmc_$op/p1/*counter_collection.csv gpurun_out/pmc_$op/p2/*counter_collection.csv gpurun_out/pmc_$op/p3/*counter_collection.csv) | grep -v "^## zero" | grep -A16 "wgrad_kernel"
done
