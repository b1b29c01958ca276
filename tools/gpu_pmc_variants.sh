#!/bin/bash
# PMC passes (tools/pmc_micro.sh) of one microbench config for the default lib
# and each variant lib given: gpu_pmc_variants.sh "<config>" v1 v2 ...
cd "$GRAFT_REPO_ROOT"
CFG=$1; shift
bash tools/pmc_micro.sh "$CFG" base > /dev/null || exit 1
python3 tools/pmc_table.py gpurun_out/pmc_base > gpurun_out/pmc_base/table.txt
for v in "$@"; do
  SRHIP_LIB=$PWD/symbolicregression.jl_amd/lib/libsrhip_$v.so bash tools/pmc_micro.sh "$CFG" $v > /dev/null || exit 1
  python3 tools/pmc_table.py gpurun_out/pmc_$v > gpurun_out/pmc_$v/table.txt
done
paste gpurun_out/pmc_base/table.txt $(for v in "$@"; do echo gpurun_out/pmc_$v/table.txt; done)
