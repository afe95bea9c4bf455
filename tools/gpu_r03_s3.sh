#!/bin/bash
# kernel traces of the CPSAM B=8 step: tuned-hipBLASLt GEMMs vs PyTorch GEMMs; new attention (vform lib)
set -o pipefail
R=$PWD
O=$R/gpurun_out/s3
mkdir -p $O
V=$R/bioengine_worker_amd/_native/variants/new_vform/libbe_hip.so
cd /tmp && export TMPDIR=/tmp
BE_HIP_LIB=$V timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/lt -o t -- python3 $R/tools/cpsam_train_bench.py --batch 8 --steps 5 --warmup 3 > $O/lt.log 2>&1 || { tail $O/lt.log; exit 1; }
BE_LT=0 BE_HIP_LIB=$V timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/torch -o t -- python3 $R/tools/cpsam_train_bench.py --batch 8 --steps 5 --warmup 3 > $O/torch.log 2>&1 || { tail $O/torch.log; exit 1; }
cd $R
python3 tools/kt_steps.py $O/lt/t_kernel_trace.csv --steps 4 > $O/lt_table.txt && python3 tools/kt_steps.py $O/torch/t_kernel_trace.csv --steps 4 > $O/torch_table.txt
head -40 $O/lt_table.txt; head -40 $O/torch_table.txt
echo done
