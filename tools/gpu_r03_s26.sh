#!/bin/bash
# conv_pair: per-channel constants in LDS (CM = 64 shared-affine variants): numerics + headline A/B
set -o pipefail
R=$PWD
export PYTHONPATH=$R
O=$R/gpurun_out/s26
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "conv or cpnet or cellpose" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
for v in base main base main; do
  if [ $v = base ]; then L=$R/bioengine_worker_amd/_native/variants/base/libbe_hip.so; else L=$R/bioengine_worker_amd/_native/libbe_hip.so; fi
  BE_HIP_LIB=$L timeout -k 10 200 python bench.py --no-extras --no-served --steps 10 > $O/bench_$v.log 2>&1 || { tail $O/bench_$v.log; exit 1; }
  echo $v $(tail -1 $O/bench_$v.log | cut -c1-200)
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o t -- python3 $R/bench.py --no-extras --no-served --steps 5 --warmup 2 > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
cd $R
python3 tools/kt_steps.py $O/kt/t_kernel_trace.csv --steps 4 --marker "conv_pair_kernel<8, 32" --top 30 --width 110 > $O/kt_table.txt || exit 1
rm -f $O/kt/t_kernel_trace.csv
head -24 $O/kt_table.txt
echo done
