#!/bin/bash
# attention fwd (main lib, VGPR-form), CPnet skip-add folded into c0's residual epilogue: GPU tests,
# headline bench, and a kernel trace of the headline step.
set -o pipefail
R=$PWD
O=$R/gpurun_out/s5
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cpnet_engine_gpu.py tests/test_cpsam_train_gpu.py tests/test_conv_pair.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 300 python3 bench.py --no-extras --no-served --steps 20 --warmup 5 > $O/bench_headline.json 2> $O/bench_headline.err || { tail $O/bench_headline.err; exit 1; }
cat $O/bench_headline.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o t -- python3 $R/bench.py --no-extras --no-served --steps 6 --warmup 3 > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
cd $R
python3 tools/kt_steps.py $O/kt/t_kernel_trace.csv --steps 4 --marker "conv_pair_kernel<8, 32" --top 45 --width 110 > $O/kt_table.txt || exit 1
cat $O/kt_table.txt
echo done
