# attention iteration: mqa parity tests, then the full gpu suite and a bench line
export TMPDIR=/tmp
tag=$1
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k mqa -x -v --timeout 120 --timeout-method thread > gpurun_out/attn_$tag.log 2>&1; rc=$?; tail -15 gpurun_out/attn_$tag.log; [ $rc -eq 0 ] && \
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1 && tail -3 gpurun_out/tests_$tag.log && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 && tail -1 gpurun_out/bench_$tag.log | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['attention']); [print(k,v) for k,v in d['kernels'].items() if 'attn' in k]"
