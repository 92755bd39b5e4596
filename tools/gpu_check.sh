# quick full check: gpu test suite, then the default bench line (no cpu baseline)
export TMPDIR=/tmp
tag=$1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1; rc=$?; tail -3 gpurun_out/tests_$tag.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 && tail -1 gpurun_out/bench_$tag.log | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], json.dumps(d['roofline']), d['attention']['frac']); [print(k,v) for k,v in list(d['kernels'].items())[:8]]"
