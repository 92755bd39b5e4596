# GPU evidence run: tests (+ parity log), the default bench (all legs), and the
# rocprofv3 kernel trace + stats of a graph-replayed bench whose per-step
# summary (tools/prof_summary.py: the last 3 replayed steps) goes to
# gpurun_out/summary_<tag>.txt.   bash tools/gpu_round.sh <tag>
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
export DV_PARITY_LOG=gpurun_out/parity_$tag.jsonl
rm -f $DV_PARITY_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1 && tail -3 gpurun_out/tests_$tag.log && \
timeout -k 10 500 python bench.py > gpurun_out/bench_$tag.log 2> gpurun_out/bench_$tag.err && tail -1 gpurun_out/bench_$tag.log | cut -c1-400 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-sampling --no-fp32 --no-config3 > gpurun_out/prof_$tag.log 2>&1 && \
python tools/prof_summary.py gpurun_out/prof_$tag/run_kernel_trace.csv 60 3 > gpurun_out/summary_$tag.txt && head -30 gpurun_out/summary_$tag.txt
