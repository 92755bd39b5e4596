# GPU tests with the parity log: bash tools/gpu_tests.sh <tag> [pytest args...]
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
export DV_PARITY_LOG=gpurun_out/parity_$tag.jsonl
rm -f $DV_PARITY_LOG
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread "$@" > gpurun_out/tests_$tag.log 2>&1
rc=$?
tail -25 gpurun_out/tests_$tag.log
exit $rc
