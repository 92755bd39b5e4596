export TMPDIR=/tmp
timeout -k 10 120 python tools/kbench.py fwd 2>&1 | grep conv
