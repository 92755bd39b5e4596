export TMPDIR=/tmp
timeout -k 10 60 python tools/redbench.py 2>&1 | grep S=
