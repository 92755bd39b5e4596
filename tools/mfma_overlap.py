"""Scan the gfx950 assembly of every csrc/*.hip for MFMAs whose destination
overlaps their own A / B operand registers (hipcc emits that for the untied
form when C is the inline constant 0; on the mid attention it corrupted P).
  python tools/mfma_overlap.py            -> one line per kernel with overlaps"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "dalle2-video_amd", "csrc")


def rng(t):
    m = re.match(r"([va])\[(\d+):(\d+)\]", t) or re.match(r"([va])(\d+)()$", t)
    if not m:
        return None
    lo = int(m.group(2))
    return m.group(1), lo, int(m.group(3) or lo)


def scan(asm):
    out, cur = {}, None
    for line in asm.split("\n"):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
        if "v_mfma" not in line:
            continue
        ops = [x.strip() for x in line.split(None, 1)[1].split(",")]
        d = rng(ops[0])
        for src in (rng(ops[1]), rng(ops[2])):
            if d and src and d[0] == src[0] and not (src[2] < d[1] or src[1] > d[2]):
                out.setdefault(cur, []).append(line.strip())
    return out


def main():
    bad = 0
    with tempfile.TemporaryDirectory() as td:
        for f in sorted(glob.glob(os.path.join(SRC, "*.hip"))):
            s = os.path.join(td, os.path.basename(f) + ".s")
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                            "--cuda-device-only", "-S", f, "-o", s], check=True, cwd=SRC)
            for k, v in scan(open(s).read()).items():
                bad += 1
                print(f"{os.path.basename(f)}: {k}: {len(v)} e.g. {v[0]}")
    print(f"{bad} kernels with an MFMA destination over its own A / B operand")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
