"""VGPR / spill / occupancy table of every kernel in a .hip file (gfx950):
python tools/resource_usage.py dalle2-video_amd/csrc/dv_conv.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                      "-Wno-unused-function", "-c", src, "-o", "/tmp/_ru.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
rows, cur = [], None
for ln in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", ln) or re.search(r"Name: (\S+) \[", ln)
    if m and "Function Name" in ln:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "VGPRs Spill", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        mm = re.search(rf"    {key}: (\d+)", ln)
        if mm and cur is not None:
            cur[key.split(" ")[0] + ("_spill" if "Spill" in key else "")] = int(mm.group(1))
for r in rows:
    if flt in r["name"]:
        dm = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        dm = re.sub(r"\(anonymous namespace\)::", "", dm)[:90]
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', 0):>4} agpr spill {r.get('VGPRs_spill', 0):>3} "
              f"occ {r.get('Occupancy', '?')}  {dm}")
