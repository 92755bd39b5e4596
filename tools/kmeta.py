"""Register / LDS / spill metadata of kernels in a hipcc -S device .s file."""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for ent in re.split(r"\n\s+- \.agpr_count:", s)[1:]:
    ent = ".agpr_count:" + ent
    name = re.search(r"\.name:\s+(\S+)", ent).group(1)
    if pat not in name:
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", ent) or [None, None])[1]
    print(f"{name[:70]:70s} vgpr {g('vgpr_count')} agpr {g('agpr_count')} lds {g('group_segment_fixed_size')} "
          f"spill {g('vgpr_spill_count')} scratch {g('private_segment_fixed_size')}")
