"""VGPR / spill / LDS / scratch of the kernels in a gfx950 assembly listing (hipcc -S
--cuda-device-only): python tools/kmeta.py kernels.s [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else "k_"
for blk in s.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if pat not in name:
        continue
    g = lambda k: re.search(rf"\.{k}:\s+(\d+)", blk).group(1)  # noqa: E731
    print(f"{name:60s} vgpr {g('vgpr_count'):>3s} spill {g('vgpr_spill_count'):>3s} sgpr {g('sgpr_count'):>3s} "
          f"lds {g('group_segment_fixed_size'):>5s} scratch {g('private_segment_fixed_size'):>4s}")
