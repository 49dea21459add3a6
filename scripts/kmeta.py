"""Per-kernel register / LDS / scratch metadata from a hipcc -S listing (amdhsa.kernels YAML)."""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in s.split("  - .agpr_count:")[1:]:
    def f(k):
        m = re.search(r"\." + k + r":\s+(\S+)", blk)
        return m.group(1) if m else "?"
    name = f("name")
    if pat in name:
        print(f"{name[:70]:70s} vgpr {f('vgpr_count'):>4} sgpr {f('sgpr_count'):>4} spill {f('vgpr_spill_count'):>3} "
              f"lds {f('group_segment_fixed_size'):>6} scratch {f('private_segment_fixed_size'):>5}")
