"""Per-kernel register / spill / scratch summary of a hipcc -save-temps .s file (metadata section)."""
import re
import sys

txt = open(sys.argv[1]).read()
for blk in re.split(r"\n\s+- \.agpr_count:", txt)[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    get = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    agpr = blk.split("\n", 1)[0].strip()
    print(f"{name.group(1) if name else '?':70s} agpr={agpr} vgpr={get('vgpr_count')} spill={get('vgpr_spill_count')} "
          f"scratch={get('private_segment_fixed_size')} sgpr={get('sgpr_count')} lds={get('group_segment_fixed_size')}")
