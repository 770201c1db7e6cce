"""Map the PCs of a glog-style crash trace ('@ 0x... ') to library + offset using a /proc/self/maps
dump of the same process (tools/diag/prof_exit.py).  Usage: resolve_pcs.py crash.log maps.txt"""
import re
import sys

log, maps = sys.argv[1], sys.argv[2]
regions = []
for ln in open(maps):
    parts = ln.split()
    if len(parts) < 6:
        continue
    lo, hi = (int(v, 16) for v in parts[0].split("-"))
    regions.append((lo, hi, int(parts[2], 16), parts[5]))
for ln in open(log):
    for pc in re.findall(r"(?:@|PC:\s*@)\s+(0x[0-9a-f]+)", ln):
        a = int(pc, 16)
        hit = next(((lo, off, path) for lo, hi, off, path in regions if lo <= a < hi), None)
        print(pc, "->", f"{hit[2]} +{a - hit[0] + hit[1]:#x}" if hit else "?")
