"""Median batch time per (library, config) and the result hashes of an
interleaved A/B log (tools/ab_head.sh, tools/box_ab.sh).
    python tools/ab_summary.py gpurun_out/<tag>/ab.log"""
import collections
import re
import sys

blocks = open(sys.argv[1]).read().split("== ")[1:]
res = collections.defaultdict(list)
hashes = collections.defaultdict(set)
for blk in blocks:
    head = blk.splitlines()[0].strip()
    lib, cfg = head.split(" ", 1)
    t = [float(x) for x in re.findall(r"gicp_batch ([\d.]+) ms", blk)][1:]
    if t:
        res[head].append(sorted(t)[len(t) // 2])
    h = re.search(r"sha1 (\w+)", blk)
    if h:
        hashes[cfg].add((lib, h.group(1)))
for k, v in res.items():
    print(f"{k:60s} {v}")
for k, v in hashes.items():
    print(k, "identical" if len({h for _, h in v}) == 1 else "DIFFER", sorted(v))
