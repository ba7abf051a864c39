"""Mean per-phase wall ms of the distributed step from CTG_DIST_DEBUG=1
stderr lines ("[dist r0] <phase> <ms> ms"), skipping the warm-up calls.
usage: dist_phases.py <stderr log> [skip]"""
import re
import sys
from collections import defaultdict

skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
acc = defaultdict(list)
for ln in open(sys.argv[1]):
    m = re.match(r'\[dist r0\] (.*?) ([0-9.]+) ms$', ln.strip())
    if m:
        acc[re.sub(r'\(.*\)', '', m.group(1)).strip()].append(float(m.group(2)))
for k, v in acc.items():
    v = v[skip:]
    print('%-22s %8.3f ms (n=%d)' % (k, sum(v) / max(len(v), 1), len(v)))
