"""Exit cost floor of a process that has opened the GPU: a child runs
startup_cost.py's kind of work (or nothing on the device), prints a stamp,
and exits; the parent times stamp -> process end.  Variants: 'none' (numpy +
library load, no device), 'init' (ctg_init only), 'tiny' (one small feature
call), 'hip_only' (the HIP runtime alone: hipInit + hipFree(0) through
ctypes, no libctg).  One JSON line per variant and repeat."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, time, ctypes
sys.path.insert(0, %r)
v = sys.argv[1]
if v == 'hip_only':
    h = ctypes.CDLL('libamdhip64.so')
    h.hipInit(0); h.hipFree(None)
else:
    import numpy as np
    from cluster_tools_amd import _lib, rag
    _lib.load()
    if v in ('init', 'tiny'):
        _lib.init_device()
    if v == 'tiny':
        lab = (np.arange(4 * 8 * 8, dtype=np.uint64) // 7).reshape(4, 8, 8)
        rag.rag_features(lab, np.random.default_rng(0).random(lab.shape, dtype=np.float32))
print(repr(time.time()), flush=True)
''' % ROOT

for rep in range(3):
    for v in ('none', 'hip_only', 'init', 'tiny'):
        p = subprocess.Popen([sys.executable, '-c', CHILD, v], stdout=subprocess.PIPE, text=True)
        line = p.stdout.readline()
        p.wait(timeout=60)
        t_end = time.time()
        ex = round(t_end - float(line), 4) if line.strip() else None
        print(json.dumps({'variant': v, 'rep': rep, 'exit_s': ex, 'rc': p.returncode}), flush=True)
