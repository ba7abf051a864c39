"""Cost of a fresh job process of the drop-in path (the reference's LocalTask
model starts one per job): import, library load, device init, then the first
call of each kind -- a pinned allocation, a small kernel (mapEdgeIds: one
ctg_reduce.hip kernel), the unique-labels call (rocPRIM sort), a feature
call -- and a repeat.  One JSON line (ms); run it several times."""
import json
import os
import sys
import time

T = [('start', time.perf_counter())]


def mark(name):
    T.append((name, time.perf_counter()))


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
mark('numpy')
from cluster_tools_amd import _lib, rag  # noqa: E402
mark('import_pkg')
lib = _lib.load()
mark('dlopen')
_lib.init_device()
mark('ctg_init')
a = rag.host_arena(1 << 20)
mark('pinned_alloc')
e = np.array([[1, 2], [1, 5], [3, 4]], np.uint64)
rag.map_edge_ids(e, e[::-1])
mark('first_small_kernel')
rag.map_edge_ids(e, e)
mark('second_small_kernel')
lab = (np.arange(4 * 8 * 8, dtype=np.uint64) // 7).reshape(4, 8, 8)
rag.unique_labels(lab)
mark('first_unique_labels')
rag.rag_features(lab, np.random.default_rng(0).random(lab.shape, dtype=np.float32))
mark('first_features')
rag.rag_features(lab, np.random.default_rng(1).random(lab.shape, dtype=np.float32))
mark('second_features')
print(json.dumps({T[i][0]: round((T[i][1] - T[i - 1][1]) * 1e3, 1) for i in range(1, len(T))}), flush=True)
