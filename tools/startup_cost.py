"""Cost of a fresh job process of the drop-in path (the reference's LocalTask
model starts one per job): import, library load, device init, first and
second library call -- printed as one JSON line (run it several times)."""
import json
import os
import sys
import time

t0 = time.perf_counter()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

t_np = time.perf_counter()
from cluster_tools_amd import _lib, rag  # noqa: E402

t_imp = time.perf_counter()
lib = _lib.load()
t_load = time.perf_counter()
_lib.init_device()
t_init = time.perf_counter()
lab = (np.arange(4 * 8 * 8, dtype=np.uint64) // 7).reshape(4, 8, 8)
rag.unique_labels(lab)
t_call1 = time.perf_counter()
rag.rag_features(lab, np.random.default_rng(0).random(lab.shape, dtype=np.float32))
t_call2 = time.perf_counter()
rag.rag_features(lab, np.random.default_rng(1).random(lab.shape, dtype=np.float32))
t_call3 = time.perf_counter()
print(json.dumps({k: round(v * 1e3, 1) for k, v in dict(
    numpy=t_np - t0, import_pkg=t_imp - t_np, dlopen=t_load - t_imp, ctg_init=t_init - t_load,
    first_call=t_call1 - t_init, first_features=t_call2 - t_call1, second_features=t_call3 - t_call2).items()}),
    flush=True)
