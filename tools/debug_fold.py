"""Debug: mean / var / min / max of the whole-volume boundary call against the
oracle, default histogram range (FAST40) and a wider one, on [0,1] data and
on negative data; one JSON line per case (CTG_LIB selects the build)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from cluster_tools_amd import rag, synthetic as S  # noqa: E402
from oracle import rag_oracle as O  # noqa: E402

lab, bnd = S.generate((20, 32, 40), cell=6, seed=5)
for name, data, rng in [('unit_fast40', bnd, (0.0, 1.0)), ('unit_wide', bnd, (-1.0, 2.0)),
                        ('neg_wide', bnd - 0.7, (-1.0, 1.0)), ('neg_fast40range', (bnd - 0.7).astype(np.float32), (0.0, 1.0))]:
    data = np.ascontiguousarray(data, dtype=np.float32)
    e_ref, f_ref = O.boundary_features(lab, data, lo=rng[0], hi=rng[1])
    out = rag.rag_features(lab, data, hist_range=rng)
    f = out['features']
    same_e = bool(np.array_equal(out['edges'], e_ref))
    res = {'case': name, 'lib': os.path.basename(os.environ.get('CTG_LIB', 'libctg.so')), 'edges_equal': same_e}
    if same_e:
        for c, nm in [(0, 'mean'), (1, 'var'), (2, 'min'), (8, 'max'), (9, 'count')]:
            d = np.abs(f[:, c] - f_ref[:, c]) / np.maximum(np.abs(f_ref[:, c]), 1e-12)
            res[nm] = [float(np.nanmax(d)), int(np.isnan(f[:, c]).sum()), int((d > 1e-5).sum())]
        bad = np.where(np.abs(f[:, 0] - f_ref[:, 0]) > 1e-5 * np.abs(f_ref[:, 0]) + 1e-12)[0][:3]
        res['bad_rows'] = [[float(x) for x in f[i, [0, 1, 2, 8, 9]]] + [float(x) for x in f_ref[i, [0, 1, 2, 8, 9]]]
                           for i in bad]
    print(json.dumps(res), flush=True)
