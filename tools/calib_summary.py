"""Per-access-width FETCH_SIZE / WRITE_SIZE factors from tools/calib.hip runs.

usage: python tools/calib_summary.py <gpurun_out/TAG> <out.json>

factor = algorithmic bytes / (counter KiB x 1024): the multiplier that turns a
kernel's FETCH_SIZE (WRITE_SIZE) of that access shape into HBM bytes.  Also
the achieved GB/s of each shape from the kernel trace.
"""
import csv
import glob
import json
import os
import sys


def rows(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def short(name):
    n = name.split('(')[0].replace('void ', '').strip()
    return n.replace('HIP_vector_type<unsigned int, 4u> ', 'uint4').replace('HIP_vector_type<unsigned int, 4u>', 'uint4')


def main():
    d, out = sys.argv[1], sys.argv[2]
    spec = json.load(open(os.path.join(d, 'calib.json')))
    stats = {short(r['Name']): float(r['AverageNs']) for r in rows(os.path.join(d, 'trace', '**', '*kernel_stats.csv'))}
    cnt = {}
    for sub, counter in (('fetch', 'FETCH_SIZE'), ('write', 'WRITE_SIZE')):
        for r in rows(os.path.join(d, sub, '**', '*counter_collection.csv')):
            if r.get('Counter_Name') != counter:
                continue
            cnt.setdefault((short(r['Kernel_Name']), counter), []).append(float(r['Counter_Value']))
    res = {}
    for k, v in spec['kernels'].items():
        kk = k.replace('unsigned long', 'unsigned long').strip()
        name = next((s for s in stats if s == kk or s.endswith(kk)), kk)
        e = {'algorithmic_bytes': v.get('read', v.get('write')), 'kind': 'read' if 'read' in v else 'write'}
        e['avg_ms'] = stats.get(name, 0.0) / 1e6
        if e['avg_ms']:
            e['achieved_GBps'] = e['algorithmic_bytes'] / (e['avg_ms'] * 1e-3) / 1e9
        for counter in ('FETCH_SIZE', 'WRITE_SIZE'):
            vals = cnt.get((name, counter))
            if vals:
                kib = sum(vals) / len(vals)
                e[counter + '_bytes'] = kib * 1024
                want = 'FETCH_SIZE' if e['kind'] == 'read' else 'WRITE_SIZE'
                if counter == want and kib:
                    e['factor'] = e['algorithmic_bytes'] / (kib * 1024)
        res[name] = e
    json.dump({'source': d, 'kernels': res}, open(out, 'w'), indent=1, sort_keys=True)
    for k, e in res.items():
        print('%-28s %-5s factor %-6s %8.1f GB/s' % (k, e['kind'], ('%.3f' % e['factor']) if 'factor' in e else '-',
                                                     e.get('achieved_GBps', 0.0)))


if __name__ == '__main__':
    main()
