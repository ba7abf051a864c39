"""Summarise rocprofv3 CSV output into profiles/<round>/*.json.

usage: python tools/pmc_summary.py <trace_dir> <pmc_dir_fetch> <pmc_dir_write> <out.json> [algorithmic_bytes [git_sha]]

* kernel stats: <trace_dir>/**/*kernel_stats.csv (Name, Calls, AverageNs ...)
* PMC: <pmc_dir>/**/*counter_collection.csv, one row per (dispatch, counter)
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  The factors that turn them
into HBM bytes come from the counter calibration (tools/calib.hip ->
profiles/r5/calib.json): every read shape the face scan uses
(8-B label and 4-B sample loads per lane, the 8 + 4 B pair, 16-B pieces) and
the 128-B record gathers measure FETCH factor 2.000; the 16-B and 8-B stores
WRITE factor 1.000.  The scan's factors are taken from that file when present.
"""
import csv
import glob
import json
import os
import sys


def _rows(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def kernel_stats(d):
    res = {}
    for r in _rows(os.path.join(d, '**', '*kernel_stats.csv')):
        name = r.get('Name') or r.get('KernelName') or ''
        res[name] = {'calls': int(r['Calls']), 'avg_ns': float(r['AverageNs']),
                     'total_ns': float(r['TotalDurationNs']), 'pct': float(r.get('Percentage', 0.0))}
    return res


def counter_per_dispatch(d, counter):
    """Median over a kernel's dispatches: the first call of a fresh process
    may overflow its initially sized record buffer and rescan (a launch that
    drops the records past the capacity -- at configs[4] it wrote 6.2 of
    17.9 GB), and a mean would count that partial launch in."""
    acc = {}
    for r in _rows(os.path.join(d, '**', '*counter_collection.csv')):
        if r.get('Counter_Name') != counter:
            continue
        name = r.get('Kernel_Name', '')
        acc.setdefault(name, []).append(float(r['Counter_Value']))
    return {k: sorted(v)[len(v) // 2] for k, v in acc.items()}


def pick(d, sub):
    """Largest per-dispatch value among the kernels whose name contains sub
    (1024^3 volumes launch the wide and the narrow face scan; the unselected
    one exits at once)."""
    vals = [v for k, v in d.items() if sub in k]
    return max(vals) if vals else None


CALIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'profiles', 'r5', 'calib.json')
# the calibration kernels standing for the face scan's access shapes
SCAN_READS = ('k_rd<unsigned long>', 'k_rd<unsigned int>', 'k_rd12', 'k_rd<uint4>')
SCAN_WRITES = ('k_wr<uint4>', 'k_wr<unsigned long>')


def factors():
    """(read factor, write factor, provenance) for the scan's access shapes."""
    try:
        k = json.load(open(CALIB))['kernels']
        rf = [k[n]['factor'] for n in SCAN_READS if 'factor' in k.get(n, {})]
        wf = [k[n]['factor'] for n in SCAN_WRITES if 'factor' in k.get(n, {})]
    except (OSError, ValueError, KeyError):
        rf = wf = []
    if rf and wf and max(rf) - min(rf) < 0.02 and max(wf) - min(wf) < 0.02:
        return sum(rf) / len(rf), sum(wf) / len(wf), 'profiles/r5/calib.json ' + ', '.join(SCAN_READS + SCAN_WRITES)
    return 2.0, 1.0, 'uncalibrated default (MI355X_MICROARCH.md HBM section)'


def main():
    trace, pf, pw, out = sys.argv[1:5]
    rfac, wfac, fsrc = factors()
    alg = float(sys.argv[5]) if len(sys.argv) > 5 else None
    sha = sys.argv[6] if len(sys.argv) > 6 else None
    stats = kernel_stats(trace)
    fetch = counter_per_dispatch(pf, 'FETCH_SIZE')
    write = counter_per_dispatch(pw, 'WRITE_SIZE')
    scan_f = pick(fetch, 'k_face_scan')
    scan_w = pick(write, 'k_face_scan')
    summary = {
        'kernel_stats': stats,
        'fetch_size_kib_per_dispatch': fetch,
        'write_size_kib_per_dispatch': write,
        'read_factor': rfac,
        'write_factor': wfac,
        'factor_source': fsrc,
        'note': 'HBM bytes = read_factor x FETCH_SIZE x 1024 + write_factor x WRITE_SIZE x 1024 '
                '(per-dispatch medians)',
        'git_sha': sha,
    }
    # the face scan's average duration from the kernel trace (the launched
    # variant: the unselected tile width exits at once and has a tiny average)
    scans = {k: v for k, v in stats.items() if 'k_face_scan' in k}
    if scans:
        name, st = max(scans.items(), key=lambda kv: kv[1]['avg_ns'])
        summary['scan_kernel'] = name
        summary['scan_avg_ns'] = st['avg_ns']
        nar = [v for k, v in stats.items() if 'k_narrow_labels' in k]
        if nar:
            summary['scan_avg_ns'] += nar[0]['avg_ns']
            summary['scan_kernel'] = 'k_narrow_labels + ' + name
        if alg:
            summary['scan_frac_from_stats'] = alg / (st['avg_ns'] * 1e-9) / 8.0e12
    # long-range affinity calls: the u32 label narrowing pass belongs to the
    # scan's roofline (bench.py times both); its bytes and time are added
    nar_f, nar_w = pick(fetch, 'k_narrow_labels'), pick(write, 'k_narrow_labels')
    if scan_f is not None and nar_f is not None:
        scan_f += nar_f
        scan_w = (scan_w or 0.0) + (nar_w or 0.0)
        summary['includes_k_narrow_labels'] = True
    if scan_f is not None and scan_w is not None:
        summary['scan_hbm_bytes_per_launch'] = rfac * scan_f * 1024 + wfac * scan_w * 1024
        summary['scan_read_bytes_per_launch'] = rfac * scan_f * 1024
        summary['scan_write_bytes_per_launch'] = wfac * scan_w * 1024
        if alg:
            summary['scan_algorithmic_bytes'] = alg
            summary['scan_traffic_over_algorithmic'] = summary['scan_hbm_bytes_per_launch'] / alg
    os.makedirs(os.path.dirname(out) or '.', exist_ok=True)
    with open(out, 'w') as fh:
        json.dump(summary, fh, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in summary.items() if k.startswith('scan')}))


if __name__ == '__main__':
    main()
