"""Print per-kernel mean counter values from rocprofv3 counter_collection CSVs.
usage: python tools/pmc_table.py <dir> [kernel-substring]"""
import csv, glob, os, sys
d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else 'k_face_scan'
acc = {}
for f in sorted(glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)):
    for r in csv.DictReader(open(f)):
        if sub not in r['Kernel_Name']:
            continue
        acc.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
        acc.setdefault('_dur_ns', []).append(float(r['End_Timestamp']) - float(r['Start_Timestamp']))
for k in sorted(acc):
    v = acc[k]
    print('%-24s %16.1f  (n=%d)' % (k, sum(v) / len(v), len(v)))
