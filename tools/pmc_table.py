"""Print per-kernel mean counter values from rocprofv3 counter_collection CSVs,
one line per distinct instantiation (template arguments tell the face scan's
modes apart).
usage: python tools/pmc_table.py <dir> [kernel-substring]"""
import csv, glob, os, re, sys
d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else 'k_face_scan'
acc = {}
for f in sorted(glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)):
    for r in csv.DictReader(open(f)):
        if sub not in r['Kernel_Name']:
            continue
        m = re.search(r'<([^>]*)>', r['Kernel_Name'])
        inst = m.group(1).replace(' ', '') if m else r['Kernel_Name'][:40]
        a = acc.setdefault(inst, {})
        a.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
        a.setdefault('_dur_ns', []).append(float(r['End_Timestamp']) - float(r['Start_Timestamp']))
for inst in sorted(acc):
    for k in sorted(acc[inst]):
        v = acc[inst][k]
        print('[%s] %-12s %16.1f (n=%d)' % (inst, k, sum(v) / len(v), len(v)))
