"""Summarise tools/pmc_trace.sh output: per kernel, counters averaged per dispatch."""
import csv, glob, sys, collections
def kname(k):
    if 'k_material' in k: return 'material'
    if 'k_shade' in k: return 'shade'
    if 'k_trace' not in k: return None
    return ('any' if 'true' in k else 'closest') + ('_p' if 'trace_p' in k else '')

for label in sys.argv[1:]:
    res = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(f'gpurun_out/pmct_{label}/p*/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name']
            kk = kname(k)
            if not kk: continue
            res[kk][r['Counter_Name']].append(float(r['Counter_Value']))
    for f in glob.glob(f'gpurun_out/pmct_{label}/p*/**/*kernel_trace.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name']
            kk = kname(k)
            if not kk: continue
            dur[kk].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    for kk, d in sorted(res.items()):
        m = {c: sum(v) / len(v) for c, v in d.items()}
        w = m.get('SQ_WAVES', 1)
        print(f"== {label} {kk}: dur(median) {sorted(dur[kk])[len(dur[kk])//2]:.1f} us, waves {w:.0f}")
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:12.4g}   per-wave {m[c]/w:10.1f}")
        if 'SQ_THREAD_CYCLES_VALU' in m and 'SQ_ACTIVE_INST_VALU' in m:
            print(f"   lane util (thread/active/64)  {m['SQ_THREAD_CYCLES_VALU']/m['SQ_ACTIVE_INST_VALU']/64:.3f}")
