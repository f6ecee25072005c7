"""Per-iteration split of an mp_ilqr_solve kernel trace (tools/ilqr_trace.sh): µs per kernel, span, gap."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
out = []; cur = None
for r in rows:
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '')
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    short = n.split('(')[0].split('<')[0].replace('void ', '')
    if short == 'ilqr_deriv_kernel':
        if cur: out.append(cur)
        cur = {'t0': int(r['Start_Timestamp'])}
    if cur is not None and 'ilqr' in short:
        cur[short] = cur.get(short, 0) + d
        cur['end'] = int(r['End_Timestamp'])
out.append(cur)
tot = {}
for i, c in enumerate(out):
    wall = (c['end'] - c['t0'])/1e3
    for k, v in c.items():
        if k not in ('t0','end'): tot[k] = tot.get(k, 0) + v
    print(i, ' '.join(f"{k[5:16]}={v:.0f}" for k, v in c.items() if k not in ('t0','end')), f"span={wall:.0f}", f"gap={(out[i+1]['t0']-c['end'])/1e3:.0f}" if i+1 < len(out) else '')
print({k: round(v/1e3,2) for k,v in tot.items()}, (out[-1]['end']-out[0]['t0'])/1e6)
