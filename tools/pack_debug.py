import sys, os, subprocess, tempfile
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import numpy as np
import pwasm_amd as pw
from test_gpu_pack import paf_records, edge_records
def run(recs, label, maxshow=6):
    ops, lits, off, out = pw.pack_cs_gpu([r[0] for r in recs], [r[1] for r in recs], [r[2] for r in recs])
    bad = []
    for i, (cs, o, ql) in enumerate(recs):
        rc, hops, hlits, tot, _ = pw.pack_cs(cs.decode("latin-1"), o, ql)
        g = out[i]
        if g["flags"] & pw.PACK_HOST:
            continue
        b = int(off[i])
        f = []
        if rc != 0: f.append("rc")
        if list(ops[b:b+g["n_ops"]]) != hops: f.append(f"ops {g['n_ops']} vs {len(hops)}")
        if bytes(lits[b:b+g["n_lits"]]) != hlits: f.append(f"lits {g['n_lits']} vs {len(hlits)}")
        for k in ("q_total","t_total","n_events_max","text_bound"):
            if int(g[k]) != int(getattr(tot,k)): f.append(f"{k} {int(g[k])} vs {int(getattr(tot,k))}")
        if f: bad.append((i, i % 8, len(cs), f))
    print(label, "bad", len(bad), "of", len(recs), flush=True)
    for x in bad[:maxshow]: print("  ", x, flush=True)
    from collections import Counter
    print("   by task position:", Counter(x[1] for x in bad), flush=True)
with tempfile.TemporaryDirectory() as tmp:
    fa, paf = os.path.join(tmp, "q.fa"), os.path.join(tmp, "a.paf")
    subprocess.run(["/root/repo/synth/build/pwsynth", "paf", "--config", "2", "--scale", "0.02", "--seed", "2", "--fa", fa, "--paf", paf], check=True, stderr=subprocess.DEVNULL)
    run(paf_records(paf), "cfg2@0.02")
run(edge_records(), "edges")
