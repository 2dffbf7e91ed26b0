"""GPU cs tokenising (pw_pack_cs_batch) against the host packer pw_pack_cs (the
restatement of pafreport.cpp:536-626 the whole report path is checked with): the same op words,
literal bytes and totals for every well-formed record; every record the kernel hands back to the
host (PW_PACK_HOST) is one the host rejects or one with an op longer than a 256-character window."""
import random
import re

import numpy as np
import pytest

import pwasm_amd as pw
from conftest import synth_paf

pytestmark = pytest.mark.gpu
GRAMMAR = re.compile(rb"(?::[0-9]{1,9}|\*[0-9A-Za-z]{2}|[+-][A-Za-z]+)*")


def paf_records(paf):
    """(cs bytes, offset, qlen) of every record of a PAF (offset: pafreport.cpp:486-490)."""
    out = []
    for line in open(paf, "rb"):
        f = line.rstrip(b"\r\n").split(b"\t")
        if len(f) < 12 or line.startswith(b"#"):
            continue
        ql, qs, qe = int(f[1]), int(f[2]), int(f[3])
        cs = next((x[5:] for x in f[12:] if x.startswith(b"cs:Z:")), None)
        if cs is None:
            continue
        out.append((cs, qs if f[4] == b"+" else ql - qe, ql))
    return out


def edge_records():
    rng = random.Random(7)
    recs = [(b"", 0, 100), (b":10", 0, 10), (b":10", 0, 9), (b":0:5", 0, 5), (b"*ag", 0, 1), (b"*ag", 1, 1),
            (b"*ag", 2, 1), (b"+acg", 0, 3), (b"+acg", 0, 2), (b"-acgt", 0, 0), (b":3*ac-gg+tt:2", 0, 8),
            (b":3*ac-gg+tt:2", -1, 8), (b":3~ac", 0, 10), (b":3=ACG", 0, 10), (b":3-", 0, 10), (b":3+", 0, 10),
            (b":3*a", 0, 10), (b":3*a:2", 0, 10), (b": 3", 0, 10), (b":-3", 0, 10), (b":1234567890", 0, 2 ** 31 - 1),
            (b":123456789", 0, 2 ** 31 - 1), (b":5a", 0, 10), (b"-ac5", 0, 10), (b"*12", 0, 10), (b"x:5", 0, 10),
            (b":2*ac" * 40, 0, 400), (b"-" + b"a" * 300 + b":5", 0, 10), (b":5-" + b"c" * 255 + b":5", 0, 10),
            (b"*NN*aT", 0, 5), (b"-acgtn", 0, 3), (b"*a1:5", 0, 10), (b"*1a-ac", 0, 10)]
    # random well-formed strings of many windows, ops straddling window boundaries
    for _ in range(200):
        parts, q = [], 0
        for _ in range(rng.randint(1, 400)):
            k = rng.random()
            if k < 0.5:
                m = rng.randint(1, 99999)
                parts.append(b":%d" % m)
                q += m
            elif k < 0.7:
                parts.append(b"*" + bytes(rng.choice(b"acgtnACGT") for _ in range(2)))
                q += 1
            elif k < 0.85:
                parts.append(b"-" + bytes(rng.choice(b"acgt") for _ in range(rng.randint(1, 40))))
            else:
                m = rng.randint(1, 40)
                parts.append(b"+" + bytes(rng.choice(b"acgt") for _ in range(m)))
                q += m
        recs.append((b"".join(parts), rng.randint(0, 3), q + rng.randint(-1, 3)))
    return recs


def check(recs):
    ops, lits, off, out = pw.pack_cs_gpu([r[0] for r in recs], [r[1] for r in recs], [r[2] for r in recs])
    n_host = 0
    for i, (cs, o, ql) in enumerate(recs):
        rc, hops, hlits, tot, _ = pw.pack_cs(cs.decode("latin-1"), o, ql)
        g = out[i]
        if g["flags"] & pw.PACK_HOST:
            # handed back only when the host packer rejects the record, or it lies outside the
            # kernel's grammar (blanks / signs / > 9 digits after ':'), or one op exceeds a window
            n_host += 1
            long_op = any(len(x) > 255 for x in cs.replace(b"*", b"\0*").replace(b":", b"\0:").replace(
                b"+", b"\0+").replace(b"-", b"\0-").split(b"\0"))
            assert rc != 0 or long_op or not GRAMMAR.fullmatch(cs), (i, cs[:60])
            continue
        assert rc == 0, (i, cs[:60], rc)
        b = int(off[i])
        assert list(ops[b: b + g["n_ops"]]) == hops, i
        assert bytes(lits[b: b + g["n_lits"]]) == hlits, i
        assert (g["q_total"], g["t_total"], g["n_ops"], g["n_lits"], g["n_events_max"], g["text_bound"]) == \
            (tot.q_total, tot.t_total, tot.n_ops, tot.n_lits, tot.n_events_max, tot.text_bound), i
        assert bool(g["flags"] & pw.PACK_ACGT) == all(c in b"ACGT" for c in hlits), i
    return n_host


def test_pack_cs_batch_edges(built):
    recs = edge_records()
    n_host = check(recs)
    assert 0 < n_host < len(recs)


@pytest.mark.parametrize("config,scale", [(1, 1.0), (2, 0.05), (3, 0.0005), (4, 0.0003)])
def test_pack_cs_batch_synth(built, tmp_path, config, scale):
    fa, paf = synth_paf(tmp_path, config, scale=scale)
    recs = paf_records(paf)
    assert recs
    assert check(recs) == 0
