"""CPU: the multi-threaded host pre-pass (pw_host.cpp Packer: chunked lines, parallel classify,
partitioned first-occurrence q~t dedupe, parallel packing, in-order concatenation) produces the
same packed batch whatever the thread count; line ends follow GLineReader (\\n, \\r, \\r\\n);
the target-genome shards of a batch partition its records (pafreport.cpp:303-382)."""
import os

import numpy as np
import pytest

import pwasm_amd as pw
from conftest import synth_paf
from test_shard import _with_duplicates_and_comments


def _arrays(fa, paf, flags=0, threads=None, shard=0, nshards=1):
    old = os.environ.get("PW_THREADS")
    if threads:
        os.environ["PW_THREADS"] = str(threads)
    try:
        b = pw.HostBatch(fa, paf, flags, shard, nshards)
    finally:
        if old is None:
            os.environ.pop("PW_THREADS", None)
        else:
            os.environ["PW_THREADS"] = old
    v = b.view
    out = {k: b.array(k) for k in ("desc", "ops", "lits")}
    out["n"] = (v.n_alns, v.n_ops, v.n_lits, v.n_events_max, v.text_total)
    return b, out


def _records(b, arrs):
    """Per record: (ref, offset, t_len, op words, literal bytes) — offsets-free content."""
    d = arrs["desc"].view(np.uint32).reshape(-1, 8)
    recs = []
    for r in d:
        ob, n, lb = int(r[0]), int(r[1]), int(r[2])
        nl = sum(2 if (w >> 30) == 1 else ((w & 0x3FFFFFFF) if (w >> 30) == 2 else 0) for w in arrs["ops"][ob:ob + n])
        recs.append((int(r[3]), int(r[4]), int(r[5]), tuple(arrs["ops"][ob:ob + n].tolist()),
                     bytes(arrs["lits"][lb:lb + nl])))
    return recs


@pytest.mark.parametrize("config,flags", [(0, 0), (2, pw.FLAG_G | pw.FLAG_C), (0, pw.FLAG_F)])
def test_thread_count_invariance(built, tmp_path, config, flags):
    fa, paf = synth_paf(tmp_path, config, seed=4, scale=0.02 if config == 2 else 1.0)
    if config == 0:
        paf = _with_duplicates_and_comments(paf, tmp_path, 3)
    _, a1 = _arrays(fa, paf, flags, threads=1)
    for t in (2, 7, 16):
        _, at = _arrays(fa, paf, flags, threads=t)
        assert at["n"] == a1["n"]
        for k in ("desc", "ops", "lits"):
            assert np.array_equal(at[k], a1[k]), (t, k)


def test_line_endings(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 0, seed=6)
    _, base = _arrays(fa, paf)
    data = open(paf, "rb").read()
    for name, sep in (("crlf", b"\r\n"), ("cr", b"\r")):
        p = tmp_path / f"{name}.paf"
        body = data.replace(b"\n", sep)
        p.write_bytes(body[:-len(sep)])  # and no line end after the last line
        _, got = _arrays(fa, str(p))
        for k in ("desc", "ops", "lits"):
            assert np.array_equal(got[k], base[k]), (name, k)


@pytest.mark.parametrize("world", [2, 3, 5])
def test_shards_partition_the_records(built, tmp_path, world):
    fa, paf = synth_paf(tmp_path, 0, seed=12)
    paf = _with_duplicates_and_comments(paf, tmp_path, 2)
    b, full = _arrays(fa, paf)
    want = sorted(_records(b, full))
    got = []
    for r in range(world):
        bs, a = _arrays(fa, paf, shard=r, nshards=world)
        got += _records(bs, a)
    assert sorted(got) == want


def test_genome_tables_host_side(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 0, seed=13)
    b = pw.HostBatch(fa, paf, 0)
    gof, taln, names = b.genomes()
    lines = [ln.split("\t") for ln in open(paf).read().splitlines() if ln and not ln.startswith("#")]
    assert len(gof) == b.view.n_alns and len(names) == len(set(n.decode() for n in names))
    assert max(gof) + 1 == len(names)
    # every record's genome is its target name; aligned bases = tend - tstart
    tn = {(f[0], f[5], f[7], f[8]) for f in lines}
    for g, t in zip(gof, taln):
        assert any(x[1] == names[g].decode() and int(x[3]) - int(x[2]) == t for x in tn)
