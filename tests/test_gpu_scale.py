"""GPU parity at the benchmarked sizes and on the rare device paths.

* cfg2 in full (100k records, -G -C), cfg3 at 100k records, cfg4 at real 1-5 Mb contigs (five
  records, auto -F, whole report diffed; the smallest also with -G -C; and 1,024 records,
  ~36 M events, CRC-checked against the chunked oracle), cfg5 at full size
  (200 rows x 1M columns, removeConsGaps=false): HIP CLI vs oracle, byte for byte.
* cfg4 property checks that do not depend on the oracle: one event line per cs event head after
  the S-merge (pafreport.cpp:556-560), rloc non-decreasing within a record (tdiffs.Reverse()
  for '-' records, :643), 9-nt query contexts (:721-733), target contexts <= 22 bytes or
  first5[n]last5 (:918-927).
* Event lengths >= 2^19 - 1 (the render record's saturated length field: the Cold record /
  op-stream path), and the modseq check failing on a reverse-strand substitution at a 'U' base
  (comp is not an involution there: U -> A -> T; pafreport.cpp:811-814).
Parity bar: bit-exact."""
import os
import random
import re

import pytest

from conftest import CLI, GA_CLI, GA_ORACLE, ORACLE, SYNTH, run, synth_paf
from test_gpu_parity import same

pytestmark = pytest.mark.gpu


def test_cfg2_full(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 2)
    out = same(["-G", "-C", "-r", fa, paf])
    assert out.count(b">") == 100000


def test_cfg3_100k(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 3, scale=0.01)
    out = same(["-G", "-C", "-r", fa, paf])
    assert out.count(b">") >= 100000


def _cs_heads(cs):
    """Event heads of a short cs string after the S-merge of directly consecutive '*' ops."""
    n, prev_sub = 0, False
    for m in re.finditer(r":\d+|\*[a-z]{2}|[-+][a-z]+", cs):
        op = m.group(0)[0]
        if op == ":":
            if m.group(0) != ":0":  # (a ':0' between '*' ops keeps them contiguous)
                prev_sub = False
            continue
        if op == "*":
            if not prev_sub:
                n += 1
            prev_sub = True
        else:
            n += 1
            prev_sub = False
    return n


def _check_report_properties(paf, report):
    recs = [ln.split("\t") for ln in open(paf).read().splitlines() if ln and not ln.startswith("#")]
    blocks = report.decode().split(">")[1:]
    assert len(blocks) == len(recs)
    for f, blk in zip(recs, blocks):
        cs = next(x[5:] for x in f if x.startswith("cs:Z:"))
        lines = blk.rstrip("\n").split("\n")[1:]
        assert len(lines) == _cs_heads(cs)
        last = -1
        for ln in lines:
            c = ln.split("\t")
            assert c[0] in ("S", "I", "D")
            rloc = int(c[1])
            assert rloc >= last
            last = rloc
            assert len(c[6]) == 9 and c[6].isupper()
            assert len(c[5]) <= 22 or re.fullmatch(r"[A-Za-z]{5}\[\d+\][A-Za-z]{5}", c[5])


def test_cfg4_megabase_contigs(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 4, extra=["--ncds", 5, "--recs", 1])
    lens = [int(ln.split("\t")[1]) for ln in open(paf)]
    assert len(lens) == 5 and min(lens) >= 1000000
    out = same(["-r", fa, paf], timeout=600)  # auto -F (FASTA > 120 kB): the config's mode
    assert out.count(b"\n") > 50000
    _check_report_properties(paf, out)
    # the smallest contig with the codon pass forced on (the oracle's O(L)-per-event suffix
    # copies, pafreport.cpp:908, keep this to one record)
    one = tmp_path / "one.paf"
    lines = open(paf).read().splitlines(keepends=True)
    one.write_text(lines[lens.index(min(lens))])
    same(["-G", "-C", "-r", fa, str(one)], timeout=600)


def test_cfg4_1k_records(built, tmp_path):
    """cfg4 at >= 1k Mb-contig records (BASELINE configs[3], scale 0.102: 1,024 records over 32
    contigs of 1-5 Mb, ~36 M events, auto -F): the CLI's whole report streamed through CRC-32
    against the oracle over byte ranges of the PAF in parallel processes (bench.oracle_crc), plus
    the oracle-independent properties on every 64th record."""
    import subprocess
    import threading

    from bench import crc_stream, host_threads, oracle_crc
    fa, paf = synth_paf(tmp_path, 4, seed=4, scale=0.102, extra=["--threads", host_threads()])
    want = oracle_crc([], fa, paf, host_threads())
    p = subprocess.Popen([str(CLI), "-r", fa, paf], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    err = {}
    th = threading.Thread(target=lambda: err.setdefault("e", p.stderr.read()))
    th.start()
    got = crc_stream(p.stdout)
    rc = p.wait(timeout=300)
    th.join()
    assert rc == 0 and err["e"] == b"", err["e"][-2000:]
    assert got == want[:3], (got, want)
    assert want[2] > 30_000_000
    sub = tmp_path / "sub.paf"
    with open(paf, "rb") as f, open(sub, "wb") as g:
        for i, line in enumerate(f):
            if i % 64 == 0:
                g.write(line)
    rp, out, ep = run([CLI, "-r", fa, sub])
    assert rp == 0, ep
    _check_report_properties(str(sub), out)


def test_cfg5_full_layout(built, tmp_path):
    lay = tmp_path / "l.pwl"
    rc, _, err = run([SYNTH, "layout", "--config", 5, "--seed", 5, "--out", lay])
    assert rc == 0, err
    ro, _, eo = run([GA_ORACLE, lay, tmp_path / "o.pwc"])
    rp, _, ep = run([GA_CLI, lay, tmp_path / "p.pwc"])
    assert (rp, ep) == (ro, eo) and ro == 0
    a, b = tmp_path / "o.pwc", tmp_path / "p.pwc"
    assert os.path.getsize(a) == os.path.getsize(b)
    with open(a, "rb") as x, open(b, "rb") as y:
        while True:
            u, v = x.read(1 << 24), y.read(1 << 24)
            assert u == v
            if not u:
                break


# ---------------------------------------------------------------- rare device paths
def _rand_cds(rng, n):
    s = "ATG" + "".join(rng.choice("ACGT") for _ in range(n - 6))
    return s + "TAA"


def _comp(s):
    return s.translate(str.maketrans("ACGTU", "TGCAA"))[::-1]


def _paf_line(q, ql, qs, qe, strand, t, tl, ts, te, cg, cs):
    return "\t".join(map(str, [q, ql, qs, qe, strand, t, tl, ts, te, 10, 20, 60, "NM:i:1", "AS:i:5",
                               f"cg:Z:{cg}", f"cs:Z:{cs}"])) + "\n"


def test_event_length_past_render_field(built, tmp_path):
    """Deletions / insertions of >= 2^19 - 1 bases: the render record's length field saturates
    and the kernels take the event length from the op stream via the Cold record."""
    rng = random.Random(99)
    L = 600000
    q = _rand_cds(rng, L)
    (tmp_path / "q.fa").write_text(f">big\n{q}\n")
    big = 530000
    a, b = 30000, 30000 + big
    ins = "".join(rng.choice("acgt") for _ in range(big))
    lines = [
        # forward: a deletion of `big` query bases (cs '+', event 'D') and a substitution after it
        _paf_line("big", L, 0, L, "+", "t1", 2 * L, 100, 100 + L - big, f"{a}M{big}I{L - b}M",
                  f":{a}+{q[a:b].lower()}:10*{'c' if q[b + 10] != 'C' else 'g'}{q[b + 10].lower()}:{L - b - 11}"),
        # forward: an insertion of `big` target bases (cs '-', event 'I')
        _paf_line("big", L, 0, L, "+", "t2", 2 * L, 100, 100 + L + big, f"{a}M{big}D{L - a}M",
                  f":{a}-{ins}:{L - a}"),
        # reverse strand: both on the aligned (reverse-complement) strand
        _paf_line("big", L, 0, L, "-", "t3", 2 * L, 100, 100 + L - big, f"{a}M{big}I{L - b}M",
                  f":{a}+{_comp(q)[a:b].lower()}:{L - b}"),
        _paf_line("big", L, 0, L, "-", "t4", 2 * L, 100, 100 + L + big, f"{a}M{big}D{L - a}M",
                  f":{a}-{ins}:{L - a}"),
    ]
    (tmp_path / "a.paf").write_text("".join(lines))
    for flags in (["-G", "-C"], []):
        out = same([*flags, "-r", "q.fa", "a.paf"], cwd=str(tmp_path), timeout=600)
        assert out.count(b">") == 4 and b"[530000]" in out


def _dense_record(rng, q, strand, tname, bad_sub_at=None, sub_run_at=None):
    """One PAF line over the whole query with an event every few bases (thousands of cs ops):
    matches of 1-6, '*' runs, 1-3 base indels.  bad_sub_at=k: the k-th op is a '*' whose query
    base is wrong (the reference's base mismatch error); sub_run_at=k: ops k-2 .. k+2 are one run
    of five directly consecutive '*' ops (an S run across op k)."""
    a = q if strand == "+" else _comp(q)
    L = len(a)
    cs, cg = [], []
    i = t = 0
    cur_m = 0

    def flush():
        nonlocal cur_m
        if cur_m:
            cg.append(f"{cur_m}M")
            cur_m = 0

    nops = 0
    while i < L:
        run = sub_run_at is not None and sub_run_at - 2 <= nops <= sub_run_at + 2
        if nops % 2 == 0 and not run:
            n = min(rng.randint(1, 6), L - i)
            cs.append(f":{n}")
            cur_m += n
            i += n
            t += n
        else:
            kind = "*" if run else rng.choice("*+-")
            if kind == "*" or i + 3 >= L:
                qb = a[i].lower()
                tb = rng.choice([c for c in "acgt" if c != qb])
                if nops == bad_sub_at:
                    qb = rng.choice([c for c in "acgt" if c != a[i].lower()])
                cs.append(f"*{tb}{qb}")
                cur_m += 1
                i += 1
                t += 1
            elif kind == "+":  # query-only bases: event 'D'
                n = min(rng.randint(1, 3), L - i - 1)
                flush()
                cs.append("+" + a[i:i + n].lower())
                cg.append(f"{n}I")
                i += n
            else:  # target-only bases: event 'I'
                n = rng.randint(1, 3)
                flush()
                cs.append("-" + "".join(rng.choice("acgt") for _ in range(n)))
                cg.append(f"{n}D")
                t += n
        nops += 1
    flush()
    return _paf_line("big", L, 0, L, strand, tname, t + 200, 100, 100 + t, "".join(cg), "".join(cs)), nops


@pytest.mark.parametrize("flags", [["-G", "-C"], []])
def test_long_records_blocks(built, tmp_path, flags):
    """Records of more than PW_BLOCK_OPS (2048) cs ops are decoded as blocks by several
    wavefronts (plan_kernel / carry_kernel / index_kernel): both strands, an S run across a block
    boundary, short records between them, and a base mismatch in a later block of a long record
    (the reference's error for that record; nothing after it)."""
    rng = random.Random(77)
    q = _rand_cds(rng, 30000)
    (tmp_path / "q.fa").write_text(f">big\n{q}\n")
    lines = []
    for r, strand in enumerate("+-+-"):
        ln, nops = _dense_record(rng, q, strand, f"t{r}", sub_run_at=2048 + 2 * r)
        assert nops > 3 * 2048
        lines.append(ln)
        lines.append(_paf_line("big", 30000, 0, 60, "+", f"s{r}", 500, 10, 70, "60M", ":60"))
    (tmp_path / "a.paf").write_text("".join(lines))
    out = same([*flags, "-r", "q.fa", "a.paf"], cwd=str(tmp_path), timeout=600)
    assert out.count(b">") == 8
    bad, _ = _dense_record(random.Random(5), q, "-", "tbad", bad_sub_at=5 * 2048 + 17)
    (tmp_path / "b.paf").write_text("".join(lines[:2]) + bad + "".join(lines[2:]))
    rc, _, err = run([ORACLE, *flags, "-r", "q.fa", "b.paf"], cwd=str(tmp_path))
    assert rc == 1 and b"base mismatch" in err
    same([*flags, "-r", "q.fa", "b.paf"], cwd=str(tmp_path), timeout=600)


def test_modseq_mismatch_reverse_u(built, tmp_path):
    """A reverse-strand substitution at a 'U' of the query passes the cs base check (comp(U) =
    A on the aligned strand) but fails predictImpact's modseq check (comp(A) = T != U): the
    reference prints the lines before it and exits 1."""
    rng = random.Random(5)
    q = list(_rand_cds(rng, 60))
    q[30] = "U"
    q = "".join(q)
    (tmp_path / "q.fa").write_text(f">qu\n{q}\n")
    rc_q = _comp(q)  # aligned strand of '-' records
    assert rc_q[29] == "A"
    alt = lambda c: "t" if c.upper() != "T" else "c"  # noqa: E731
    cs = f":10*{alt(rc_q[10])}{rc_q[10].lower()}:18*{alt(rc_q[29])}{rc_q[29].lower()}:30"
    lines = [
        _paf_line("qu", 60, 0, 60, "+", "t0", 200, 10, 70, "60M", f":5*{alt(q[5])}{q[5].lower()}:54"),
        _paf_line("qu", 60, 0, 60, "-", "t1", 200, 10, 70, "60M", cs),
        _paf_line("qu", 60, 0, 60, "+", "t2", 200, 10, 70, "60M", ":60"),
    ]
    (tmp_path / "a.paf").write_text("".join(lines))
    rc, out, err = run([ORACLE, "-r", "q.fa", "a.paf"], cwd=str(tmp_path))
    assert rc == 1 and b"modseq" in err
    same(["-r", "q.fa", "a.paf"], cwd=str(tmp_path))


# ---------------------------------------------------------------- pipelined CLI batches
@pytest.mark.parametrize("chunk,kind", [(3000, None), (20000, None), (5000, "mismatch"), (7000, "crlf")])
def test_cli_many_batches(built, tmp_path, chunk, kind, monkeypatch):
    """The CLI reads the PAF in chunks (PW_CHUNK_BYTES), packs chunk k+1 while the GPU runs
    chunk k, and the q~t dedupe state carries across chunks: same bytes as one pass."""
    from test_gpu_parity import _inject
    from test_shard import _with_duplicates_and_comments
    fa, paf = synth_paf(tmp_path, 0, seed=23)
    paf = _with_duplicates_and_comments(paf, tmp_path, 3)
    if kind == "mismatch":
        paf = _inject(paf, tmp_path, "mismatch", seed=9)
    elif kind == "crlf":
        p = tmp_path / "crlf.paf"
        p.write_bytes(open(paf, "rb").read().replace(b"\n", b"\r\n"))
        paf = str(p)
    monkeypatch.setenv("PW_CHUNK_BYTES", str(chunk))
    same(["-r", fa, paf])


@pytest.mark.parametrize("chunk,kind", [(None, None), (3000, None), (20000, "dups"), (5000, "mismatch"),
                                        (None, "cfg2"), (None, "long"), (60000, "long"), (None, "arena"),
                                        (None, "cfg2img")])
def test_cli_output_file(built, tmp_path, chunk, kind, monkeypatch):
    """-o to a regular file (a stale longer file is truncated), one batch or many, clean batches and
    batches with messages / a fatal record: same bytes, stderr and exit code as the oracle."""
    from test_gpu_parity import _inject
    from test_shard import _with_duplicates_and_comments
    if kind in ("cfg2", "cfg2img"):  # (~90 MB of report: three pinned text windows, written by threads)
        fa, paf = synth_paf(tmp_path, 2, seed=31, scale=0.3)
        flags = ["-G", "-C"]
        if kind == "cfg2img":  # windows cut into 1 MB image groups
            monkeypatch.setenv("PW_EMIT_IMG_BYTES", str(1 << 20))
    elif kind == "arena":  # every line kilobytes: most text in arena pages; images capped at 64 KB so
        # windows are cut into groups and pieces past the cap are written from their sources
        fa, paf = synth_paf(tmp_path, 0, seed=21, extra=["--subrun", 1.0, "--psub", 1.0, "--pdel", 0, "--pins", 0,
                                                         "--err", 0.2, "--rev", 0.5])
        flags = []
        monkeypatch.setenv("PW_EMIT_IMG_BYTES", "65536")
    elif kind == "long":  # long lines (fixup_kernel) and pages that overflow into the arena
        fa, paf = synth_paf(tmp_path, 0, seed=21, extra=["--longindel", 0.5, "--subrun", 0.6, "--err", 0.05])
        flags = []
    else:
        fa, paf = synth_paf(tmp_path, 0, seed=29)
        flags = []
    if kind == "dups":
        paf = _with_duplicates_and_comments(paf, tmp_path, 3)
    elif kind == "mismatch":
        paf = _inject(paf, tmp_path, "mismatch", seed=13)
    if chunk:
        monkeypatch.setenv("PW_CHUNK_BYTES", str(chunk))
    want, got = tmp_path / "o.txt", tmp_path / "h.txt"
    got.write_bytes(b"stale\n" * 3_000_000)
    ro, _, eo = run([ORACLE, *flags, "-r", fa, paf, "-o", want])
    rp, _, ep = run([CLI, *flags, "-r", fa, paf, "-o", got])
    assert (rp, ep) == (ro, eo), (rp, ro, ep[-2000:], eo[-2000:])
    assert got.read_bytes() == want.read_bytes()
