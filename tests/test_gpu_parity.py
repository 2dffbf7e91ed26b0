"""GPU parity: the HIP path (pwasm_amd/bin/pafreport -> libpwasm_amd.so kernels) against the
oracle on the same inputs — byte-identical stdout, stderr and exit code.

Inputs: the hand-derived KATs (tests/golden/kat), seeded synthetic PAF for every config shape
 at sizes the oracle finishes in seconds, injected errors at random records,
all -G/-F/-C/-N modes, the torch-stream batch API, and the GapAssem column consensus.
Parity bar: bit-exact (integer/byte work only)."""
import os
import random
import shutil
import struct

import numpy as np
import pytest

import pwasm_amd as pw
from conftest import CLI, GA_CLI, GA_ORACLE, KAT_DIR, ORACLE, SYNTH, run, synth_paf
from test_oracle_kat import read_pwc, run_case, write_pwl

pytestmark = pytest.mark.gpu

CASES = sorted(d for d in os.listdir(KAT_DIR) if os.path.isdir(KAT_DIR / d))


@pytest.mark.parametrize("case", CASES)
def test_kat_on_gpu(built, case, tmp_path):
    run_case(CLI, case, tmp_path)


def same(args, cwd=None, timeout=900):
    """Run oracle and product with the same args; compare everything the reference prints."""
    ro, oo, eo = run([ORACLE, *args], cwd=cwd, timeout=timeout)
    rp, op, ep = run([CLI, *args], cwd=cwd, timeout=timeout)
    assert rp == ro, (rp, ro, ep[-2000:], eo[-2000:])
    if op != oo:
        a, b = oo.decode(errors="replace").splitlines(), op.decode(errors="replace").splitlines()
        for i, (x, y) in enumerate(zip(a, b)):
            if x != y:
                pytest.fail(f"first difference at line {i}:\noracle: {x!r}\nhip:    {y!r}")
        pytest.fail(f"length differs: oracle {len(a)} lines, hip {len(b)} lines")
    assert ep == eo
    return oo


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_edge_mix(built, tmp_path, seed):
    fa, paf = synth_paf(tmp_path, 0, seed=seed)
    out = same(["-r", fa, paf])
    assert out.count(b"\n") > 100


@pytest.mark.parametrize("seed", [1, 7])
def test_edge_mix_host_packer(built, tmp_path, seed, monkeypatch):
    """The CLI packs cs strings on the GPU by default (pw_pack_cs_batch); PW_PACK_HOST=1 keeps the
    host packer (the -w path uses it always): same bytes either way."""
    monkeypatch.setenv("PW_PACK_HOST", "1")
    fa, paf = synth_paf(tmp_path, 0, seed=seed)
    same(["-r", fa, paf])


@pytest.mark.parametrize("flags", [["-G", "-C"], ["-F", "-N"]])
def test_cli_report_args_poisoned(built, tmp_path, monkeypatch, flags):
    """PW_ARGS_POISON=1 fills the CLI's pw_report_args with 0xFF before its fields are assigned
    (flags / n_queries were left as stack garbage): a field left unset then shows up as
    PW_E_ARG or a wrong report, never as whatever the stack held."""
    monkeypatch.setenv("PW_ARGS_POISON", "1")
    fa, paf = synth_paf(tmp_path, 0, seed=12)
    same([*flags, "-r", fa, paf])


@pytest.mark.parametrize("flags", [[], ["-C"], ["-N"], ["-G"], ["-F"], ["-G", "-C"], ["-F", "-C"]])
def test_modes(built, tmp_path, flags):
    fa, paf = synth_paf(tmp_path, 0, seed=11)
    same([*flags, "-r", fa, paf])


def test_cfg1_plumbing(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 1)
    out = same(["-r", fa, paf])
    assert out.count(b">") == 20


def test_cfg2_subsample(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 2, scale=0.05)
    same(["-G", "-C", "-r", fa, paf])


def test_cfg3_subsample(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 3, scale=0.0004)
    same(["-G", "-C", "-r", fa, paf])


def test_cfg4_long_contigs_full_genome_mode(built, tmp_path):
    # dense cs over long queries (auto -F: FASTA > 120 kB); contigs shortened so the oracle's
    # O(L) per-event suffix copy (pafreport.cpp:908) stays within seconds
    fa, paf = synth_paf(tmp_path, 4, extra=["--ncds", 2, "--len-min", 150000, "--len-max", 250000, "--recs", 3,
                                            "--err", 0.02])
    assert os.path.getsize(fa) > 120000
    out = same(["-r", fa, paf])
    assert out.count(b"\n") > 5000


def test_long_indels_and_runs(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 0, seed=21, extra=["--longindel", 0.5, "--subrun", 0.6, "--err", 0.05])
    same(["-r", fa, paf])


def test_arena_pages(built, tmp_path):
    """Records of nothing but long '*' runs: every line is kilobytes (fixup_kernel) and chunks reserve
    up to ~150 KB, far past a page (PW_PAGE_BYTES - kPageSlack): render's arena pages and their
    per-lane copy-out (the in-place pages go through the LDS page image instead)."""
    for seed in (21, 22):
        fa, paf = synth_paf(tmp_path, 0, seed=seed, extra=["--subrun", 1.0, "--psub", 1.0, "--pdel", 0, "--pins", 0,
                                                           "--err", 0.2, "--rev", 0.5])
        same(["-r", fa, paf])


def test_long_lines_many_chunks(built, tmp_path):
    """~300 chunks of lines with long indels and S runs: dozens of lines longer than render's LDS
    line buffer (kLine = 108 bytes with the newline: held or re-emitted by render, or rewritten in
    place by fixup_kernel), and hundreds of 93-108 byte lines, built by render in the line buffer's
    slack (kLine was 92 until round 4)."""
    fa, paf = synth_paf(tmp_path, 0, seed=21, scale=10, extra=["--longindel", 0.5, "--subrun", 0.6, "--err", 0.05])
    out = same(["-r", fa, paf])
    lines = [l for l in out.split(b"\n") if l[:2] in (b"S\t", b"I\t", b"D\t")]
    assert len(lines) > 4 * 64 * 64
    assert sum(len(l) >= 108 for l in lines) > 40  # (the oracle: 55)
    assert sum(92 <= len(l) < 108 for l in lines) > 500  # (681)


@pytest.mark.parametrize("opts,lo,hi", [
    # S runs of 5+ bases (a general-path wave's long lines: render's per-wave list and epilogue,
    # several per chunk)
    (["--err", 0.05, "--subrun", 0.5, "--psub", 1.0, "--pdel", 0, "--pins", 0], 20, 0),
    # every line a long S run past 212 bytes (more long lines per chunk than render holds or lists,
    # and lines past the epilogue's buffer: fixup_kernel)
    (["--err", 0.1, "--subrun", 1.0, "--psub", 1.0, "--pdel", 0, "--pins", 0], 100, 100),
])
def test_long_lines_render_paths(built, tmp_path, opts, lo, hi):
    """Lines past render's line buffer (kLine = 108): a fast wave's first one is held in the
    interleaved rows and stored by the copy-out, a wave's others of up to 212 bytes go to its list
    (kLongCap = 4) and are emitted again after its last chunk, the rest to fixup_kernel — same
    bytes as the oracle on each route."""
    fa, paf = synth_paf(tmp_path, 0, seed=5, scale=2, extra=opts)
    out = same(["-r", fa, paf])
    lines = [l for l in out.split(b"\n") if l[:2] in (b"S\t", b"I\t", b"D\t")]
    assert sum(len(l) >= 108 for l in lines) >= lo
    assert sum(len(l) >= 212 for l in lines) >= hi


@pytest.mark.parametrize("err", [0.25, 0.45])
def test_dense_target_contexts(built, tmp_path, err):
    """Events every few bases: most target contexts need the op walk (tctx_kernel's batches of
    128, and groups of slots with more flagged events than its list holds beside the carried ones)."""
    fa, paf = synth_paf(tmp_path, 0, seed=11, scale=2, extra=["--err", err])
    out = same(["-r", fa, paf])
    assert out.count(b"\n") > 1000


def test_reverse_only_and_forward_only(built, tmp_path):
    for rev in (0.0, 1.0):
        fa, paf = synth_paf(tmp_path, 0, seed=31, extra=["--rev", rev])
        same(["-r", fa, paf])


def _inject(paf, tmp_path, kind, seed):
    lines = open(paf).read().splitlines(keepends=True)
    rng = random.Random(seed)
    idx = [i for i, l in enumerate(lines) if not l.startswith("#") and "*" in l]
    k = rng.choice(idx[len(idx) // 3:])
    f = lines[k].rstrip("\n").split("\t")
    cs = [i for i, x in enumerate(f) if x.startswith("cs:Z:")][0]
    if kind == "mismatch":  # flip the query base of one '*' op
        s = f[cs]
        j = s.index("*", 5)
        q = s[j + 2]
        f[cs] = s[:j + 2] + ("c" if q != "c" else "g") + s[j + 3:]
    elif kind in ("mismatch_splice", "star_bad"):
        # a '*' op (its query base flipped, or clean) right before a '~' / an unknown op byte: the
        # GPU packer hands the record back, and the host-packed prefix must reach index_kernel
        # so the first error in cs order is the one reported (pafreport.cpp:545-548, 620-624)
        s = f[cs]
        j = s.index("*", 5)
        q = s[j + 2]
        if kind == "mismatch_splice":
            f[cs] = s[:j + 2] + ("c" if q != "c" else "g") + "~gt10ag" + s[j + 3:]
        else:
            f[cs] = s[:j + 3] + "Q" + s[j + 3:]
    elif kind == "bounds":
        f[cs] = f[cs] + ":1000000"
    elif kind == "cigar":
        cg = [i for i, x in enumerate(f) if x.startswith("cg:Z:")][0]
        f[cg] = f[cg] + "3Q"
    lines[k] = "\t".join(f) + "\n"
    out = os.path.join(tmp_path, f"inj_{kind}.paf")
    open(out, "w").write("".join(lines))
    return out


@pytest.mark.parametrize("kind", ["mismatch", "bounds", "cigar", "mismatch_splice", "star_bad"])
def test_error_midway(built, tmp_path, kind):
    fa, paf = synth_paf(tmp_path, 0, seed=41)
    bad = _inject(paf, tmp_path, kind, seed=5)
    same(["-r", fa, bad])


def test_empty_and_comment_only_input(built, tmp_path):
    fa, _ = synth_paf(tmp_path, 1)
    p = tmp_path / "c.paf"
    p.write_text("# nothing here\n")
    same(["-r", fa, str(p)])
    p2 = tmp_path / "e.paf"
    p2.write_text("")
    same(["-r", fa, str(p2)])


def test_stdin_input(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 1)
    import subprocess
    a = subprocess.run([str(ORACLE), "-r", fa], stdin=open(paf), stdout=subprocess.PIPE).stdout
    b = subprocess.run([str(CLI), "-r", fa], stdin=open(paf), stdout=subprocess.PIPE).stdout
    assert a == b and len(a) > 0


def test_batch_api_on_torch_stream(built, tmp_path):
    """Stage a packed batch in torch device memory, launch on torch's stream, render the
    report from the device results: must equal the CLI output."""
    import torch
    fa, paf = synth_paf(tmp_path, 0, seed=3)
    b = pw.HostBatch(fa, paf, 0)
    dev = pw.stage_batch(b, "cuda:0")
    pw.run_report(b, dev, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    res = dev["results"].cpu().numpy()
    outp = str(tmp_path / "batch.txt")
    rc = b.write_report_from(dev, outp)
    assert rc == 0
    _, want, _ = run([ORACLE, "-r", fa, paf])
    assert open(outp, "rb").read() == want
    n_events = pw.results_array(res)["n_events"][: b.view.n_alns].sum()
    assert n_events == want.count(b"\n") - want.count(b">")


def test_report_events_after_side_stream(built, tmp_path):
    """pw_report_events_after: the next-stop table built on another stream (behind a long
    dependency there), the pass waiting for its event before render — same report as the oracle,
    twice in a row on the same buffers (the side stream waits for the previous pass)."""
    import torch
    fa, paf = synth_paf(tmp_path, 2, seed=11, scale=0.05)
    b = pw.HostBatch(fa, paf, pw.FLAG_G | pw.FLAG_C)
    v = b.view
    dev = pw.stage_batch(b, "cuda:0")
    main, side = torch.cuda.current_stream(), torch.cuda.Stream()
    ready, done = torch.cuda.Event(), torch.cuda.Event()
    L = pw.lib()
    _, want, _ = run([ORACLE, "-G", "-C", "-r", fa, paf])
    for it in range(2):
        dev["next_stop"].fill_(-7)  # stale table on the main stream: the side stream must come after it
        done.record(main)
        side.wait_event(done)
        with torch.cuda.stream(side):
            torch.cuda._sleep(2000000)  # keep the table build late on the side stream
        assert L.pw_stop_table_build(dev["qseq"].data_ptr(), dev["qoff"].data_ptr(), dev["qlen"].data_ptr(),
                                     int(v.n_queries), dev["next_stop"].data_ptr(), side.cuda_stream) == 0
        ready.record(side)
        a = pw.report_args(b, dev)
        assert L.pw_report_events_after(pw.ctypes.byref(a), main.cuda_stream, ready.cuda_event) == 0
        torch.cuda.synchronize()
        outp = str(tmp_path / f"after{it}.txt")
        assert b.write_report_from(dev, outp) == 0
        assert open(outp, "rb").read() == want


def test_report_builds_next_stop_in_pass(built, tmp_path):
    """PW_REPORT_BUILD_NEXT_STOP: the pass's first kernel builds the next-stop table itself (its
    first workgroups) and clears the pass counters — the table equals pw_stop_table_build's, the
    report equals the oracle's, twice on the same buffers (a stale table and stale counters from
    the previous pass are overwritten), with 16- and 32-byte event records; and a batch of no
    records still gets its table."""
    import torch
    fa, paf = synth_paf(tmp_path, 2, seed=13, scale=0.05)
    b = pw.HostBatch(fa, paf, pw.FLAG_G | pw.FLAG_C)
    v = b.view
    dev = pw.stage_batch(b, "cuda:0")
    L = pw.lib()
    s = torch.cuda.current_stream().cuda_stream
    _, want, _ = run([ORACLE, "-G", "-C", "-r", fa, paf])
    dev["next_stop"].fill_(-7)  # (the padding between queries is never written)
    assert L.pw_stop_table_build(dev["qseq"].data_ptr(), dev["qoff"].data_ptr(), dev["qlen"].data_ptr(),
                                 int(v.n_queries), dev["next_stop"].data_ptr(), s) == 0
    torch.cuda.synchronize()
    ref_ns = dev["next_stop"].clone()
    for it, hot32 in enumerate((False, False, True)):
        dev["next_stop"].fill_(-7)
        dev["work"][:64].fill_(0xFF)  # stale counters: the pass must clear them
        a = pw.report_args(b, dev)
        assert a.max_rec_ops <= 2048  # (no plan pass: index clears the counters)
        if hot32:
            a.hot_pbits = 0
        a.flags = pw.REPORT_BUILD_NEXT_STOP
        assert L.pw_report_events(pw.ctypes.byref(a), s) == 0
        torch.cuda.synchronize()
        assert torch.equal(dev["next_stop"], ref_ns), it
        outp = str(tmp_path / f"inpass{it}.txt")
        assert b.write_report_from(dev, outp) == 0
        assert open(outp, "rb").read() == want, it
    dev["next_stop"].fill_(-7)
    a = pw.report_args(b, dev)
    a.n_alns = 0
    a.flags = pw.REPORT_BUILD_NEXT_STOP
    assert L.pw_report_events(pw.ctypes.byref(a), s) == 0
    torch.cuda.synchronize()
    assert torch.equal(dev["next_stop"], ref_ns)


# ---------------------------------------------------------------- GapAssem consensus
def ga_same(layout, tmp_path, extra=(), writers=True):
    """gapassem_consensus (GapAssem C++ API on the GPU) against the oracle: exit code, stderr, the
    PWC1 result and — with `writers` — the writeACE / writeInfo / writeMSA outputs."""
    outs = ["--ace", "--info", "--msa"] if writers else []
    ro, _, eo = run([GA_ORACLE, layout, tmp_path / "o.pwc", *extra,
                     *[a for o in outs for a in (o, tmp_path / ("o" + o[1:]))]])
    rp, _, ep = run([GA_CLI, layout, tmp_path / "p.pwc", *extra,
                     *[a for o in outs for a in (o, tmp_path / ("p" + o[1:]))]])
    assert rp == ro, (rp, ro, ep, eo)
    assert ep == eo
    if ro == 0:
        assert open(tmp_path / "p.pwc", "rb").read() == open(tmp_path / "o.pwc", "rb").read()
        for o in outs:
            a, b = (open(tmp_path / (x + o[1:]), "rb").read() for x in "op")
            assert a == b, o
    return ro


def test_gapassem_hand_layouts(built, tmp_path):
    lay = tmp_path / "l.pwl"
    write_pwl(lay, [(0, "ACGT", [0, 0, 1, 0], 0, 0, 0), (1, "CNGA", [0, 0, 1, 0], 0, 0, 0),
                    (2, "-G", [0, 0], 0, 0, 0)])
    assert ga_same(lay, tmp_path) == 0
    assert read_pwc(tmp_path / "p.pwc")["cons"] == "AC*GGA"
    lay2 = tmp_path / "z.pwl"
    write_pwl(lay2, [(0, "ACG", [0, 0, 0], 0, 0, 0), (4, "TT", [0, 0], 0, 0, 0)])
    assert ga_same(lay2, tmp_path) == 5


def test_gapassem_clipped_rows(built, tmp_path):
    rng = random.Random(7)
    rows = []
    for r in range(12):
        n = rng.randint(20, 60)
        seq = "".join(rng.choice("ACGTN") for _ in range(n))
        ofs = [0] + [rng.choice([0, 0, 0, 1, 2, -1]) for _ in range(n - 1)]
        rows.append((rng.randint(0, 30), seq, ofs, rng.randint(0, 4), rng.randint(0, 4), r % 2))
    lay = tmp_path / "c.pwl"
    write_pwl(lay, rows)
    for extra in (["--no-refine-clipping"], [], ["--remove-gaps"], ["--remove-gaps", "--no-refine-clipping"]):
        ga_same(lay, tmp_path, extra)


@pytest.mark.parametrize("seed", range(6))
def test_gapassem_refine_clipping_random(built, tmp_path, seed):
    """refineClipping (X-drop, GapAssem.cpp:182-349) + removeClipGaps per row, deleted bases
    (ofs -1: removeColumn replayed on the host) — library defaults, both removeConsGaps modes."""
    from test_gapassem_refine import random_layout
    rng = random.Random(700 + seed)
    rows = random_layout(rng, rng.randint(3, 25), clip=True, dels=seed % 2 == 1)
    lay = tmp_path / "r.pwl"
    write_pwl(lay, rows)
    ga_same(lay, tmp_path)
    ga_same(lay, tmp_path, ["--remove-gaps"])


@pytest.mark.parametrize("scale,clip,dels", [(0.002, 0.5, 0.0), (0.01, 0.3, 0.002), (0.02, 0.5, 0.001)])
def test_gapassem_clipped_synthetic(built, tmp_path, scale, clip, dels):
    lay = tmp_path / "s.pwl"
    rc, _, err = run([SYNTH, "layout", "--config", 5, "--scale", scale, "--rows", 40, "--clip", clip, "--dels", dels,
                      "--out", lay])
    assert rc == 0, err
    assert ga_same(lay, tmp_path) == 0
    assert ga_same(lay, tmp_path, ["--remove-gaps"]) == 0


@pytest.mark.parametrize("scale", [0.0005, 0.002, 0.01])
def test_gapassem_synthetic(built, tmp_path, scale):
    lay = tmp_path / "s.pwl"
    rc, _, err = run([SYNTH, "layout", "--config", 5, "--scale", scale, "--out", lay])
    assert rc == 0, err
    assert ga_same(lay, tmp_path) == 0


@pytest.mark.parametrize("seed", range(3))
def test_gapassem_odd_characters(built, tmp_path, seed):
    """tile_counts classifies A C G T N - * (and H) with a fast check and redoes a wave's groups
    with the general bin rule (toupper, anything else N) when a byte is outside that set: rows over
    several 2048-column tiles, some pure A/C/G/T/N, some with lower case, '*', '-' and other bytes."""
    rng = random.Random(900 + seed)
    rows = []
    for r in range(24):
        n = rng.randint(2000, 9000)
        odd = r % 3 != 0
        pool = "ACGTACGTACGTN" + ("acgtn*-RYxH." if odd else "")
        seq = "".join(rng.choice(pool) if rng.random() < (0.05 if odd else 1.0) else rng.choice("ACGT")
                      for _ in range(n))
        ofs = [0] + [rng.choice([0] * 40 + [1, 2, 5, 70]) for _ in range(n - 1)]
        rows.append((rng.randint(0, 6000), seq, ofs, rng.randint(0, 30), rng.randint(0, 30), r % 2))
    rows[0] = (0, "".join(rng.choice("ACGT") for _ in range(20000)), [0] * 20000, 0, 0, 0)  # coverage
    lay = tmp_path / "o.pwl"
    write_pwl(lay, rows)
    assert ga_same(lay, tmp_path, writers=False) == 0
    assert ga_same(lay, tmp_path, ["--remove-gaps"], writers=False) == 0


def test_gapassem_tile_boundaries(built, tmp_path):
    # rows long enough to cross several 2048-column tiles and 256-base chunks with gaps
    lay = tmp_path / "b.pwl"
    rc, _, err = run([SYNTH, "layout", "--config", 5, "--scale", 0.02, "--rows", 40, "--out", lay])
    assert rc == 0, err
    assert ga_same(lay, tmp_path) == 0


# ---------------------------------------------------------------- multi-GPU shard path
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_run_on_gpu(built, tmp_path, world):
    """Each shard through the HIP batch path (the per-rank work of a multi-GPU run, here all on
    cuda:0), item streams merged by global line: must equal the single-process oracle run."""
    import torch
    from pwasm_amd import shard
    from test_shard import _with_duplicates_and_comments
    fa, paf = synth_paf(tmp_path, 0, seed=8)
    dup = _with_duplicates_and_comments(paf, tmp_path, 2)
    parts = shard.split_paf(dup, world, str(tmp_path))
    got = []
    for r, (p, gmap) in enumerate(parts):
        b = pw.HostBatch(fa, p, 0)
        dev = pw.stage_batch(b, "cuda:0")
        pw.run_report(b, dev, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ip = str(tmp_path / f"s{r}.pwi")
        assert b.write_items_from(dev, ip) == 0
        got.append((shard.read_items(ip), gmap))
    out, err, rc = shard.merge_items(got)
    assert (rc, out, err) == run([ORACLE, "-r", fa, dup])


# ---------------------------------------------------------------- GapAssem refineMSA, removeConsGaps
def test_gapassem_remove_gaps_hand(built, tmp_path):
    lay = tmp_path / "l.pwl"
    write_pwl(lay, [(0, "ACGT", [0, 0, 1, 0], 0, 0, 0), (1, "CNGA", [0, 0, 1, 0], 0, 0, 0),
                    (2, "-G", [0, 0], 0, 0, 0)])
    assert ga_same(lay, tmp_path, ["--remove-gaps"]) == 0
    r = read_pwc(tmp_path / "p.pwc")
    assert r["cons"] == "ACGGA" and r["removed"] == 1


@pytest.mark.parametrize("seed", range(8))
def test_gapassem_remove_gaps_random(built, tmp_path, seed):
    from test_gapassem_refine import random_layout
    rng = random.Random(500 + seed)
    rows = random_layout(rng, rng.randint(2, 30), clip=seed % 2 == 1)
    lay = tmp_path / "r.pwl"
    write_pwl(lay, rows)
    ga_same(lay, tmp_path, ["--remove-gaps", "--no-refine-clipping"])
    ga_same(lay, tmp_path, ["--no-refine-clipping"])


@pytest.mark.parametrize("scale", [0.0005, 0.005, 0.02])
def test_gapassem_remove_gaps_synthetic(built, tmp_path, scale):
    lay = tmp_path / "s.pwl"
    rc, _, err = run([SYNTH, "layout", "--config", 5, "--scale", scale, "--rows", 40, "--out", lay])
    assert rc == 0, err
    assert ga_same(lay, tmp_path, ["--remove-gaps"]) == 0
    assert read_pwc(tmp_path / "p.pwc")["removed"] > 0


def test_gapassem_remove_gaps_deleted_bases(built, tmp_path):
    """Deleted bases (ofs < 0, as GASeq::removeBase leaves them) under removeConsGaps: the raw-ofs
    walk of removeColumn (GapAssem.cpp:766-771) replayed per row on the host (former D8)."""
    lay = tmp_path / "n.pwl"
    # (toMSA still places a deleted base in a column: rows holding one end before the longest row)
    write_pwl(lay, [(0, "ACGT", [0, -1, 0, 0], 0, 0, 0), (0, "ACGTAC", [0] * 6, 0, 0, 0),
                    (1, "CGTA", [0, 1, -1, 0], 0, 0, 1), (0, "AGGTAC", [0, 0, 2, 0, 0, 0], 0, 1, 0),
                    (0, "ACGTAC", [0, 0, 1, 0, 0, 0], 0, 0, 0)])
    assert ga_same(lay, tmp_path, ["--remove-gaps"]) == 0
    assert read_pwc(tmp_path / "p.pwc")["removed"] > 0


# ---------------------------------------------------------------- multi-GPU GapAssem driver
def _ga_cli(lay, tmp_path, remove, refine=True):
    extra = (["--remove-gaps"] if remove else []) + ([] if refine else ["--no-refine-clipping"])
    rc, _, err = run([GA_CLI, lay, tmp_path / "c.pwc", *extra])
    return rc, err.decode(), (open(tmp_path / "c.pwc", "rb").read() if rc == 0 else None)


@pytest.mark.parametrize("remove", [False, True])
def test_gapassem_driver_single_rank_on_gpu(built, tmp_path, remove):
    from pwasm_amd import gapassem
    lay = tmp_path / "s.pwl"
    rc, _, err = run([SYNTH, "layout", "--config", 5, "--scale", 0.005, "--rows", 30, "--out", lay])
    assert rc == 0, err
    got = gapassem.consensus(str(lay), remove_gaps=remove)
    assert got == _ga_cli(lay, tmp_path, remove)
    assert got[0] == 0
    # clipped rows + deleted bases: the driver's host row tail (pw_ga_row_*) after the GPU edits
    lay2 = tmp_path / "c.pwl"
    rc, _, err = run([SYNTH, "layout", "--config", 5, "--scale", 0.005, "--rows", 30, "--clip", 0.5, "--dels", 0.002,
                      "--out", lay2])
    assert rc == 0, err
    for refine in (True, False):
        got = gapassem.consensus(str(lay2), remove_gaps=remove, refine_clipping=refine)
        assert got == _ga_cli(lay2, tmp_path, remove, refine)
        assert got[0] == 0


def _ga_rank(rank, world, port, lay, remove, q):
    import torch.distributed as dist
    from pwasm_amd import gapassem
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = gapassem.consensus(lay, remove_gaps=remove)  # HIP engine on cuda:0
        if rank == 0:
            q.put(res)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gapassem_sharded_on_gpu(built, tmp_path):
    """Two ranks (both on cuda:0, gloo): partial histograms of each half of the rows on the GPU,
    merged by the all-reduce, refined per shard — same bytes as the single-GPU CLI."""
    import socket
    import torch.multiprocessing as mp
    lay = tmp_path / "s.pwl"
    rc, _, err = run([SYNTH, "layout", "--config", 5, "--scale", 0.003, "--rows", 12, "--out", lay])
    assert rc == 0, err
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ga_rank, args=(r, 2, port, str(lay), True, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == _ga_cli(lay, tmp_path, True)


# ---------------------------------------------------------------- reads past the query end
def _comp(s):
    return s.translate(str.maketrans("ACGT", "TGCA"))[::-1]


def query_end_case(tmp_path):
    """Events in the last, partial codon of a query that is followed by another query in the
    FASTA: the codon reads run past the end (the reference reads the NUL terminator; DESIGN.md
    D6), never into the next query's bases."""
    qa = "ATGAAACCCGGGTTTAAACCCGGGTTTAAACG"  # 32 nt: the last codon is partial
    qb = "GGGGGGGGGGGGGGGGGGGGGGGG"
    fa = tmp_path / "q.fa"
    fa.write_text(f">qa\n{qa}\n>qb\n{qb}\n")
    alt = lambda c: "t" if c != "T" else "c"  # noqa: E731
    rc_qa = _comp(qa)
    recs = [
        ("qa", 32, 0, 32, "+", "t1", 100, 10, 42, "32M", f":31*{alt(qa[31])}{qa[31].lower()}"),
        ("qa", 32, 0, 32, "+", "t2", 100, 10, 40, "29M2I1M", f":29+{qa[29:31].lower()}:1"),
        ("qa", 32, 0, 32, "-", "t3", 100, 5, 37, "32M", f":1*{alt(rc_qa[1])}{rc_qa[1].lower()}:30"),
        ("qa", 32, 0, 32, "+", "t4", 100, 10, 43, "31M1D1M", f":31-a:1"),
    ]
    lines = []
    for q, ql, qs, qe, st, t, tl, ts, te, cg, cs in recs:
        lines.append("\t".join(map(str, [q, ql, qs, qe, st, t, tl, ts, te, 30, 32, 60, "NM:i:1", "AS:i:9",
                                         f"cg:Z:{cg}", f"cs:Z:{cs}"])) + "\n")
    paf = tmp_path / "e.paf"
    paf.write_text("".join(lines))
    return str(fa), str(paf)


def test_reads_past_query_end(built, tmp_path):
    fa, paf = query_end_case(tmp_path)
    out = same(["-G", "-C", "-r", fa, paf])
    assert out.count(b">") == 4 and b"(X)" in out


# ---------------------------------------------------------------- -w (MSA of the last query run)
def same_w(args, tmp_path, msa_ok=True):
    """CLI and oracle with `-w`: stdout, stderr, exit code and the MSA file bytes."""
    mo, mp = tmp_path / "oracle.mfa", tmp_path / "hip.mfa"
    ro, oo, eo = run([ORACLE, "-w", mo, *args])
    rp, op, ep = run([CLI, "-w", mp, *args])
    assert (rp, op, ep) == (ro, oo, eo), (rp, ro, ep[-2000:], eo[-2000:])
    assert mp.exists() == mo.exists()
    if not mo.exists():
        return ro, None
    if msa_ok:
        assert mp.read_bytes() == mo.read_bytes()
    return ro, mo.read_bytes()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_w_edge_mix(built, tmp_path, seed):
    fa, paf = synth_paf(tmp_path, 0, seed=seed)
    rc, msa = same_w(["-r", fa, paf], tmp_path)
    assert rc == 0 and msa.count(b">") >= 2


def test_w_cfg2_subsample(built, tmp_path):
    fa, paf = synth_paf(tmp_path, 2, seed=5, scale=0.05)
    rc, _ = same_w(["-G", "-C", "-r", fa, paf], tmp_path)
    assert rc == 0


@pytest.mark.parametrize("seed,rev", [(7, 0.5), (8, 1.0)])
def test_w_long_run(built, tmp_path, seed, rev):
    fa, paf = str(tmp_path / "r.fa"), str(tmp_path / "r.paf")
    rc, _, err = run([SYNTH, "paf", "--config", 0, "--seed", seed, "--ncds", 2, "--recs", 300, "--rev", rev,
                      "--fa", fa, "--paf", paf])
    assert rc == 0, err
    rc, msa = same_w(["-r", fa, paf], tmp_path)
    assert rc == 0 and msa.count(b">") > 100


def _w_error_paf(tmp_path, kind):
    fa, paf = query_end_case(tmp_path)
    rec = {  # a gap at the sequence end: GASeq::setGap refuses it (GapAssem.cpp:212-233)
        "ref_end_fwd": ["qa", 32, 0, 32, "+", "t5", 100, 10, 43, 30, 33, 60, "cg:Z:32M1D", "cs:Z::32-a"],
        "ref_start_rev": ["qa", 32, 0, 32, "-", "t6", 100, 10, 43, 30, 33, 60, "cg:Z:1D32M", "cs:Z:-a:32"],
        "target_end": ["qa", 32, 0, 32, "+", "t7", 100, 10, 40, 30, 32, 60, "cg:Z:30M2I", "cs:Z::30+cg"],
    }[kind]
    rec = rec[:12] + ["NM:i:1", "AS:i:9"] + rec[12:]
    p = tmp_path / f"{kind}.paf"
    p.write_text(open(paf).read() + "\t".join(map(str, rec)) + "\n")
    return fa, str(p)


@pytest.mark.parametrize("kind", ["ref_end_fwd", "ref_start_rev", "target_end"])
def test_w_invalid_gap_position(built, tmp_path, kind):
    fa, paf = _w_error_paf(tmp_path, kind)
    rc, msa = same_w(["-r", fa, paf], tmp_path)
    assert rc == 1 and msa == b""


def test_w_refused_in_genome_mode_and_bad_path(built, tmp_path):
    fa, paf = query_end_case(tmp_path)
    rc, _ = same_w(["-F", "-r", fa, paf], tmp_path, msa_ok=False)
    assert rc == 1
    ro, oo, eo = run([ORACLE, "-w", tmp_path / "no" / "x.mfa", "-r", fa, paf])
    rp, op, ep = run([CLI, "-w", tmp_path / "no" / "x.mfa", "-r", fa, paf])
    assert (rp, op, ep) == (ro, oo, eo) and ro == 1


@pytest.mark.parametrize("zero", [False, True])
def test_msa_columns_fused_equals_count_call(built, tmp_path, zero):
    """pw_msa_columns (bestChar in tile_counts' epilogue) against pw_msa_count + pw_msa_call on the
    same staged layout: counts, consensus and minmax identical, over several 2048-column tiles and
    a partial last tile; `zero` leaves a zero-coverage stretch inside [mincol, maxcol]."""
    import torch
    from pwasm_amd import gapassem
    rng = random.Random(31 + zero)
    rows = []
    for r in range(30):
        n = rng.randint(500, 4000)
        seq = "".join(rng.choice("ACGTACGTNacgt*-") for _ in range(n))
        if zero:  # two groups of rows with uncovered columns between them
            ofs = [0] + [rng.choice([0] * 30 + [1]) for _ in range(n - 1)]
            off = rng.randint(0, 300) if r % 2 else rng.randint(20000, 20300)
        else:
            ofs = [0] + [rng.choice([0] * 30 + [1, 3, 80]) for _ in range(n - 1)]
            off = rng.randint(0, 3000)
        rows.append((off, seq, ofs, rng.randint(0, 20), rng.randint(0, 20), r % 2))
    lay_p = tmp_path / "f.pwl"
    write_pwl(lay_p, rows)
    lay = gapassem.Layout(str(lay_p))
    eng = gapassem.HipEngine("cuda:0")
    st = eng.stage(lay, range(lay.n), lay.length)
    counts, mm = eng.count(st)
    cons, mm = eng.call(st)
    torch.cuda.synchronize()
    want = (counts.clone(), cons.clone(), mm.clone())
    st["d"]["cons"].fill_(7)
    st["d"]["counts"].fill_(-1)
    counts, mm = eng.columns(st)
    torch.cuda.synchronize()
    assert torch.equal(counts, want[0])
    assert torch.equal(st["d"]["cons"], want[1])
    assert mm.tolist() == want[2].tolist()
    assert (int(mm[3]) != 2 ** 31 - 1) == zero  # (the zero-coverage column is found by both)


@pytest.mark.gpu
@pytest.mark.parametrize("remove", [False, True])
def test_msa_columns_refine_equals_columns_then_refine(built, tmp_path, remove):
    """pw_msa_columns_refine (without removeConsGaps: the consensus string written by tile_counts'
    call epilogue) against pw_msa_columns + pw_msa_refine on the same staged layout: consensus
    string, its length, minmax and (remove) every row's offset / numgaps / ofs identical."""
    import torch
    from pwasm_amd import gapassem
    rng = random.Random(77 + remove)
    rows = []
    for r in range(40):
        n = rng.randint(300, 5000)
        seq = "".join(rng.choice("ACGTACGTNacgt-") for _ in range(n))
        ofs = [0] + [rng.choice([0] * 40 + [1, 2, 7]) for _ in range(n - 1)]
        rows.append((rng.randint(0, 6000), seq, ofs, rng.randint(0, 15), rng.randint(0, 15), r % 2))
    lay_p = tmp_path / "cr.pwl"
    write_pwl(lay_p, rows)
    lay = gapassem.Layout(str(lay_p))
    eng = gapassem.HipEngine("cuda:0")
    st = eng.stage(lay, range(lay.n), lay.length)
    d = st["d"]
    eng.columns(st)
    cons, rws = eng.refine_host(st, remove)
    want_mm = d["mm"].clone()
    d["cout"].fill_(7)
    d["clen"].fill_(-5)
    d["cons"].fill_(9)
    eng.columns_refine(st, remove)
    torch.cuda.synchronize()
    clen = int(d["clen"].cpu().item())
    assert clen == len(cons)
    assert bytes(d["cout"][:clen].cpu().numpy()) == cons
    assert d["mm"].tolist() == want_mm.tolist()
    if remove:
        offo, ngo, ofso = d["offo"].cpu().numpy(), d["ngo"].cpu().numpy(), d["ofso"].cpu().numpy()
        for k, r in enumerate(st["rows"]):
            o = int(st["row_off"][k])
            assert (int(offo[k]), int(ngo[k])) == rws[r][:2]
            assert (ofso[o:o + int(st["lens"][k])] == rws[r][2]).all()


# ---------------------------------------------------------------- RCCL collectives C-ABI
def test_msa_counts_allreduce_world1(built, tmp_path):
    """pw_comm_* + pw_msa_counts_allreduce / reduce_scatter on a one-rank RCCL communicator:
    the merged histograms equal the shard's own, the bad row comes back global (row_base)."""
    import ctypes
    import torch
    from pwasm_amd import gapassem, lib
    L = lib()
    lay_p = tmp_path / "s.pwl"
    rc, _, err = run([SYNTH, "layout", "--config", 5, "--scale", 0.003, "--rows", 12, "--out", lay_p])
    assert rc == 0, err
    lay = gapassem.Layout(str(lay_p))
    eng = gapassem.HipEngine("cuda:0")
    st = eng.stage(lay, range(lay.n), lay.length)
    counts, mm = eng.count(st)
    ref_counts, ref_mm = counts.clone(), mm.clone()
    uid = ctypes.create_string_buffer(128)
    assert L.pw_comm_unique_id(uid) == 0
    comm = ctypes.c_void_p()
    assert L.pw_comm_init(ctypes.byref(comm), 1, uid, 0) == 0
    try:
        counts, mm = eng.merge(st, 5, comm)
        torch.cuda.synchronize()
        assert torch.equal(counts, ref_counts)
        assert mm[:2].tolist() == ref_mm[:2].tolist() and int(mm[2]) == int(ref_mm[2])  # INT_MAX stays
        part = torch.empty_like(counts)
        assert L.pw_msa_counts_reduce_scatter(counts.data_ptr(), part.data_ptr(), lay.length, comm,
                                              torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        assert torch.equal(part, ref_counts)
    finally:
        assert L.pw_comm_destroy(comm) == 0


def _ga_rank_nccl(lay, q):
    import torch.distributed as dist
    from pwasm_amd import gapassem
    os.environ.update(MASTER_ADDR="127.0.0.1", PW_GA_COMM="rccl")
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        q.put(gapassem.consensus(lay, remove_gaps=True))
    finally:
        dist.destroy_process_group()


def test_gapassem_driver_rccl_world1(built, tmp_path):
    """The driver with the nccl backend merges through pw_msa_counts_allreduce on its own RCCL
    communicator (PW_GA_COMM=rccl forces that path at world 1): same bytes as the CLI."""
    import socket
    import torch.multiprocessing as mp
    lay = tmp_path / "s.pwl"
    rc, _, err = run([SYNTH, "layout", "--config", 5, "--scale", 0.003, "--rows", 12, "--out", lay])
    assert rc == 0, err
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_ga_rank_nccl, args=(str(lay), q))
    p.start()
    res = q.get(timeout=100)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert res == _ga_cli(lay, tmp_path, True)


def _short_fraction(paf):
    """Records whose cs string packs to at most 64 ops (index_pair_kernel's records)."""
    import re
    n = short = 0
    for ln in open(paf):
        if ln.startswith("#"):
            continue
        cs = next((x[5:] for x in ln.rstrip("\n").split("\t")[12:] if x.startswith("cs:Z:")), None)
        if cs is None:
            continue
        n += 1
        short += len(re.findall(r"[:*+-]", cs)) <= 64
    return short / max(n, 1)


@pytest.mark.parametrize("seed,extra", [(51, []), (52, ["--subrun", 0.6, "--rev", 0.8]), (53, ["--longindel", 0.4])])
def test_pair_index_short_records(built, tmp_path, seed, extra, monkeypatch):
    """Mostly short records: index_pair_kernel decodes two per wavefront (one per 32-lane half);
    the same bytes with PW_NO_PAIRS=1 (one record per wavefront) and from the oracle — odd record
    counts, a mismatch injected into a short record, reverse strands, S runs, long indels."""
    fa, paf = synth_paf(tmp_path, 0, seed=seed, extra=["--len-min", 90, "--len-max", 700, "--ncds", 31, "--recs", 9, *extra])
    assert _short_fraction(paf) >= 0.8
    same(["-r", fa, paf])
    bad = _inject(paf, tmp_path, "mismatch", seed=seed)
    same(["-r", fa, bad])
    monkeypatch.setenv("PW_NO_PAIRS", "1")
    same(["-r", fa, paf])


@pytest.mark.parametrize("cfg,hot32", [(0, "0"), (0, "1"), (4, "0"), (4, "1")])
def test_event_record_formats(built, tmp_path, monkeypatch, cfg, hot32):
    """The report pass keeps 16-byte event records between its kernels when the queries' lengths
    and count fit (query index and position in one word; start, length and literal bytes loaded
    by the readers) and 32-byte ones otherwise (PW_HOT32=1 forces them): the same bytes either
    way, on gene-length queries and on 150-250 kb contigs (18 position bits, auto -F)."""
    monkeypatch.setenv("PW_HOT32", hot32)
    if cfg == 0:
        fa, paf = synth_paf(tmp_path, 0, seed=21)
        same(["-r", fa, paf])
    else:
        fa, paf = synth_paf(tmp_path, 4, extra=["--ncds", 2, "--len-min", 150000, "--len-max", 250000, "--recs", 3,
                                                "--err", 0.02])
        same(["-r", fa, paf])
