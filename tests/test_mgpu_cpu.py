"""CPU: the pieces of the multi-GPU pafreport driver (pwasm_amd/mgpu.py) that need no GPU — the
ragged all-gather of per-genome rows / names over gloo (world 2), the C++ k-way merge of the
shards' item streams (pw_items_merge) against the Python reference merge (shard.merge_items),
GArgs-style option parsing and the genome-table writer."""
import os
import socket
import struct

import numpy as np
import pytest
import torch.multiprocessing as mp

import pwasm_amd as pw
from pwasm_amd import mgpu, shard


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gather_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = torch.arange(3 + 4 * rank, dtype=torch.int64) + 100 * rank
        got = mgpu.gather_ragged(t)
        q.put((rank, [x.tolist() for x in got]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gather_ragged_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_gather_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [list(range(3)), [100 + k for k in range(7)]]
    assert res[0] == want and res[1] == want


def _write_items(path, items):
    with open(path, "wb") as f:
        f.write(b"PWI1")
        for line, st, o, e in items:
            f.write(struct.pack("<QiII", line, st, len(o), len(e)) + o + e)


@pytest.mark.parametrize("stop", [None, 7])
def test_items_merge_matches_python_merge(built, tmp_path, stop):
    rng = np.random.default_rng(3)
    lines = rng.permutation(40)
    shards = [sorted(lines[k::3].tolist()) for k in range(3)]
    paths, parts = [], []
    for k, ls in enumerate(shards):
        items = [(ln, 1 if ln == stop else -1, f"out{ln}\n".encode() * (ln % 3), f"err{ln}\n".encode() * (ln % 2))
                 for ln in ls]
        p = tmp_path / f"s{k}.pwi"
        _write_items(p, items)
        paths.append(p)
        parts.append((shard.read_items(str(p)), list(range(100))))  # identity line map
    want_out, want_err, want_rc = shard.merge_items(parts)
    rc = pw.items_merge(paths, tmp_path / "o.txt", tmp_path / "e.txt")
    assert rc == want_rc
    assert (tmp_path / "o.txt").read_bytes() == want_out
    assert (tmp_path / "e.txt").read_bytes() == want_err


def test_parse_args():
    o, n, x = mgpu.parse_args(["-G", "-C", "-rq.fa", "a.paf", "-o", "r.txt", "--genome-table", "t.tsv"])
    assert o == {"G": "", "C": "", "r": "q.fa", "o": "r.txt"} and n == ["a.paf"] and x == {"genome-table": "t.tsv"}
    o, n, _ = mgpu.parse_args(["-GC", "-r", "q.fa", "a.paf"])
    assert o == {"G": "", "C": "", "r": "q.fa"}
    with pytest.raises(SystemExit):
        mgpu.parse_args(["-x"])


def test_genome_table_writer(tmp_path):
    rows = np.zeros(32, np.uint8)
    rows[0:4] = np.frombuffer(np.uint32(3).tobytes(), np.uint8)
    rows[4:8] = np.frombuffer(np.uint32(17).tobytes(), np.uint8)
    rows[8:16] = np.frombuffer(np.uint64(12345).tobytes(), np.uint8)
    rows[16:20] = np.frombuffer(np.uint32(1).tobytes(), np.uint8)
    p = tmp_path / "t.tsv"
    mgpu.write_genome_table(p, [rows], [[b"tA", b"tB"]])
    assert p.read_text().splitlines()[1:] == ["tA\t3\t17\t12345", "tB\t1\t0\t0"]


# ---------------------------------------------------------------- byte-range exchange + offset writes
def _paf_with_everything(tmp_path, fatal):
    """An edge-mix PAF with duplicate q~t pairs (dedupe warnings), comments, CRLF line ends on some
    lines and, optionally, a short line two thirds in (the fatal that ends the run)."""
    from conftest import synth_paf
    from test_shard import _with_duplicates_and_comments
    fa, paf = synth_paf(tmp_path, 0, seed=41)
    dup = _with_duplicates_and_comments(paf, tmp_path, 2)
    lines = open(dup, "rb").read().splitlines(keepends=True)
    lines = [ln.replace(b"\n", b"\r\n") if k % 7 == 3 else ln for k, ln in enumerate(lines)]
    if fatal:
        lines.insert(2 * len(lines) // 3, b"cds0\t30\t0\t30\t+\n")
    p = tmp_path / "all.paf"
    p.write_bytes(b"".join(lines))
    return fa, str(p)


def _exchange_rank(rank, world, port, fa, paf, out_path, errf, q, window=None, mode="exchange"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PW_MGPU_WRITE=mode)
    fd = os.open(errf, os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
    os.dup2(fd, 2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        text, line_no, n_total = mgpu.exchange(paf, world, rank, "cpu", "gloo")
        # every received line belongs to this rank: target genome hash (column 6) mod world
        got = bytes(text).split(b"\n")[:-1]
        for ln in got:
            assert shard.shard_of(ln, world) == rank
        # the batches of this rank without a GPU: every record "ran" with zero events (results of
        # zeros), so each prints its header — headers, messages, dedupe and the fatal stop all go
        # through the offset-write path
        outs = []
        prev = None
        for b0, b1, l0, l1 in mgpu.batch_cuts(text, line_no, 3000):
            b = pw.HostBatch.from_buffer(fa, text[b0:b1], line_no[l0:l1], 0, prev)
            prev = b
            res = np.zeros(max(int(b.view.n_alns), 1) * 48, np.uint8)
            pages, txt = np.zeros(16, np.uint8), np.zeros(16, np.uint8)
            outs.append((b, txt, res, pages, b.items(txt, res, pages)))
        if window is None:
            code = mgpu.write_items_at(outs, n_total, out_path, world, rank, "cpu")
        else:  # windows of a few lines, each batch handed over before the windows it completes
            w = mgpu.OffsetWriter(n_total, out_path, world, rank, "cpu", window=window)
            pool, released = mgpu.HostTextPool(2), []  # (the text buffers of main(): released once written)
            for k, o in enumerate(outs):
                slot = []
                t = pool.take(16, slot)
                t.zero_()
                w.add((o[0], t.numpy()) + o[2:], lambda i=slot[0], k=k: (released.append(k), pool.give(i)))
                w.advance(int(o[4][0][-1]) + 1 if len(o[4][0]) else 0)
                assert released == sorted(released) and len(released) <= k + 1
            # (finish_run closes the writer; a run ended by a fatal line writes no genome table)
            gtab = {f"t{rank}".encode(): np.array([1, 2, 3], np.uint64)}
            code = mgpu.finish_run(w, None, gtab, {"genome-table": out_path + ".gt"}, world, rank, "cpu")
            if not w.fatal:  # every batch's buffer went back to the pool
                assert released == list(range(len(outs))), (released, len(outs))
        q.put((rank, code, n_total, [int(x) for x in line_no]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fatal,window,mode", [(2, False, None, "exchange"), (2, True, None, "exchange"),
                                                     (3, True, None, "exchange"), (2, False, 7, "exchange"),
                                                     (3, True, 5, "exchange"), (3, False, 7, "exchange"),
                                                     (2, True, 5, "pwrite"), (3, False, None, "pwrite")])
def test_exchange_and_offset_write_gloo(built, tmp_path, world, fatal, window, mode):
    """mgpu's scalable host path on the CPU (gloo): each rank reads 1/N of the PAF by byte range
    (pw_paf_split), lines are exchanged by target genome (all_to_all_single), packed in several
    batches per rank (the q~t dedupe state carried over), and written at offsets from an
    exclusive scan of the all-reduced per-line byte counts.  The file, stderr and exit code must
    equal the single-process batch (pw_batch_from_files + write_items + merge) on the same zero
    results."""
    fa, paf = _paf_with_everything(tmp_path, fatal)
    single = pw.HostBatch(fa, paf, 0)
    res = np.zeros(max(int(single.view.n_alns), 1) * 48, np.uint8)
    z = np.zeros(16, np.uint8)
    items = tmp_path / "single.pwi"
    assert single.write_items(z, res, z, str(items)) == 0
    want_rc = pw.items_merge([items], tmp_path / "want.out", tmp_path / "want.err")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    out = tmp_path / "got.out"
    ps = [ctx.Process(target=_exchange_rank, args=(r, world, port, fa, paf, str(out), str(tmp_path / f"e{r}"), q,
                                                   window, mode))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r, (c, n, ln)) for r, c, n, ln in (q.get(timeout=90) for _ in range(world)))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    n_lines = len(open(paf, "rb").read().replace(b"\r\n", b"\n").split(b"\n")) - 1
    assert all(v[1] == n_lines for v in res.values())
    assert {v[0] for v in res.values()} == {want_rc}
    assert want_rc == (1 if fatal else 0)
    noise = (b"/opt/amdgpu/", b"[W", b"[Gloo]", b"[I")
    err = b"".join(ln for ln in open(tmp_path / "e0", "rb").read().splitlines(keepends=True)
                   if not ln.startswith(noise))
    assert out.read_bytes() == (tmp_path / "want.out").read_bytes()
    assert err == (tmp_path / "want.err").read_bytes()
    if window is not None:  # no timing-dependent genome table after a fatal line
        assert os.path.exists(str(out) + ".gt") == (not fatal)
    # every non-comment line went to exactly one rank, with its global line number
    got = sorted(x for v in res.values() for x in v[2])
    lines = open(paf, "rb").read().replace(b"\r\n", b"\n").split(b"\n")[:-1]
    assert got == [k for k, ln in enumerate(lines) if not ln.startswith(b"#")]


def _finish_rank(rank, world, port, out_path, gt_path, errf, fail_rank, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    fd = os.open(errf, os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
    os.dup2(fd, 2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = mgpu.OffsetWriter(5, out_path, world, rank, "cpu")
        # fail_rank could not read its batch (e.g. an unreadable -r FASTA); every other rank got no
        # lines at all (lines go to the owner of their target genome)
        err = "pw_batch_from_buffer: Error: invalid FASTA file q.fa !\n" if rank == fail_rank else None
        code = mgpu.finish_run(w, err, {}, {"genome-table": gt_path}, world, rank, "cpu")
        q.put((rank, code, w.failed))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank", [(2, 0), (2, 1), (3, 2), (2, None)])
def test_input_error_on_one_rank_ends_every_rank(tmp_path, world, fail_rank):
    """an input error that only some ranks hit must end the run on every rank (exit 1,
    the message once, from rank 0) — the lineless ranks may not wait in the genome-table gather or
    the final barrier for ranks that already returned."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    gt = tmp_path / "gt.tsv"
    ps = [ctx.Process(target=_finish_rank, args=(r, world, port, str(tmp_path / "o.txt"), str(gt),
                                                 str(tmp_path / f"e{r}"), fail_rank, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = {r: (c, f) for r, c, f in (q.get(timeout=90) for _ in range(world))}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = 0 if fail_rank is None else 1
    assert {c for c, _ in res.values()} == {want}
    assert {f for _, f in res.values()} == {fail_rank is not None}
    noise = (b"/opt/amdgpu/", b"[W", b"[Gloo]", b"[I")
    err0 = b"".join(ln for ln in open(tmp_path / "e0", "rb").read().splitlines(keepends=True)
                    if not ln.startswith(noise))
    assert err0 == (b"Error: invalid FASTA file q.fa !\n" if fail_rank is not None else b"")
    assert gt.exists() == (fail_rank is None)


# ---------------------------------------------------------------- host helpers of the write paths (round 6)
def _old_batch_cuts(text, target):
    """The pre-round-6 numpy form of mgpu.batch_cuts (every line end indexed)."""
    n = text.size
    ends = np.flatnonzero(text == 10) + 1
    cuts, b0, l0 = [], 0, 0
    while b0 < n:
        k = int(np.searchsorted(ends, b0 + target, side="left"))
        k = min(max(k, l0 + 1), ends.size) - 1
        b1 = int(ends[k])
        cuts.append((b0, b1, l0, k + 1))
        b0, l0 = b1, k + 1
    return cuts


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_batch_cuts_c_matches_numpy(built, seed):
    """pw_batch_cuts (memchr scans, threaded line counts) cuts exactly where the numpy form did:
    batches of at most `target` bytes, at least one line, at line ends."""
    rng = np.random.default_rng(seed)
    for _ in range(200):
        lens = rng.integers(1, 60, int(rng.integers(1, 80)))
        text = np.concatenate([np.append(np.full(int(x), 65, np.uint8), np.uint8(10)) for x in lens]).astype(np.uint8)
        for t in (1, 2, 3, 7, 30, 100, 10 ** 6):
            assert mgpu.batch_cuts(text, None, t) == _old_batch_cuts(text, t)
    assert mgpu.batch_cuts(np.zeros(0, np.uint8), None, 10) == []


@pytest.mark.parametrize("img", [None, 1 << 20, 4099])
def test_gather_write_spans(built, tmp_path, monkeypatch, img):
    """pw_gather_write: spans of a source in order, written contiguously at an offset (host threads
    fill 64 MB images, one pwrite each; small images: many images, spans cut between images)."""
    if img:
        monkeypatch.setenv("PW_EMIT_IMG_BYTES", str(img))
    rng = np.random.default_rng(4)
    src = rng.integers(0, 256, 24 << 20, dtype=np.uint8)
    lens = rng.integers(0, 5000, 8000).astype(np.uint64)
    offs = rng.integers(0, src.size - 5000, lens.size).astype(np.uint64)
    want = b"".join(src[int(o):int(o) + int(n)].tobytes() for o, n in zip(offs, lens))
    p = tmp_path / "g.bin"
    p.write_bytes(b"x" * 100)
    fd = os.open(p, os.O_WRONLY)
    try:
        pw.gather_write(fd, 37, src, offs, lens)
    finally:
        os.close(fd)
    got = p.read_bytes()
    assert got[:37] == b"x" * 37 and got[37:37 + len(want)] == want


@pytest.mark.parametrize("img", [None, 1000])
def test_render_range_equals_write_range(built, tmp_path, monkeypatch, img):
    """pw_batch_render_range's bytes back to back are what pw_batch_write_range pwrites at the items'
    offsets (plain items, messages, dedupe warnings; zero results: header-only records).  Contiguous
    offsets take the image path (small images: a run cut into many)."""
    if img:
        monkeypatch.setenv("PW_EMIT_IMG_BYTES", str(img))
    from test_shard import _with_duplicates_and_comments
    from conftest import synth_paf
    fa, paf = synth_paf(tmp_path, 0, seed=43)
    dup = _with_duplicates_and_comments(paf, tmp_path, 2)
    b = pw.HostBatch(fa, dup, 0)
    n = int(b.view.n_alns)
    res = np.zeros(max(n, 1) * 48, np.uint8)
    z = np.zeros(16, np.uint8)
    ln, st, on, en = b.items(z, res, z)
    k = len(ln)
    out, eb = b.render_range(z, res, z, 0, int(on.sum()), k, int(en.sum()))
    offs = np.concatenate([[0], np.cumsum(on.astype(np.int64))[:-1]]).astype(np.uint64)
    p = tmp_path / "w.bin"
    p.write_bytes(b"")
    fd = os.open(p, os.O_WRONLY)
    try:
        eb2 = b.write_range(z, res, z, fd, 0, offs, int(en.sum()))
    finally:
        os.close(fd)
    assert bytes(out) == p.read_bytes() and eb == eb2
    assert k > 10 and int(en.sum()) > 0
    big = np.full(int(on.sum()) + 64, 0xAB, np.uint8)  # into a caller's buffer (the exchange write's)
    _, eb3 = b.render_range(z, res, z, 0, int(on.sum()), k, int(en.sum()), out=big[16:16 + int(on.sum())])
    assert bytes(big[16:16 + int(on.sum())]) == bytes(out) and eb3 == eb
    assert (big[:16] == 0xAB).all() and (big[16 + int(on.sum()):] == 0xAB).all()


def test_write_range_scattered_destinations(built, tmp_path):
    """pw_batch_write_range with every item's destination out of order (the per-thread pwrite path,
    not the image path): each item's bytes land at its own offset."""
    from conftest import synth_paf
    fa, paf = synth_paf(tmp_path, 0, seed=44)
    b = pw.HostBatch(fa, paf, 0)
    n = int(b.view.n_alns)
    res = np.zeros(max(n, 1) * 48, np.uint8)
    z = np.zeros(16, np.uint8)
    ln, st, on, en = b.items(z, res, z)
    k = len(ln)
    out, eb = b.render_range(z, res, z, 0, int(on.sum()), k, int(en.sum()))
    on = on.astype(np.int64)
    src = np.concatenate([[0], np.cumsum(on)[:-1]])
    order = np.random.default_rng(5).permutation(k)  # item order in the file
    dst = np.zeros(k, np.int64)
    dst[order] = np.concatenate([[0], np.cumsum(on[order])[:-1]])
    p = tmp_path / "s.bin"
    p.write_bytes(b"")
    fd = os.open(p, os.O_WRONLY)
    try:
        b.write_range(z, res, z, fd, 0, dst.astype(np.uint64), int(en.sum()))
    finally:
        os.close(fd)
    got = p.read_bytes()
    ob = bytes(out)
    assert k > 10 and len(got) == len(ob)
    for j in range(k):
        assert got[dst[j]:dst[j] + on[j]] == ob[src[j]:src[j] + on[j]]


def test_host_text_pool():
    """HostTextPool: a free slot large enough is reused, a small free slot is regrown, and with every
    slot busy take() falls back to a fresh tensor (no slot: give(None) is a no-op)."""
    p = mgpu.HostTextPool(2)
    s = []
    a = p.take(100, s)  # slot 0; slot 1 allocated at the same size on the helper thread
    b = p.take(50, s)
    c = p.take(10, s)
    assert s == [0, 1, None] and a.numel() == 100 and b.numel() == 50 and c.numel() == 10
    assert p.bufs[0].numel() == p.bufs[1].numel() >= 150
    p.give(1)
    p.give(None)
    d = p.take(40, s)  # slot 1 fits
    assert s[-1] == 1 and d.data_ptr() == b.data_ptr()
    p.give(0)
    e = p.take(1 << 22, s)  # slot 0 too small: regrown
    assert s[-1] == 0 and e.numel() == 1 << 22


def test_from_buffer_threaded_split_matches_files(built, tmp_path):
    """pw_batch_from_buffer copies and splits its lines on host threads (byte ranges snapped to line
    starts, > 4 MB): the packed batch equals pw_batch_from_files on the same PAF (arrays, and the
    items of a zero-results pass)."""
    from conftest import synth_paf
    fa, paf = synth_paf(tmp_path, 2, seed=7, scale=0.3)
    raw = open(paf, "rb").read()
    assert len(raw) > (12 << 20)
    text = np.frombuffer(raw, np.uint8)
    line_no = np.arange(raw.count(b"\n"), dtype=np.uint64)
    flags = pw.FLAG_G | pw.FLAG_C
    a = pw.HostBatch(fa, paf, flags)
    b = pw.HostBatch.from_buffer(fa, text, line_no, flags, None)
    for name in ("desc", "ops", "lits", "qseq", "qoff", "qlen"):
        assert np.array_equal(a.array(name), b.array(name)), name
    n = int(a.view.n_alns)
    res = np.zeros(max(n, 1) * 48, np.uint8)
    z = np.zeros(16, np.uint8)
    ia, ib = a.items(z, res, z), b.items(z, res, z)
    for x, y in zip(ia, ib):
        assert np.array_equal(x, y)
