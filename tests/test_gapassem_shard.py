"""Multi-GPU GapAssem path (pwasm_amd/gapassem.py): rows sharded over ranks,
partial column histograms summed with one all-reduce, mincol/maxcol/bad-row reduced, refineMSA
on every rank, edited rows gathered on rank 0 — must write the same PWC1 bytes, stderr and exit
code as the single-process oracle.  On the CPU the device work is done by a small numpy model
(ModelEngine, test code: toMSA/bestChar/closed-form refine) so the collective choreography runs
over gloo with world_size 2 and 3; the HIP engine of the same driver is covered on the GPU in
test_gpu_parity.py::test_gapassem_sharded_on_gpu."""
import os
import random
import socket

import numpy as np
import pytest

from conftest import GA_ORACLE, SYNTH, run
from test_gapassem_refine import model, random_layout, read_clips
from test_oracle_kat import write_pwl

INT_MAX = 2 ** 31 - 1


class ModelEngine:
    """CPU stand-in for HipEngine (test infrastructure only)."""

    def stage(self, lay, rows, ncols, nranks=1):
        return dict(lay=lay, rows=list(rows), ncols=ncols)

    def count(self, st):
        import torch
        lay, ncols = st["lay"], st["ncols"]
        cnt = np.zeros((ncols, 6), dtype=np.int32)
        lo_c, hi_c, bad = INT_MAX, -1, INT_MAX
        for k, r in enumerate(st["rows"]):
            cl, cr = lay.clips(r)
            L = int(lay.seqlen[r])
            col = int(lay.offset[r]) - lay.minoffset
            rmin, rmax = INT_MAX, -1
            for i in range(L):
                clipped = i < cl or i >= L - cr
                if not clipped and rmin == INT_MAX:
                    rmin = col
                g = int(lay.ofs[r][i])
                for _ in range(max(g, 0)):
                    if not clipped:
                        if not 0 <= col < ncols:
                            bad = min(bad, k)
                        else:
                            cnt[col, 5] += 1
                    col += 1
                if not 0 <= col < ncols:
                    bad = min(bad, k)
                elif not clipped:
                    ch = chr(lay.seq[r][i]).upper()
                    cnt[col, "ACGT".index(ch) if ch in "ACGT" else (5 if ch in "-*" else 4)] += 1
                    rmax = col
                col += 1
            lo_c, hi_c = min(lo_c, rmin), max(hi_c, rmax)
        st["counts"] = torch.from_numpy(cnt.reshape(-1).copy())
        st["mm"] = torch.tensor([lo_c, hi_c, bad, INT_MAX], dtype=torch.int32)
        return st["counts"], st["mm"]

    def call(self, st):
        c = st["counts"].numpy().reshape(-1, 6)
        cons = np.zeros(len(c), dtype=np.uint8)
        for i, v in enumerate(c):
            if v.sum() == 0:
                continue
            bi = int(np.argmax(v))
            cons[i] = ord("-") if bi == 4 and v[5] == v[4] else ord("ACGTN-"[bi])
        st["cons"] = cons
        lo, hi = int(st["mm"][0]), int(st["mm"][1])
        z = [i for i in range(lo, hi + 1) if lo != INT_MAX and cons[i] == 0]
        st["mm"][3] = z[0] if z else INT_MAX
        return cons, st["mm"]

    def refine_host(self, st, remove_gaps):
        lay, cons = st["lay"], st["cons"]
        lo, hi = int(st["mm"][0]), int(st["mm"][1])
        s = bytes(cons[lo:hi + 1]).replace(b"-", b"" if remove_gaps else b"*")
        rows = {}
        if remove_gaps:
            counts = st["counts"].numpy().reshape(-1, 6).tolist()
            res = dict(minoff=lay.minoffset, mincol=lo, maxcol=hi, length=st["ncols"], counts=counts)
            mine = [(int(lay.offset[r]), bytes(lay.seq[r]).decode(), lay.ofs[r].tolist(), int(lay.clp5[r]),
                     int(lay.clp3[r]), int(lay.rev[r])) for r in st["rows"]]
            for r, (off, ng, ofs) in zip(st["rows"], model(mine, res, clip_gaps=False)):
                rows[r] = (off, ng, np.array(ofs, dtype=np.int16))
        return s, rows


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, world, port, lay, remove, q, refine=True):
    import torch.distributed as dist
    from pwasm_amd import gapassem
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = gapassem.consensus(lay, remove_gaps=remove, engine=ModelEngine(), refine_clipping=refine)
        if rank == 0:
            q.put(res)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _sharded(lay, world, remove, refine=True):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, str(lay), remove, q, refine)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def _oracle(lay, tmp_path, remove, refine=True):
    extra = ([] if refine else ["--no-refine-clipping"]) + (["--remove-gaps"] if remove else [])
    rc, _, err = run([GA_ORACLE, lay, tmp_path / "o.pwc", *extra])
    return rc, err.decode(), (open(tmp_path / "o.pwc", "rb").read() if rc == 0 else None)


@pytest.mark.parametrize("refine", [False, True])
def test_single_process_model_equals_oracle(built, tmp_path, refine):
    """The driver's host per-row tail (pw_ga_row_finish / pw_ga_row_remove_columns through the
    C-ABI: refineClipping X-drop, removeClipGaps, removeColumn replay for deleted bases) on top of
    the model engine, against the oracle's literal refineMSA."""
    from pwasm_amd import gapassem
    n_clip_moves = 0
    for seed in range(10):
        rng = random.Random(900 + seed)
        rows = random_layout(rng, 9, clip=seed % 2 == 1, dels=seed >= 6)
        lay = tmp_path / f"l{seed}.pwl"
        write_pwl(lay, rows)
        for remove in (False, True):
            want = _oracle(lay, tmp_path, remove, refine)
            assert gapassem.consensus(str(lay), remove_gaps=remove, engine=ModelEngine(), refine_clipping=refine) == want
            if want[0] == 0 and refine:
                got = read_clips(want[2], [len(r[1]) for r in rows])
                n_clip_moves += sum(c != (r[3], r[4]) for c, r in zip(got, rows))
    if refine:
        assert n_clip_moves > 0  # refineClipping moved some clip boundary


@pytest.mark.parametrize("world,remove", [(2, True), (2, False), (3, True)])
def test_gloo_sharded_consensus(built, tmp_path, world, remove):
    lay = tmp_path / "s.pwl"
    rc, _, err = run([SYNTH, "layout", "--config", 5, "--scale", 0.0003, "--rows", 7, "--out", lay])
    assert rc == 0, err
    want = _oracle(lay, tmp_path, remove)
    assert want[0] == 0
    assert _sharded(lay, world, remove) == want


def test_gloo_sharded_errors(built, tmp_path):
    # zero-coverage column (exit 5) and a trimmed row warning, reported once in row order
    lay = tmp_path / "z.pwl"
    write_pwl(lay, [(0, "ACG", [0, 0, 0], 0, 0, 0), (0, "ACG", [0, 0, 0], 2, 1, 0), (4, "TT", [0, 0], 0, 0, 1)])
    want = _oracle(lay, tmp_path, False)
    assert want[0] == 5 and "trimmed too badly" in want[1]
    assert _sharded(lay, 2, False) == want


def test_shard_rows_balanced_and_nonempty():
    from pwasm_amd.gapassem import shard_rows
    assert shard_rows([10, 10, 10, 10], 2) == [(0, 2), (2, 4)]
    b = shard_rows([1000, 1, 1, 1], 4)
    assert [hi - lo for lo, hi in b] == [1, 1, 1, 1]
    b = shard_rows([5] * 9, 3)
    assert b == [(0, 3), (3, 6), (6, 9)]


def test_finish_rows_message_overflow(built, tmp_path, monkeypatch):
    """pw_ga_rows_finish with a message buffer far too small: the overflowing call must leave every
    row as it was, so the retry with the reported size applies each row's edits exactly once
    (a retry on already-edited rows applied removeColumn / refineClipping twice)."""
    from pwasm_amd import gapassem
    real = gapassem.finish_rows
    monkeypatch.setattr(gapassem, "finish_rows", lambda *a, **k: real(*a, **{**k, "msg_cap": 1}))
    with_msgs = 0
    for seed in range(10):
        rng = random.Random(900 + seed)
        rows = random_layout(rng, 9, clip=True, dels=seed >= 5)
        lay = tmp_path / f"m{seed}.pwl"
        write_pwl(lay, rows)
        for remove in (False, True):
            want = _oracle(lay, tmp_path, remove)
            with_msgs += bool(want[1])
            assert gapassem.consensus(str(lay), remove_gaps=remove, engine=ModelEngine()) == want
    assert with_msgs > 0  # some row printed a message, so the first call overflowed
